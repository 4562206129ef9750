#!/bin/bash
# GPU parity suite against the default library and the IEEE-generic variant
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_fast.log 2>&1
echo "fast rc=$?"; tail -8 gpurun_out/pytest_fast.log | grep -i "passed\|failed"
BRAX_AMD_LIB=brax_amd/_lib_gp/libbrax_amd.so timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gp.log 2>&1
echo "gp rc=$?"; tail -8 gpurun_out/pytest_gp.log | grep -i "passed\|failed"
exit 0
