#!/bin/bash
# GPU: phase-kernel parity, full gpu suite, bench with the phase roofline leg.
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_phases.py -q -p no:cacheprovider > gpurun_out/pytest_phases.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_phases.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc2=$?; tail -5 gpurun_out/pytest_gpu.log
if [ $rc2 -ne 0 ] && [ $rc2 -ne 1 ]; then exit $rc2; fi
timeout -k 10 300 python bench.py --steps 500 --warmup 50 --no-cpu-baseline > gpurun_out/bench_phase.log 2>&1 || exit $?
tail -1 gpurun_out/bench_phase.log
