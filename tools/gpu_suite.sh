#!/bin/bash
# The whole GPU suite without stopping at the first failure (every failing
# gate reported) -> gpurun_out/pytest_<tag>.log, then the margins file
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-all}; shift
if [ $# -eq 0 ]; then set -- tests; fi
timeout -k 10 1000 python -u -m pytest "$@" -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
cp gpurun_out/parity_margins.json gpurun_out/parity_margins_$TAG.json 2>/dev/null
grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/pytest_$TAG.log | tail -25
exit $rc
