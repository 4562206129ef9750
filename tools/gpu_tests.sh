# GPU test suite (or the test files given) -> gpurun_out/pytest_<tag>.log; stops on failure
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-all}; shift
timeout -k 10 900 python -u -m pytest ${@:-tests} -m gpu -x -v -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/pytest_$TAG.log | tail -15
exit $rc
