# GPU test suite (or the pytest args given) -> gpurun_out/pytest_<tag>.log; stops on failure
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-all}; shift
if [ $# -eq 0 ]; then set -- tests; fi
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/pytest_$TAG.log | tail -15
exit $rc
