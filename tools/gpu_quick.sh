# quick GPU pass: the given test files, smoke, then the driver's bench
# command and a 1000-step bench (no secondary legs)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-q}; shift
if [ $# -gt 0 ]; then bash tools/gpu_tests.sh $TAG "$@" || exit 1; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/bench20_${TAG}_$i.log 2>&1 || { tail -20 gpurun_out/bench20_${TAG}_$i.log; exit 1; }
python tools/bench_line.py gpurun_out/bench20_${TAG}_$i.log
done
timeout -k 10 300 python bench.py --steps 1000 --warmup 50 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/bench1000_$TAG.log 2>&1 || { tail -20 gpurun_out/bench1000_$TAG.log; exit 1; }
python tools/bench_line.py gpurun_out/bench1000_$TAG.log
