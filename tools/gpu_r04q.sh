# the round-end record at HEAD (kernels unchanged since r04m; the parity
# tests' ill-conditioned gates now binding): the full GPU suite, smoke, the
# driver's 20-step bench command and the default bench
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04q}
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
for e in ant humanoid; do cp gpurun_out/long_horizon_$e.json gpurun_out/long_horizon_${e}_$TAG.json 2>/dev/null; done
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 || exit 8
timeout -k 10 400 python bench.py > gpurun_out/bench_default_$TAG.log 2>&1 || exit 9
exit $rc
