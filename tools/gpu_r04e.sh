# validation of a kernel change set: the opt-in spherical halves, the MULTI
# occupancy scan, the full GPU suite (+ long-horizon JSONs), smoke, the
# halves A/B, then the rocprof + PMC profile and the driver's bench command
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04e}
ok() { local r=$1; case $r in 0|1) return 0;; *) exit $r;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_sph_halves.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sph_$TAG.log 2>&1; ok $?
timeout -k 10 150 python -u tools/multi_occ.py 0 > gpurun_out/occ_$TAG.log 2>&1; ok $?
timeout -k 10 150 python -u tools/multi_occ.py 36 256 512 768 1024 2048 >> gpurun_out/occ_$TAG.log 2>&1; ok $?
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
for e in ant humanoid; do cp gpurun_out/long_horizon_$e.json gpurun_out/long_horizon_${e}_$TAG.json 2>/dev/null; done
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
timeout -k 10 150 python -u tools/sph_ab.py > gpurun_out/sph_ab_$TAG.log 2>&1; ok $?
bash tools/run_prof.sh $TAG || exit 7
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 || exit 8
# against the previous build, when one is staged (brax_amd/_lib_prev)
if [ -f brax_amd/_lib_prev/libbrax_amd.so ]; then bash tools/gpu_ab_prev.sh ab_$TAG || exit 9; fi
exit $rc
