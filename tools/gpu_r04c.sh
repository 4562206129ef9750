# the GPU suite (every failure listed), smoke, stamps / mstamps diagnostics,
# the rocprof + PMC passes and the driver's bench command
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04c}
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
# diagnostics: a Python error (e.g. a stale diagnostic build) skips the step;
# a time limit, abort or fault ends the script
diag() { "$@"; local r=$?; case $r in 0|1|2) return 0;; *) exit $r;; esac; }
if [ -f brax_amd/_lib_stamps/libbrax_amd.so ]; then
  BRAX_AMD_LIB=brax_amd/_lib_stamps/libbrax_amd.so diag timeout -k 10 120 python tools/stamps.py ant > gpurun_out/stamps_${TAG}_ant.log 2>&1
  BRAX_AMD_LIB=brax_amd/_lib_stamps/libbrax_amd.so diag timeout -k 10 120 python tools/stamps.py humanoid > gpurun_out/stamps_${TAG}_humanoid.log 2>&1
fi
if [ -f brax_amd/_lib_mstamps/libbrax_amd.so ]; then
  BRAX_AMD_LIB=brax_amd/_lib_mstamps/libbrax_amd.so diag timeout -k 10 120 python tools/mstamps.py 0 > gpurun_out/mstamps_${TAG}_0.log 2>&1
fi
diag timeout -k 10 120 python tools/lanes_ab.py humanoid ant halfcheetah > gpurun_out/lanes_ab_$TAG.log 2>&1
# the Humanoid long-horizon drift of an IEEE-division / IEEE-sqrt build (A/B)
if [ -f brax_amd/_lib_precise/libbrax_amd.so ]; then
  cp gpurun_out/long_horizon_humanoid.json gpurun_out/long_horizon_humanoid_$TAG.json 2>/dev/null
  cp gpurun_out/long_horizon_ant.json gpurun_out/long_horizon_ant_$TAG.json 2>/dev/null
  BRAX_AMD_LIB=brax_amd/_lib_precise/libbrax_amd.so diag timeout -k 10 300 python -u -m pytest tests/test_gpu_long_horizon.py -k humanoid -q -p no:cacheprovider > gpurun_out/long_horizon_precise_$TAG.log 2>&1
  cp gpurun_out/long_horizon_humanoid.json gpurun_out/long_horizon_humanoid_precise_$TAG.json 2>/dev/null
fi
bash tools/run_prof.sh $TAG || exit 7
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 || exit 8
exit $rc
