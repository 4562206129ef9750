# Humanoid long-horizon drift (tests/test_gpu_long_horizon.py) under builds
# that differ only in fp32 division / square-root rounding (diagnostic A/B)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04e}
for L in _lib _lib_iCONTACT _lib_iBODY _lib_iJOINT; do
  [ -f brax_amd/$L/libbrax_amd.so ] || continue
  BRAX_AMD_LIB=brax_amd/$L/libbrax_amd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_long_horizon.py -k humanoid -q -p no:cacheprovider > gpurun_out/drift_${TAG}_$L.log 2>&1
  r=$?; case $r in 0|1) ;; *) exit $r;; esac
  cp gpurun_out/long_horizon_humanoid.json gpurun_out/drift_${TAG}_$L.json
done
