# the Humanoid drift under the rounding builds, then the spherical halves'
# tests and the Humanoid parity gates (default and halves)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04f}
bash tools/gpu_drift_ab.sh $TAG || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_sph_halves.py tests/test_gpu_parity.py -k "sph or humanoid" -v --timeout 170 --timeout-method thread -p no:cacheprovider > gpurun_out/hum_$TAG.log 2>&1
r=$?; grep -E "passed|failed" gpurun_out/hum_$TAG.log | tail -3; exit $r
