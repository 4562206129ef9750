# the spherical joint halves (partner exchange, bit-identity with the 16-lane
# kernel, timing A/B), the MULTI occupancy scan (this tree, its 128-VGPR
# variant and the pre-diet build under ab_prediet/), the full GPU suite, then
# the Humanoid drift under the division / square-root rounding builds
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04d}
ok() { local r=$1; case $r in 0|1) return 0;; *) exit $r;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_sph_halves.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/sph_$TAG.log 2>&1; ok $?
timeout -k 10 150 python -u tools/sph_ab.py > gpurun_out/sph_ab_$TAG.log 2>&1; ok $?
timeout -k 10 150 python -u tools/multi_occ.py 0 > gpurun_out/occ_cur_$TAG.log 2>&1; ok $?
BX_MULTI_WPE=4 timeout -k 10 150 python -u tools/multi_occ.py 0 > gpurun_out/occ_w4_$TAG.log 2>&1; ok $?
if [ -d ab_prediet ]; then
  timeout -k 10 150 python -u ab_prediet/tools/multi_occ.py 0 > gpurun_out/occ_pre_$TAG.log 2>&1; ok $?
fi
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
bash tools/gpu_drift_ab.sh $TAG || exit $?
exit $rc
