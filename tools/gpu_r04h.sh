# the Humanoid drift with IEEE division in one function group at a time, and
# the MULTI kernel at three waves per SIMD against two
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r04h}
ok() { local r=$1; case $r in 0|1) return 0;; *) exit $r;; esac; }
bash tools/gpu_drift_ab.sh $TAG || exit $?
timeout -k 10 150 python -u tools/multi_occ.py 0 256 512 768 1024 2048 > gpurun_out/occ_w2_$TAG.log 2>&1; ok $?
BX_MULTI_WPE=3 timeout -k 10 150 python -u tools/multi_occ.py 0 256 512 768 1024 2048 > gpurun_out/occ_w3_$TAG.log 2>&1; ok $?
