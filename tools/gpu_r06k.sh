#!/bin/bash
# MULTI: Mountain tests, bitwise 128 vs 256 lanes, timing against round 5's
# library in the early (10 warm steps) and the piled-up (200) state
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06k}
timeout -k 10 400 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_nan.py -k "mountain or twin_cull" -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_mtn_$TAG.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|Timeout" gpurun_out/pytest_mtn_$TAG.log | tail -15
[ $rc -le 1 ] || exit $rc
for l in 128 256; do
  BX_MULTI_LANES=$l timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_$l.npz > gpurun_out/mbc_$TAG.log 2>&1 || { tail -5 gpurun_out/mbc_$TAG.log; exit 5; }
done
python tools/multi_bitcmp.py cmp gpurun_out/mb_128.npz gpurun_out/mb_256.npz | grep -c bitwise
for warm in 10 200; do
  export BX_MULTI_WARM=$warm
  for v in "_lib_prev default" "_lib 128"; do
    set -- $v
    if [ $2 = default ]; then unset BX_MULTI_LANES; else export BX_MULTI_LANES=$2; fi
    BRAX_AMD_LIB=brax_amd/$1/libbrax_amd.so timeout -k 10 300 python tools/multi_ab.py > gpurun_out/mab.tmp 2>&1 || { tail -5 gpurun_out/mab.tmp; exit 4; }
    tail -1 gpurun_out/mab.tmp | tee -a gpurun_out/multi_ab_$TAG.log
  done
done
