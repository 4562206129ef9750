#!/bin/bash
# MULTI joint phases ordered by a wave fence when their lanes all sit in the
# first wave (default) against the workgroup barriers (_lib_nw,
# BX_MULTI_NO_WSYNC): bitwise states, the Mountain tests, the A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05ai}
timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_base.npz > gpurun_out/mb_$TAG.log 2>&1 || exit 3
BRAX_AMD_LIB=brax_amd/_lib_nw/libbrax_amd.so timeout -k 10 200 python tools/multi_bitcmp.py save gpurun_out/mb_nw.npz >> gpurun_out/mb_$TAG.log 2>&1 || exit 3
python tools/multi_bitcmp.py cmp gpurun_out/mb_base.npz gpurun_out/mb_nw.npz >> gpurun_out/mb_$TAG.log 2>&1
tail -4 gpurun_out/mb_$TAG.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "mountain or near or cull" > gpurun_out/pyt_m_$TAG.log 2>&1 || { tail -30 gpurun_out/pyt_m_$TAG.log; exit 6; }
tail -1 gpurun_out/pyt_m_$TAG.log
bash tools/multi_ab.sh $TAG nw
