#!/bin/bash
# MULTI joint halves with the damping folded into the actuator slots against the
# unfolded build (_lib_nf, BX_MULTI_NOFOLD): the Mountain tests, the A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05af}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "mountain or near or cull" > gpurun_out/pyt_m_$TAG.log 2>&1 || { tail -30 gpurun_out/pyt_m_$TAG.log; exit 6; }
tail -1 gpurun_out/pyt_m_$TAG.log
bash tools/multi_ab.sh $TAG nf
