#!/bin/bash
# MULTI joint halves (H.mjh; BX_NO_MULTI_JH=1: one lane per joint): the MULTI
# parity tests under both, then the interleaved A/B
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05s}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "mountain" > gpurun_out/pyt_m_$TAG.log 2>&1 || { tail -30 gpurun_out/pyt_m_$TAG.log; exit 6; }
tail -1 gpurun_out/pyt_m_$TAG.log
for round in 1 2; do
  for v in 0 1; do
    BX_NO_MULTI_JH=$v timeout -k 10 200 python tools/multi_ab.py > gpurun_out/mab.tmp 2>&1 || { tail -5 gpurun_out/mab.tmp; exit 4; }
    echo "no_mjh=$v $(tail -1 gpurun_out/mab.tmp)" | tee -a gpurun_out/multi_ab_$TAG.log
  done
done
