#!/bin/bash
# NearNeighbors lists by a per-wave bitonic sort (MULTI): the NearNeighbors /
# Mountain tests, the stamps of the culled scene, the A/B line
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05v}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_scale.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "mountain or near or cull" > gpurun_out/pyt_m_$TAG.log 2>&1 || { tail -30 gpurun_out/pyt_m_$TAG.log; exit 6; }
tail -1 gpurun_out/pyt_m_$TAG.log
BRAX_AMD_LIB=brax_amd/_lib_mst/libbrax_amd.so timeout -k 10 200 python tools/mstamps.py 36 > gpurun_out/mstamps_${TAG}_36.log 2>&1 || exit 3
grep -v amdgpu.ids gpurun_out/mstamps_${TAG}_36.log | head -3
for round in 1 2; do
  timeout -k 10 200 python tools/multi_ab.py > gpurun_out/mab.tmp 2>&1 || { tail -5 gpurun_out/mab.tmp; exit 4; }
  tail -1 gpurun_out/mab.tmp | tee -a gpurun_out/multi_ab_$TAG.log
done
