#!/bin/bash
# round 5: the single-step kernel's prologue part by part (BX_PSTAMPS build),
# the MULTI A/B (geometry + impulse-constant loads together in the position
# pass, none for non-penetrating rows in the velocity pass), and the
# legacy_spring Grasp gate's failing samples dumped for offline analysis.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05e}
for e in ant humanoid; do
  BRAX_AMD_LIB=brax_amd/_lib_pst/libbrax_amd.so timeout -k 10 120 python tools/pstamps.py $e > gpurun_out/pstamps_${e}_$TAG.log 2>&1 || exit 2
  cat gpurun_out/pstamps_${e}_$TAG.log | grep -v amdgpu.ids
done
bash tools/multi_ab.sh $TAG prev || exit 6
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "grasp_spring or mountain" -m gpu -q -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
tail -3 gpurun_out/pytest_$TAG.log
ls gpurun_out/gate_fail_* 2>/dev/null
exit 0
