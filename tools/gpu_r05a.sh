#!/bin/bash
# round 5, first GPU pass: the per-env parity gate in record-only mode (every
# env's HIP_i / max(1e-5, 2 E32_i), 66 fp32 realisations per env) for the
# default build and for PRECISE=1 (IEEE division), then the `bench.py --gpus 2`
# rehearsal (the parent spawns its ranks; gloo, both on GPU 0), smoke and the
# driver's bench command.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05a}
BX_PARITY_RECORD_ONLY=1 bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
if [ -f brax_amd/_lib_precise/libbrax_amd.so ]; then
  BX_PARITY_RECORD_ONLY=1 BRAX_AMD_LIB=brax_amd/_lib_precise/libbrax_amd.so \
    bash tools/gpu_suite.sh ${TAG}_precise tests/test_gpu_parity.py tests/test_gpu_scale.py; r2=$?
  [ $r2 -le 1 ] || exit $r2
fi
bash tools/rehearse_2rank.sh $TAG || exit 5
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/bench20_$TAG.log 2>&1 || exit 8
python tools/bench_line.py gpurun_out/bench20_$TAG.log
exit $rc
