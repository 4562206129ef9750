#!/bin/bash
# round 5: IEEE division in the legacy_spring impulse functions, the per-env
# gate asserting: bitwise comparison of the SINGLE-kernel rollouts against the
# previous build (brax_amd/_lib_prev), then the whole GPU suite with the
# per-env gate recording (asserting), then the driver's bench command.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05c}
if [ -f brax_amd/_lib_prev/libbrax_amd.so ]; then
  BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_prev.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
  timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
  python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1
  tail -5 gpurun_out/bc_$TAG.log
fi
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-phases --no-secondary --no-cpu-baseline > gpurun_out/bench20_$TAG.log 2>&1 || exit 8
python tools/bench_line.py gpurun_out/bench20_$TAG.log
exit $rc
