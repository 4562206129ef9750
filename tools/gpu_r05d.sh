#!/bin/bash
# round 5: the MULTI kernel's split row image (geometry for every near row,
# impulse constants for penetrating rows only) and the correctly rounded
# Angle-actuator target: bitwise SINGLE rollouts vs brax_amd/_lib_prev, the
# whole GPU suite (per-env gate asserting), smoke, the MULTI A/B.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05d}
BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_prev.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -c bitwise gpurun_out/bc_$TAG.log
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
tail -1 gpurun_out/smoke_$TAG.log
bash tools/multi_ab.sh $TAG prev || exit 6
exit $rc
