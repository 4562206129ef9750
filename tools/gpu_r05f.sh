#!/bin/bash
# round 5: axis_angle's correctly rounded normalisations (legacy_spring
# Grasp's 2-dof thumb): the SINGLE rollouts vs the previous build, the whole
# GPU suite with the per-env gate asserting, smoke, and the MULTI A/B of the
# Newton-corrected body quotients (_lib) against the fast ones (_lib_fq) and
# the round's starting build (_lib_prev).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r05f}
BRAX_AMD_LIB=brax_amd/_lib_prev/libbrax_amd.so timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_prev.npz > gpurun_out/bc_$TAG.log 2>&1 || exit 3
timeout -k 10 200 python tools/bitcmp.py save gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1 || exit 3
python tools/bitcmp.py cmp gpurun_out/bc_prev.npz gpurun_out/bc_new.npz >> gpurun_out/bc_$TAG.log 2>&1
grep -v bitwise gpurun_out/bc_$TAG.log | grep -v amdgpu.ids | tail -8
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
tail -1 gpurun_out/smoke_$TAG.log
bash tools/multi_ab.sh $TAG fq prev || exit 6
exit $rc
