#!/bin/bash
# one-step kernels for every env's Env.step: GPU suite, then the 17-env scan
# on this build and on the base build, interleaved
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06w}
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
for v in _lib _lib_base _lib; do
  BRAX_AMD_LIB=brax_amd/$v/libbrax_amd.so timeout -k 10 300 python tools/env_scan.py > gpurun_out/env_scan_${TAG}$v.log 2>&1 || exit 9
  echo "== $v"; grep -v "^{\"batch\|amdgpu.ids" gpurun_out/env_scan_${TAG}$v.log | python3 -c "
import sys, json
for l in sys.stdin:
    k, _, j = l.partition(' ')
    try: print(k, json.loads(j)['gpu_us_per_step'].__round__(1))
    except Exception: pass
" | tr '\n' ' '; echo
done
exit $rc
