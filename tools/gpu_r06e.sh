#!/bin/bash
# checkpoint of the NaN commit: the whole GPU suite + margins, smoke, the
# driver's command, the RCCL spawn parent on the one-GPU box, the 17-env scan
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06e}
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 60 python tools/check_parent_nohip.py 2 > gpurun_out/parent_nohip_$TAG.log 2>&1; echo "parent check rc $?"; cat gpurun_out/parent_nohip_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 || exit 8
python tools/bench_line.py gpurun_out/bench20_$TAG.log
timeout -k 10 300 python tools/env_scan.py > gpurun_out/env_scan_$TAG.log 2>&1 || exit 9
tail -20 gpurun_out/env_scan_$TAG.log
exit $rc
