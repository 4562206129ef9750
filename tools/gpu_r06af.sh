#!/bin/bash
# round 6 record of one build: the whole GPU suite (per-env gate asserting)
# + margins, smoke, the driver's 20-step command, the default bench (CPU
# baseline leg included), the rocprof kernel-trace + PMC passes
# (tools/run_prof.sh), the 2-rank `--gpus 2` rehearsal.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r06af}
bash tools/gpu_suite.sh $TAG; rc=$?
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 4
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench20_$TAG.log 2>&1 || exit 8
python tools/bench_line.py gpurun_out/bench20_$TAG.log
timeout -k 10 500 python bench.py > gpurun_out/bench_default_$TAG.log 2>&1 || exit 9
python tools/bench_line.py gpurun_out/bench_default_$TAG.log
bash tools/run_prof.sh $TAG || exit 10
bash tools/rehearse_2rank.sh $TAG || exit 11
timeout -k 10 60 python tools/check_parent_nohip.py 2 > gpurun_out/parent_nohip_$TAG.log 2>&1 || exit 12
tail -1 gpurun_out/parent_nohip_$TAG.log
exit $rc
