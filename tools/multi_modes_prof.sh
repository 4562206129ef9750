#!/bin/bash
# Per-mode rocprofv3 record of the MULTI kernel (Ant Mountain(4), 2,048 envs):
# for each of Info on / off x cutoff 0 / 36, a kernel-trace pass, FETCH_SIZE
# and WRITE_SIZE passes and an SQ pass, each in its own run of
# tools/multi_traffic.py (30 launches of that one mode), so every figure
# names one configuration. Summarised by tools/multi_modes_summary.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r06}
OUT=gpurun_out/mmodes_$TAG
mkdir -p $OUT
for mode in noinfo info; do
  for cut in 0 36; do
    M=$OUT/${mode}_$cut
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $M/trace -o run --output-format csv -- python3 tools/multi_traffic.py $mode $cut > $M.trace.log 2>&1 || { echo "trace $mode $cut failed"; tail -5 $M.trace.log; exit 1; }
    tail -1 $M.trace.log
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $M/fetch -o run --output-format csv -- python3 tools/multi_traffic.py $mode $cut > $M.fetch.log 2>&1 || { echo "fetch $mode $cut failed"; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $M/write -o run --output-format csv -- python3 tools/multi_traffic.py $mode $cut > $M.write.log 2>&1 || { echo "write $mode $cut failed"; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU -d $M/sq -o run --output-format csv -- python3 tools/multi_traffic.py $mode $cut > $M.sq.log 2>&1 || { echo "sq $mode $cut failed"; exit 1; }
  done
done
python3 tools/multi_modes_summary.py $OUT $TAG
