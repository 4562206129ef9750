#!/bin/bash
# rocprofv3 passes over single-env step runs: kernel trace, then two SQ
# counter passes (each its own run). usage: bash tools/run_env_prof.sh TAG env...
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
for E in "$@"; do
  OUT=gpurun_out/eprof_${TAG}_$E
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/env_prof.py $E > $OUT.trace.log 2>&1 || { echo "$E trace failed"; tail -5 $OUT.trace.log; exit 1; }
  tail -1 $OUT.trace.log
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_INSTS_SALU SQ_ACTIVE_INST_VALU -d $OUT/sq -o run --output-format csv -- python3 tools/env_prof.py $E --steps 5 > $OUT.sq.log 2>&1 || { echo "$E sq failed"; tail -5 $OUT.sq.log; exit 1; }
done
echo ok
