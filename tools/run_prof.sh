#!/bin/bash
# rocprofv3 passes over bench.py: kernel-trace stats, then separate PMC passes
# (FETCH_SIZE, WRITE_SIZE, SQ counters), each in its own run.
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
ARGS="--steps 300 --warmup 30 --no-cpu-baseline --phase-envs 1048576"
PARGS="--steps 50 --warmup 5 --no-cpu-baseline --phase-envs 1048576"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py $ARGS > $OUT.trace.log 2>&1 || { echo trace failed; tail -20 $OUT.trace.log; exit 1; }
tail -1 $OUT.trace.log
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py $PARGS > $OUT.fetch.log 2>&1 || { echo fetch failed; tail -20 $OUT.fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py $PARGS > $OUT.write.log 2>&1 || { echo write failed; tail -20 $OUT.write.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE -d $OUT/sq -o run --output-format csv -- python3 bench.py $PARGS > $OUT.sq.log 2>&1 || { echo sq failed; tail -20 $OUT.sq.log; }
# the stall split (MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY +
# ACTIVE_INST_ANY ~ WAVE_CYCLES; WAIT_INST_LDS a sub-bucket of WAIT_INST_ANY)
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/sq2 -o run --output-format csv -- python3 bench.py $PARGS > $OUT.sq2.log 2>&1 || { echo sq2 failed; tail -20 $OUT.sq2.log; }
find $OUT -name "*.csv"
