#!/bin/bash
# SQ counter passes on the fused env-step kernel (bench, no phase leg)
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sq}
OUT=gpurun_out/$TAG
A="--steps 20 --warmup 5 --no-cpu-baseline --no-phases"
timeout -k 10 120 rocprofv3 -L > $OUT.list.txt 2>&1 || true
grep -oE "SQ_[A-Z_0-9]+" $OUT.list.txt | sort -u > $OUT.sqnames.txt || true
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SALU -d $OUT/p1 -o run --output-format csv -- python3 bench.py $A > $OUT.p1.log 2>&1 || { tail -5 $OUT.p1.log; exit 1; }
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_IFETCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_LDS -d $OUT/p2 -o run --output-format csv -- python3 bench.py $A > $OUT.p2.log 2>&1 || { tail -5 $OUT.p2.log; exit 1; }
echo ok
