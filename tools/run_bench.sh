#!/bin/bash
# Default bench (with the CPU baseline leg) -> gpurun_out/bench_<tag>.log
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r01}
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
