# the MULTI kernel's wait split: vector-memory / LDS / scalar instruction
# counts and the L2 (TCC) and L1 (TCP) request volume, Info off, 2,048 envs
# (tools/multi_traffic.py; one --pmc pass per block group)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/mq/sq -o run --output-format csv -- python3 tools/multi_traffic.py noinfo > gpurun_out/mq_sq.log 2>&1 || exit 5
timeout -s KILL 90 rocprofv3 --pmc TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/mq/tc -o run --output-format csv -- python3 tools/multi_traffic.py noinfo > gpurun_out/mq_tc.log 2>&1 || exit 6
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/mq/sq_ant -o run --output-format csv -- python3 tools/env_prof.py ant > gpurun_out/mq_sq_ant.log 2>&1 || exit 7
exit 0
