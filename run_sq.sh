#!/bin/bash
mkdir -p gpurun_out
export TMPDIR=/tmp
OUT=gpurun_out/sq_$1
shift
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -d $OUT -o run --output-format csv -- python3 bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > $OUT.log 2>&1 || { tail -20 $OUT.log; exit 1; }
python3 - $OUT <<'PY'
import csv, collections, sys
rows=list(csv.DictReader(open(sys.argv[1]+'/run_counter_collection.csv')))
agg=collections.defaultdict(list)
for r in rows:
    if 'env_step' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
waves=1024
for k,v in sorted(agg.items()):
    print(f"{k:24s} per-dispatch {sum(v)/len(v):14.0f}")
PY
