#!/bin/bash
# SQ counters of one env's step kernel across library builds (A/B):
#   bash tools/sq_ab.sh TAG ENV lib_dir...   (lib dirs under brax_amd/, e.g. _lib _lib_base)
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=$1; E=$2; shift 2
for n in "$@"; do
  OUT=gpurun_out/sqab_${TAG}_${E}_$n
  BRAX_AMD_LIB=brax_amd/$n/libbrax_amd.so timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY -d $OUT -o run --output-format csv -- python3 tools/env_prof.py $E --steps 5 > $OUT.log 2>&1 || { echo "$n failed"; tail -5 $OUT.log; exit 1; }
  python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + '/**/run_counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
  if 'env_step' in r['Kernel_Name']:
    acc[r['Counter_Name']].append(float(r['Counter_Value']))
m = {k: sum(v) / len(v) for k, v in acc.items()}
w = m.get('SQ_WAVES', 1)
print(sys.argv[1].split('sqab_')[1], {k: round(v / w, 1) for k, v in sorted(m.items()) if k != 'SQ_WAVES'})
PY
done
