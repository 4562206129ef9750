#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for n in _lib _lib_prev _lib_pk; do
  BRAX_AMD_LIB=brax_amd/$n/libbrax_amd.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/diag_$n -o run --output-format csv -- python3 tools/diag_rollout_graph.py > gpurun_out/diag_$n.log 2>&1 || exit 2
  grep "us/step" gpurun_out/diag_$n.log
  python3 - gpurun_out/diag_$n <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
  if 'env_' in r['Name'] or 'uniform' in r['Name']:
    print('   ', r['Name'][:90], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
