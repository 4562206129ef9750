"""Per-wave SQ counters of the env-step kernel from a run_sq.sh output dir."""
import collections
import csv
import sys

d = sys.argv[1]
for p in ('p1', 'p2'):
  acc = collections.defaultdict(list)
  for r in csv.DictReader(open(f'{d}/{p}/run_counter_collection.csv')):
    if 'env_step' in r['Kernel_Name']:
      acc[r['Counter_Name']].append(float(r['Counter_Value']))
  waves = 1024
  print(p, ' '.join(f'{k.replace("SQ_", "")}={sum(v) / len(v) / waves:.0f}' for k, v in acc.items()))
