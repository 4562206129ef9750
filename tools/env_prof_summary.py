"""Per-kernel summary of run_env_prof.sh output: average duration at the
most frequent grid, and per-wave SQ counters (VALU / LDS instructions, wave
cycles, waits), VGPRs and scratch of the env-step kernels.

    python tools/env_prof_summary.py gpurun_out/eprof_<tag>_<env> ...
"""
import collections
import csv
import json
import sys


def summarize(d):
  out = {}
  tr = collections.defaultdict(list)
  for r in csv.DictReader(open(f'{d}/trace/run_kernel_trace.csv')):
    if 'env_step' not in r['Kernel_Name']:
      continue
    k = r['Kernel_Name'].split('(')[0].replace('void ', '')
    tr[k].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
  for k, v in tr.items():
    out[k] = {'calls': len(v), 'avg_us': sum(v) / len(v) / 1e3}
  acc = collections.defaultdict(lambda: collections.defaultdict(list))
  meta = {}
  for r in csv.DictReader(open(f'{d}/sq/run_counter_collection.csv')):
    if 'env_step' not in r['Kernel_Name']:
      continue
    k = r['Kernel_Name'].split('(')[0].replace('void ', '')
    acc[k][r['Counter_Name']].append(float(r['Counter_Value']))
    meta[k] = {'vgpr': int(r['VGPR_Count']), 'agpr': int(r.get('Accum_VGPR_Count', 0) or 0),
               'scratch': int(r['Scratch_Size']), 'lds': int(r['LDS_Block_Size'])}
  for k, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    w = m.get('SQ_WAVES', 1)
    e = out.setdefault(k, {})
    e.update(meta.get(k, {}))
    e['waves'] = w
    e['valu_per_wave'] = m.get('SQ_INSTS_VALU', 0) / w
    e['lds_per_wave'] = m.get('SQ_INSTS_LDS', 0) / w
    e['salu_per_wave'] = m.get('SQ_INSTS_SALU', 0) / w
    cyc = 4 * m.get('SQ_WAVE_CYCLES', 0) / w
    e['cycles_per_wave'] = cyc
    e['valu_issue_frac'] = 4 * e['valu_per_wave'] / cyc if cyc else None
    e['wait_lds_frac'] = 4 * m.get('SQ_WAIT_INST_LDS', 0) / w / cyc if cyc else None
    e['wait_any_frac'] = 4 * m.get('SQ_WAIT_ANY', 0) / w / cyc if cyc else None
  return out


if __name__ == '__main__':
  res = {d: summarize(d) for d in sys.argv[1:]}
  print(json.dumps(res, indent=1))
