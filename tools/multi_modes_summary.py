"""Summarise tools/multi_modes_prof.sh into profiles/<tag>_multi_modes.json.

    python tools/multi_modes_summary.py gpurun_out/mmodes_<tag> <tag>

Per mode (Info on / off x cutoff 0 / 36) of the MULTI kernel: the average
launch (kernel trace), HBM bytes per launch and per env-step (2 x FETCH_SIZE +
WRITE_SIZE, KB -> B, the gfx950 correction of MI355X_MICROARCH.md, as
tools/prof_summary.py) against the algorithmic bytes per env-step
tools/multi_traffic.py prints, and the SQ issue split per wave (SQ_WAVE_CYCLES
in quad-cycles).
"""
import csv
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _rows(p, kern='system_step_multi_kernel'):
  if not os.path.exists(p):
    return []
  with open(p) as f:
    return [r for r in csv.DictReader(f) if kern in r['Kernel_Name']]


def _mean(v):
  return sum(v) / len(v) if v else None


def mode(d):
  out = {}
  with open(d + '.trace.log') as f:
    line = [l for l in f if l.startswith('mode ')][-1].split()
  kv = dict(zip(line[0::2], line[1::2]))
  envs = int(kv['envs'])
  alg = int(kv['algorithmic_bytes_per_env_step'])
  tr = _rows(os.path.join(d, 'trace', 'run_kernel_trace.csv'))
  dur = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in tr]
  out['kernel'] = tr[0]['Kernel_Name'].split('(')[0].replace('void ', '') if tr else None
  out['launches'] = len(dur)
  out['avg_us'] = _mean(dur) / 1e3 if dur else None
  # the later half: past the drop's first contacts
  out['avg_us_last_half'] = _mean(dur[len(dur) // 2:]) / 1e3 if dur else None
  out['system_steps_per_s'] = envs / (out['avg_us'] * 1e-6) if dur else None
  c = defaultdict(list)
  for sub in ('fetch', 'write', 'sq'):
    for r in _rows(os.path.join(d, sub, 'run_counter_collection.csv')):
      c[r['Counter_Name']].append(float(r['Counter_Value']))
      out.setdefault('vgpr', int(r['VGPR_Count']))
      out.setdefault('lds_bytes', int(r['LDS_Block_Size']))
      out.setdefault('scratch', int(r['Scratch_Size']))
      out.setdefault('workgroup', int(r['Workgroup_Size']))
  m = {k: _mean(v) for k, v in c.items()}
  if 'FETCH_SIZE' in m and 'WRITE_SIZE' in m:
    rd, wr = 2 * m['FETCH_SIZE'] * 1024, m['WRITE_SIZE'] * 1024
    out['hbm_read_bytes_per_env_step'] = rd / envs
    out['hbm_write_bytes_per_env_step'] = wr / envs
    out['hbm_bytes_per_env_step'] = (rd + wr) / envs
    out['raw_fetch_bytes_per_env_step'] = m['FETCH_SIZE'] * 1024 / envs
    out['algorithmic_bytes_per_env_step'] = alg
    out['info_bytes_per_env_step'] = int(kv.get('info_bytes', 0))
    out['traffic_over_algorithmic'] = (rd + wr) / envs / alg
  if m.get('SQ_WAVES'):
    w = m['SQ_WAVES']
    wc = m['SQ_WAVE_CYCLES']
    sq = {'waves': w, 'valu_insts_per_wave': m['SQ_INSTS_VALU'] / w,
          'cycles_per_wave': 4 * wc / w, 'valu_issue_frac': 4 * m['SQ_INSTS_VALU'] / (4 * wc)}
    for name, k in (('wait_any_frac', 'SQ_WAIT_ANY'), ('wait_inst_any_frac', 'SQ_WAIT_INST_ANY'),
                    ('active_inst_any_frac', 'SQ_ACTIVE_INST_ANY')):
      if k in m:
        sq[name] = m[k] / wc
    sq['lds_insts_per_wave'] = m.get('SQ_INSTS_LDS', 0) / w
    sq['salu_insts_per_wave'] = m.get('SQ_INSTS_SALU', 0) / w
    out['sq'] = sq
  return out


def main():
  d, tag = sys.argv[1], sys.argv[2]
  res = {'round': tag, 'tool': 'tools/multi_modes_prof.sh (tools/multi_traffic.py: Ant Mountain(4), '
                              '2,048 envs, 30 launches from the drop of one mode per run)',
         'modes': {}}
  for info in ('noinfo', 'info'):
    for cut in (0, 36):
      k = f'{info}_cutoff{cut}'
      p = os.path.join(d, f'{info}_{cut}')
      if os.path.exists(p + '.trace.log'):
        res['modes'][k] = mode(p)
  with open(os.path.join(ROOT, 'profiles', f'{tag}_multi_modes.json'), 'w') as f:
    json.dump(res, f, indent=1)
  for k, v in res['modes'].items():
    print(k, 'us', round(v['avg_us'] or 0, 1), 'late', round(v['avg_us_last_half'] or 0, 1),
          'M/s', round((v['system_steps_per_s'] or 0) / 1e6, 2),
          'traffic/alg', round(v.get('traffic_over_algorithmic', 0), 3),
          'valu_issue', round(v.get('sq', {}).get('valu_issue_frac', 0), 3),
          'wait_any', round(v.get('sq', {}).get('wait_any_frac', 0), 3))


if __name__ == '__main__':
  main()
