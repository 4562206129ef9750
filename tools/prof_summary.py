"""Summarise a run_prof.sh output directory into profiles/.

    python tools/prof_summary.py gpurun_out/prof_<tag> <tag> [phase_envs]

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats), and
profiles/<tag>_counters.json + profiles/traffic.json: per kernel, the mean
PMC counters per dispatch and the HBM bytes per launch, corrected as
MI355X_MICROARCH.md prescribes for gfx950 (FETCH_SIZE reports half of a wide
coalesced read: doubled; WRITE_SIZE exact for 16-B-per-lane stores; both in KB).
"""
import csv
import hashlib
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# algorithmic bytes per env-step of the fused env kernels the bench runs,
# keyed by the exact rocprof instantiation: QP in+out 2*52*N,
# action 4*A, obs 4*O, reward/done 8.
ENV_STEP_B = {
    'bx::env_step_kernel<16, 1, 160, 4, 1>': 1428,  # Ant: N=10, A=8, O=87
    'bx::env_step_kernel<16, 1, 33, 4, 2>': 2284,   # Humanoid: N=12, A=17, O=240
    # Env.step's packed-layout single step (bx_env_step_packed)
    'bx::env_step_packed_kernel<16, 1, 160, 4, 1>': 1428,
    'bx::env_step_packed_kernel<16, 1, 33, 4, 2>': 2284,
    # the same per env-step, K steps per launch (bx_env_rollout_packed)
    'bx::env_rollout_kernel<16, 1, 160, 4, 1>': 1428,
    'bx::env_rollout_kernel<16, 1, 33, 4, 2>': 2284,
}


def rollout_steps(d):
  """Env steps per rollout launch in the profiled bench run (its JSON line's
  config.steps_per_launch), 1 if absent."""
  try:
    with open(d.rstrip('/') + '.trace.log') as f:
      lines = [l for l in f if l.startswith('{')]
    return int(json.loads(lines[-1])['config'].get('steps_per_launch', 1))
  except (OSError, IndexError, KeyError, ValueError):
    return 1
PHASE_B = {'kinetic_kernel': 80 * 10, 'update_acc_kernel': 72 * 10, 'vproj_kernel': 96 * 10,
           'capsule_plane_kernel': 120 * 5}


def short(name):
  n = name.split('(')[0].replace('void ', '')
  return n


def bench_grids(d):
  """Per kernel, the grid size of its most frequent launch in the trace
  pass: the bench configuration. Other grids of the same instantiation (the
  32,768-env leg runs the Ant kernel on 8x the grid) are summarised apart
  so they do not mix into the bench kernel's averages."""
  n = defaultdict(lambda: defaultdict(list))
  p = os.path.join(d, 'trace', 'run_kernel_trace.csv')
  with open(p) as f:
    for r in csv.DictReader(f):
      k = short(r['Kernel_Name'])
      # the total grid (the counter passes report X * Y * Z; the phase
      # kernels launch 2-D grids)
      g = int(r['Grid_Size_X']) * int(r.get('Grid_Size_Y') or 1) * int(r.get('Grid_Size_Z') or 1)
      n[k][g].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
  grids, stats = {}, {}
  for k, by in n.items():
    g = max(by, key=lambda x: len(by[x]))
    grids[k] = g
    stats[k] = {'calls': len(by[g]), 'avg_ns': sum(by[g]) / len(by[g]), 'grid': g}
    if 'rollout' in k:
      # a rollout kernel runs K-step launches and (Env.step on a wide batch)
      # one-step launches: split the durations at 4x the shortest, so each
      # average covers launches of one length
      d = sorted(by[g])
      long_ = [x for x in d if x > 4 * d[0]]
      if long_:
        short_ = [x for x in d if x <= 4 * d[0]]
        stats[k].update({'calls': len(long_), 'avg_ns': sum(long_) / len(long_),
                         'one_step_launches': {'calls': len(short_),
                                               'avg_ns': sum(short_) / len(short_)}})
    other = {str(x): {'calls': len(v), 'avg_ns': sum(v) / len(v)} for x, v in by.items() if x != g}
    if other:
      stats[k]['other_grids'] = other
  return grids, stats


def counters(d, grids):
  out = defaultdict(lambda: defaultdict(list))
  meta = {}
  for sub in ('fetch', 'write', 'sq', 'sq2'):
    p = os.path.join(d, sub, 'run_counter_collection.csv')
    if not os.path.exists(p):
      continue
    with open(p) as f:
      for r in csv.DictReader(f):
        k = short(r['Kernel_Name'])
        if not k.startswith('bx::') and 'bx::' not in k:
          continue
        if k in grids and int(r['Grid_Size']) != grids[k]:
          continue
        out[k][r['Counter_Name']].append(float(r['Counter_Value']))
        meta[k] = {'grid': int(r['Grid_Size']), 'workgroup': int(r['Workgroup_Size']),
                   'vgpr': int(r['VGPR_Count']), 'sgpr': int(r['SGPR_Count']),
                   'lds_bytes': int(r['LDS_Block_Size']), 'scratch': int(r['Scratch_Size'])}
  return out, meta


def main():
  d, tag = sys.argv[1], sys.argv[2]
  prof = os.path.join(ROOT, 'profiles')
  shutil.copy(os.path.join(d, 'trace', 'run_kernel_stats.csv'),
              os.path.join(prof, f'{tag}_kernel_stats.csv'))
  # per-kernel averages from the dispatch trace at the bench grid (the
  # --stats CSV copied above averages every grid of an instantiation)
  grids, stats = bench_grids(d)
  K = rollout_steps(d)
  for k in stats:
    if 'env_rollout_kernel' in k:
      stats[k]['steps_per_launch'] = K
    elif 'env_rollout_wide_kernel' in k:
      stats[k]['steps_per_launch'] = 50  # bench.py secondary_configs: 50-step rollouts
  cnt, meta = counters(d, grids)
  res = {}
  for k, cs in cnt.items():
    e = {'counters': {c: {'dispatches': len(v), 'mean': sum(v) / len(v)} for c, v in cs.items()}}
    e.update(meta.get(k, {}))
    e['trace'] = stats.get(k)
    f = e['counters'].get('FETCH_SIZE', {}).get('mean')
    w = e['counters'].get('WRITE_SIZE', {}).get('mean')
    if f is not None and w is not None:
      e['hbm_read_bytes_per_launch'] = 2 * f * 1024
      e['hbm_write_bytes_per_launch'] = w * 1024
      e['hbm_bytes_per_launch'] = e['hbm_read_bytes_per_launch'] + e['hbm_write_bytes_per_launch']
    res[k] = e
  with open(os.path.join(prof, f'{tag}_counters.json'), 'w') as f:
    json.dump(res, f, indent=1)
  # traffic.json: what bench.py reports as roofline.traffic
  traffic = {'round': tag, 'source': f'profiles/{tag}_counters.json',
             'note': 'HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB -> B), '
                     'gfx950 correction per MI355X_MICROARCH.md', 'kernels': {}}
  for k, e in res.items():
    if 'hbm_bytes_per_launch' not in e:
      continue
    ent = {'hbm_bytes_per_launch': e['hbm_bytes_per_launch'],
           'hbm_read_bytes_per_launch': e['hbm_read_bytes_per_launch'],
           'hbm_write_bytes_per_launch': e['hbm_write_bytes_per_launch'],
           'grid': e.get('grid'), 'avg_ns': (e.get('trace') or {}).get('avg_ns')}
    base = k.split('::')[-1].split('<')[0]
    if k in ENV_STEP_B:
      ent['batch'] = e['grid'] // 64 * 4  # 16 lanes per env, 4 envs per 64-wide workgroup
      spl = K if 'env_rollout_kernel' in k else 1
      ent['steps_per_launch'] = spl
      ent['algorithmic_bytes_per_launch'] = ENV_STEP_B[k] * ent['batch'] * spl
    elif base in PHASE_B:
      envs = int(sys.argv[3]) if len(sys.argv) > 3 else 1 << 20  # bench --phase-envs
      ent['envs'] = envs
      ent['algorithmic_bytes_per_launch'] = PHASE_B[base] * envs
    traffic['kernels'][k] = ent
  with open(os.path.join(prof, 'traffic.json'), 'w') as f:
    json.dump(traffic, f, indent=1)
  # rocprof_latest.json: the kernel-trace averages, keyed to the library build
  # they were measured on (bench.py reports them only for that exact build)
  lib = os.path.join(ROOT, 'brax_amd', '_lib', 'libbrax_amd.so')
  with open(lib, 'rb') as f:
    sha = hashlib.sha1(f.read()).hexdigest()
  # per-wave SQ issue figures of the kernels the SQ pass counted
  # (SQ_WAVE_CYCLES counts quad-cycles; one wave issues at most one VALU
  # instruction per 4 cycles, MI355X_MICROARCH.md)
  for k, e in res.items():
    c = e.get('counters', {})
    waves = c.get('SQ_WAVES', {}).get('mean')
    if k in stats and waves and 'SQ_INSTS_VALU' in c and 'SQ_WAVE_CYCLES' in c:
      valu = c['SQ_INSTS_VALU']['mean'] / waves
      cyc = 4 * c['SQ_WAVE_CYCLES']['mean'] / waves
      wc = c['SQ_WAVE_CYCLES']['mean']
      stats[k]['sq'] = {'source': f'profiles/{tag}_counters.json', 'waves': waves,
                        'valu_insts_per_wave': valu,
                        'lds_insts_per_wave': c.get('SQ_INSTS_LDS', {}).get('mean', 0) / waves,
                        'salu_insts_per_wave': c.get('SQ_INSTS_SALU', {}).get('mean', 0) / waves,
                        'cycles_per_wave': cyc, 'valu_issue_frac': 4 * valu / cyc}
      # the stall split of the wave cycles (quad-cycle counters over quad-cycles)
      for name, ctr in (('wait_any_frac', 'SQ_WAIT_ANY'), ('wait_inst_any_frac', 'SQ_WAIT_INST_ANY'),
                        ('active_inst_any_frac', 'SQ_ACTIVE_INST_ANY'),
                        ('wait_inst_lds_frac', 'SQ_WAIT_INST_LDS')):
        if ctr in c:
          stats[k]['sq'][name] = c[ctr]['mean'] / wc
  # the MULTI kernel's bench launches mix four modes (Info on / off x cutoff
  # 0 / 36): its per-mode record (tools/multi_modes_prof.sh), when present,
  # keyed beside the mixed average
  mm = None
  mp = os.path.join(prof, f'{tag}_multi_modes.json')
  if os.path.exists(mp):
    with open(mp) as f:
      mm = json.load(f)
    for k in stats:
      if 'system_step_multi_kernel' in k:
        stats[k]['note'] = ('averages the bench\'s four MULTI modes; per mode: '
                            f'profiles/{tag}_multi_modes.json (multi_modes below)')
  with open(os.path.join(prof, 'rocprof_latest.json'), 'w') as f:
    sys.path.insert(0, ROOT)
    from bench import src_sha1
    out = {'round': tag, 'source': f'profiles/{tag}_kernel_stats.csv', 'lib_sha1': sha,
           'src_sha1': src_sha1(), 'kernels': stats}
    if mm is not None:
      out['multi_modes'] = mm
    json.dump(out, f, indent=1)
  print(json.dumps(traffic, indent=1))


if __name__ == '__main__':
  main()
