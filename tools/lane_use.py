"""Per-phase lane use of the SINGLE-mode env kernels (diagnostic), next to the
static per-phase instruction mix (tools/phase_mix.py): for each phase of one
substep, the lanes of an env's 16 that execute it and the distinct items
they cover, from the compiled system (the lane roles of bx_capi.cpp's lane
image: joint halves put joint j's parent side on lane j and its child side
on lane j + 8; with body copies (JB) every side lane integrates its side's
body; contact rows sit one per lane).

    python tools/lane_use.py ant [--mix profiles/<tag>_phase_mix_ant.json] [--json out]

With --mix, the VALU-weighted fraction of issued lane slots that do distinct
work is reported (per step: every phase's static VALU count times its trip
count, times its distinct-item lanes / 64 per wave... per 16-lane env).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tests.helpers import compiled  # noqa: E402

LANES = 16


def roles(name):
  _, d, _, _ = compiled(name)
  N, J = int(d['n_bodies']), len(d['joint_type'])
  K = len(d['act_type']) if 'act_type' in d else J
  R = len(d['row_group'])
  jh = J <= 8 and set(d['joint_type'].tolist()) <= {1}  # revolute joint halves
  out = {}
  if jh:
    side_bodies = [int(d['joint_body_p'][j]) for j in range(J)] + [int(d['joint_body_c'][j])
                                                                   for j in range(J)]
    out['actuators + damping'] = (2 * K, 2 * K)   # both halves are work
    out['joints'] = (2 * J, 2 * J)
    body = (2 * J, len(set(side_bodies)))          # copies: active lanes, distinct bodies
  else:
    out['actuators + damping'] = (K, K)
    out['joints'] = (J, J)
    body = (N, N)
  for ph in ('body acc + kinetic', 'body pos update (+ vproj)', 'body contact pos + vproj',
             'body contact vel'):
    out[ph] = body
  out['contact position pass'] = (R, R)
  out['contact velocity pass'] = (R, R)
  return {'system': name, 'bodies': N, 'joints': J, 'actuators': K, 'rows': R,
          'joint_halves': jh,
          'phases': {k: {'active_lanes': a, 'distinct_items': u, 'of_lanes': LANES,
                         'distinct_frac': u / LANES} for k, (a, u) in out.items()}}


# trips per env step of each loop depth of the Ant rollout kernel's ISA
# (tools/phase_mix.py): depth 4 = the substep loop (10 per step), depth 3 =
# the collision part of a substep pair (5), depths 1-2 = once per step
TRIPS = {4: 10, 3: 5, 2: 1, 1: 1}


def main():
  name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith('--') else 'ant'
  r = roles(name)
  if '--mix' in sys.argv:
    mix = json.load(open(sys.argv[sys.argv.index('--mix') + 1]))
    tot = useful = 0.0
    per = {}
    for row in mix['rows']:
      n = row['valu'] * TRIPS.get(row['loop_depth'], 1)
      frac = r['phases'].get(row['name'], {}).get('distinct_frac', 1.0)
      per.setdefault(row['name'], [0.0, frac])[0] += n
      tot += n
      useful += n * frac
    r['valu_per_step'] = {k: {'valu': v[0], 'distinct_frac': v[1]} for k, v in per.items()}
    r['valu_weighted_distinct_frac'] = useful / tot if tot else None
  print(json.dumps(r, indent=1))
  if '--json' in sys.argv:
    with open(sys.argv[sys.argv.index('--json') + 1], 'w') as f:
      json.dump(r, f, indent=1)


if __name__ == '__main__':
  main()
