"""Static per-phase instruction mix of a step kernel (diagnostic).

Build the SINGLE-mode translation unit's assembly with the phase marks (the
stamp points as `;BXPHASE k` comments, code not scheduled across them):

  cd brax_amd/csrc && hipcc <the Makefile's CXXFLAGS + SCHED> -DBX_TU_FAST \
      -DBX_PHASE_MARKS --cuda-device-only -S pbd_kernels.hip -o single_marks.s
  python tools/phase_mix.py single_marks.s <mangled kernel name> [--json out]

Every instruction is attributed to the phase whose mark ENDS its stretch of
code (the next `;BXPHASE` in program order), with the loop depth LLVM
annotates on its basic block. A loop's block laid out past the loop's marks
(its stretch ends at a mark outside the loop) goes to the loop body's last
phase. Per loop depth the totals are exact; the per-phase split follows the
layout. Per env step (the Ant rollout kernel): depth 4 = the substep loop (10
trips), depth 3 = the collision part of a substep pair (5), depths 1-2 once
(tools/lane_use.py TRIPS).

Instruction classes: VALU arithmetic (fma / mul / add), transcendental,
compare / select, DPP lane moves, SGPR-lane moves (readlane / writelane:
SGPR spills and uniform reads), other VALU (integer, conversion, moves), LDS,
global memory, waitcnt, SALU / SMEM.
"""
import json
import re
import sys
from collections import Counter, defaultdict

PHASES = {
    '0': 'actuators + damping', '1': 'body acc + kinetic', '2': 'joints',
    '3': 'body pos update (+ vproj)', '4': 'contact position pass', '5': 'body contact pos + vproj',
    '6': 'contact velocity pass', '7': 'body contact vel', '9': 'pbd tail (Info sums)',
    '10': 'prologue / action row', '11': 'pbd step entry', '12': 'observation',
    '13': 'reward / metrics', '14': 'outputs / AutoReset / loop', 'end': 'after the last mark',
}


def cls(op, s):
  if 'row_' in s or 'quad_perm' in s or '_dpp' in op:
    return 'dpp'
  if op.startswith(('v_readlane', 'v_writelane', 'v_readfirstlane')):
    return 'sgpr_lane'
  if op.startswith(('v_fma', 'v_fmac', 'v_mad_f32', 'v_pk_fma')):
    return 'fma'
  if op.startswith(('v_mul_f32', 'v_pk_mul_f32')):
    return 'mul'
  if op.startswith(('v_add_f32', 'v_sub_f32', 'v_subrev_f32', 'v_pk_add_f32')):
    return 'add'
  if op.startswith(('v_rcp', 'v_sqrt', 'v_rsq', 'v_sin', 'v_cos', 'v_exp', 'v_log')):
    return 'transcendental'
  if op.startswith(('v_cndmask', 'v_cmp', 'v_max', 'v_min', 'v_med')):
    return 'cmp_select'
  if op.startswith('v_'):
    return 'valu_other'
  if op.startswith('ds_'):
    return 'lds'
  if op.startswith(('global_', 'buffer_', 'scratch_', 'flat_')):
    return 'vmem'
  if op == 's_waitcnt':
    return 'waitcnt'
  if op.startswith('s_'):
    return 'salu_smem'
  return 'other'


VALU = ('fma', 'mul', 'add', 'transcendental', 'cmp_select', 'dpp', 'sgpr_lane', 'valu_other')


def parse(path, sym):
  lines = open(path).read().splitlines()
  start = next(i for i, l in enumerate(lines) if l.startswith(sym + ':'))
  pending = []  # (depth, class) since the last mark
  out = defaultdict(Counter)  # (phase, depth) -> class counts
  depth = 0
  marks_at = defaultdict(list)  # loop depth -> the marks seen at that depth
  for l in lines[start + 1:]:
    if l.startswith('.Lfunc_end'):
      break
    if l.startswith('.LBB'):
      m = re.search(r'Depth=(\d)', l)
      depth = int(m.group(1)) if m else 0
      continue
    s = l.strip()
    m = re.match(r';\s*BXPHASE (\d+)', s)
    if m:
      marks_at[depth].append(int(m.group(1)))
      for d, c in pending:
        # a loop's block that LLVM laid out past the loop's marks (the mark
        # ending the stretch sits at a shallower depth) is the loop body's
        # last phase: the one ending at the loop's highest mark
        ph = m.group(1)
        if d > depth and marks_at.get(d):
          ph = str(max(marks_at[d]))
        out[(ph, d)][c] += 1
      pending = []
      continue
    if not s or s.startswith((';', '.')):
      continue
    op = s.split()[0]
    pending.append((depth, cls(op, s)))
  for d, c in pending:
    out[('end', d)][c] += 1
  return out


def main():
  path, sym = sys.argv[1], sys.argv[2]
  js = sys.argv[sys.argv.index('--json') + 1] if '--json' in sys.argv else None
  out = parse(path, sym)
  rows = []
  for (ph, d), c in sorted(out.items(), key=lambda x: (x[0][1], x[0][0])):
    valu = sum(c[k] for k in VALU)
    arith = c['fma'] + c['mul'] + c['add']
    rows.append({'phase': ph, 'name': PHASES.get(ph, ph), 'loop_depth': d, 'valu': valu,
                 'arith_frac_of_valu': arith / valu if valu else None, **dict(c)})
    print(f"{PHASES.get(ph, ph):30s} depth {d}  VALU {valu:5d}  "
          + '  '.join(f'{k} {c[k]}' for k in VALU + ('lds', 'vmem', 'waitcnt', 'salu_smem') if c[k]))
  if js:
    with open(js, 'w') as f:
      json.dump({'source': path, 'kernel': sym, 'rows': rows}, f, indent=1)


if __name__ == '__main__':
  main()
