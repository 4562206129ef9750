"""Static instruction mix of one kernel's ISA per loop depth (diagnostic).

  hipcc ... --cuda-device-only -S pbd_kernels.hip -o single.s
  python tools/isa_loops.py single.s '_ZN2bx15env_step_kernelILi16ELi1ELi0ELi4E'

Counts VALU, LDS, waitcnt, SGPR-spill lane moves and scratch accesses by the
loop depth LLVM annotates on each basic block.
"""
import re
import sys
from collections import Counter, defaultdict


def main():
  path, sym = sys.argv[1], sys.argv[2]
  lines = open(path).read().splitlines()
  start = next(i for i, l in enumerate(lines) if l.startswith(sym) and l.rstrip().endswith(':') or
               (l.startswith(sym) and ':' in l))
  depth = 0
  cnt = defaultdict(Counter)
  for l in lines[start + 1:]:
    if l.startswith('.Lfunc_end'):
      break
    if l.startswith('.LBB'):
      m = re.search(r'Depth=(\d)', l)
      depth = int(m.group(1)) if m else 0
      continue
    s = l.strip()
    if not s or s.startswith(';') or s.startswith('.'):
      continue
    op = s.split()[0]
    c = cnt[depth]
    if op.startswith('v_readlane') or op.startswith('v_writelane'):
      c['sgpr_spill_lane'] += 1
    elif op.startswith('v_'):
      c['valu'] += 1
    if op.startswith('ds_'):
      c['lds'] += 1
    if op.startswith('scratch_'):
      c['scratch'] += 1
    if op == 's_waitcnt':
      c['waitcnt'] += 1
    if op.startswith('global_') or op.startswith('buffer_'):
      c['global'] += 1
  for d in sorted(cnt):
    print(d, dict(cnt[d]))


if __name__ == '__main__':
  main()
