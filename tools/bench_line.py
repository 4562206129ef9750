"""One-line summary of a bench.py log's JSON line."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d['roofline']
loops = {k: round(d[k]['ms_per_step'] * 1e3, 2) for k in ('eager_loop', 'graph_loop', 'rollout_loop', 'direct_loop')
         if k in d and 'ms_per_step' in d[k]}
print(f"value {d['value'] / 1e6:.2f} M/s ({d.get('timed_loop')}), us/step {d['ms_per_step'] * 1e3:.2f}, "
      f"loops us/step {loops}, kernel {r['kernel'].split('::')[-1]} {r.get('kernel_ms_per_step', r['kernel_ms']) * 1e3:.2f} us/step, "
      f"single-step kernel {r.get('single_step_kernel_ms', 0) * 1e3:.2f} us, frac {r['frac']:.4f}")
