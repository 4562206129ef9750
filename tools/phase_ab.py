"""Phase-kernel roofline A/B across library builds: python phase_ab.py lib..."""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] != '--child':
  for rep in range(2):
    for lib in sys.argv[1:]:
      env = dict(os.environ, BRAX_AMD_LIB=os.path.join(ROOT, lib))
      r = subprocess.run([sys.executable, __file__, '--child'], env=env, capture_output=True,
                         text=True, timeout=120)
      if r.returncode:
        print(r.stderr[-2000:]); sys.exit(r.returncode)
      d = json.loads(r.stdout.strip().splitlines()[-1])
      print(lib, ' '.join(f"{k}={v['achieved']:.0f}({v['frac']:.3f})" for k, v in d['kernels'].items()), flush=True)
  sys.exit(0)
sys.path.insert(0, ROOT)
import torch
import bench
from brax_amd import envs
dev = torch.device('cuda', 0)
env = envs.create('ant', batch_size=64, device=dev)
print(json.dumps(bench.phase_bench(env.unwrapped.sys, dev, 1 << 20, reps=50)))
