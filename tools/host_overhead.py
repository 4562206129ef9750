"""Host cost of one Env.step call (Ant, 4096 envs): wall per call with the
launch queue absorbing the kernels, then the synchronised rate, plus a
cProfile of the Python path. Diagnostic, not part of the product."""
import cProfile, pstats, sys, time, os
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from brax_amd import envs
dev = torch.device('cuda', 0)
B = 4096
env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
st = env.reset(0)
acts = torch.rand((64, B, 8), device=dev) * 2 - 1
for k in range(50):
  st = env.step(st, acts[k % 64])
torch.cuda.synchronize()
n = 200
t0 = time.perf_counter()
for k in range(n):
  st = env.step(st, acts[k % 64])
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f'host us/step {1e6*(t1-t0)/n:.1f}  total us/step {1e6*(t2-t0)/n:.1f}')
pr = cProfile.Profile()
pr.enable()
for k in range(n):
  st = env.step(st, acts[k % 64])
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats('tottime').print_stats(18)
