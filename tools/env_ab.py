"""Per-step kernel time of one env at 4,096 envs on the library BRAX_AMD_LIB
names: the 50-step rollout launch (RolloutRunner) and the single Env.step
launch, HIP events over back-to-back launches; one JSON line
(tools/env_ab.sh interleaves builds).  python tools/env_ab.py humanoid"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
  from brax_amd import envs
  from brax_amd.envs.rollout import RolloutRunner
  name = sys.argv[1] if len(sys.argv) > 1 else 'humanoid'
  dev = torch.device('cuda', 0)
  B = 4096
  env = envs.create(name, batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  st = env.reset(np.array([0, 7], np.uint32))
  r = RolloutRunner(env, st, 50, seed=3)
  for _ in range(4):
    r.run()
  torch.cuda.synchronize()
  a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  a.record()
  for _ in range(20):
    r.run()
  b.record()
  torch.cuda.synchronize()
  roll = a.elapsed_time(b) * 1e3 / (20 * 50)
  act = torch.rand((B, env.action_size), device=dev) * 2 - 1
  s = [st]

  def step():
    s[0] = env.step(s[0], act)
  for _ in range(20):
    step()
  torch.cuda.synchronize()
  a.record()
  for _ in range(200):
    step()
  b.record()
  torch.cuda.synchronize()
  one = a.elapsed_time(b) * 1e3 / 200
  print(json.dumps({'lib': os.environ.get('BRAX_AMD_LIB', 'brax_amd/_lib'), 'env': name,
                    'rollout_us_per_step': round(roll, 2), 'env_step_us': round(one, 2)}), flush=True)


if __name__ == '__main__':
  main()
