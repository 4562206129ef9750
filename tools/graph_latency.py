"""Fixed per-replay overhead of the bench's graph loop (one MI355X).

For K-step StepGraphs of the Ant bench env: wall time of one replay + sync,
the HIP-event span of the same replay on the launch stream, and the kernel
train, to split a short timed run's overhead into launch latency, the
graph's tail (state copies, epoch bump) and completion detection.

    python tools/graph_latency.py [--spin]
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

if '--spin' in sys.argv:
  # hipDeviceScheduleSpin (1) before the context exists: host waits spin
  hip = C.CDLL('libamdhip64.so')
  print('hipSetDeviceFlags(spin) ->', hip.hipSetDeviceFlags(C.c_uint(1)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from brax_amd import envs  # noqa: E402
from brax_amd.envs.graph import StepGraph  # noqa: E402


def main():
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(dev)
  B = 4096
  env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  st = env.reset(np.array([0, 0x5EED], np.uint32))
  act = torch.rand((B, 8), device=dev) * 2 - 1
  for _ in range(5):
    st = env.step(st, act)
  kern = bench.kernel_train(env, st, act)
  res = {'kernel_ms': kern}
  for K in (1, 5, 20, 50):
    g = StepGraph(env, st, K, seed=1)
    for _ in range(3):
      g.replay()
    torch.cuda.synchronize()
    walls, evs = [], []
    for _ in range(10):
      a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      a.record()
      g.replay()
      b.record()
      torch.cuda.synchronize()
      walls.append((time.perf_counter() - t0) * 1e3)
      evs.append(a.elapsed_time(b))
    # back-to-back replays (the 1000-step bench's shape)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = max(1, 200 // K)
    for _ in range(n):
      g.replay()
    torch.cuda.synchronize()
    bb = (time.perf_counter() - t0) * 1e3 / (n * K)
    res[f'K{K}'] = {'wall_ms_median': float(np.median(walls)), 'event_ms_median': float(np.median(evs)),
                    'wall_per_step_ms': float(np.median(walls)) / K,
                    'overhead_ms': float(np.median(walls)) - K * kern,
                    'back_to_back_per_step_ms': bb}
    del g
  print(json.dumps(res, indent=1))


if __name__ == '__main__':
  main()
