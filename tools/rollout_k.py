"""Fixed per-launch cost of the direct rollout loop (one MI355X, Ant bench env).

For K-step `RolloutRunner`s: the HIP-event span of back-to-back runs (GPU
time per launch) and the wall time of ONE run bracketed by
torch.cuda.synchronize() (what a one-launch timed region sees), so the
launch's cost splits into K x per-step + a fixed part (prologue, slowest-wave
tail, launch and completion latency).

    python tools/rollout_k.py [--spin] [K ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SPIN = '--spin' in sys.argv
if SPIN:
  # hipDeviceScheduleSpin (1) before the context exists: host waits spin
  import ctypes
  sys.argv.remove('--spin')
  print('hipSetDeviceFlags(spin) ->', ctypes.CDLL('libamdhip64.so').hipSetDeviceFlags(ctypes.c_uint(1)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from brax_amd import envs  # noqa: E402
from brax_amd.envs.rollout import RolloutRunner  # noqa: E402


def main():
  ks = [int(a) for a in sys.argv[1:]] or [1, 2, 5, 10, 20, 50, 100]
  dev = torch.device('cuda', 0)
  torch.cuda.set_device(dev)
  env = envs.create('ant', batch_size=4096, episode_length=1000, auto_reset=True, device=dev)
  state = env.reset(np.array([0, 0x5EED], np.uint32))
  rows = []
  for K in ks:
    r = RolloutRunner(env, state, K)
    t_end = time.perf_counter() + 0.05
    while time.perf_counter() < t_end:
      r.run()
      torch.cuda.synchronize()
    n = max(2, 2000 // K)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
      r.run()
    b.record()
    torch.cuda.synchronize()
    gpu_us = a.elapsed_time(b) * 1e3 / n
    walls = []
    for _ in range(30):
      for _ in range(3):  # keep the clocks up between samples
        r.run()
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      r.run()
      torch.cuda.synchronize()
      walls.append((time.perf_counter() - t0) * 1e6)
    w = float(np.median(walls))
    # the same one-launch region after the GPU idled (a host pause of 5 ms,
    # e.g. a garbage collection between warm-up and t0): the clock drops
    idle = []
    for _ in range(10):
      for _ in range(3):
        r.run()
      torch.cuda.synchronize()
      time.sleep(0.005)
      t0 = time.perf_counter()
      r.run()
      torch.cuda.synchronize()
      idle.append((time.perf_counter() - t0) * 1e6)
    # host time of one run() call (ctypes + the C entry point + the launch)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
      r.run()
    host = (time.perf_counter() - t0) * 1e6 / 20
    torch.cuda.synchronize()
    rows.append({'K': K, 'gpu_us_per_launch': gpu_us, 'gpu_us_per_step': gpu_us / K,
                 'wall_us_one_launch': w, 'wall_us_per_step': w / K,
                 'wall_minus_gpu_us': w - gpu_us,
                 'wall_us_one_launch_after_5ms_idle': float(np.median(idle)),
                 'host_us_per_run_call': host})
    print(json.dumps(rows[-1]), flush=True)
    del r
  # least-squares fit of the back-to-back GPU time: per-step + fixed
  kk = np.array([x['K'] for x in rows], float)
  g = np.array([x['gpu_us_per_launch'] for x in rows])
  s, f = np.polyfit(kk, g, 1)
  print(json.dumps({'fit_gpu_us_per_step': s, 'fit_gpu_fixed_us_per_launch': f}), flush=True)


if __name__ == '__main__':
  main()
