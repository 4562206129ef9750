"""A/B: the bench loop's per-step action draw on the env's stream vs on a
side stream one step ahead (double-buffered slabs, event-ordered). Diagnostic."""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from brax_amd import _native, envs  # noqa: E402

dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
B = 4096
env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
lib = _native.lib()
A = env.action_size


def serial(n):
  st = env.reset(np.array([0, 7], np.uint32))
  act = torch.empty((B, A), device=dev)
  s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
  def one(st, k):
    lib.bx_uniform(C.c_void_p(act.data_ptr()), B * A, 1, k * B * A, -1.0, 1.0, s)
    return env.step(st, act)
  for k in range(50):
    st = one(st, k)
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for k in range(n):
    st = one(st, 50 + k)
  torch.cuda.synchronize()
  return (time.perf_counter() - t0) / n


def overlapped(n):
  st = env.reset(np.array([0, 7], np.uint32))
  acts = [torch.empty((B, A), device=dev) for _ in range(2)]
  main = torch.cuda.current_stream()
  side = torch.cuda.Stream()
  ss = C.c_void_p(side.cuda_stream)
  drawn = [torch.cuda.Event() for _ in range(2)]
  used = [torch.cuda.Event() for _ in range(2)]
  def draw(k):
    b = k % 2
    side.wait_event(used[b])
    lib.bx_uniform(C.c_void_p(acts[b].data_ptr()), B * A, 1, k * B * A, -1.0, 1.0, ss)
    drawn[b].record(side)
  for b in range(2):
    used[b].record(main)
  draw(0)
  def one(st, k):
    b = k % 2
    main.wait_event(drawn[b])
    st = env.step(st, acts[b])
    used[b].record(main)
    draw(k + 1)
    return st
  for k in range(50):
    st = one(st, k)
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for k in range(n):
    st = one(st, 50 + k)
  torch.cuda.synchronize()
  return (time.perf_counter() - t0) / n


for rep in range(2):
  a = serial(1000)
  b = overlapped(1000)
  print(f'serial {a * 1e6:.2f} us/step ({B / a / 1e6:.1f} M/s)   overlapped {b * 1e6:.2f} us/step '
        f'({B / b / 1e6:.1f} M/s)', flush=True)
