"""hipGraph-captured Env.step rollouts.

The reference compiles `env.step` with `jax.jit` and calls the executable in
a Python loop (`/root/reference/notebooks/environments.ipynb:386-423`); each
call is one device dispatch. Here one `Env.step` is already one fused kernel
launch through the C ABI, but the ~20 µs of Python per step (the wrapper
chain, the State, the ctypes call, the action draw's launch) can exceed the
~29 µs kernel on a slow or busy host and leave the GPU idle between launches.

`StepGraph` records K consecutive steps once into a HIP graph (stream
capture through `torch.cuda.CUDAGraph`) and replays it: the device runs the
eager loop's work (the action draws, the fused env step per step, and an
optional per-step hook such as the episodic (reward, done) sum), and the host
pays one graph launch per K steps. Nothing is skipped or cached: every replay
steps the state forward K steps, and the actions are fresh on every replay
because the draw reads its offset from a device epoch counter the graph bumps
at its end. By default the K action slabs of a replay are drawn by ONE
`bx_uniform_slabs` launch (ABI 9) at the head of the graph, slab t at the
offset the eager loop's `bx_uniform` uses for step t, so a replayed rollout
steps on the same bits as the eager loop with
`action_offset(rank, B, A, step, world)`, one draw kernel per K steps instead
of one per step (`draw='per_step'` keeps the per-step launch).
"""
from typing import Callable, Optional

import ctypes as C
import torch

from brax_amd import _native
from brax_amd.base import PackedQP, packed_buffer
from brax_amd.envs.env import State
from brax_amd.system import _stream


def _static(x):
  return None if x is None else x.detach().clone().contiguous()


class StepGraph:
  """K `env.step` calls with on-device action draws, captured as one graph.

  Args:
    env: an env from `brax_amd.envs.create` (any wrapper chain).
    state: the state to start from (copied into the graph's static inputs).
    k: steps per graph replay.
    seed, offset, step_stride: the action stream. Step t of replay r draws
      `U(seed, offset + (r * k + t) * step_stride + i)` for the (B, A) slab,
      `lo`/`hi` its range; `step_stride = world * B * A` and
      `offset = action_offset(rank, B, A, first_step, world)` reproduce the
      eager loop's slabs.
    hook: called as `hook(state)` after each captured step (device work
      only: it is recorded into the graph and runs on every replay; the
      warm-up pass before capture does not call it).
    draw: 'batched' (default): the K slabs of a replay in one
      `bx_uniform_slabs` launch at the head of the graph, (K, B, A) floats;
      'per_step': one `bx_uniform_epoch` launch before each step (the
      reference loop's shape, one draw per step). Same bits either way.
  """

  def __init__(self, env, state: State, k: int, seed: int = 1, offset: int = 0,
               step_stride: Optional[int] = None, lo: float = -1.0, hi: float = 1.0,
               hook: Optional[Callable[[State], None]] = None, draw: str = 'batched'):
    if k < 1:
      raise ValueError(f'k must be >= 1, got {k}')
    if draw not in ('batched', 'per_step'):
      raise ValueError(f"draw must be 'batched' or 'per_step', got {draw!r}")
    u = env.unwrapped
    dev = u.sys.device
    self.env, self.k, self.device, self.draw = env, int(k), dev, draw
    buf = packed_buffer(state.qp)
    B = (buf if buf is not None else state.qp.pos).shape[0]
    A = env.action_size
    self.batch_size = B
    stride = B * A if step_stride is None else int(step_stride)
    # static inputs: exactly the tensors Env.step reads (the QP, done, the
    # episode counters, the target envs' streams); first_qp / first_obs pass
    # through by reference
    if buf is None:
      buf = torch.zeros(state.qp.pos.shape[:-1] + (16,), dtype=torch.float32, device=dev)
      for lo_, f in ((0, state.qp.pos), (3, state.qp.rot), (7, state.qp.vel), (10, state.qp.ang)):
        buf[..., lo_:lo_ + f.shape[-1]] = f
    self._qp = _static(buf)
    self._done = _static(state.done)
    info = dict(state.info)
    self._steps = _static(info.get('steps'))
    rng = info.get('rng')
    if rng is None and getattr(u, 'needs_rng', False):
      # a hand-built state of a target env: the step would start a zero
      # stream per call; make it a static input so replays advance it
      rng = torch.zeros((B,), dtype=torch.int32, device=dev)
    self._rng = _static(rng)
    if self._steps is not None:
      info['steps'] = self._steps
    if self._rng is not None:
      info['rng'] = self._rng
    self._in = State(qp=PackedQP(self._qp), obs=state.obs, reward=state.reward,
                     done=self._done, metrics=state.metrics, info=info)
    self._acts = torch.empty((self.k if draw == 'batched' else 1, B, A), dtype=torch.float32,
                             device=dev)
    self._epoch = torch.zeros((1,), dtype=torch.int64, device=dev)
    lib = _native.lib()

    def draw_slabs(first, n):
      _native.check(lib.bx_uniform_slabs(
          C.c_void_p(self._acts.data_ptr()), B * A, n, seed, offset + first * stride, stride,
          C.c_void_p(self._epoch.data_ptr()), self.k * stride, lo, hi, _stream(dev.index)))

    def body(hook=hook):
      st = self._in
      if self.draw == 'batched':
        draw_slabs(0, self.k)
      for t in range(self.k):
        if self.draw == 'per_step':
          draw_slabs(t, 1)
        st = env.step(st, self._acts[t if self.draw == 'batched' else 0])
        if hook is not None:
          hook(st)
      # feed the K-th state back into the static inputs, advance the epoch
      self._qp.copy_(packed_buffer(st.qp))
      self._done.copy_(st.done)
      if self._steps is not None:
        self._steps.copy_(st.info['steps'])
      if self._rng is not None:
        self._rng.copy_(st.info['rng'])
      self._epoch.add_(1)
      return st

    with torch.cuda.device(dev):
      # one eager pass on a side stream fills the host-side caches (the env's
      # parameter block) and the allocator, as torch's capture recipe asks;
      # the state it produces is discarded and the statics restored. The hook
      # is left out of it (its side effects would count K extra steps).
      statics = [t for t in (self._qp, self._done, self._steps, self._rng) if t is not None]
      snap = [t.clone() for t in statics]
      side = torch.cuda.Stream(dev)
      side.wait_stream(torch.cuda.current_stream(dev))
      with torch.cuda.stream(side):
        body(hook=None)
      torch.cuda.current_stream(dev).wait_stream(side)
      for dst, src in zip(statics, snap):
        dst.copy_(src)
      self._epoch.zero_()
      self.graph = torch.cuda.CUDAGraph()
      # thread_local: only this thread's calls are checked during capture, so
      # a process group's watchdog thread polling its collectives' events (the
      # bench's barrier just before) cannot invalidate the capture
      with torch.cuda.graph(self.graph, capture_error_mode='thread_local'):
        self._out = body()
      torch.cuda.current_stream(dev).synchronize()

  @property
  def epoch(self) -> int:
    """Replays done so far (a device read: synchronises)."""
    return int(self._epoch.item())

  def replay(self) -> State:
    """Steps the rollout K steps forward; returns the K-th state."""
    self.graph.replay()
    return self._out
