"""hipGraph-captured Env.step rollouts.

The reference compiles `env.step` with `jax.jit` and calls the executable in
a Python loop (`/root/reference/notebooks/environments.ipynb:386-423`); each
call is one device dispatch. Here one `Env.step` is already one fused kernel
launch through the C ABI, but the ~20 µs of Python per step (the wrapper
chain, the State, the ctypes call, the action draw's launch) can exceed the
~29 µs kernel on a slow or busy host and leave the GPU idle between launches.

`StepGraph` records K consecutive steps once into a HIP graph (stream
capture through `torch.cuda.CUDAGraph`) and replays it: per step the device
runs exactly the eager loop's kernels (the action draw, the fused env step,
and an optional per-step hook such as the episodic (reward, done) sum), and
the host pays one graph launch per K steps. Nothing is skipped or cached:
every replay steps the state forward K steps, and the actions are fresh on
every replay because the draw reads its offset from a device epoch counter
(`bx_uniform_epoch`, ABI 8) the graph bumps at its end; a replayed rollout
therefore draws the same slabs, step for step, as the eager loop with
`bx_uniform` at offset `action_offset(rank, B, A, step, world)`.

The output buffers of the K captured steps live in the graph's private
memory pool and are overwritten by the next replay: `replay()` returns the
state after the K-th step, valid until the following replay (clone what you
keep, as with any captured graph).
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
    overlap_draw: draw step t+1's actions on a forked stream while step t
      runs (same slabs, same bits). Off by default: the cross-stream edges
      cost more than the draw they hide (Ant 4,096 envs: 36.3 us per step
      against 30.9 us in line, profiles/r02zl_bench.log).
  """

  def __init__(self, env, state: State, k: int, seed: int = 1, offset: int = 0,
               step_stride: Optional[int] = None, lo: float = -1.0, hi: float = 1.0,
               hook: Optional[Callable[[State], None]] = None, overlap_draw: bool = False):
    if k < 1:
      raise ValueError(f'k must be >= 1, got {k}')
    u = env.unwrapped
    dev = u.sys.device
    self.env, self.k, self.device = env, int(k), dev
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
    self._rng = _static(info.get('rng'))
    if self._steps is not None:
      info['steps'] = self._steps
    if self._rng is not None:
      info['rng'] = self._rng
    self._in = State(qp=PackedQP(self._qp), obs=state.obs, reward=state.reward,
                     done=self._done, metrics=state.metrics, info=info)
    # two action slabs: with overlap_draw, step t+1's draw runs on a forked
    # stream beside step t (the step kernel holds one wave per SIMD at the
    # bench size, so the draw's waves find idle SIMD slots); each draw waits
    # only for the step that last read its slab
    self._acts = [torch.empty((B, A), dtype=torch.float32, device=dev) for _ in range(2)]
    self._epoch = torch.zeros((1,), dtype=torch.int64, device=dev)
    self.overlap_draw = bool(overlap_draw)
    lib = _native.lib()
    draw_stream = torch.cuda.Stream(dev)

    def draw(t):
      _native.check(lib.bx_uniform_epoch(
          C.c_void_p(self._acts[t % 2].data_ptr()), B * A, seed, offset + t * stride,
          C.c_void_p(self._epoch.data_ptr()), self.k * stride, lo, hi, _stream(dev.index)))

    def body(hook=hook):
      st = self._in
      main = torch.cuda.current_stream(dev)
      ready = [None, None]
      if self.overlap_draw:
        draw(0)
      for t in range(self.k):
        if not self.overlap_draw:
          draw(t)
        else:
          if ready[t % 2] is not None:
            main.wait_event(ready[t % 2])
          if t + 1 < self.k:  # fork: after step t-1, the last reader of slab (t+1) % 2
            draw_stream.wait_stream(main)
            with torch.cuda.stream(draw_stream):
              draw(t + 1)
              ev = torch.cuda.Event()
              ev.record(draw_stream)
            ready[(t + 1) % 2] = ev
        st = env.step(st, self._acts[t % 2])
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

    # one eager pass on a side stream fills the host-side caches (the env's
    # parameter block) and the allocator, as torch's capture recipe asks;
    # the state it produces is discarded and the statics restored. The hook
    # is left out of it (its side effects would count K extra steps).
    snap = [t.clone() for t in (self._qp, self._done, self._steps, self._rng) if t is not None]
    side = torch.cuda.Stream(dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
      body(hook=None)
    torch.cuda.current_stream(dev).wait_stream(side)
    for dst, src in zip([t for t in (self._qp, self._done, self._steps, self._rng)
                         if t is not None], snap):
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
