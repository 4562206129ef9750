"""Open-loop rollouts: K `Env.step`s in ONE kernel launch.

The reference collects trajectories by scanning `env.step` under `jit`
(`brax/training/acting.py:53-77`, `generate_unroll`: `jax.lax.scan` of
`actor_step`); when the actions are known up front (random-action rollouts,
replayed action sequences, the reference notebook's benchmark loop) the scan
is open-loop. `rollout(env, state, actions)` runs that scan through
`bx_env_rollout_packed`: one launch steps every env K times, the state held on
chip between steps, and writes every step's complete output (state, obs,
reward, done, episode counters, metrics, the target envs' streams) to HBM -
bit for bit the outputs of K chained `env.step` calls
(`tests/test_gpu_rollout.py`).
"""
import ctypes as C
import dataclasses
from typing import Any, Optional, Tuple

import torch

from brax_amd import _native
from brax_amd.base import PackedQP, packed_buffer
from brax_amd.envs.env import PhysicsEnv, State, Wrapper, _f32, _Metrics
from brax_amd.system import _stream


@dataclasses.dataclass(frozen=True)
class Trajectory:
  """Every step of a rollout, leading axis K (steps) then B (envs):
  qp (K, B, N, 16) packed (pos 0:3, rot 3:7, vel 7:10, ang 10:13), obs
  (K, B, O), reward / done / steps / truncation (K, B), metrics (K, B, M)
  with `metric_keys` naming the columns, rng (K, B) for the target envs."""
  qp: Any
  obs: Any
  reward: Any
  done: Any
  steps: Any
  truncation: Any
  metrics: Any
  metric_keys: Tuple[str, ...]
  rng: Optional[Any] = None


def chain_options(env):
  """The PhysicsEnv under a wrapper chain and the options the fused kernel
  applies for it: EpisodeWrapper (episode_length, action_repeat),
  AutoResetWrapper (auto_reset); Vector / Vmap wrappers pass through.
  Other wrappers have no fused form: NotImplementedError."""
  from brax_amd.envs import wrappers  # pylint: disable=import-outside-toplevel
  opts = {}
  w = env
  while isinstance(w, Wrapper):
    if isinstance(w, wrappers.EpisodeWrapper):
      opts['episode_length'] = w.episode_length
      opts['action_repeat'] = w.action_repeat
    elif isinstance(w, wrappers.AutoResetWrapper):
      opts['auto_reset'] = True
    elif not isinstance(w, (wrappers.VectorWrapper, wrappers.VmapWrapper)):
      raise NotImplementedError(f'{type(w).__name__} has no fused rollout')
    w = w.env
  if not isinstance(w, PhysicsEnv):
    raise NotImplementedError(f'{type(w).__name__} is not a kernel env')
  return w, opts


def rollout(env, state: State, actions, out: Optional[torch.Tensor] = None
            ) -> Tuple[State, Trajectory]:
  """K consecutive `env.step(state, actions[t])` in one launch.

  Args:
    env: an env from `brax_amd.envs.create` (Episode / AutoReset / Vector
      wrappers over a kernel env).
    state: the state to start from (a batch of B envs).
    actions: (K, B, A) float32 on the env's device (any strides with a
      unit last-axis stride).
    out: optional flat float32 buffer of K * B * (N*16 + O + 4 + M) floats
      for the trajectory (reused across calls by graph captures).
  Returns:
    (the state after the K-th step, the Trajectory of all K steps); the
    state's tensors are views into the trajectory's last step.
  """
  u, opts = chain_options(env)
  dev = u.sys.device
  qbuf = packed_buffer(state.qp)
  if qbuf is None:
    qbuf = torch.zeros(state.qp.pos.shape[:-1] + (16,), dtype=torch.float32, device=dev)
    for lo, f in ((0, state.qp.pos), (3, state.qp.rot), (7, state.qp.vel), (10, state.qp.ang)):
      qbuf[..., lo:lo + f.shape[-1]] = f
  if qbuf.dtype != torch.float32 or qbuf.device != dev or not qbuf.is_contiguous():
    qbuf = qbuf.to(dev, torch.float32).contiguous()
  B = qbuf.shape[0]
  act = actions
  if type(act) is not torch.Tensor or act.dtype != torch.float32 or act.device != dev:
    act = torch.as_tensor(act, dtype=torch.float32, device=dev)
  if act.dim() != 3 or act.shape[1] != B or act.shape[2] != u.action_size:
    raise ValueError(f'actions {tuple(act.shape)} != (K, {B}, {u.action_size})')
  if act.stride(-1) != 1:
    act = act.contiguous()
  K = act.shape[0]
  auto = bool(opts.get('auto_reset'))
  info_in = state.info
  first_qp = info_in.get('first_qp') if auto else None
  first_obs = info_in.get('first_obs') if auto else None
  if auto and (first_qp is None or first_obs is None):
    raise ValueError('AutoResetWrapper state lacks first_qp / first_obs')
  p = u._cached_params(opts, first_qp, first_obs)  # pylint: disable=protected-access
  done_in = _f32(state.done, dev)
  steps_in = info_in.get('steps')
  if steps_in is not None:
    steps_in = _f32(steps_in, dev)
  rng_in = info_in.get('rng')
  if rng_in is None and getattr(u, 'needs_rng', False):
    rng_in = torch.zeros((B,), dtype=torch.int32, device=dev)
  N, O, M = u.sys.num_bodies, u.obs_size, len(u.metric_keys)
  block = B * (N * 16 + O + 4 + M)
  if out is None:
    out = torch.empty((K * block,), dtype=torch.float32, device=dev)
  elif (out.numel() < K * block or out.dtype != torch.float32 or not out.is_contiguous()
        or out.device != dev):
    raise ValueError(f'out must hold {K * block} contiguous float32 on {dev}')
  rng_out = torch.empty((K, B), dtype=torch.int32, device=dev) if rng_in is not None else None
  _native.check(_native.lib().bx_env_rollout_packed(
      u.sys._h, C.byref(p), B, K, qbuf.data_ptr(), done_in.data_ptr(),  # pylint: disable=protected-access
      None if steps_in is None else steps_in.data_ptr(),
      None if rng_in is None else rng_in.data_ptr(), act.data_ptr(), act.stride(1),
      act.stride(0), act.shape[2], out.data_ptr(),
      None if rng_out is None else rng_out.data_ptr(), _stream(dev.index)))
  blocks = out[:K * block].view(K, block)
  q, obs, sc, met = torch.split(blocks, (B * N * 16, B * O, 4 * B, B * M), dim=1)
  q = q.view(K, B, N, 16)
  obs = obs.view(K, B, O)
  sc = sc.view(K, 4, B)
  met = met.view(K, B, M)
  traj = Trajectory(qp=q, obs=obs, reward=sc[:, 0], done=sc[:, 1], steps=sc[:, 2],
                    truncation=sc[:, 3], metrics=met, metric_keys=tuple(u.metric_keys),
                    rng=rng_out)
  info = dict(info_in)
  if p.episode_length > 0:
    info['steps'] = sc[K - 1, 2]
    info['truncation'] = sc[K - 1, 3]
  if rng_out is not None:
    info['rng'] = rng_out[K - 1]
  keys = u.metric_keys
  m_in = state.metrics
  extra = m_in.carried(keys) if type(m_in) is _Metrics else {
      k: v for k, v in m_in.items() if k not in keys}
  final = State(qp=PackedQP(q[K - 1]), obs=obs[K - 1], reward=sc[K - 1, 0], done=sc[K - 1, 1],
                metrics=_Metrics(met[K - 1] if M else None, keys, extra), info=info)
  return final, traj


class RolloutGraph:
  """`rollout` of K steps with on-device action draws, captured as one HIP
  graph: per replay ONE `bx_uniform_slabs` launch draws the K action slabs
  (slab t at `offset + (r * K + t) * step_stride`, the eager loop's
  `bx_uniform` offsets, as `StepGraph` draws them), ONE
  `bx_env_rollout_packed` launch steps every env K times, and the K-th state
  is fed back into the graph's static inputs. `hook(traj)` (device work
  only) is recorded after the rollout, e.g. the episodic (reward, done) sum
  over the K steps. `replay()` returns (state after the K-th step,
  trajectory), valid until the next replay."""

  def __init__(self, env, state: State, k: int, seed: int = 1, offset: int = 0,
               step_stride: Optional[int] = None, lo: float = -1.0, hi: float = 1.0,
               hook=None):
    from brax_amd.envs.graph import _static  # pylint: disable=import-outside-toplevel
    if k < 1:
      raise ValueError(f'k must be >= 1, got {k}')
    u, _ = chain_options(env)
    dev = u.sys.device
    self.env, self.k, self.device = env, int(k), dev
    buf = packed_buffer(state.qp)
    B = (buf if buf is not None else state.qp.pos).shape[0]
    A = env.action_size
    stride = B * A if step_stride is None else int(step_stride)
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
      rng = torch.zeros((B,), dtype=torch.int32, device=dev)
    self._rng = _static(rng)
    if self._steps is not None:
      info['steps'] = self._steps
    if self._rng is not None:
      info['rng'] = self._rng
    self._in = State(qp=PackedQP(self._qp), obs=state.obs, reward=state.reward,
                     done=self._done, metrics=state.metrics, info=info)
    self._acts = torch.empty((self.k, B, A), dtype=torch.float32, device=dev)
    N, O, M = u.sys.num_bodies, u.obs_size, len(u.metric_keys)
    self._out = torch.empty((self.k * B * (N * 16 + O + 4 + M),), dtype=torch.float32,
                            device=dev)
    self._epoch = torch.zeros((1,), dtype=torch.int64, device=dev)
    lib = _native.lib()

    def body(hook=hook):
      _native.check(lib.bx_uniform_slabs(
          C.c_void_p(self._acts.data_ptr()), B * A, self.k, seed, offset, stride,
          C.c_void_p(self._epoch.data_ptr()), self.k * stride, lo, hi, _stream(dev.index)))
      st, tr = rollout(env, self._in, self._acts, out=self._out)
      if hook is not None:
        hook(tr)
      self._qp.copy_(packed_buffer(st.qp))
      self._done.copy_(st.done)
      if self._steps is not None:
        self._steps.copy_(st.info['steps'])
      if self._rng is not None:
        self._rng.copy_(st.info['rng'])
      self._epoch.add_(1)
      return st, tr

    with torch.cuda.device(dev):
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
      with torch.cuda.graph(self.graph, capture_error_mode='thread_local'):
        self._res = body()
      torch.cuda.current_stream(dev).synchronize()

  def replay(self):
    """Steps every env K steps forward; returns (state, trajectory)."""
    self.graph.replay()
    return self._res


class RolloutRunner:
  """Back-to-back open-loop rollouts of K steps with on-device action draws,
  launched directly: per `run()` ONE `bx_env_rollout_random` launch that
  draws each step's actions inside the kernel (the K slabs at the eager
  loop's `bx_uniform` offsets: chunk c's slab t at `offset + (c * K + t) *
  step_stride`, recorded in `actions()`) and steps every env K times; for a
  system whose staged action row is narrower than the env's action (`draw`
  False), one `bx_uniform_slabs` launch and one `bx_env_rollout_packed`
  launch instead. Two trajectory buffers alternate: chunk c reads its input
  state from chunk c - 1's last step in place (no copies); one C call of host
  time per run, on the caller's current stream. `hook(traj)` runs after each
  rollout (device work, e.g. the episodic sums). `state()` is the state after
  the last run."""

  def __init__(self, env, state: State, k: int, seed: int = 1, offset: int = 0,
               step_stride: Optional[int] = None, lo: float = -1.0, hi: float = 1.0,
               hook=None):
    if k < 1:
      raise ValueError(f'k must be >= 1, got {k}')
    u, opts = chain_options(env)
    dev = u.sys.device
    self.env, self.k, self.device, self.hook = env, int(k), dev, hook
    self._u = u
    buf = packed_buffer(state.qp)
    B = (buf if buf is not None else state.qp.pos).shape[0]
    A = env.action_size
    self.B, self.A = B, A
    self.seed, self.offset, self.lo, self.hi = seed, int(offset), float(lo), float(hi)
    self.stride = B * A if step_stride is None else int(step_stride)
    N, O, M = u.sys.num_bodies, u.obs_size, len(u.metric_keys)
    self.N, self.O, self.M = N, O, M
    self.block = B * (N * 16 + O + 4 + M)
    self._out = torch.empty((2, self.k * self.block), dtype=torch.float32, device=dev)
    needs_rng = state.info.get('rng') is not None or getattr(u, 'needs_rng', False)
    self._rng = torch.zeros((2, self.k, B), dtype=torch.int32, device=dev) if needs_rng else None
    self._acts = torch.empty((self.k, B, A), dtype=torch.float32, device=dev)
    auto = bool(opts.get('auto_reset'))
    self._first = (state.info.get('first_qp'), state.info.get('first_obs')) if auto else (None, None)
    if auto and None in self._first:
      raise ValueError('AutoResetWrapper state lacks first_qp / first_obs')
    self._p = u._params(opts, *self._first)  # pylint: disable=protected-access
    self._has_steps = self._p.episode_length > 0
    # the starting state goes into buffer 1's last step: chunk 0 reads it there
    last = self._views(1)
    if buf is None:
      for lo_, f in ((0, state.qp.pos), (3, state.qp.rot), (7, state.qp.vel), (10, state.qp.ang)):
        last['qp'][..., lo_:lo_ + f.shape[-1]] = f
    else:
      last['qp'].copy_(buf)
    last['done'].copy_(torch.as_tensor(state.done, dtype=torch.float32, device=dev))
    if state.info.get('steps') is not None:
      last['steps'].copy_(torch.as_tensor(state.info['steps'], dtype=torch.float32, device=dev))
    else:
      last['steps'].zero_()
    if self._rng is not None and state.info.get('rng') is not None:
      self._rng[1, self.k - 1].copy_(state.info['rng'])
    self._metrics_in = state.metrics
    self._info_in = dict(state.info)
    self._c = 0
    self._cur = 1  # the buffer holding the latest trajectory
    self._lib = _native.lib()
    # one-launch draws when the system stages the whole action row (probed
    # with a zero-step call: argument checks only)
    self.draw = self._lib.bx_env_rollout_random(
        self._u.sys._h, C.byref(self._p), B, 0, None, None, None, None, 0, 0, 0,  # pylint: disable=protected-access
        0.0, 1.0, A, None, None, None, None) == 0
    # the launch's C arguments per buffer parity, built once (run() then
    # passes ctypes objects straight through: the host half of a launch is
    # on the critical path of a short timed region)
    self._args = {}
    self._stream_key = None

  def _views(self, i):
    K, B, N, O, M = self.k, self.B, self.N, self.O, self.M
    blk = self._out[i].view(K, self.block)[K - 1]
    q, obs, sc, met = torch.split(blk, (B * N * 16, B * O, 4 * B, B * M))
    sc = sc.view(4, B)
    return {'qp': q.view(B, N, 16), 'obs': obs.view(B, O), 'reward': sc[0], 'done': sc[1],
            'steps': sc[2], 'truncation': sc[3], 'metrics': met.view(B, M)}

  def _launch_args(self, src, stream):
    """(the arguments before the draw offset, the ones after it) of the
    launch that reads buffer `src` and writes the other, on `stream`."""
    dst = 1 - src
    K, B, N, O = self.k, self.B, self.N, self.O
    base = self._out[src].data_ptr() + 4 * (K - 1) * self.block
    sc = base + 4 * B * (N * 16 + O)
    rng_in = None if self._rng is None else self._rng[src, K - 1].data_ptr()
    rng_out = None if self._rng is None else self._rng[dst].data_ptr()
    steps_in = sc + 8 * B if self._has_steps else None
    vp = C.c_void_p
    h = self._u.sys._h  # pylint: disable=protected-access
    if self.draw:
      pre = (h, C.byref(self._p), C.c_int64(B), C.c_int32(K), vp(base), vp(sc + 4 * B),
             vp(steps_in), vp(rng_in), C.c_uint64(self.seed))
      post = (C.c_uint64(self.stride), C.c_float(self.lo), C.c_float(self.hi),
              C.c_int64(self.A), vp(self._acts.data_ptr()), vp(self._out[dst].data_ptr()),
              vp(rng_out), stream)
    else:
      pre = (vp(self._acts.data_ptr()), C.c_int64(B * self.A), C.c_int64(K),
             C.c_uint64(self.seed))
      post = ((C.c_uint64(self.stride), None, C.c_uint64(0), C.c_float(self.lo),
               C.c_float(self.hi), stream),
              (h, C.byref(self._p), C.c_int64(B), C.c_int32(K), vp(base), vp(sc + 4 * B),
               vp(steps_in), vp(rng_in), vp(self._acts.data_ptr()), C.c_int64(self.A),
               C.c_int64(B * self.A), C.c_int64(self.A), vp(self._out[dst].data_ptr()),
               vp(rng_out), stream))
    return pre, post

  def run(self):
    """Draws the next K action slabs and steps every env K steps."""
    src = self._cur
    stream = _stream(self.device.index)
    if stream.value != self._stream_key:  # the caller's current stream moved
      self._args = {}
      self._stream_key = stream.value
    a = self._args.get(src)
    if a is None:
      a = self._args[src] = self._launch_args(src, stream)
    pre, post = a
    off = C.c_uint64(self.offset + self._c * self.k * self.stride)
    if self.draw:
      _native.check(self._lib.bx_env_rollout_random(*pre, off, *post))
    else:
      _native.check(self._lib.bx_uniform_slabs(*pre, off, *post[0]))
      _native.check(self._lib.bx_env_rollout_packed(*post[1]))
    self._cur = 1 - src
    self._c += 1
    if self.hook is not None:
      self.hook(self.trajectory())

  def actions(self):
    """The last run's (K, B, A) actions."""
    return self._acts

  def trajectory(self) -> Trajectory:
    K, B, N, O, M = self.k, self.B, self.N, self.O, self.M
    blocks = self._out[self._cur].view(K, self.block)
    q, obs, sc, met = torch.split(blocks, (B * N * 16, B * O, 4 * B, B * M), dim=1)
    sc = sc.view(K, 4, B)
    return Trajectory(qp=q.view(K, B, N, 16), obs=obs.view(K, B, O), reward=sc[:, 0],
                      done=sc[:, 1], steps=sc[:, 2], truncation=sc[:, 3],
                      metrics=met.view(K, B, M), metric_keys=tuple(self._u.metric_keys),
                      rng=None if self._rng is None else self._rng[self._cur])

  def state(self) -> State:
    """The state after the last run (views of the current trajectory)."""
    v = self._views(self._cur)
    info = dict(self._info_in)
    if self._has_steps:
      info['steps'] = v['steps']
      info['truncation'] = v['truncation']
    if self._rng is not None:
      info['rng'] = self._rng[self._cur, self.k - 1]
    keys = self._u.metric_keys
    m_in = self._metrics_in
    extra = m_in.carried(keys) if type(m_in) is _Metrics else {
        k: v_ for k, v_ in m_in.items() if k not in keys}
    return State(qp=PackedQP(v['qp']), obs=v['obs'], reward=v['reward'], done=v['done'],
                 metrics=_Metrics(v['metrics'] if self.M else None, keys, extra), info=info)
