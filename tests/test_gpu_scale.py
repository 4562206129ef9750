"""Full-size configurations and the single-call reset boundary, on the GPU.

* `bx_env_reset` (one C call: noise, default_qp, reset-time Info, obs) gives
  the same bits as the explicit three-call path `reset_from(reset_noise(...))`.
* Ant at 32,768 envs (BASELINE configs[3], all envs on one GPU): determinism,
  unit quaternions, sampled fp64-oracle parity — and 8 shards of 4,096 envs,
  reset and stepped with global-env-id keyed noise and actions, reproduce the
  single 32,768 batch bit for bit (the reference shards by
  global index, `agents/ppo/train.py:276-283`).
* Ant Mountain(4) at 2,048 envs (configs[4]), all pairs and NearNeighbors
  cutoff 36: determinism, batch independence and sampled oracle parity.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from tests.helpers import QP_FIELDS, compiled, config_for

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
  assert torch.cuda.is_available(), 'GPU tests need a GPU'
  return torch.device('cuda', 0)


def _actions(B, A, step, seed, dev, rank=0, world=1):
  """(B, A) U[-1,1) actions keyed by (step, global env id), as bench.py."""
  from brax_amd import _native
  from brax_amd import distributed as bd
  out = torch.empty((B, A), dtype=torch.float32, device=dev)
  _native.check(_native.lib().bx_uniform(
      C.c_void_p(out.data_ptr()), B * A, seed, bd.action_offset(rank, B, A, step, world),
      -1.0, 1.0, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)))
  return out


@pytest.mark.parametrize('name', ['ant', 'humanoid', 'halfcheetah', 'humanoidstandup'])
def test_env_reset_matches_explicit_path(dev, name):
  """bx_env_reset == default_qp + info + obs of the same noise, bit for bit;
  reward/done/metrics start at zero."""
  from brax_amd import envs
  env = envs.get_environment(name, device=dev)
  B, off = 300, 1234
  key = np.array([5, 77], np.uint32)
  st = env.reset_batch(key, B, env_offset=off)
  qpos, qvel = env.reset_noise(key, B, env_offset=off)
  ref = env.reset_from(qpos, qvel)
  torch.cuda.synchronize()
  for f in ('pos', 'rot', 'vel', 'ang'):
    assert torch.equal(getattr(st.qp, f), getattr(ref.qp, f)), f
  assert torch.equal(st.obs, ref.obs)
  assert not st.reward.any() and not st.done.any()
  for k in env.metric_keys:
    assert not st.metrics[k].any(), k
  # noise is keyed by global env id: env 1234 + 7 reset alone is row 7
  one = env.reset_batch(key, 1, env_offset=off + 7)
  assert torch.equal(one.qp.pos[0], st.qp.pos[7]) and torch.equal(one.obs[0], st.obs[7])


def test_ant_32768_shards_reproduce_one_batch(dev, oracle_lib):
  """BASELINE configs[3] (Ant, 32,768 envs over 8 GPUs), rehearsed on one
  GPU: 8 shards of 4,096 envs with env_offset = r * 4096 reset to, and step
  through 3 Env.steps to, exactly the bits of the one 32,768-env batch."""
  from brax_amd import envs
  from brax_amd import distributed as bd
  from tests.test_gpu_parity import Envelope, _env_err, _gate
  world, Bs = 8, 4096
  B = world * Bs
  key = np.array([0, 0x5EED], np.uint32)
  big_env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  big = big_env.reset(key)
  shard_envs = [bd.shard_env(envs.create('ant', batch_size=Bs, episode_length=1000,
                                         auto_reset=True, device=dev), r, Bs)
                for r in range(world)]
  shards = [e.reset(key) for e in shard_envs]
  T = 3
  prev = None
  for t in range(T + 1):
    for r in range(world):
      sl = slice(r * Bs, (r + 1) * Bs)
      assert torch.equal(shards[r].qp.pos, big.qp.pos[sl]), (t, r)
      assert torch.equal(shards[r].qp.rot, big.qp.rot[sl]), (t, r)
      assert torch.equal(shards[r].qp.vel, big.qp.vel[sl]), (t, r)
      assert torch.equal(shards[r].obs, big.obs[sl]), (t, r)
      assert torch.equal(shards[r].reward, big.reward[sl]), (t, r)
    if t == T:
      break
    act = _actions(B, 8, t, 1, dev)
    prev = (big, act)
    big = big_env.step(big, act)
    shards = [shard_envs[r].step(shards[r], _actions(Bs, 8, t, 1, dev, r, world))
              for r in range(world)]
  torch.cuda.synchronize()
  # full-batch properties of the 32,768 batch
  st, act = prev
  again = big_env.step(st, act)
  assert torch.equal(again.qp.pos, big.qp.pos) and torch.equal(again.obs, big.obs)
  q = big.qp.rot
  assert torch.allclose(q.norm(dim=-1), torch.ones_like(q[..., 0]), atol=1e-5)
  assert torch.isfinite(big.obs).all()
  # sampled parity with the fp64 oracle (System.step of the last step)
  vc, d, rd, meta = compiled('ant')
  o64 = oracle_lib.Oracle(d, rd, np.float64, safe_guard=True)
  env32 = Envelope(oracle_lib, 'ant')
  idx = np.random.default_rng(7).choice(B, 256, replace=False)
  done = st.done.cpu().numpy()[idx]
  idx = idx[done == 0]  # auto-reset envs restart from first_qp instead
  qp_in = st.qp.numpy()[idx]
  an = act.cpu().numpy()[idx].astype(np.float64)
  ref, _ = o64.system_step(qp_in, an)
  outs = env32.system(qp_in, an)
  keep = big.done.cpu().numpy()[idx] == 0
  got = big.qp.numpy()[idx]
  for f, sl in QP_FIELDS.items():
    _gate(got[keep][..., sl], ref[keep][..., sl],
          _env_err([o[0][keep][..., sl] for o in outs], ref[keep][..., sl]), f)


@pytest.mark.parametrize('variant', ['multi', 'multi256', 'itemloop'])
@pytest.mark.parametrize('cutoff', [0, 36, 300])
def test_mountain4_full_batch(dev, oracle_lib, cutoff, variant):
  """BASELINE configs[4]: Ant Mountain(4) System.step at 2,048 envs
  (37 bodies, 630 capsule-capsule + 72 capsule-plane rows; NearNeighbors
  cutoff 36 as published): determinism, batch independence, unit
  quaternions and parity with the fp64 oracle on sampled envs. Both large-
  scene kernels: MULTI (the default: 128 threads per env, four envs per CU,
  gather tasks; and the same at 256 threads per env) and the item loops at
  256 threads per env. Cutoff 300 keeps more cells than
  one wave's 256 candidate keys: the NearNeighbors lists past a wave's
  sorted keys are empty (the bitonic lists' padding)."""
  import brax_amd
  from brax_amd import _native
  from tests.test_gpu_parity import Envelope, _env_err, _gate
  cfg = config_for('mountain4')
  cfg.collider_cutoff = cutoff
  sys_ = brax_amd.System(cfg, device=dev)
  assert sys_.lanes == 128  # the MULTI kernel's default width here: four envs per CU
  from tests.helpers import set_variant
  _native.check(set_variant(sys_, variant))
  B = 2048
  q0 = sys_.default_qp()
  qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                     for t in (q0.pos, q0.rot, q0.vel, q0.ang)))
  A = sys_.action_size
  for t in range(2):  # diverge the envs first
    qp, _ = sys_.step(qp, _actions(B, A, t, 3, dev))
  act = _actions(B, A, 2, 3, dev)
  a, ia = sys_.step(qp, act)
  b, _ = sys_.step(qp, act)
  torch.cuda.synchronize()
  assert torch.equal(a.pos, b.pos) and torch.equal(a.ang, b.ang)
  sub = brax_amd.QP(*(x[:3].contiguous() for x in (qp.pos, qp.rot, qp.vel, qp.ang)))
  c, ic = sys_.step(sub, act[:3])
  assert torch.equal(c.pos, a.pos[:3]) and torch.equal(c.vel, a.vel[:3])
  assert torch.equal(ic.contact_penetration, ia.contact_penetration[:3])
  assert torch.allclose(a.rot.norm(dim=-1), torch.ones_like(a.rot[..., 0]), atol=1e-5)
  assert torch.isfinite(a.vel).all()
  from brax_amd.compiler import compile_reset
  vc, d, meta = brax_amd.compiler.compile_system(cfg)
  rd = compile_reset(vc, meta['body_index'])
  o64 = oracle_lib.Oracle(d, rd, np.float64, safe_guard=True)
  env32 = Envelope(oracle_lib, None, desc=(d, rd))
  idx = np.random.default_rng(11).choice(B, 8, replace=False)
  qp_in = qp.numpy()[idx]
  an = act.cpu().numpy()[idx].astype(np.float64)
  ref, _ = o64.system_step(qp_in, an)
  outs = env32.system(qp_in, an)
  got = a.numpy()[idx]
  for f, sl in QP_FIELDS.items():
    _gate(got[..., sl], ref[..., sl], _env_err([o[0][..., sl] for o in outs], ref[..., sl]), f)


@pytest.mark.parametrize('cutoff', [0, 36])
def test_mountain4_multi_vs_item_loops(dev, oracle_lib, cutoff):
  """The two large-scene kernels round differently: the MULTI kernel's body
  integration keeps the build's fast quotients (`qnormalize(r, true)`: v_rcp
  + multiply, ~1.5 ulp), the item loops take Newton-corrected ones (`ndiv`,
  correctly rounded but for ties); a scene whose MULTI tables do not fit runs
  the item loops, so a system's rounding can change with its size. Recorded
  here: on the same 2,048 diverged envs, each env's normwise distance between
  the two kernels' states, against the sum of their two parity bounds
  (2 x max(1e-5, 2 x E32_i): each kernel within its own bound of the float64
  reference, sampled envs), and the distances themselves in the margins file
  (`multi_vs_items:<field>`)."""
  import brax_amd
  from brax_amd import _native
  from tests.margins import record_margin
  from tests.test_gpu_parity import Envelope, _env_err
  from tests.helpers import normwise
  cfg = config_for('mountain4')
  cfg.collider_cutoff = cutoff
  sys_ = brax_amd.System(cfg, device=dev)
  B = 2048
  q0 = sys_.default_qp()
  qp = brax_amd.QP(*(t.unsqueeze(0).expand((B,) + t.shape).contiguous()
                     for t in (q0.pos, q0.rot, q0.vel, q0.ang)))
  A = sys_.action_size
  for t in range(2):  # diverge the envs first (on the default kernel)
    qp, _ = sys_.step(qp, _actions(B, A, t, 3, dev))
  act = _actions(B, A, 2, 3, dev)
  out = {}
  from tests.helpers import set_variant
  for variant in ('multi', 'items'):
    _native.check(set_variant(sys_, variant))
    out[variant] = sys_.step(qp, act, info=False)[0].numpy()
  from brax_amd.compiler import compile_reset
  vc, d, meta = brax_amd.compiler.compile_system(cfg)
  rd = compile_reset(vc, meta['body_index'])
  o64 = oracle_lib.Oracle(d, rd, np.float64, safe_guard=True)
  env32 = Envelope(oracle_lib, None, desc=(d, rd))
  idx = np.random.default_rng(12).choice(B, 8, replace=False)
  qp_in = qp.numpy()[idx]
  an = act.cpu().numpy()[idx].astype(np.float64)
  ref, _ = o64.system_step(qp_in, an)
  outs = env32.system(qp_in, an)
  for f, sl in QP_FIELDS.items():
    dist = normwise(out['multi'][..., sl], out['items'][..., sl])
    e32 = np.asarray(_env_err([o[0][..., sl] for o in outs], ref[..., sl]))
    bound = 2 * np.maximum(1e-5, 2 * e32)
    ds = dist[idx]
    k = int(np.argmax(ds / bound))
    record_margin(f'multi_vs_items:{f}', float(ds[k]), float(bound[k]), n=len(idx),
                  pair_ratios=(ds / bound).tolist(), role='record', full_batch_max=float(dist.max()),
                  full_batch_p50=float(np.median(dist)))
    assert (ds <= bound).all(), (f, ds, bound)
    assert np.isfinite(dist).all()
