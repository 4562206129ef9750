"""Benchmark: env-steps/sec of Ant at 4096 envs per GPU (BASELINE.json).

One step = one `Env.step` of `envs.create('ant', batch_size=B,
episode_length=1000, auto_reset=True)`, i.e. ONE fused kernel launch doing
10 PBD substeps + observation + reward + Episode/AutoReset, on synthetic
U[-1,1] actions drawn on the device each step. Inputs are resident in HBM.

    python bench.py [--gpus N --steps K --warmup W --batch B]
    torchrun --nproc-per-node N bench.py --gpus N   (one rank per GPU)

Multi-GPU: every rank owns B envs (weak scaling, env ids offset by rank) and
the only collective is an RCCL all-gather of the per-env (reward, done) pair
each step. Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic HBM bytes per Ant env-step: QP in 520 + QP out
# 520 + action 32 + obs 348 + reward/done 8 = 1,428 B.
ANT_BYTES_PER_ENV_STEP = 1428
ANT_KERNEL = 'bx::env_step_kernel<16, 1, 32, 4>'  # rocprof name of the Ant env step (F_G1)
# Counted flops per Ant Env.step (reference numpy path).
ANT_FLOPS_PER_ENV_STEP = 87382
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8 TB/s HBM3E
FP32_VALU_PEAK_TFLOPS = 157.3


def _dist():
  ws = int(os.environ.get('WORLD_SIZE', '1'))
  if ws > 1:
    import torch.distributed as dist
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    local = int(os.environ.get('LOCAL_RANK', '0'))
    torch.cuda.set_device(local)
    dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    return dist, dist.get_rank(), ws, local
  return None, 0, 1, 0


def cpu_baseline(batch, min_seconds=10.0, max_steps=100000):
  """The oracle's float32 C restatement (OpenMP over envs) on this host's
  cores, on a bounded sample of the same workload."""
  from oracle.oracle import Oracle
  from tests.helpers import compiled
  _, d, rd, _ = compiled('ant')
  o = Oracle(d, rd, np.float32)
  threads = o.max_threads()
  rng = np.random.default_rng(0)
  B = batch
  T = np.load(os.path.join(ROOT, 'tests', 'golden', 'traj_ant.npz'))
  qp = np.repeat(T['qp'][0], (B + 63) // 64, axis=0)[:B].astype(np.float32)
  o.env_step('ant', qp[:64], rng.uniform(-1, 1, (64, 8)), 87, 10)  # warm
  t0 = time.perf_counter()
  steps = 0
  while steps < max_steps and (time.perf_counter() - t0) < min_seconds:
    act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
    qp, _, _, _, _ = o.env_step('ant', qp, act, 87, 10)
    steps += 1
  dt = time.perf_counter() - t0
  return {'value': B * steps / dt, 'unit': 'env-steps/s', 'cores': threads, 'kind': 'port',
          'sample': f'Ant, {B} envs x {steps} env-steps ({dt:.1f} s), float32 C '
                    f'restatement (oracle/pbd_oracle.c), {threads} OpenMP threads, '
                    f'{platform.processor() or platform.machine()}'}


PHASE_KERNELS = {'kinetic': 'bx::kinetic_kernel', 'update_acc': 'bx::update_acc_kernel',
                 'velocity_projection': 'bx::vproj_kernel',
                 'capsule_plane': 'bx::capsule_plane_kernel'}


def phase_bench(sys_, dev, batch=1 << 20, reps=20):
  """The integrator and collider phases as standalone SoA kernels
  (brax_amd.phases) over `batch` envs: algorithmic GB/s vs the HBM peak,
  timed with HIP events on the launch stream."""
  from brax_amd import phases
  from brax_amd.base import QP
  N = sys_.num_bodies
  g = torch.Generator(device=dev).manual_seed(0)
  soa = torch.rand((13, N, batch), device=dev, generator=g) - 0.5
  soa[3:7] += 1.0  # quaternion planes away from zero norm
  aux = torch.rand((13, N, batch), device=dev, generator=g) - 0.5
  aux[3:7] += 1.0
  out = soa.clone()
  contacts = torch.empty((10, sys_.num_rows, batch), device=dev)
  runs = {
      'kinetic': (lambda: phases.kinetic(sys_, soa, out), phases.BYTES[0] * N),
      'update_acc': (lambda: phases.update_acc(sys_, soa, aux[:6], out), phases.BYTES[1] * N),
      'velocity_projection': (lambda: phases.velocity_projection(sys_, soa, aux, out),
                              phases.BYTES[2] * N),
      'capsule_plane': (lambda: phases.capsule_plane(sys_, soa, contacts),
                        phases.BYTES['capsule_plane'] * sys_.num_rows),
  }
  res = {}
  for name, (fn, per_env) in runs.items():
    for _ in range(3):
      fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
      fn()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / reps
    gbs = per_env * batch / (us * 1e-6) / 1e9
    res[name] = {'us': us, 'bytes_per_launch': per_env * batch, 'achieved': gbs,
                 'frac': gbs / HBM_PEAK_GBS, 'traffic': None}
    k = ((_traffic() or {}).get('kernels') or {}).get(PHASE_KERNELS[name])
    if k and k.get('envs') == batch:
      res[name]['traffic'] = k['hbm_bytes_per_launch']
  del soa, aux, out, contacts
  return {'envs': batch, 'unit': 'GB/s', 'peak': HBM_PEAK_GBS, 'kernels': res}


def _time(fn, steps, warmup):
  """Wall-clock and HIP-event time of `steps` calls of fn after `warmup`."""
  for _ in range(warmup):
    fn()
  torch.cuda.synchronize()
  a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  t0 = time.perf_counter()
  a.record()
  for _ in range(steps):
    fn()
  b.record()
  torch.cuda.synchronize()
  return time.perf_counter() - t0, a.elapsed_time(b) * 1e-3


def secondary_configs(dev, steps=50):
  """BASELINE.json's other single-GPU configs, one short leg each:
  Humanoid Env.step at 4096 envs (configs[2]) and Ant Mountain(4)
  System.step at 2048 envs, all pairs and NearNeighbors cutoff 36 (configs[4];
  the reference's V100 plot, multiagent.ipynb:222-267, is at 1024 envs)."""
  from brax_amd import envs
  from brax_amd.envs.mountain import ant_mountain_config
  import brax_amd
  out = {}
  B = 4096
  env = envs.create('humanoid', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  st = [env.reset(np.array([0, 7], np.uint32))]
  act = torch.rand((B, env.action_size), device=dev) * 2 - 1

  def hstep():
    st[0] = env.step(st[0], act)
  wall, gpu = _time(hstep, steps, 5)
  out['humanoid_4096'] = {'value': B * steps / wall, 'unit': 'env-steps/s',
                          'ms_per_step': wall * 1e3 / steps, 'gpu_ms_per_step': gpu * 1e3 / steps}
  for cutoff in (0, 36):
    cfg = ant_mountain_config(4)
    cfg.collider_cutoff = cutoff
    sys_ = brax_amd.System(cfg, device=dev)
    Bm = 2048
    qp0 = sys_.default_qp()
    qp = [brax_amd.QP(*(t.unsqueeze(0).expand((Bm,) + t.shape).contiguous()
                        for t in (qp0.pos, qp0.rot, qp0.vel, qp0.ang)))]
    a = torch.rand((Bm, sys_.action_size), device=dev) * 2 - 1

    def mstep():
      qp[0], _ = sys_.step(qp[0], a)
    n = max(steps // 5, 5)
    wall, gpu = _time(mstep, n, 2)
    out[f'mountain4_2048_cutoff{cutoff}'] = {
        'value': Bm * n / wall, 'unit': 'env-steps/s (System.step)',
        'ms_per_step': wall * 1e3 / n, 'gpu_ms_per_step': gpu * 1e3 / n,
        'contact_rows': sys_.num_rows, 'lanes_per_env': sys_.lanes}
  return out


def _traffic():
  """HBM bytes per launch from the committed PMC profile, if present."""
  p = os.path.join(ROOT, 'profiles', 'traffic.json')
  if os.path.exists(p):
    with open(p) as f:
      return json.load(f)
  return None


def main():
  ap = argparse.ArgumentParser()
  ap.add_argument('--gpus', type=int, default=1)
  ap.add_argument('--steps', type=int, default=1000)
  ap.add_argument('--warmup', type=int, default=50)
  ap.add_argument('--batch', type=int, default=4096)
  ap.add_argument('--no-cpu-baseline', action='store_true')
  ap.add_argument('--no-phases', action='store_true',
                  help='skip the standalone SoA phase-kernel roofline leg')
  ap.add_argument('--phase-envs', type=int, default=1 << 20)
  ap.add_argument('--no-secondary', action='store_true',
                  help='skip the Humanoid / Ant Mountain legs')
  ap.add_argument('--generic', action='store_true',
                  help='force the generic item-loop kernel variant (A/B)')
  ap.add_argument('--block', type=int, default=0,
                  help='threads per workgroup of the step kernel (A/B; default 64)')
  ap.add_argument('--variant', default='',
                  help='lanes,mode kernel variant (mode 0 global, 1 single, 2 lds)')
  args = ap.parse_args()

  dist, rank, world, local = _dist()
  dev = torch.device('cuda', local)
  torch.cuda.set_device(dev)
  from brax_amd import _native, envs
  import ctypes as C

  B = args.batch
  env = envs.create('ant', batch_size=B, episode_length=1000, auto_reset=True, device=dev)
  if args.generic:
    _native.check(_native.lib().bx_system_set_single(env.sys._h, 0))
  if args.variant:
    lanes, mode = (int(x) for x in args.variant.split(','))
    _native.check(_native.lib().bx_system_set_variant(env.sys._h, lanes, mode))
  if args.block:
    _native.check(_native.lib().bx_system_set_block(env.sys._h, args.block))
  from brax_amd import distributed as bd
  state = env.reset(bd.rank_key(np.array([0, 0x5EED], np.uint32), rank))
  # synthetic U[-1,1] actions, one (B, 8) slab per step, drawn on the device by
  # the counter RNG before the timed region (inputs resident in HBM)
  n_act = args.warmup + args.steps
  acts = torch.empty((n_act, B, 8), dtype=torch.float32, device=dev)
  lib = _native.lib()
  _native.check(lib.bx_uniform(C.c_void_p(acts.data_ptr()), acts.numel(), 1 + rank, 0, -1.0,
                               1.0, C.c_void_p(torch.cuda.current_stream().cuda_stream)))
  exchange = bd.EpisodeExchange(B, dev) if world > 1 else None

  def one_step(st, k, ev=None):
    if ev is not None:
      ev[0].record()
    st = env.step(st, acts[k])
    if ev is not None:
      ev[1].record()
    if exchange is not None:
      exchange(st.reward, st.done)  # the one RCCL collective: (reward, done) all-gather
    return st

  for k in range(args.warmup):
    state = one_step(state, k)
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  torch.cuda.synchronize()
  # per-launch HIP events on every EVENT_EVERY-th step (the stream the kernel
  # runs on): the kernel's average launch duration for `roofline`, without
  # putting event packets between every pair of launches
  EVENT_EVERY = 8
  events = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            if k % EVENT_EVERY == 0 else None for k in range(args.steps)]
  span = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
  span[0].record()
  t0 = time.perf_counter()
  for k in range(args.steps):
    state = one_step(state, args.warmup + k, events[k])
  span[1].record()
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  torch.cuda.synchronize()
  elapsed = time.perf_counter() - t0
  kern_ms = float(np.mean([ev[0].elapsed_time(ev[1]) for ev in events if ev is not None]))
  span_ms = span[0].elapsed_time(span[1]) / args.steps
  if dist is not None:
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

  total = B * world * args.steps
  value = total / elapsed
  if rank != 0:
    dist.destroy_process_group()
    return
  bytes_per_launch = ANT_BYTES_PER_ENV_STEP * B
  achieved_gbs = bytes_per_launch / (kern_ms * 1e-3) / 1e9
  # PMC traffic of THIS kernel instantiation (Ant: 16 lanes, SINGLE mode,
  # feature mask 0, gather width 4), not the Humanoid one that shares its name
  tr = _traffic()
  k = ((tr or {}).get('kernels') or {}).get(ANT_KERNEL)
  traffic = k['hbm_bytes_per_launch'] if k and k.get('batch') == B else None
  out = {
      'metric': 'env-steps/sec (Ant, 4096 envs/GPU)',
      'value': value,
      'unit': 'env-steps/s',
      'n_gpus': world,
      'steps': args.steps,
      'warmup': args.warmup,
      'ms_per_step': elapsed * 1e3 / args.steps,
      'higher_is_better': True,
      'scaling': 'weak',
      'vs_baseline': None,
      'dtype': 'f32',
      'data': 'synthetic: U[-1,1] actions (device counter RNG, one slab per step, '
              'resident in HBM); reset from the Ant config with device-RNG joint noise',
      'config': {'workload': 'Ant-v1 Env.step (10 PBD substeps + obs/reward + '
                             'Episode/AutoReset), envs.create(ant)',
                 'envs_per_gpu': B, 'episode_length': 1000, 'substeps': 10,
                 'parallelism': f'env-shard x{world}'},
      'roofline': {'bound': 'hbm', 'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS,
                   'unit': 'GB/s', 'frac': achieved_gbs / HBM_PEAK_GBS,
                   'traffic': traffic,
                   'kernel': ANT_KERNEL, 'kernel_ms': kern_ms,
                   'span_ms_per_step': span_ms,
                   'bytes_per_launch': bytes_per_launch,
                   'note': 'fused env-step is VALU/latency-bound (AI ~61 flop/B, '
                           'SURVEY 8(d)); compute view below',
                   'valu_tflops': ANT_FLOPS_PER_ENV_STEP * B / (kern_ms * 1e-3) / 1e12,
                   'valu_peak_tflops': FP32_VALU_PEAK_TFLOPS},
  }
  out['secondary_configs'] = None if args.no_secondary else secondary_configs(dev)
  out['phase_roofline'] = (None if args.no_phases else
                           phase_bench(env.unwrapped.sys, dev, args.phase_envs))
  if world == 1 and not args.no_cpu_baseline:
    out['cpu_baseline'] = cpu_baseline(B)
  else:
    out['cpu_baseline'] = None
  print(json.dumps(out), flush=True)
  if dist is not None:
    dist.destroy_process_group()


if __name__ == '__main__':
  main()
