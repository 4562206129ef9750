"""Benchmark: env-steps/sec of Ant at 4096 envs per GPU (BASELINE.json).

One step = a fresh (B, 8) slab of synthetic U[-1,1] actions drawn on the
device by the counter RNG (keyed by step and global env id; the reference's
published loop draws one per step, notebooks/environments.ipynb:386-423) + one
`Env.step` of `envs.create('ant', batch_size=B, episode_length=1000,
auto_reset=True)`: 10 PBD substeps + observation + reward + Episode/AutoReset.
Inputs are resident in HBM.

`value` is the `direct` loop, by design: `RolloutRunner`, ONE
`bx_env_rollout_random` launch per K steps (K = steps up to 200, else
gcd(steps, 50)) that draws each step's actions inside the kernel and steps
every env K times, the state read in place from the previous launch's last
step (the reference's lax.scan of env.step with the random actions drawn in
the loop). Its timed region (barrier + synchronisation on both sides,
exactly `--steps` steps) runs `--repeats` times (default 5) and `value` is the
median region: at the driver's 20 steps a region is ONE launch, and a lone
launch or clock hiccup would move a single sample by several percent (every
sample is in `timed_regions`). The other loops are reported beside it for the
record:
`eager_loop` (Python: bx_uniform + Env.step per step), `graph_loop`
(StepGraph: a hipGraph of one draw + K Env.step launches: the closed-loop
per-step path) and `rollout_loop` (RolloutGraph: a hipGraph of one draw + one
bx_env_rollout_packed launch). Only if the direct loop cannot run is `value`
taken from the next loop in that order, and `timed_loop` says which.
`roofline.kernel_ms` times the headline loop's own launch (back-to-back
RolloutRunner.run() calls bracketed by HIP events on their stream).

    python bench.py [--gpus N --steps K --warmup W --batch B]
    torchrun --nproc-per-node N bench.py --gpus N   (one rank per GPU)

Multi-GPU: rank r owns the global envs [r*B, (r+1)*B) (weak scaling). Reset
noise and actions are keyed by global env id with one shared seed, so the
ranks together step exactly the envs of one N*B batch; the only collective is
the episodic exchange: each rank sums its envs' (reward, done) on the device
every step, and the sums are all-gathered over RCCL once per episode length
(1000 steps), or once per timed run when that is shorter, so the timed region
always holds at least one collective (`collectives_in_timed_region`). Prints
ONE JSON line on rank 0.
"""
import argparse
import gc
import json
import math
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
# rocprof name of the Ant env step: 16 lanes, SINGLE mode, features F_G1 |
# F_JH (one collider group per body, joint halves), gather width 4, the Ant
# env program only (EK_ANT)
ANT_KERNEL = 'bx::env_step_packed_kernel<16, 1, 160, 4, 1>'
# the same instantiation under its multi-step name: K-step open-loop rollout
# launches (bx_env_rollout_packed)
ANT_ROLLOUT_KERNEL = 'bx::env_rollout_kernel<16, 1, 160, 4, 1>'
# Counted flops per Ant Env.step (reference numpy path).
ANT_FLOPS_PER_ENV_STEP = 87382
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: 8 TB/s HBM3E
FP32_VALU_PEAK_TFLOPS = 157.3
# the reference's published Ant 4,096-env rollout rate
REF_PUBLISHED = 895723.0
# steps per captured graph of the timed loop: the whole timed run up to
# GRAPH_MAX steps (one replay, one action draw), else gcd(steps, GRAPH_STEPS)
GRAPH_STEPS = 50
GRAPH_MAX = 200
# least warm-up of each replayed loop, seconds of its own work
WARM_S = 0.02
# the timed loops, in order: the eager Python loop, StepGraph replays,
# RolloutGraph replays, RolloutRunner (direct rollout launches)
KINDS = ('eager', 'step', 'rollout', 'direct')


def graph_steps(steps):
  return steps if steps <= GRAPH_MAX else math.gcd(steps, GRAPH_STEPS)


def _dist():
  ws = int(os.environ.get('WORLD_SIZE', '1'))
  # BX_DIST_FORCE=1: the process group (and the episodic RCCL exchange) even
  # at world size 1, e.g. `torchrun --nproc-per-node 1`: the one-GPU box then
  # executes the N-GPU run's collective path on RCCL
  if ws > 1 or os.environ.get('BX_DIST_FORCE') == '1':
    import torch.distributed as dist
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # BX_DIST_BACKEND=gloo: a rehearsal of the N-rank path with several ranks
    # on one GPU (RCCL refuses duplicate devices); the product run is RCCL
    backend = os.environ.get('BX_DIST_BACKEND', 'nccl')
    if backend != 'nccl':
      local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    if backend == 'nccl':
      dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
      dist.init_process_group(backend)
    return dist, dist.get_rank(), ws, local
  return None, 0, 1, 0


def rank_plan(gpus, environ):
  """What `bench.py --gpus N` does in a process with environment `environ`:
  ('run', None) when it is a rank of an N-process world (or N = 1 alone);
  ('spawn', None) when N > 1 and no launcher set WORLD_SIZE, so this parent
  must start the N ranks itself; ('refuse', why) when the world a launcher
  made disagrees with --gpus (the line would name the wrong experiment)."""
  if gpus < 1:
    return 'refuse', f'--gpus {gpus}: need at least one GPU'
  ws = environ.get('WORLD_SIZE')
  if ws is None:
    return ('spawn', None) if gpus > 1 else ('run', None)
  if int(ws) != gpus:
    return 'refuse', (f'--gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks: '
                      'run with --gpus equal to the world size')
  return 'run', None


def rank_env(environ, rank, world, port):
  """The environment of rank `rank` of a `world`-process run started by
  `spawn_ranks` (torchrun's variables, one process per local GPU)."""
  e = dict(environ)
  e.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
           LOCAL_WORLD_SIZE=str(world), GROUP_RANK='0', MASTER_ADDR='127.0.0.1',
           MASTER_PORT=str(port))
  return e


def _count_list(v):
  return len([x for x in v.split(',') if x.strip() != ''])


def visible_gpus(environ, topology='/sys/class/kfd/kfd/topology/nodes'):
  """GPUs this process would see, without touching HIP: the device lists of
  HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (indices into what
  ROCR_VISIBLE_DEVICES leaves), else ROCR_VISIBLE_DEVICES, else the GPU nodes
  of the KFD topology (sysfs text; a node with SIMDs is a GPU, CPU nodes have
  none). None when neither says."""
  rocr = environ.get('ROCR_VISIBLE_DEVICES')
  for k in ('HIP_VISIBLE_DEVICES', 'CUDA_VISIBLE_DEVICES'):
    v = environ.get(k)
    if v is not None:
      n = _count_list(v)
      return min(n, _count_list(rocr)) if rocr is not None else n
  if rocr is not None:
    return _count_list(rocr)
  try:
    nodes = os.listdir(topology)
  except OSError:
    return None
  n = 0
  for d in nodes:
    try:
      with open(os.path.join(topology, d, 'properties')) as f:
        props = dict(line.split()[:2] for line in f if len(line.split()) >= 2)
    except OSError:
      continue
    if int(props.get('simd_count', '0')) > 0:
      n += 1
  return n


def spawn_ranks(gpus, argv, script=None):
  """`python bench.py --gpus N` without a launcher: start N fresh rank
  processes of this script (one per GPU, torchrun's environment) BEFORE this
  parent touches the GPU, wait for all of them, and return the first failing
  rank's exit status (the others are stopped then, since they would wait at a
  barrier forever). Rank 0 prints the JSON line. (`script`: another program
  in the ranks' place, for the CPU test of this contract.)"""
  import signal
  import socket
  import subprocess
  backend = os.environ.get('BX_DIST_BACKEND', 'nccl')
  if backend == 'nccl':
    # counted from the environment / the KFD topology: no HIP call in this
    # parent (torch.cuda.device_count() falls back to hipGetDeviceCount when
    # amdsmi is unavailable, which would initialise HIP before the ranks start)
    have = visible_gpus(os.environ)
    if have is not None and have < gpus:
      print(f'bench.py: --gpus {gpus} but {have} GPUs visible', file=sys.stderr)
      return 2
  with socket.socket() as s:
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
  procs = [subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + list(argv),
                            env=rank_env(os.environ, r, gpus, port))
           for r in range(gpus)]

  def stop(*_):
    for q in procs:  # our own children, by PID
      if q.poll() is None:
        q.terminate()
  # a launcher that stops this parent stops its ranks too
  prev = signal.signal(signal.SIGTERM, lambda *a: (stop(), sys.exit(143)))
  try:
    return _wait_ranks(procs, stop)
  except BaseException:
    # KeyboardInterrupt / SystemExit / an error while waiting: no rank is
    # left running (a rank blocked at a barrier would hold its GPU)
    stop()
    for q in procs:
      try:
        q.wait(timeout=15)
      except subprocess.TimeoutExpired:
        q.kill()
        q.wait()
    raise
  finally:
    signal.signal(signal.SIGTERM, prev)


def _wait_ranks(procs, stop):
  rc, t_stop = 0, None
  live = list(procs)
  while live:
    for p in list(live):
      code = p.poll()
      if code is None:
        continue
      live.remove(p)
      if code != 0 and rc == 0:
        rc = code if code > 0 else 128 - code
        stop()
        t_stop = time.monotonic()
    if t_stop is not None and live and time.monotonic() - t_stop > 15:
      for q in live:
        q.kill()
      t_stop = None
    time.sleep(0.05)
  return rc


def host_cpu():
  """This host's CPU: `nproc`, the CPUs this process may run on, and the
  /proc/cpuinfo model name."""
  model = platform.processor() or platform.machine()
  try:
    with open('/proc/cpuinfo') as f:
      for line in f:
        if line.startswith('model name'):
          model = line.split(':', 1)[1].strip()
          break
  except OSError:
    pass
  try:
    allowed = len(os.sched_getaffinity(0))
  except AttributeError:
    allowed = os.cpu_count()
  return {'nproc': os.cpu_count(), 'allowed_cpus': allowed, 'model': model}


def cpu_baseline(batch, min_seconds=10.0, max_steps=100000):
  """The oracle's float32 C restatement (OpenMP over envs) on this host's
  cores, on a bounded sample of the same workload. The thread count is
  OpenMP's default: every CPU this process may use, or OMP_NUM_THREADS
  where the host sets it (the GPU box sets it to its CPU share per GPU)."""
  from oracle.oracle import Oracle
  from tests.helpers import compiled
  _, d, rd, _ = compiled('ant')
  o = Oracle(d, rd, np.float32)
  threads = o.max_threads()
  cpu = host_cpu()
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
          'nproc': cpu['nproc'], 'allowed_cpus': cpu['allowed_cpus'], 'cpu_model': cpu['model'],
          'omp_num_threads': os.environ.get('OMP_NUM_THREADS'),
          # the box's CPU share is OMP_NUM_THREADS (the operator's setting);
          # nproc counts the whole shared host
          'per_core': B * steps / dt / max(threads, 1),
          # the reference's own JAX-CPU floor for this env
          'reference_cpu_floor': {'value': 990.0, 'unit': 'env-steps/s',
                                  'source': 'brax/tests/env_test.py:27,75 (Ant, B=128, lax.scan of 1,000 zero-action steps, > 0.99 x 1000 SPS)'},
          'sample': f'Ant, {B} envs x {steps} env-steps ({dt:.1f} s), float32 C '
                    f'restatement (oracle/pbd_oracle.c), {threads} OpenMP threads '
                    f'(nproc {cpu["nproc"]}, {cpu["allowed_cpus"]} CPUs allowed, '
                    f'OMP_NUM_THREADS={os.environ.get("OMP_NUM_THREADS")}), {cpu["model"]}'}


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
  Humanoid Env.step at 4096 envs (configs[2]), Ant Env.step at configs[3]'s
  32,768-env global batch on one GPU, and Ant Mountain(4)
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
                          'ms_per_step': wall * 1e3 / steps, 'gpu_ms_per_step': gpu * 1e3 / steps,
                          'actions': 'one fixed slab (no per-step draw)'}
  # Humanoid replayed from a captured graph (StepGraph), with the headline's
  # per-step on-device action draw (one more kernel per step than the leg above)
  from brax_amd.envs.graph import StepGraph
  g = StepGraph(env, st[0], 10, seed=3)
  wall, gpu = _time(g.replay, steps // 10, 2)
  out['humanoid_4096_graph'] = {'value': B * (steps // 10) * 10 / wall, 'unit': 'env-steps/s',
                                'ms_per_step': wall * 1e3 / (steps // 10 * 10),
                                'actions': 'drawn on the device every step'}
  # the same through K-step rollout launches (RolloutRunner; the Humanoid
  # program reads the raw action row, so one slab draw + one rollout per K)
  from brax_amd.envs.rollout import RolloutRunner
  r = RolloutRunner(env, st[0], 50, seed=3)
  wall, gpu = _time(r.run, max(steps // 50, 1), 2)
  n_r = max(steps // 50, 1) * 50
  out['humanoid_4096_rollout'] = {'value': B * n_r / wall, 'unit': 'env-steps/s',
                                  'ms_per_step': wall * 1e3 / n_r, 'gpu_ms_per_step': gpu * 1e3 / n_r,
                                  'actions': 'drawn on the device every step (50 per launch)'}
  del env, st, g, r
  # configs[3]'s global batch (32,768 Ant envs) on ONE GPU: what one rank of
  # the 8-GPU run would hold if the whole batch sat on a single card.
  Bg = 32768
  env = envs.create('ant', batch_size=Bg, episode_length=1000, auto_reset=True, device=dev)
  st = [env.reset(np.array([0, 7], np.uint32))]
  act = torch.rand((Bg, env.action_size), device=dev) * 2 - 1

  def gstep():
    st[0] = env.step(st[0], act)
  wall, gpu = _time(gstep, steps, 5)
  out['ant_32768_one_gpu'] = {'value': Bg * steps / wall, 'unit': 'env-steps/s',
                              'ms_per_step': wall * 1e3 / steps, 'gpu_ms_per_step': gpu * 1e3 / steps}
  r = RolloutRunner(env, st[0], 50, seed=3)
  wall, gpu = _time(r.run, max(steps // 50, 1), 2)
  out['ant_32768_one_gpu_rollout'] = {'value': Bg * n_r / wall, 'unit': 'env-steps/s',
                                      'ms_per_step': wall * 1e3 / n_r,
                                      'gpu_ms_per_step': gpu * 1e3 / n_r,
                                      'actions': 'drawn inside the rollout launch (50 steps)'}
  del env, st, r
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

    def mstep_noinfo():
      qp[0], _ = sys_.step(qp[0], a, info=False)
    n = max(steps // 5, 5)
    # (10 untimed steps first: the first call sizes the overflow buffer, and
    # the clock settles)
    wall, gpu = _time(mstep, n, 10)
    out[f'mountain4_2048_cutoff{cutoff}'] = {
        'value': Bm * n / wall, 'unit': 'env-steps/s (System.step)',
        'ms_per_step': wall * 1e3 / n, 'gpu_ms_per_step': gpu * 1e3 / n,
        'contact_rows': sys_.num_rows, 'lanes_per_env': sys_.lanes,
        'lds_bytes_per_env': sys_.lds_bytes,
        'envs_per_cu_by_lds': (160 * 1024) // max(sys_.lds_bytes, 1),
        # the MULTI kernel holds 256 registers (two waves per SIMD): eight
        # waves per CU, i.e. four 128-thread envs
        'envs_per_cu_by_registers': 8 // (sys_.lanes // 64) if sys_.lanes >= 128 else None}
    # the same steps without Info (System.step(..., info=False): the state
    # only, as jit drops the Info a caller ignores)
    wall, gpu = _time(mstep_noinfo, n, 10)
    out[f'mountain4_2048_cutoff{cutoff}_noinfo'] = {
        'value': Bm * n / wall, 'unit': 'env-steps/s (System.step, no Info)',
        'ms_per_step': wall * 1e3 / n, 'gpu_ms_per_step': gpu * 1e3 / n}
  return out


def _traffic():
  """HBM bytes per launch from the committed PMC profile, if present."""
  p = os.path.join(ROOT, 'profiles', 'traffic.json')
  if os.path.exists(p):
    with open(p) as f:
      return json.load(f)
  return None


def kernel_train(env, state, act, n=200):
  """Duration of the fused env-step kernel alone: `n` back-to-back
  `bx_env_step_packed` launches (Env.step's call; fixed input state and
  action, in and out never alias) bracketed by HIP events on the stream they
  run on. The span covers the launches and their inter-kernel gaps, never
  host work, so it cannot exceed a timed step."""
  import ctypes as C
  from brax_amd import _native
  from brax_amd.base import packed_buffer
  from brax_amd.system import _stream
  u = env.unwrapped
  dev = u.sys.device
  qb = packed_buffer(state.qp)
  B = qb.shape[0]
  N, O, M = u.sys.num_bodies, u.obs_size, len(u.metric_keys)
  out = torch.empty((B * (N * 16 + O + 4 + M),), dtype=torch.float32, device=dev)
  p = u._params({'episode_length': 1000, 'action_repeat': 1, 'auto_reset': True},  # pylint: disable=protected-access
                state.info['first_qp'], state.info['first_obs'])
  lib = _native.lib()
  stream = _stream(dev.index)
  args = (u.sys._h, C.byref(p), B, qb.data_ptr(), state.done.data_ptr(),  # pylint: disable=protected-access
          state.info['steps'].data_ptr(), None, C.c_void_p(act.data_ptr()), act.stride(0),
          act.shape[1], out.data_ptr(), None, stream)
  for _ in range(10):
    _native.check(lib.bx_env_step_packed(*args))
  torch.cuda.synchronize()
  a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  a.record()
  for _ in range(n):
    lib.bx_env_step_packed(*args)
  b.record()
  torch.cuda.synchronize()
  return a.elapsed_time(b) / n


def clone_state(st):
  """A copy of a graph's output state that outlives the graph's memory pool."""
  from brax_amd.base import PackedQP, packed_buffer
  info = {k: (v.clone() if isinstance(v, torch.Tensor) else v) for k, v in st.info.items()}
  return st.replace(qp=PackedQP(packed_buffer(st.qp).clone()), obs=st.obs.clone(),
                    reward=st.reward.clone(), done=st.done.clone(), info=info)


def runner_train(env, state, k, n=20):
  """Per-step duration of the headline loop's own launch: `n` back-to-back
  `RolloutRunner.run()` calls of `k` steps (one `bx_env_rollout_random`
  launch each, the actions drawn inside it, each launch reading the previous
  one's last step in place) bracketed by HIP events on the stream they run on,
  divided by n * k. Returns (ms per step, the runner's `draw`)."""
  from brax_amd.envs.rollout import RolloutRunner
  r = RolloutRunner(env, state, k, seed=1)
  for _ in range(3):
    r.run()
  torch.cuda.synchronize()
  a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
  a.record()
  for _ in range(n):
    r.run()
  b.record()
  torch.cuda.synchronize()
  return a.elapsed_time(b) / (n * k), r.draw


def src_sha1():
  """sha1 over the native sources and build files of libbrax_amd.so."""
  import hashlib
  h = hashlib.sha1()
  csrc = os.path.join(ROOT, 'brax_amd', 'csrc')
  for n in sorted(os.listdir(csrc)):
    if n.endswith(('.hip', '.h', '.cpp')) or n == 'Makefile':
      with open(os.path.join(csrc, n), 'rb') as f:
        h.update(n.encode() + b'\0' + f.read())
  with open(os.path.join(ROOT, 'include', 'brax_amd.h'), 'rb') as f:
    h.update(f.read())
  return h.hexdigest()


def _rocprof_avg(kernel, steps_per_launch=1):
  """The committed rocprof average of `kernel` (profiles/rocprof_latest.json),
  when it was profiled from this exact library build, scaled to launches of
  `steps_per_launch` env steps (the profile records its own launches')."""
  import hashlib
  p = os.path.join(ROOT, 'profiles', 'rocprof_latest.json')
  if not os.path.exists(p):
    return None
  from brax_amd import _native
  with open(_native.LIB_PATH, 'rb') as f:
    sha = hashlib.sha1(f.read()).hexdigest()
  with open(p) as f:
    d = json.load(f)
  k = d.get('kernels', {}).get(kernel)
  # the library build, or (hipcc output is not byte-reproducible across build
  # directories) the exact kernel sources and build flags it was built from
  if not k or (d.get('lib_sha1') != sha and d.get('src_sha1') != src_sha1()):
    return None
  spl = k.get('steps_per_launch', 1)
  per_step = k['avg_ns'] * 1e-6 / spl
  # the profiled launch as measured, and the same rate scaled to this run's
  # launch length (labelled apart: a 50-step launch profiled at 1.03 ms is
  # 0.41 ms scaled to 20 steps, not a 0.41 ms 50-step launch)
  return {'profiled_launch_ms': k['avg_ns'] * 1e-6, 'profiled_steps_per_launch': spl,
          'avg_ms_per_step': per_step,
          'scaled_to_steps_per_launch': steps_per_launch,
          'scaled_launch_ms': per_step * steps_per_launch, 'calls': k.get('calls'),
          'source': d.get('source'), 'lib_sha1': sha, 'sq': k.get('sq')}


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
  ap.add_argument('--repeats', type=int, default=5,
                  help='timed regions of the direct (headline) loop; value = their median')
  ap.add_argument('--generic', action='store_true',
                  help='force the generic item-loop kernel variant (A/B)')
  ap.add_argument('--block', type=int, default=0,
                  help='threads per workgroup of the step kernel (A/B; default 64)')
  ap.add_argument('--variant', default='',
                  help='lanes,mode kernel variant (mode 0 global, 1 single, 2 lds)')
  args = ap.parse_args()

  plan, why = rank_plan(args.gpus, os.environ)
  if plan == 'refuse':
    print(f'bench.py: {why}', file=sys.stderr)
    sys.exit(2)
  if plan == 'spawn':
    sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
  dist, rank, world, local = _dist()
  dev = torch.device('cuda', local)
  torch.cuda.set_device(dev)
  from brax_amd import _native, envs
  from brax_amd import distributed as bd
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
  # rank r resets the global envs [r*B, (r+1)*B) of one shared seed
  bd.shard_env(env, rank, B)
  state = env.reset(np.array([0, 0x5EED], np.uint32))
  A = env.action_size
  lib = _native.lib()
  stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
  act = torch.empty((B, A), dtype=torch.float32, device=dev)
  # the episodic (reward, done) exchange: summed on the device every step,
  # all-gathered over RCCL once per period: the episode length (1000), or the
  # timed step count when shorter, so every timed region holds >= 1 collective
  K = graph_steps(args.steps)
  period = bd.exchange_period(1000, args.steps, K)
  exchange = bd.EpisodeExchange(B, dev, every=period) if dist is not None else None

  def one_step(st, k):
    # the step's action slab, keyed by (step, global env id): drawn on the
    # device inside the timed region
    lib.bx_uniform(C.c_void_p(act.data_ptr()), B * A, 1,
                   bd.action_offset(rank, B, A, k, world), -1.0, 1.0, stream)
    st = env.step(st, act)
    if exchange is not None:
      exchange(st.reward, st.done)  # the RCCL all-gather once per period
    return st

  for k in range(args.warmup):
    state = one_step(state, k)
  # no collector pause inside a timed region; collected BEFORE the warm-up
  # work: a collection between the warm-up and t0 idles the GPU for
  # milliseconds, its clock drops, and a short timed region (the driver's
  # 20 steps are ONE rollout launch) runs on the ramp
  gc.collect()
  gc.disable()
  # the step kernel alone (its launch train also brings the clocks up before
  # the timed loops)
  kern_ms = single_ms = kernel_train(env, state, act)
  if exchange is not None:
    exchange.reset()
  torch.cuda.synchronize()
  if dist is not None:
    dist.barrier()
  torch.cuda.synchronize()
  t0 = time.perf_counter()
  for k in range(args.steps):
    state = one_step(state, args.warmup + k)
  torch.cuda.synchronize()
  if dist is not None:  # (one rank: the synchronisation above is the bracket)
    dist.barrier()
    torch.cuda.synchronize()
  elapsed = time.perf_counter() - t0
  gc.enable()
  eager_elapsed = elapsed
  eager_collectives = exchange.flushes if exchange is not None else 0
  # the same loop replayed from hipGraphs, the actions continuing the eager
  # loop's (step, global env id) stream: (1) StepGraph: K steps per graph
  # launch (one draw of the K action slabs, then K x (Env.step + the episodic
  # sum)); (2) RolloutGraph: the K steps as ONE open-loop rollout launch
  # (bx_env_rollout_packed: the state stays on chip between steps, every
  # step's outputs written; the reference's lax.scan of env.step) after the
  # one draw. `value` is the faster loop that completed on every rank.
  from brax_amd.envs.graph import StepGraph
  from brax_amd.envs.rollout import RolloutGraph, RolloutRunner

  def timed_replays(g, advance_hook, repeats=1):
    """Warm replays, then `repeats` timed regions of args.steps // K replays
    each (barrier + sync on both sides of every region); the elapsed wall
    time of each region, the collectives inside each and the replays run
    untimed + timed. The warm-up is max(warmup // K, 2) replays, extended
    to WARM_S of the loop's own work: the GPU's clock ramps over ~10 ms of
    load (a 20-step rollout launch runs 506 us cold, 471 us warm in one
    rocprof trace), so the timed region starts at the steady state."""
    fire = g.run if isinstance(g, RolloutRunner) else g.replay
    gc.collect()  # before the warm replays (see the eager loop)
    gc.disable()
    n_warm = max(args.warmup // K, 2)
    t_w = time.perf_counter()
    for _ in range(n_warm):
      fire()
    torch.cuda.synchronize()
    per = (time.perf_counter() - t_w) / n_warm
    extra = max(0, math.ceil((WARM_S - per * n_warm) / max(per, 1e-6)))
    for _ in range(extra):
      fire()
    n_warm += extra
    els, cols = [], []
    for _ in range(repeats):
      if exchange is not None:
        exchange.reset()
      torch.cuda.synchronize()
      if dist is not None:
        dist.barrier()
      torch.cuda.synchronize()
      t0 = time.perf_counter()
      for _ in range(args.steps // K):
        fire()
        if advance_hook is not None:
          advance_hook(K)  # the RCCL all-gather once per period, on the host
      torch.cuda.synchronize()
      if dist is not None:  # (one rank: the synchronisation above is the bracket)
        dist.barrier()
        torch.cuda.synchronize()
      els.append(time.perf_counter() - t0)
      cols.append(exchange.flushes if exchange is not None else 0)
    gc.enable()
    return els, min(cols), n_warm + (repeats - 1) * (args.steps // K)

  def build(kind, st, k0):
    try:
      off = bd.action_offset(rank, B, A, k0, world)
      if kind == 'step':
        return StepGraph(env, st, K, seed=1, offset=off, step_stride=world * B * A,
                         hook=None if exchange is None else (
                             lambda s_: exchange.accumulate(s_.reward, s_.done))), None
      cls = RolloutGraph if kind == 'rollout' else RolloutRunner
      return cls(env, st, K, seed=1, offset=off, step_stride=world * B * A,
                 hook=None if exchange is None else (
                     lambda tr: exchange.accumulate_steps(tr.reward, tr.done))), None
    except Exception as e:  # pylint: disable=broad-except
      # a failed capture must not sink the run: every rank falls back, and
      # the line says so
      return None, f'{type(e).__name__}: {e}'

  def agreed(ok):
    if dist is None:
      return ok
    f = torch.tensor([int(ok)], dtype=torch.int32, device=dev)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    return bool(f.item())

  adv = None if exchange is None else exchange.advance
  # per loop: the timed regions' elapsed times (the direct loop's timed
  # region runs `--repeats` times; the others once), collectives, error
  R = max(int(args.repeats), 1)
  loops = {'eager': ([eager_elapsed], eager_collectives, None)}
  k0 = args.warmup + args.steps
  for kind in KINDS[1:]:
    g, err = build(kind, state, k0)
    if agreed(g is not None):
      els, col, n_run = timed_replays(g, adv, R if kind == 'direct' else 1)
      loops[kind] = (els, col, None)
      k0 += (n_run + args.steps // K) * K
      state = clone_state(g.state() if kind == 'direct' else  # pylint: disable=protected-access
                          g._res[0] if kind == 'rollout' else g._out)
    else:
      loops[kind] = (None, 0, err)
    del g
  if dist is not None:
    # each region's time is its slowest rank's
    t = torch.tensor([loops[k][0][i] if loops[k][0] is not None else -1.0
                      for k in KINDS for i in range(R if k == 'direct' else 1)],
                     dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    v = t.tolist()
    for k in KINDS:
      n = R if k == 'direct' else 1
      part, v = v[:n], v[n:]
      loops[k] = ((part if part[0] >= 0 else None),) + loops[k][1:]
  # a loop's time: the median of its timed regions (one region but the
  # direct loop's; its region is one K-step launch at the driver's 20 steps,
  # so a single launch or clock hiccup would move a lone sample by several %)
  samples = {k: loops[k][0] for k in KINDS}
  loops = {k: ((float(np.median(e)) if e is not None else None),) + loops[k][1:]
           for k, e in ((k, loops[k][0]) for k in KINDS)}
  # the headline is the direct loop by design; another loop only if it failed
  best = next(k for k in ('direct', 'rollout', 'step', 'eager') if loops[k][0] is not None)
  elapsed, collectives = loops[best][0], loops[best][1]
  eager_elapsed = loops['eager'][0]

  total = B * world * args.steps
  value = total / elapsed
  if rank != 0:
    dist.destroy_process_group()
    return
  # the dominant kernel of the timed loop: the K-step rollout kernel (one
  # launch = K x B env-steps) or the single-step kernel (one launch = B
  # env-steps); achieved = algorithmic flops (bytes) per launch / launch time
  direct_draw = None
  if best in ('rollout', 'direct'):
    kname, spl = ANT_ROLLOUT_KERNEL, K
    ms_step, direct_draw = runner_train(env, state, K)
    kern_ms = ms_step * K
    kern_src = (f'HIP events over 20 back-to-back {K}-step RolloutRunner.run() launches '
                f'({"bx_env_rollout_random: actions drawn inside the launch" if direct_draw else "bx_uniform_slabs + bx_env_rollout_packed"}) '
                'on the launch stream (runner_train): the headline loop\'s own launch')
  else:
    kname, spl = ANT_KERNEL, 1
    kern_src = ('HIP events over 200 back-to-back bx_env_step_packed launches on the launch '
                'stream (kernel_train)')
  bytes_per_launch = ANT_BYTES_PER_ENV_STEP * B * spl
  flops_per_launch = ANT_FLOPS_PER_ENV_STEP * B * spl
  tflops = flops_per_launch / (kern_ms * 1e-3) / 1e12
  achieved_gbs = bytes_per_launch / (kern_ms * 1e-3) / 1e9
  # PMC traffic of THIS kernel instantiation (Ant: 16 lanes, SINGLE mode,
  # features F_G1 | F_JH, gather width 4), per env-step x the launch's steps
  tr = _traffic()
  k = ((tr or {}).get('kernels') or {}).get(kname)
  traffic = (k['hbm_bytes_per_launch'] / k.get('steps_per_launch', 1) * spl
             if k and k.get('batch') == B else None)
  rp = _rocprof_avg(kname, spl)
  sq = (rp or {}).get('sq') or {}
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
      # BASELINE.md's published number for this workload: Ant, 4,096 envs,
      # U[-1,1] actions, one (Colab) GPU, notebooks/environments.ipynb:386-423
      'vs_baseline': value / REF_PUBLISHED,
      'baseline': {'value': REF_PUBLISHED, 'unit': 'env-steps/s',
                   'source': 'BASELINE.md (notebooks/environments.ipynb:386-423: Ant, 4096 '
                             'envs, random actions, Colab GPU)'},
      'dtype': 'f32',
      'data': 'synthetic: U[-1,1] actions drawn on the device each step inside the timed '
              'region (counter RNG keyed by step and global env id); reset from the Ant '
              'config with device-RNG joint noise keyed by global env id',
      'config': {'workload': 'Ant-v1 Env.step (10 PBD substeps + obs/reward + '
                             'Episode/AutoReset), envs.create(ant)',
                 'launch': {
                     'rollout': f'hipGraph replays of one on-device draw of {K} action slabs + '
                                f'one {K}-step open-loop rollout launch (bx_env_rollout_packed)',
                     'direct': (f'per {K} steps: ONE {K}-step open-loop rollout launch that '
                                'draws each step\'s actions inside the kernel '
                                '(bx_env_rollout_random), launched directly from prebuilt C '
                                'arguments, the state read in place from the previous launch\'s '
                                'last step (RolloutRunner)' if direct_draw else
                                f'per {K} steps: one on-device draw of {K} action slabs '
                                f'(bx_uniform_slabs) + one {K}-step open-loop rollout launch '
                                '(bx_env_rollout_packed), launched directly from prebuilt C '
                                'arguments (RolloutRunner)'),
                     'step': f'hipGraph replays of one on-device draw of {K} action slabs + {K} '
                             'fused Env.step launches (+ the episodic sum per step when N>1)',
                     'eager': 'a Python loop of bx_uniform + Env.step per step'}[best],
                 'envs_per_gpu': B, 'episode_length': 1000, 'substeps': 10,
                 'steps_per_launch': K if best != 'eager' else 1,
                 'parallelism': f'env-shard x{world}',
                 'exchange_period': period if exchange is not None else None,
                 'dist_backend': dist.get_backend() if dist is not None else None},
      # RCCL all-gathers of the episodic (reward, done) sums inside the timed
      # region (0 at N = 1: there is no collective on one GPU)
      'collectives_in_timed_region': collectives,
      # the fused env step is VALU/latency-bound (AI ~61 flop/B):
      # headline = counted flops / kernel time vs the FP32 VALU peak; the HBM
      # view (algorithmic bytes / kernel time vs 8 TB/s) is kept beside it
      'roofline': {'bound': 'valu', 'achieved': tflops, 'peak': FP32_VALU_PEAK_TFLOPS,
                   'unit': 'TFLOP/s', 'frac': tflops / FP32_VALU_PEAK_TFLOPS,
                   'traffic': traffic,
                   'kernel': kname, 'kernel_ms': kern_ms, 'steps_per_launch': spl,
                   'kernel_ms_per_step': kern_ms / spl,
                   'kernel_ms_source': kern_src,
                   'single_step_kernel_ms': single_ms,
                   # the SQ issue view of the same kernel (committed counters of
                   # this library build): VALU instructions x 4 cycles / wave cycles
                   'valu_issue_frac': sq.get('valu_issue_frac'),
                   'rocprof': rp,
                   'flops_per_launch': flops_per_launch,
                   'bytes_per_launch': bytes_per_launch,
                   'hbm': {'achieved': achieved_gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                           'frac': achieved_gbs / HBM_PEAK_GBS, 'traffic': traffic}},
  }
  # the same steps from the plain Python loop (one Env.step call per step):
  # host-bound on a slow host, hence the graph above
  # every loop's rate (value is the fastest); a loop that failed says why
  for kind, key in (('eager', 'eager_loop'), ('step', 'graph_loop'), ('rollout', 'rollout_loop'),
                    ('direct', 'direct_loop')):
    el, col, err = loops[kind]
    out[key] = ({'value': total / el, 'unit': 'env-steps/s', 'ms_per_step': el * 1e3 / args.steps,
                 'collectives_in_timed_region': col} if el is not None else {'error': err})
  out['timed_loop'] = best
  out['timed_regions'] = {'repeats': len(samples[best]) if samples[best] else 0,
                          'ms_per_step': [e * 1e3 / args.steps for e in (samples[best] or [])],
                          'statistic': 'median'}
  out['timed_loop_policy'] = ('the direct loop by design (RolloutRunner); rollout, step, eager '
                              'only when it could not run')
  out['warmup_policy'] = (f'{args.warmup} warm-up steps; each replayed loop warms on >= '
                          f'{WARM_S * 1e3:.0f} ms of its own untimed replays (steady-state clocks)')
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
