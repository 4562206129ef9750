"""The RCCL path of the multi-GPU run, executed on the one GPU the box has.

The N-GPU bench shards envs by global id and exchanges only the episodic
(reward, done) sums (the reference's pmap sharding,
`brax/training/agents/ppo/train.py:276-283`). Those sums are all-gathered by
`EpisodeExchange.flush` with `all_gather_into_tensor` on device tensors under
backend "nccl" (= RCCL on ROCm). Here a world-size-1 RCCL process group runs
that exact call, and `bench.py` runs under `torchrun --nproc-per-node 1` with
the process group forced (BX_DIST_FORCE=1), so its timed region holds the
RCCL gather. Each runs in a child process (its own process group)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_EXCHANGE = r'''
import os, sys, torch, torch.distributed as dist
sys.path.insert(0, os.environ['BX_ROOT'])
from brax_amd import distributed as bd
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
dist.init_process_group('nccl', rank=0, world_size=1, device_id=dev)
assert dist.get_backend() == 'nccl'
B = 4096
ex = bd.EpisodeExchange(B, dev, every=3)
g = torch.Generator(device=dev).manual_seed(5)
host = torch.zeros((2, B), dtype=torch.float64)
outs = []
for t in range(6):
  scal = torch.rand((4, B), device=dev, generator=g)  # one env step's (4, B) scalars
  scal[1] = (scal[1] > 0.5).float()                     # done flags
  host += scal[:2].double().cpu()
  r = ex(*scal.unbind(0)[:2])
  if r is not None:
    outs.append((r.clone(), host.clone()))
    host.zero_()
assert ex.flushes == 2 and len(outs) == 2
for got, want in outs:
  assert got.shape == (1, 2, B) and got.is_cuda
  # float32 sums of 3 steps on the device vs the float64 host sums
  err = (got[0].double().cpu() - want).abs().max().item()
  assert err < 1e-5, err
  # the gathered tensor holds exactly the rank's device sums
torch.cuda.synchronize()
dist.destroy_process_group()
print('rccl exchange ok')
'''


def _free_port():
  s = socket.socket()
  s.bind(('127.0.0.1', 0))
  p = s.getsockname()[1]
  s.close()
  return p


def _env(**kw):
  e = dict(os.environ)
  e.update({'BX_ROOT': ROOT, 'MASTER_ADDR': '127.0.0.1', 'MASTER_PORT': str(_free_port()),
            'HSA_ENABLE_IPC_MODE_LEGACY': '0'})
  e.update(kw)
  return e


def test_rccl_episode_exchange_world1():
  """`EpisodeExchange.flush`'s device all_gather_into_tensor on RCCL
  (`brax_amd/distributed.py:119-125`) gathers the rank's device sums of
  every exchange period, equal to the host sums of the same steps."""
  r = subprocess.run([sys.executable, '-c', _EXCHANGE], env=_env(), capture_output=True,
                     text=True, timeout=150)
  assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
  assert 'rccl exchange ok' in r.stdout


def test_bench_rccl_world1_under_torchrun():
  """`torchrun --nproc-per-node 1 bench.py` with the process group forced:
  backend nccl, and every timed loop holds one RCCL gather."""
  cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
         '--master-addr', '127.0.0.1', '--master-port', str(_free_port()),
         os.path.join(ROOT, 'bench.py'), '--gpus', '1', '--steps', '20', '--warmup', '5',
         '--no-secondary', '--no-phases', '--no-cpu-baseline']
  r = subprocess.run(cmd, env=_env(BX_DIST_FORCE='1'), capture_output=True, text=True,
                     timeout=170, cwd=ROOT)
  assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
  line = [l for l in r.stdout.splitlines() if l.startswith('{')][-1]
  d = json.loads(line)
  print(json.dumps({k: d[k] for k in ('value', 'timed_loop', 'collectives_in_timed_region')}))
  assert d['config']['dist_backend'] == 'nccl'
  assert d['collectives_in_timed_region'] >= 1
  for k in ('eager_loop', 'graph_loop', 'rollout_loop', 'direct_loop'):
    assert d[k].get('collectives_in_timed_region', 0) >= 1, (k, d[k])
