"""Diagnostic: the bench's rollout_loop (RolloutGraph) per-step time and the
AutoReset target's layout at its construction (BRAX_AMD_LIB selects the
build)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
  import bench
  from brax_amd import envs
  from brax_amd.envs.graph import StepGraph
  from brax_amd.envs.rollout import RolloutGraph
  dev = torch.device('cuda', 0)
  env = envs.create('ant', batch_size=4096, episode_length=1000, auto_reset=True, device=dev)
  st = env.reset(np.array([0, 0x5EED], np.uint32))
  g = StepGraph(env, st, 20, seed=1)
  g.replay()
  st2 = bench.clone_state(g._out)  # pylint: disable=protected-access
  for name, s in (('reset state', st), ('after StepGraph', st2)):
    fq = s.info['first_qp']
    print(name, type(fq).__name__, getattr(fq, '_buf', None).shape if hasattr(fq, '_buf') else None,
          fq.pos.stride(), fq.pos.data_ptr() % 16, fq.rot.data_ptr() - fq.pos.data_ptr())
    r = RolloutGraph(env, s, 20, seed=1)
    for _ in range(3):
      r.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(10):
      r.replay()
    b.record()
    torch.cuda.synchronize()
    print('  RolloutGraph us/step', a.elapsed_time(b) * 1e3 / 200, flush=True)


if __name__ == '__main__':
  main()
