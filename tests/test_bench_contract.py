"""bench.py's bookkeeping, on the CPU: the committed rocprof averages it
reports are keyed to the native build they were measured on, and the
profile summary's per-kernel numbers are internally consistent."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_src_sha1_is_stable_and_covers_the_native_sources():
  a = bench.src_sha1()
  assert a == bench.src_sha1() and len(a) == 40


def test_committed_profile_is_keyed_to_this_build():
  """profiles/rocprof_latest.json must describe the current sources (the
  bench refuses to quote it otherwise), and its Ant kernel entry must be the
  4,096-env bench grid with SQ figures attached."""
  with open(os.path.join(ROOT, 'profiles', 'rocprof_latest.json')) as f:
    d = json.load(f)
  assert d['src_sha1'] == bench.src_sha1(), 'profile predates the current kernel sources'
  k = d['kernels'][bench.ANT_KERNEL]
  assert k['grid'] == 4096 * 16  # 16 lanes per env
  assert 20e3 < k['avg_ns'] < 60e3
  sq = k['sq']
  assert abs(sq['valu_issue_frac'] - 4 * sq['valu_insts_per_wave'] / sq['cycles_per_wave']) < 1e-9
  assert sq['waves'] == 1024


def test_traffic_carries_algorithmic_bytes_per_env_kernel():
  with open(os.path.join(ROOT, 'profiles', 'traffic.json')) as f:
    t = json.load(f)['kernels']
  ant = t[bench.ANT_KERNEL]
  assert ant['algorithmic_bytes_per_launch'] == bench.ANT_BYTES_PER_ENV_STEP * 4096
  hum = t['bx::env_step_packed_kernel<16, 1, 33, 4, 2>']
  assert hum['algorithmic_bytes_per_launch'] == 2284 * 4096
