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


def test_rank_plan_follows_gpus_and_the_launcher():
  """`--gpus N` is the experiment the line names: alone it spawns N ranks, a
  launcher's world must match it, and N = 1 runs in place."""
  assert bench.rank_plan(1, {}) == ('run', None)
  assert bench.rank_plan(8, {}) == ('spawn', None)
  assert bench.rank_plan(2, {'WORLD_SIZE': '2'}) == ('run', None)
  assert bench.rank_plan(1, {'WORLD_SIZE': '1'}) == ('run', None)
  for gpus, env in ((8, {'WORLD_SIZE': '1'}), (1, {'WORLD_SIZE': '4'}), (0, {})):
    plan, why = bench.rank_plan(gpus, env)
    assert plan == 'refuse' and why


def test_rank_env_is_torchruns():
  e = bench.rank_env({'X': '1'}, 3, 8, 29999)
  assert (e['RANK'], e['LOCAL_RANK'], e['WORLD_SIZE'], e['MASTER_ADDR'], e['MASTER_PORT'],
          e['X']) == ('3', '3', '8', '127.0.0.1', '29999', '1')


def _script(tmp_path, body):
  p = tmp_path / 'rank.py'
  p.write_text('import os, sys, time\n' + body)
  return str(p)


def test_spawn_ranks_starts_n_ranks(tmp_path, monkeypatch):
  monkeypatch.setenv('BX_DIST_BACKEND', 'gloo')
  out = tmp_path / 'seen'
  out.mkdir()
  s = _script(tmp_path, f"open(os.path.join({str(out)!r}, os.environ['RANK']), 'w').write("
                        "os.environ['WORLD_SIZE'] + ' ' + ' '.join(sys.argv[1:]))\n")
  assert bench.spawn_ranks(3, ['--gpus', '3'], script=s) == 0
  assert sorted(os.listdir(out)) == ['0', '1', '2']
  assert (out / '2').read_text() == '3 --gpus 3'


def test_spawn_ranks_fails_when_a_rank_fails(tmp_path, monkeypatch):
  """A failing rank fails the run, and the ranks left waiting (as at a
  barrier) are stopped instead of hanging the parent."""
  monkeypatch.setenv('BX_DIST_BACKEND', 'gloo')
  s = _script(tmp_path, "sys.exit(3) if os.environ['RANK'] == '1' else time.sleep(600)\n")
  import time
  t0 = time.monotonic()
  assert bench.spawn_ranks(2, [], script=s) == 3
  assert time.monotonic() - t0 < 60


def test_spawn_ranks_refuses_more_rccl_ranks_than_gpus(monkeypatch):
  """The RCCL parent counts GPUs from the environment (or the KFD
  topology), never through HIP: device_count() here would be a HIP call."""
  monkeypatch.delenv('BX_DIST_BACKEND', raising=False)
  monkeypatch.setenv('HIP_VISIBLE_DEVICES', '0')

  def no_hip():
    raise AssertionError('the parent must not call into HIP')
  monkeypatch.setattr(bench.torch.cuda, 'device_count', no_hip)
  assert bench.spawn_ranks(8, []) == 2


def test_visible_gpus_without_hip(tmp_path):
  assert bench.visible_gpus({'HIP_VISIBLE_DEVICES': '0,1,2'}) == 3
  assert bench.visible_gpus({'CUDA_VISIBLE_DEVICES': '3'}) == 1
  assert bench.visible_gpus({'ROCR_VISIBLE_DEVICES': '0,1,2,3'}) == 4
  # HIP's list indexes into what ROCR leaves
  assert bench.visible_gpus({'ROCR_VISIBLE_DEVICES': '2', 'HIP_VISIBLE_DEVICES': '0,1'}) == 1
  assert bench.visible_gpus({'HIP_VISIBLE_DEVICES': ''}) == 0
  # the KFD topology: CPU nodes have no SIMDs
  for i, simds in enumerate((0, 1024, 1024)):
    d = tmp_path / str(i)
    d.mkdir()
    (d / 'properties').write_text(f'cpu_cores_count 8\nsimd_count {simds}\ngfx_target_version 0\n')
  assert bench.visible_gpus({}, topology=str(tmp_path)) == 2
  assert bench.visible_gpus({}, topology=str(tmp_path / 'absent')) is None


def test_spawn_ranks_stops_ranks_when_the_parent_is_interrupted(tmp_path, monkeypatch):
  """An exception while waiting (e.g. KeyboardInterrupt) leaves no rank
  running."""
  monkeypatch.setenv('BX_DIST_BACKEND', 'gloo')
  s = _script(tmp_path, "time.sleep(600)\n")
  started = []
  real_popen = __import__('subprocess').Popen

  def popen(*a, **k):
    p = real_popen(*a, **k)
    started.append(p)
    return p
  monkeypatch.setattr('subprocess.Popen', popen)

  def interrupted(procs, stop):
    raise KeyboardInterrupt
  monkeypatch.setattr(bench, '_wait_ranks', interrupted)
  import pytest
  with pytest.raises(KeyboardInterrupt):
    bench.spawn_ranks(2, [], script=s)
  assert len(started) == 2 and all(p.poll() is not None for p in started)
