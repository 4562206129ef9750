"""The kernel plan each system compiles to, on the host (bx_system_plan: the
host half of bx_system_create, no device): which step kernel runs it and the
LDS its workgroup needs, i.e. how many envs a CU holds at once."""
import pytest

from brax_amd.system import System
from tests.helpers import config_for

LDS_CU = 160 * 1024  # MI355X LDS per CU


@pytest.mark.parametrize('name', ['ant', 'humanoid', 'halfcheetah', 'humanoidstandup'])
def test_env_systems_run_the_register_hoisted_kernel(name):
  p = System.plan(config_for(name))
  assert p['mode'] == 1 and p['lanes'] == 16, p
  # four envs per one-wave workgroup
  assert 0 < p['lds_bytes'] <= LDS_CU // 4, p


@pytest.mark.parametrize('cutoff', [0, 36])
def test_ant_mountain4_runs_four_envs_per_cu(cutoff):
  """BASELINE configs[4]: Ant Mountain(4) runs the large-scene kernel at 128
  threads per env (two waves). The kernel is built for two waves per SIMD
  (256 registers), so the register file holds four such envs per CU, and
  since round 6 the LDS does too: only the penetrating rows get contact
  slots (64 per chunk) and a contact record (128 in LDS), the rows' bounds
  are 12 bytes, and the Info accumulators, the NearNeighbors ranks / lists
  and the near-row list share words that are dead while they live, so an
  env's tail fits 40 KB with all pairs (cutoff 0) and culled (cutoff 36)."""
  cfg = config_for('mountain4')
  cfg.collider_cutoff = cutoff
  p = System.plan(cfg)
  assert p['mode'] == 3 and p['lanes'] == 128, p
  assert p['lds_bytes'] * 4 <= LDS_CU, p
  assert p['envs_per_cu_by_lds'] == 4, p
  assert p['envs_per_cu_by_registers'] == 4 and p['envs_per_cu'] == 4, p


def test_plan_refuses_a_null_descriptor():
  import ctypes as C
  from brax_amd import _native
  v = C.c_int32()
  rc = _native.lib().bx_system_plan(None, None, C.byref(v), C.byref(v), C.byref(v))
  assert rc != 0 and b'null' in _native.lib().bx_last_error()


def test_mountain4_with_many_materials_takes_the_item_loops():
  """The MULTI kernel assembles rows from LDS tables with <= 255 distinct
  (friction, elasticity, scale, threshold) materials; a scene with more
  (here every row its own friction) takes the item-loop kernels instead of
  failing to build."""
  import ctypes as C
  import numpy as np
  from brax_amd import _native, abi, compiler
  cfg = config_for('mountain4')
  vc, desc, meta = compiler.compile_system(cfg)
  rdesc = compiler.compile_reset(vc, meta['body_index'])
  n = len(desc['row_friction'])
  desc['row_friction'] = np.linspace(0.5, 1.5, n)
  cd, keep = abi.make_desc(desc)
  rd, keep_r = abi.make_reset_desc(rdesc, meta['num_joint_dof'])
  mode, lanes, lds = C.c_int32(), C.c_int32(), C.c_int32()
  _native.check(_native.lib().bx_system_plan(C.byref(cd), C.byref(rd), C.byref(mode),
                                             C.byref(lanes), C.byref(lds)))
  del keep, keep_r
  assert mode.value == 0, (mode.value, lanes.value, lds.value)
