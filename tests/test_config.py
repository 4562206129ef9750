"""Config parser (brax.Config text format without protobuf)."""
import numpy as np
import pytest

from brax_amd import config as C
from brax_amd import compiler
from brax_amd.envs import configs


def test_floats_are_fp32():
  cfg = C.parse('dt: 0.05 substeps: 10 gravity { z: -9.8 }')
  assert cfg.dt == float(np.float32(0.05)) == 0.05000000074505806
  assert cfg.gravity.z == float(np.float32(-9.8))
  assert cfg.substeps == 10


def test_defaults_and_presence():
  cfg = C.parse('bodies { name: "a" }')
  b = cfg.bodies[0]
  assert b.mass == 0.0 and not b.HasField('frozen')
  assert b.frozen.all is False and not b.HasField('frozen')  # reading does not set
  b.frozen.position.x = 1
  assert b.HasField('frozen') and b.frozen.HasField('position')


def test_oneof_and_copy():
  c = C.Message('Collider')
  c.sphere.radius = 0.5
  assert c.WhichOneof('type') == 'sphere'
  c.capsule.radius = 0.1
  assert c.WhichOneof('type') == 'capsule' and not c.HasField('sphere')
  d = C.Message('Collider')
  d.CopyFrom(c)
  d.capsule.radius = 0.2
  assert c.capsule.radius == pytest.approx(0.1)


def test_bundled_configs_roundtrip():
  for txt in (configs.ANT_CONFIG, configs.HUMANOID_CONFIG, configs.HALFCHEETAH_CONFIG):
    a = C.parse(txt)
    b = C.parse(a.to_text())
    assert a.to_compact() == b.to_compact()


def test_repeated_add_and_lists():
  cfg = C.parse('bodies { name: "a" colliders { plane {} } } '
                'collide_include { first: "a" second: "b" } '
                'mesh_geometries { name: "m" faces: [0, 1, 2] }')
  j = cfg.joints.add(name='j')
  j.angle_limit.add(min=-10, max=10)
  assert cfg.joints[0].angle_limit[0].max == 10.0
  assert list(cfg.mesh_geometries[0].faces) == [0, 1, 2]


def test_validation_errors():
  with pytest.raises(ValueError):
    compiler.validate_config(C.parse('dt: 0'))
  with pytest.raises(RuntimeError):
    compiler.validate_config(C.parse('dt: 0.1 bodies { name: "a" } bodies { name: "a" }'))
  with pytest.raises(ValueError):
    compiler.validate_config(C.parse(
        'dt: 0.1 dynamics_mode: "pbd" joints { name: "j" stiffness: 5 }'))


def test_parse_error():
  with pytest.raises((ValueError, AttributeError)):
    C.parse('bodies { nonsense: 1 }')
