"""Test scenes (input data for goldens and parity tests; test infrastructure).

BOX_TEST_CONFIG is the BoxTest scene of the reference
(`brax/tests/physics_test.py:51-65`): default 0 drops the box, default 1 slides
it (`test_box_hits_ground` / `test_box_slide`, :67-83).

mesh_test_config() is the MeshTest scene (`physics_test.py:364-390`) without
its capsule body and with an inline mesh: the reference loads `cylinder.stl`
through trimesh (`brax/io/mesh.py:25-57`), which this image lacks, so the
cylinder is a hexagonal prism given as vertices / faces / face normals (the
inline form `brax/physics/base.py:206-211` accepts without loading).
"""
import numpy as np

BOX_TEST_CONFIG = """
dt: 1.5 substeps: 2000 friction: 0.77459666924
gravity { z: -9.8 }
bodies {
  name: "box" mass: 1
  colliders { box { halfsize { x: 0.5 y: 0.5 z: 0.5 }}}
  colliders { box { halfsize { x: 1 y: 1 z: 1 }} no_contact: true }
  inertia { x: 1 y: 1 z: 1 }
}
bodies { name: "Ground" frozen: { all: true } colliders { plane {}}}
defaults { qps { name: "box" pos { z: 1 }}}
defaults { qps { name: "box" pos { z: 2 } vel {x: 2}}}
"""


def _prism(n=6):
  """Vertices, triangle faces and outward face normals of an n-gon prism of
  radius 1 and half-height 1 around the z axis."""
  ang = 2 * np.pi * np.arange(n) / n
  ring = np.stack([np.cos(ang), np.sin(ang)], -1)
  verts = np.concatenate([np.c_[ring, -np.ones(n)], np.c_[ring, np.ones(n)]])
  faces, normals = [], []
  for k in range(1, n - 1):  # caps, fanned from vertex 0 / n
    faces += [(0, k + 1, k), (n, n + k, n + k + 1)]
    normals += [(0., 0., -1.), (0., 0., 1.)]
  for k in range(n):  # sides, two triangles per quad
    k1 = (k + 1) % n
    mid = ring[k] + ring[k1]
    mid = mid / np.linalg.norm(mid)
    faces += [(k, k1, n + k1), (k, n + k1, n + k)]
    normals += [(mid[0], mid[1], 0.)] * 2
  return verts, np.array(faces), np.array(normals)


def _vec(name, v):
  return f'{name} {{ x: {v[0]:.9g} y: {v[1]:.9g} z: {v[2]:.9g} }}'


def mesh_test_config(height=1.5):
  verts, faces, normals = _prism()
  geom = ' '.join([_vec('vertices', v) for v in verts]
                  + [f'faces: {int(i)}' for i in faces.reshape(-1)]
                  + [_vec('face_normals', v) for v in normals])
  return f"""
dt: 0.05 substeps: 10 friction: 1.0
gravity {{ z: -9.8 }}
bodies {{
  name: "Mesh" mass: 1
  colliders {{ mesh {{ name: "Cylinder" scale: 0.1 }} }}
  inertia {{ x: 1 y: 1 z: 1 }}
}}
bodies {{ name: "Ground" frozen: {{ all: true }} colliders {{ plane {{}} }} }}
defaults {{ qps {{ name: "Mesh" pos: {{ x: 0 y: 0 z: {height} }} }} }}
defaults {{ qps {{ name: "Mesh" pos: {{ x: 0 y: 0 z: 0.2 }} rot: {{ x: 20 y: 10 }} ang {{ x: 3 }} }} }}
mesh_geometries {{ name: "Cylinder" {geom} }}
"""
