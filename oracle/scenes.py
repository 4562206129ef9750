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


def mesh_capsule_config():
  """MeshTest's `test_mesh_hits_capsule` scene (`physics_test.py:409-423`):
  the capsule moved under the falling mesh (here the inline prism, scale 0.1
  as there). Capsule-mesh contacts: one row per mesh triangle."""
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
bodies {{
  name: "Capsule" mass: 1
  colliders {{ capsule {{ length: 2 radius: 0.2 }} }}
  inertia {{ x: 1 y: 1 z: 1 }}
}}
bodies {{ name: "Ground" frozen: {{ all: true }} colliders {{ plane {{}} }} }}
defaults {{
  qps {{ name: "Mesh" pos: {{ x: 0 y: 0 z: 0.7 }} }}
  qps {{ name: "Capsule" pos: {{ x: 0 y: 0 z: 0.2 }} rot: {{ x: 0 y: 90 z: 0 }} }}
}}
mesh_geometries {{ name: "Cylinder" {geom} }}
"""


# BoxCapsuleTest (`physics_test.py:141-205`): boxes fall onto capsules
# (capsule-box contacts against the box's 12 triangles, TwoWay), a capsule
# falls onto a frozen box (OneWay)
BOX_CAPSULE_TEST_CONFIG = """
dt: 0.05 substeps: 30 friction: 1
gravity { z: -9.8 }
bodies { name: "box1" mass: 1 colliders { box { halfsize { x: 0.5 y: 0.5 z: 0.5 }}} inertia { x: 1 y: 1 z: 1 } }
bodies { name: "capsule1" mass: 1 colliders { capsule { length: 2 radius: 0.2 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "box2" mass: 10 colliders { box { halfsize { x: 0.5 y: 0.5 z: 0.5 }}} inertia { x: 1 y: 1 z: 1 } }
bodies { name: "capsule2" mass: 1 colliders { capsule { length: 2 radius: 0.2 } } inertia { x: 1 y: 1 z: 1 } }
bodies { name: "box3" colliders { box { halfsize: { x: 0.5 y: 0.5 z: 0.5 } } } mass: 1.0 frozen { all: true } }
bodies { name: "capsule3" colliders { capsule { radius: 0.5 length: 1.0 } } inertia { x: 1.0 y: 1.0 z: 1.0 } mass: 1.0 }
bodies { name: "Ground" frozen: { all: true } colliders { plane {}}}
defaults {
  qps { name: "capsule1" pos { x: 8 y: 0 z: 1 } }
  qps { name: "box1" pos { x: 8 y: 0 z: 3.5 } }
  qps { name: "capsule2" pos { x: 2 y: 0 z: 1 } }
  qps { name: "box2" pos { x: 2 y: 0 z: 3.5 } }
  qps { name: "capsule3" pos { x: 0 y: 0 z: 3 } }
}
defaults {
  qps { name: "capsule1" pos { x: 8 y: 0 z: 1 } }
  qps { name: "box1" pos { x: 8.1 y: 0.05 z: 2.48 } rot { x: 5 z: 10 } vel { z: -0.5 } }
  qps { name: "capsule2" pos { x: 2 y: 0 z: 1 } }
  qps { name: "box2" pos { x: 2 y: 0.1 z: 2.53 } rot { y: 8 } }
  qps { name: "capsule3" pos { x: 0.1 y: 0 z: 1.423 } rot { x: 30 } }
}
solver_scale_collide: .3
"""
# the same scene with its box-box (hull-hull SAT) pairs left out through
# collide_include (only the listed pairs collide, colliders.py:969-972)
BOX_CAPSULE_NO_HULL_CONFIG = BOX_CAPSULE_TEST_CONFIG + """
collide_include { first: "capsule1" second: "box1" }
collide_include { first: "capsule2" second: "box2" }
collide_include { first: "capsule3" second: "box3" }
collide_include { first: "capsule1" second: "Ground" }
collide_include { first: "capsule2" second: "Ground" }
collide_include { first: "capsule3" second: "Ground" }
collide_include { first: "box1" second: "Ground" }
collide_include { first: "box2" second: "Ground" }
collide_include { first: "capsule1" second: "capsule2" }
"""


def heightmap_config(dt=2.0, substeps=1000):
  """HeightMapTest (`physics_test.py:228-250`): a box falls onto the bottom
  left quadrant of a 3 x 3 height map of size 10."""
  return f"""
dt: {dt} substeps: {substeps} friction: 1 elasticity: 0
gravity {{ z: -9.8 }}
bodies {{ name: "box" mass: 1 colliders {{ box {{ halfsize {{ x: 0.3 y: 0.3 z: 0.3 }}}} }} inertia {{ x: 0.1 y: 0.1 z: 0.1 }} }}
bodies {{ name: "ground" frozen: {{ all: true }}
  colliders {{ heightMap {{ size: 10 data: [1, 2, 3, 1, 2, 3, 1, 2, 3] }} }} }}
defaults {{ qps {{ name: "box" pos: {{x: 1.5 y: -7.5 z: 4}} }} }}
defaults {{ qps {{ name: "box" pos: {{x: 1.5 y: -7.5 z: 1.35}} rot {{ x: 10 y: 5 }} vel {{ x: 1 }} }} }}
"""


def clipped_plane_config(dt=2.0, substeps=800):
  """CapsuleClippedPlaneTest (`physics_test.py:426-461`): three spheres, one
  above a clipped plane at z = 2, two beside it falling to the ground."""
  return f"""
dt: {dt} substeps: {substeps} friction: 0.6
gravity {{ z: -9.8 }}
bodies {{ name: "Sphere1" mass: 1 colliders {{ sphere {{ radius: 0.5 }} }} inertia {{ x: 1 y: 1 z: 1 }} }}
bodies {{ name: "Sphere2" mass: 1 colliders {{ sphere {{ radius: 0.5 }} }} inertia {{ x: 1 y: 1 z: 1 }} }}
bodies {{ name: "Sphere3" mass: 1 colliders {{ sphere {{ radius: 0.5 }} }} inertia {{ x: 1 y: 1 z: 1 }} }}
bodies {{ name: "ClippedPlane" mass: 1
  colliders {{ clipped_plane {{ halfsize_x: 3 halfsize_y: 1 }} position {{ z: 2 }} }}
  frozen {{ all: true }} }}
bodies {{ name: "Ground" frozen: {{ all: true }} colliders {{ plane {{}}}} }}
defaults {{
  qps {{ name: "Sphere1" pos {{ z: 3 }} }}
  qps {{ name: "Sphere2" pos {{ z: 3 x: -4 }} }}
  qps {{ name: "Sphere3" pos {{ z: 3 y: -2 }} }}
  qps {{ name: "ClippedPlane" pos {{ x: 0 }} }}
}}
defaults {{
  qps {{ name: "Sphere1" pos {{ z: 2.55 x: 2.8 }} vel {{ x: 1 }} }}
  qps {{ name: "Sphere2" pos {{ z: 0.52 x: -4 }} }}
  qps {{ name: "Sphere3" pos {{ z: 1.0 y: -1.2 }} vel {{ y: 1 }} }}
  qps {{ name: "ClippedPlane" pos {{ x: 0 }} }}
}}
"""


def box_box_config(dt=0.5, substeps=200):
  """BoxBoxTest (`physics_test.py:85-117`): a small box (rotated 45 degrees)
  falls onto a box resting on the ground (hull-hull SAT contacts)."""
  return f"""
dt: {dt} substeps: {substeps} friction: 0.8 elasticity: 0.5
gravity {{ z: -9.8 }}
bodies {{ name: "box1" mass: 1 colliders {{ box {{ halfsize {{ x: 0.2 y: 0.2 z: 0.2 }}}} }} inertia {{ x: 1 y: 1 z: 1 }} }}
bodies {{ name: "box2" mass: 1 colliders {{ box {{ halfsize {{ x: 0.1 y: 0.1 z: 0.1 }}}} }} inertia {{ x: 1 y: 1 z: 1 }} }}
bodies {{ name: "Ground" frozen: {{ all: true }} colliders {{ plane {{}}}} }}
defaults {{
  qps {{ name: "box1" pos {{ x: 0 y: 1 z: .2 }} rot {{z: 0}} }}
  qps {{ name: "box2" pos {{ x: 0.1 y: 1 z: .6 }} rot {{z: 45}} }}
}}
defaults {{
  qps {{ name: "box1" pos {{ x: 0 y: 1 z: .2 }} rot {{z: 0}} }}
  qps {{ name: "box2" pos {{ x: 0.1 y: 1 z: .49 }} rot {{x: 7 y: 4 z: 45}} vel {{ z: -0.3 }} }}
}}
"""


# NearNeighbors past its allowed cells (colliders.py:55-89, 1005-1013): two
# bodies with two capsules each give 4 capsule-capsule pairs (> cutoff 3, so
# the group is culled) over U = 4 candidates, but the mask is set with BODY
# indices, so it allows one cell only, (0, 1). top_k(3) then also returns
# the two masked (-inf) cells of lowest flat index: (0, 0), a capsule against
# itself, and (0, 2).
TWIN_CULL_CONFIG = """
dt: 0.05 substeps: 10 friction: 0.6 gravity { z: -9.8 }
bodies { name: "A" mass: 1 inertia { x: 1 y: 1 z: 1 }
  colliders { capsule { radius: 0.25 length: 1.0 } }
  colliders { position { x: 0.5 } rotation { y: 90 } capsule { radius: 0.2 length: 0.8 } } }
bodies { name: "B" mass: 1 inertia { x: 1 y: 1 z: 1 }
  colliders { capsule { radius: 0.25 length: 1.0 } }
  colliders { position { y: 0.5 } rotation { x: 90 } capsule { radius: 0.2 length: 0.8 } } }
bodies { name: "Ground" frozen { all: true } colliders { plane {} } }
collider_cutoff: 3
defaults { qps { name: "A" pos { z: 1 } } qps { name: "B" pos { x: 0.3 y: 0.2 z: 1.5 } } }
"""
