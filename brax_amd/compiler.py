"""System compiler: `brax.Config` -> flat constant arrays (the descriptor).

Host-side, once per System, float64 numpy (the reference builds these in
Python double from fp32 proto fields and lets `jit` cast them to fp32). The
ordering rules and quirks are the reference's, restated:

  validate_config      `brax/physics/base.py:156-254`
  Body                 `brax/physics/bodies.py:38-44`   (stores INVERSE inertia)
  colliders.get        `brax/physics/colliders.py:891-1023`
  Collidable/Capsule*  `brax/physics/geometry.py:78-99,242-288`
  joints.get / Joint   `brax/physics/joints.py:418-474,36-77`
  spring_joints.get    `brax/physics/spring_joints.py:40-87,302-331` (legacy_spring)
  actuators.get        `brax/physics/actuators.py:115-164`
  Euler.__init__       `brax/physics/integrators.py:32-48`
  Collider.__init__    `brax/physics/colliders.py:95-114`

The descriptor keys match `oracle/gen_golden.py:dump_desc`, so the reference's
own compiled arrays pin this compiler (tests/test_compiler.py).
"""
import copy
import warnings

import itertools

import numpy as np

from brax_amd import config as cfgmod

# joint kinds (descriptor `joint_type`)
REVOLUTE, UNIVERSAL, SPHERICAL = 1, 2, 3
# dynamics modes (descriptor `dynamics_mode`)
DYN_PBD, DYN_LEGACY_SPRING = 0, 1
# actuator kinds (descriptor `act_type`)
TORQUE, ANGLE = 0, 1
# contact functions (descriptor `col_fn`)
CAPSULE_PLANE, CAPSULE_CAPSULE, HEIGHTMAP, CLIPPED_PLANE, CAPSULE_MESH, HULL_HULL = 0, 1, 2, 3, 4, 5
ROW_EXT = 16  # per-row extra constants of the extended contact functions
# force kinds
THRUSTER, TWISTER = 0, 1


# --------------------------------------------------------------------------
# float64 math helpers (same formulas as `brax/math.py:25-77`)
# --------------------------------------------------------------------------

def vec(v):
  return np.array([v.x, v.y, v.z], np.float64)


def euler_to_quat(v):
  """x-y'-z'' intrinsic Tait-Bryan, degrees -> wxyz (`math.py:68-77`)."""
  c1, c2, c3 = np.cos(v * np.pi / 360)
  s1, s2, s3 = np.sin(v * np.pi / 360)
  w = c1 * c2 * c3 - s1 * s2 * s3
  x = s1 * c2 * c3 + c1 * s2 * s3
  y = c1 * s2 * c3 - s1 * c2 * s3
  z = c1 * c2 * s3 + s1 * s2 * c3
  return np.array([w, x, y, z])


def rotate(vv, q):
  """Rotates vector vv by unit quaternion q (`math.py:25-40`)."""
  s, u = q[0], q[1:]
  r = 2 * (np.dot(u, vv) * u) + (s * s - np.dot(u, u)) * vv
  return r + 2 * s * np.cross(u, vv)


# --------------------------------------------------------------------------
# validate_config
# --------------------------------------------------------------------------

_AXES = tuple((part, ax) for part in ('position', 'rotation') for ax in 'xyz')
_NAMED = ('bodies', 'joints', 'actuators', 'mesh_geometries')


def _reify_frozen(frozen, inherited=None):
  """Makes one Frozen message explicit: `all` <-> six set axes.

  With `inherited` (the config-level Frozen) an unset axis takes the
  inherited value first (`base.py:219-224`). Returns the final `all` flag.
  """
  if inherited is not None:
    for part, ax in _AXES:
      own = getattr(getattr(frozen, part), ax)
      setattr(getattr(frozen, part), ax, own or getattr(getattr(inherited, part), ax))
  if frozen.all:
    for part, ax in _AXES:
      setattr(getattr(frozen, part), ax, 1.0)
  if all(getattr(getattr(frozen, part), ax) for part, ax in _AXES):
    frozen.all = True
  return bool(frozen.all)


def _resolve_dynamics_mode(config):
  """`base.py:181-204`: an explicit mode is checked against the joints'
  stiffness; anything else is inferred from it, with the reference's warning."""
  stiff = [j.stiffness != 0 for j in config.joints]
  mode = config.dynamics_mode
  if mode == 'legacy_spring' and not all(stiff):
    raise ValueError('joint.stiffness must be >0 when dynamics_mode == legacy_spring')
  if mode == 'pbd':
    if any(stiff):
      raise ValueError('joint.stiffness is invalid when dynamics_mode == pbd')
    if config.baumgarte_erp:
      raise ValueError('baumgarte_erp is invalid when dynamics_mode == pbd')
  if mode in ('legacy_spring', 'pbd'):
    return
  config.dynamics_mode = 'legacy_spring' if any(stiff) else 'pbd'
  warnings.warn('dynamics_mode not specified, but joint.stiffness >0. '
                'Setting dynamics_mode="legacy_spring".' if any(stiff) else
                'dynamics_mode not specified, defaulting to "pbd".')


def validate_config(config):
  """Returns a normalised deep copy of `config`, as `base.py:156-254` does.

  Steps: positive dt, substeps >= 1, solver_scale_collide defaults to 1;
  unique names per named collection; the dynamics mode; explicit frozen
  axes (config level, then each body inheriting it); unit inertia for
  bodies that give none; collider materials from the config defaults. Mesh
  files are not loaded (inline `mesh_geometries` only).
  """
  config = copy.deepcopy(config)
  if config.dt <= 0:
    raise ValueError('config.dt must be positive')
  config.substeps = config.substeps or 1
  config.solver_scale_collide = config.solver_scale_collide or 1.0
  for coll in _NAMED:
    names = [o.name for o in getattr(config, coll)]
    dup = next((n for i, n in enumerate(names) if n in names[:i]), None)
    if dup is not None:
      raise RuntimeError(f'duplicate name in config: {dup}')
  _resolve_dynamics_mode(config)

  _reify_frozen(config.frozen)
  body_all = []
  for b in config.bodies:
    if not (b.inertia.x or b.inertia.y or b.inertia.z):
      b.inertia.x = b.inertia.y = b.inertia.z = 1
    body_all.append(_reify_frozen(b.frozen, config.frozen))
    for c in b.colliders:
      if not c.HasField('material'):
        c.material.friction = config.friction
        c.material.elasticity = config.elasticity
  config.frozen.all = all(body_all)
  return config


# --------------------------------------------------------------------------
# pieces
# --------------------------------------------------------------------------

def _bodies(config):
  inv_inertia = 1. / np.array([vec(b.inertia) for b in config.bodies])
  mass = np.array([b.mass for b in config.bodies], np.float64)
  index = {b.name: i for i, b in enumerate(config.bodies)}
  return mass, inv_inertia, index


def _integrator(config):
  pos_mask = 1. * np.logical_not(
      np.array([vec(b.frozen.position) for b in config.bodies]))
  rot_mask = 1. * np.logical_not(
      np.array([vec(b.frozen.rotation) for b in config.bodies]))
  quat_mask = 1. * np.logical_not(
      np.array([[0.] + list(vec(b.frozen.rotation)) for b in config.bodies]))
  return pos_mask, rot_mask, quat_mask


def _capsule_axis(col):
  return rotate(np.array([0., 0., 1.]), euler_to_quat(vec(col.rotation)))


def _near_neighbors(pairs, index, cutoff):
  """NearNeighbors candidates (`colliders.py:55-89`, built at :1005-1013).

  The candidates are the group's unique collidables in first-appearance
  order (a, then b, per pair). The allowed-pair mask is set with BODY indices
  (`col_a.body.idx`, `col_b.body.idx`) into the candidates' U x U distance
  matrix (`jp.index_update(dist_mask, mask, 0)`), so entry (i, j) pairs
  candidate i with candidate j, whichever bodies those are; the rows are
  those entries, in flat (i * U + j) order. Each step keeps the `cutoff`
  entries with the smallest candidate-centre distance (top_k of -dist; ties
  to the lower flat index, as jax.lax.top_k).

  Mask cells outside U x U follow the jit path: `.at[].set` drops
  out-of-bounds scatter indices (the numpy backend raises IndexError there,
  e.g. for Ant Mountain(2+)). With more cutoff than allowed cells, top_k
  also returns masked (sim = -inf) cells: every allowed cell first, then the
  masked cells of lowest flat index (jax.lax.top_k keeps equal values in
  index order). Those cells are rows too, flagged `masked`; the kernels rank
  them after every allowed cell."""
  uniq, seen = [], {}
  for ca, ca_idx, ba, cb, cb_idx, bb in pairs:
    for c, c_idx, b in ((ca, ca_idx, ba), (cb, cb_idx, bb)):
      if (b.name, c_idx) not in seen:
        seen[(b.name, c_idx)] = len(uniq)
        uniq.append((c, c_idx, b))
  U = len(uniq)
  cells = sorted({(index[ba.name], index[bb.name]) for _, _, ba, _, _, bb in pairs})
  cells = [(i, j) for i, j in cells if i < U and j < U]
  allowed = {i * U + j for i, j in cells}
  if cutoff > U * U:
    raise ValueError(f'collider_cutoff {cutoff} exceeds the {U * U} NearNeighbors cells')
  extra = [f for f in range(U * U) if f not in allowed][:max(cutoff - len(cells), 0)]
  flat = sorted(allowed | set(extra))
  rows = [(uniq[f // U][0], uniq[f // U][1], uniq[f // U][2],
           uniq[f % U][0], uniq[f % U][1], uniq[f % U][2]) for f in flat]
  return dict(pairs=rows, flat=flat, masked=[int(f not in allowed) for f in flat],
              cutoff=int(cutoff))


_BOX_CORNERS = np.array(list(itertools.product((-1, 1), (-1, 1), (-1, 1))), np.float64)
# `geometry.py:34-56`: the 12 triangles of a box (indices into _BOX_CORNERS)
# and their outward normals
_TRI_BOX_FACES = [0, 4, 1, 4, 1, 5, 0, 4, 2, 2, 4, 6, 6, 4, 5, 6, 5, 7,
                  2, 6, 3, 3, 6, 7, 1, 3, 5, 5, 3, 7, 0, 2, 1, 1, 2, 3]
_TRI_BOX_NORMALS = [[0, -1., 0], [0, -1., 0], [0, 0, -1.], [0, 0, -1.], [1., 0, 0], [1., 0, 0],
                    [0, 1., 0], [0, 1., 0], [0, 0, 1.], [0, 0, 1.], [-1., 0, 0], [-1., 0, 0]]


# `geometry.py:57-73`: the box's 6 quads (clockwise) and their normals
_BOX_QUADS = [0, 1, 5, 4, 0, 4, 6, 2, 6, 4, 5, 7, 2, 6, 7, 3, 1, 3, 7, 5, 0, 2, 3, 1]
_BOX_QUAD_NORMALS = [[0, -1., 0], [0, 0, -1.], [1., 0, 0], [0, 1., 0], [0, 0, 1.], [-1., 0, 0]]


def _hull_box(col):
  """HullBox (`geometry.py:201-206` via BoxMesh/BaseMesh :138-198): the 8
  corners, the 6 quads (winding fixed as for every mesh) and their normals,
  in the body frame."""
  rot = euler_to_quat(vec(col.rotation))
  vert = np.array([rotate(c, rot) for c in _BOX_CORNERS * vec(col.box.halfsize)])
  vert = vert + vec(col.position)
  normals = np.array([rotate(np.array(n), rot) for n in _BOX_QUAD_NORMALS])
  faces = vert[np.array(_BOX_QUADS)].reshape(-1, 4, 3)
  out = []
  for f, n in zip(faces, normals):
    wind = np.dot(np.cross(f[0] - f[-1], f[0] - f[1]), n) >= 0
    out.append(f if wind else f[::-1])
  return vert, np.array(out), normals


def _mesh_faces(col, mesh_geoms):
  """Triangles (F,3,3) and face normals (F,3) in the body frame of a
  TriangulatedBox (`geometry.py:157-198`) or a Mesh (`geometry.py:291-331`),
  with BaseMesh's winding fix (`geometry.py:138-154`): a face whose first two
  edges wind against its normal has its vertex order reversed."""
  rot = euler_to_quat(vec(col.rotation))
  if col.WhichOneof('type') == 'box':
    vert = np.array([rotate(c, rot) for c in _BOX_CORNERS * vec(col.box.halfsize)])
    vert = vert + vec(col.position)
    normals = np.array([rotate(np.array(n), rot) for n in _TRI_BOX_NORMALS])
    faces = vert[np.array(_TRI_BOX_FACES)].reshape(-1, 3, 3)
  else:
    g = mesh_geoms[col.mesh.name]
    scale = col.mesh.scale if col.mesh.scale else 1
    vert = np.array([[v.x * scale, v.y * scale, v.z * scale] for v in g.vertices], np.float64)
    vert = np.array([rotate(v, rot) for v in vert]) + vec(col.position)
    faces = vert[np.array(list(g.faces), np.int64)].reshape(-1, 3, 3)
    normals = np.array([rotate(vec(n), rot) for n in g.face_normals])
  out = []
  for f, n in zip(faces, normals):
    wind = np.dot(np.cross(f[0] - f[-1], f[0] - f[1]), n) >= 0
    out.append(f if wind else f[::-1])
  return np.array(out), normals


def _point_ends(col, mesh_geoms):
  """Body-frame contact points of a box (8 corners, `geometry.py:123-137`) or
  a point mesh (its scaled vertices, `geometry.py:312-357`)."""
  rot = euler_to_quat(vec(col.rotation))
  if col.WhichOneof('type') == 'box':
    pts = _BOX_CORNERS * vec(col.box.halfsize)
  else:
    g = mesh_geoms[col.mesh.name]
    scale = col.mesh.scale if col.mesh.scale else 1
    pts = np.array([[v.x * scale, v.y * scale, v.z * scale] for v in g.vertices], np.float64)
  return [rotate(p, rot) + vec(col.position) for p in pts]


def _colliders(config, index):
  """Collider groups and flattened contact rows (`colliders.py:891-1023`)."""
  # only the capsule/sphere/plane subset of `collider_pairs` is on the path
  # (SURVEY §2); other supported-by-reference types raise.
  pair_types = [('box', 'plane'), ('box', 'heightMap'), ('capsule', 'box'),
                ('capsule', 'plane'), ('capsule', 'capsule'),
                ('capsule', 'mesh'), ('capsule', 'clipped_plane'),
                ('mesh', 'plane'), ('box', 'box')]
  # box-plane and mesh-plane contacts are point-plane contacts of the box
  # corners / mesh vertices (`colliders.py:667-696`): exactly capsule_plane
  # with a zero radius, so they compile to CAPSULE_PLANE rows
  supported = {('capsule', 'plane'): CAPSULE_PLANE,
               ('capsule', 'capsule'): CAPSULE_CAPSULE,
               ('box', 'plane'): CAPSULE_PLANE,
               ('mesh', 'plane'): CAPSULE_PLANE,
               ('box', 'heightMap'): HEIGHTMAP,
               ('capsule', 'clipped_plane'): CLIPPED_PLANE,
               ('capsule', 'box'): CAPSULE_MESH,
               ('capsule', 'mesh'): CAPSULE_MESH,
               ('box', 'box'): HULL_HULL}
  mesh_geoms = {mg.name: mg for mg in config.mesh_geometries}
  unique_meshes = {}
  cols = []
  for b in config.bodies:
    for c_idx, c in enumerate(b.colliders):
      if c.no_contact:
        continue
      if c.WhichOneof('type') == 'sphere':
        nc = cfgmod.Message('Collider')
        nc.CopyFrom(c)
        nc.capsule.radius = c.sphere.radius
        nc.capsule.length = 2 * c.sphere.radius
        nc.capsule.end = 1
        c = nc
      if c.WhichOneof('type') == 'mesh':
        unique_meshes[c.mesh.name] = 1
      cols.append((c, b, c_idx))

  include = {(ci.first, ci.second) for ci in config.collide_include}
  # NB: a generator, consumed by the first membership test (App. A.1)
  parents = ((j.parent, j.child) for j in config.joints)
  groups = []

  def pairs_of(cols_a, cols_b):
    cols_a = [x for x in cols_a if not x[1].frozen.all]
    cols_ab = []
    pair_count = {}
    for ca, ba, ca_idx in cols_a:
      for cb, bb, cb_idx in cols_b:
        included = (ba.name, bb.name) in include or (bb.name, ba.name) in include
        if ((ba.name, ca_idx, bb.name, cb_idx) in pair_count or
            (bb.name, cb_idx, ba.name, ca_idx) in pair_count):
          continue
        if ba.name == bb.name:
          continue
        if ba.frozen.all and bb.frozen.all:
          continue
        # `A or B and not included` binds as `A or (B and not included)`
        if (ba.name, bb.name) in parents or (bb.name, ba.name) in parents and not included:
          continue
        if ca.no_contact or cb.no_contact:
          continue
        if not include or included:
          cols_ab.append((ca, ca_idx, ba, cb, cb_idx, bb))
          pair_count[(ba.name, ca_idx, bb.name, cb_idx)] = 1
          pair_count[(bb.name, cb_idx, ba.name, ca_idx)] = 1
    return cols_ab

  for (type_a, type_b) in pair_types:
    # mesh pairs form one collider per unique mesh name (colliders.py:941-949)
    replicas = list(unique_meshes) if 'mesh' in (type_a, type_b) else [None]
    for mesh_name in replicas:
      def of_type(t, mesh_name=mesh_name):
        return [x for x in cols if x[0].WhichOneof('type') == t and
                (t != 'mesh' or x[0].mesh.name == mesh_name)]
      cols_ab = pairs_of(of_type(type_a), of_type(type_b))
      for b_is_frozen in (True, False):
        flt = [x for x in cols_ab if x[-1].frozen.all == b_is_frozen]
        if not flt:
          continue
        if (type_a, type_b) not in supported:
          raise NotImplementedError(
              f'collider pair {type_a}/{type_b} is outside the MI355X path')
        grp = dict(oneway=b_is_frozen, fn=supported[(type_a, type_b)], pairs=flt, cutoff=0,
                   kind=type_a)
        if (config.collider_cutoff and len(flt) > config.collider_cutoff and
            (type_a, type_b) == ('capsule', 'capsule')):
          grp.update(_near_neighbors(flt, index, config.collider_cutoff))
        groups.append(grp)

  h = config.dt / config.substeps
  g_norm = np.linalg.norm(vec(config.gravity))
  out = dict(col_oneway=[], col_fn=[], col_scale=[], col_velocity_threshold=[],
             col_baumgarte_erp=[])
  rows = {k: [] for k in ('group', 'body_a', 'body_b', 'a_pos', 'a_end',
                          'a_radius', 'b_pos', 'b_end', 'b_radius', 'friction',
                          'elasticity', 'flat', 'nn_masked', 'ext', 'hm')}
  hm_data = []
  hulls = {}  # (body name, collider index) -> hull index (HullBox data)
  hull_vert, hull_face, hull_norm = [], [], []

  def hull_of(c, c_idx, b):
    key = (b.name, c_idx)
    if key not in hulls:
      v, f, n = _hull_box(c)
      hulls[key] = len(hull_vert)
      hull_vert.append(v)
      hull_face.append(f)
      hull_norm.append(n)
    return hulls[key]
  out['col_cutoff'] = []
  for gi, g in enumerate(groups):
    out['col_oneway'].append(1 if g['oneway'] else 0)
    out['col_fn'].append(g['fn'])
    out['col_scale'].append(config.solver_scale_collide)
    out['col_velocity_threshold'].append(g_norm * h * 4.0)
    out['col_baumgarte_erp'].append(config.baumgarte_erp * config.substeps / config.dt)
    out['col_cutoff'].append(g['cutoff'])
    ext_l = None
    if g['fn'] == HULL_HULL:
      # hull_hull (`colliders.py:851-888`): SAT gives 4 contacts per pair
      # (edge contact padded, or the face manifold); row e of a pair is
      # contact e, ext = (hull a, hull b, e)
      ends_l, ext_l = [], []
      for ca, ca_idx, ba, cb, cb_idx, bb in g['pairs']:
        ha, hb = hull_of(ca, ca_idx, ba), hull_of(cb, cb_idx, bb)
        ends_l.append([np.zeros(3)] * 4)
        ext_l.append([np.concatenate([[ha, hb, e], np.zeros(ROW_EXT - 3)]) for e in range(4)])
    elif g['kind'] in ('box', 'mesh'):
      # Box corners (`geometry.py:123-137`) / PointMesh vertices (:312-357)
      # in the body frame, as zero-radius capsule ends
      ends_l = [_point_ends(ca, mesh_geoms) for ca, _, _, _, _, _ in g['pairs']]
    elif g['fn'] == CAPSULE_MESH:
      # one row per triangle of the box / mesh (`colliders.py:822-848`)
      ends_l, ext_l = [], []
      for ca, _, _, cb, _, _ in g['pairs']:
        faces, normals = _mesh_faces(cb, mesh_geoms)
        ends_l.append([_capsule_axis(ca) * (ca.capsule.length * 0.5 - ca.capsule.radius)]
                      * len(faces))
        ext_l.append([np.concatenate([f.reshape(-1), n, np.zeros(ROW_EXT - 12)])
                      for f, n in zip(faces, normals)])
    elif g['fn'] in (CAPSULE_PLANE, CLIPPED_PLANE):
      # CapsuleEnd (`geometry.py:261-288`): 1 or 2 ends; mixed -> pad by dup
      ends_l = []
      for ca, _, _, _, _, _ in g['pairs']:
        axis = _capsule_axis(ca)
        seg = ca.capsule.length * 0.5 - ca.capsule.radius
        ends_l.append([vec(ca.position) + e * axis * seg
                       for e in ([ca.capsule.end] if ca.capsule.end else [-1, 1])])
      if len({len(e) for e in ends_l}) != 1:
        for e in ends_l:
          if len(e) == 1:
            e.append(e[0])
    flats = g.get('flat', [-1] * len(g['pairs']))
    masked = g.get('masked', [0] * len(g['pairs']))
    for pi, (ca, _, ba, cb, _, bb) in enumerate(g['pairs']):
      fa = ca.material.friction * cb.material.friction
      ea = ca.material.elasticity * cb.material.elasticity
      a_rad = 0. if g['kind'] in ('box', 'mesh') else ca.capsule.radius
      if g['fn'] == HULL_HULL:
        a_rad = 0.
      ext, hm = [np.zeros(ROW_EXT)] * len(ends_l[pi]) if g['fn'] != CAPSULE_CAPSULE else [
          np.zeros(ROW_EXT)], (-1, 0)
      if g['fn'] == HEIGHTMAP:
        # HeightMap (`geometry.py:270-288`): a square grid, row-major, cell
        # size = size / (mesh_size - 1)
        data = np.asarray(list(cb.heightMap.data), np.float64)
        m = int(np.sqrt(len(data)))
        if m * m != len(data):
          raise ValueError('height map data length should be a perfect square.')
        hm = (len(hm_data), m)
        hm_data.extend(data.tolist())
        ext = [np.concatenate([[cb.heightMap.size / (m - 1)], np.zeros(ROW_EXT - 1)])] * 8
      elif g['fn'] == CLIPPED_PLANE:
        # ClippedPlane (`geometry.py:214-239`): normal, x, y of the collider
        # rotation, position, half sizes (body frame)
        rot = euler_to_quat(vec(cb.rotation))
        e = np.concatenate([rotate(np.array([0., 0., 1.]), rot), rotate(np.array([1., 0., 0.]), rot),
                            rotate(np.array([0., 1., 0.]), rot), vec(cb.position),
                            [cb.clipped_plane.halfsize_x, cb.clipped_plane.halfsize_y],
                            np.zeros(ROW_EXT - 14)])
        ext = [e] * len(ends_l[pi])
      elif ext_l is not None:
        ext = ext_l[pi]
      if g['fn'] in (CAPSULE_PLANE, HEIGHTMAP, CLIPPED_PLANE, CAPSULE_MESH, HULL_HULL):
        ends = ends_l[pi]
        b_end, b_rad = np.zeros(3), 0.
      else:
        ends = [_capsule_axis(ca) * (ca.capsule.length * 0.5 - ca.capsule.radius)]
        b_end = _capsule_axis(cb) * (cb.capsule.length * 0.5 - cb.capsule.radius)
        b_rad = cb.capsule.radius
      for ei, e in enumerate(ends):
        rows['ext'].append(ext[ei])
        rows['hm'].append(hm)
        rows['flat'].append(flats[pi])
        rows['nn_masked'].append(masked[pi])
        rows['group'].append(gi)
        rows['body_a'].append(index[ba.name])
        rows['body_b'].append(index[bb.name])
        rows['a_pos'].append(vec(ca.position))
        rows['a_end'].append(e)
        rows['a_radius'].append(a_rad)
        rows['b_pos'].append(vec(cb.position))
        rows['b_end'].append(b_end)
        rows['b_radius'].append(b_rad)
        rows['friction'].append(fa)
        rows['elasticity'].append(ea)
  d = {}
  d['col_oneway'] = np.asarray(out['col_oneway'], np.int32)
  d['col_fn'] = np.asarray(out['col_fn'], np.int32)
  d['col_cutoff'] = np.asarray(out['col_cutoff'], np.int32)
  for k in ('col_scale', 'col_velocity_threshold', 'col_baumgarte_erp'):
    d[k] = np.asarray(out[k], np.float64)
  d['row_ext'] = np.asarray(rows.pop('ext'), np.float64).reshape(-1, ROW_EXT)
  d['row_hm'] = np.asarray(rows.pop('hm'), np.int32).reshape(-1, 2)
  d['hm_data'] = np.asarray(hm_data, np.float64)
  d['hull_vert'] = np.asarray(hull_vert, np.float64).reshape(-1, 8, 3)
  d['hull_face'] = np.asarray(hull_face, np.float64).reshape(-1, 6, 4, 3)
  d['hull_norm'] = np.asarray(hull_norm, np.float64).reshape(-1, 6, 3)
  if not any(rows['nn_masked']):
    rows.pop('nn_masked')  # the key exists only where a masked cell is a row
  for k, v in rows.items():
    if k in ('group', 'body_a', 'body_b', 'flat', 'nn_masked'):
      d['row_' + k] = np.asarray(v, np.int32)
    elif k.endswith(('pos', 'end')):
      d['row_' + k] = np.asarray(v, np.float64).reshape(-1, 3)
    else:
      d['row_' + k] = np.asarray(v, np.float64)
  return d


def _joint_geometry(j):
  """Offsets and axes shared by both joint families (`joints.py:58-77`,
  `spring_joints.py:72-86`)."""
  axis_c = np.array([rotate(e, euler_to_quat(vec(j.rotation))) for e in np.eye(3)])
  ref = euler_to_quat(vec(j.reference_rotation))
  axis_p = np.array([rotate(a, ref) for a in axis_c])
  return vec(j.parent_offset), vec(j.child_offset), axis_p, axis_c


def _spring_joints(config, index):
  """Springy joint groups of `legacy_spring` (`spring_joints.py:302-331`):
  every joint (stiffness > 0 is enforced by validate_config) goes to its dof's
  group, groups in dof order, Revolute / Universal / Spherical; no
  sphericalisation. Defaults (`spring_joints.py:59-67`): spring_damping =
  coeff * sqrt(stiffness) with coeff 0.5 for Revolute (`:120`) and 2.0
  otherwise; limit_strength = stiffness."""
  groups = {}
  for joint in config.joints:
    if joint.stiffness > 0:
      groups.setdefault(len(joint.angle_limit), []).append(joint)
  groups = sorted(groups.items(), key=lambda kv: kv[0])
  keys = ('type', 'dof', 'free_dofs', 'body_p', 'body_c', 'off_p', 'off_c', 'axis_p',
          'axis_c', 'limit', 'damping', 'scale_pos', 'scale_ang', 'group', 'stiffness',
          'spring_damping', 'limit_strength')
  J = {k: [] for k in keys}
  meta = []
  for gi, (dof, v) in enumerate(groups):
    if dof not in (1, 2, 3):
      raise RuntimeError(f'invalid number of joint limits: {dof}')
    jtype = {1: REVOLUTE, 2: UNIVERSAL, 3: SPHERICAL}[dof]
    coeff = 0.5 if dof == 1 else 2.0
    meta.append((dof, [j.name for j in v], None))
    for j in v:
      off_p, off_c, axis_p, axis_c = _joint_geometry(j)
      J['type'].append(jtype)
      J['dof'].append(dof)
      J['free_dofs'].append(-1)
      J['body_p'].append(index[j.parent])
      J['body_c'].append(index[j.child])
      J['off_p'].append(off_p)
      J['off_c'].append(off_c)
      J['axis_p'].append(axis_p)
      J['axis_c'].append(axis_c)
      lim = np.zeros((3, 2))
      lim[:dof] = np.array([[i.min, i.max] for i in j.angle_limit]) / 180.0 * np.pi
      J['limit'].append(lim)
      J['damping'].append(j.angular_damping)
      J['scale_pos'].append(0.)
      J['scale_ang'].append(0.)
      J['group'].append(gi)
      J['stiffness'].append(j.stiffness)
      J['spring_damping'].append(j.spring_damping if j.HasField('spring_damping')
                                 else coeff * np.sqrt(np.float64(j.stiffness)))
      J['limit_strength'].append(j.limit_strength if j.HasField('limit_strength')
                                 else j.stiffness)
  return _joint_arrays(J), meta


def _joint_arrays(J):
  d = {}
  for k in ('type', 'dof', 'free_dofs', 'body_p', 'body_c', 'group'):
    d['joint_' + k] = np.asarray(J[k], np.int32)
  d['joint_off_p'] = np.asarray(J['off_p'], np.float64).reshape(-1, 3)
  d['joint_off_c'] = np.asarray(J['off_c'], np.float64).reshape(-1, 3)
  d['joint_axis_p'] = np.asarray(J['axis_p'], np.float64).reshape(-1, 3, 3)
  d['joint_axis_c'] = np.asarray(J['axis_c'], np.float64).reshape(-1, 3, 3)
  d['joint_limit'] = np.asarray(J['limit'], np.float64).reshape(-1, 3, 2)
  for k in ('damping', 'scale_pos', 'scale_ang', 'stiffness', 'spring_damping',
            'limit_strength'):
    d['joint_' + k] = np.asarray(J.get(k, [0.] * len(J['type'])), np.float64)
  return d


def _joints(config, mass, inv_inertia, index):
  """Joint groups (`joints.py:418-474`). MUTATES config.joints (App. A.2)."""
  if config.dynamics_mode == 'legacy_spring':
    return _spring_joints(config, index)
  groups = {}
  dofs = {len(j.angle_limit) for j in config.joints}
  sphericalize = len(dofs) > 1
  sphericalize |= 2 in dofs
  for joint in config.joints:
    dof = len(joint.angle_limit)
    free = dof
    while sphericalize and dof < 3:
      joint.angle_limit.add()
      dof += 1
    groups.setdefault(dof, {'joint': [], 'free_dofs': []})
    groups[dof]['joint'].append(joint)
    groups[dof]['free_dofs'].append(free)
  groups = sorted(groups.items(), key=lambda kv: kv[0])
  scale_pos = config.solver_scale_pos or .6
  scale_ang = config.solver_scale_ang or .2
  J = {k: [] for k in ('type', 'dof', 'free_dofs', 'body_p', 'body_c', 'off_p',
                       'off_c', 'axis_p', 'axis_c', 'limit', 'damping',
                       'scale_pos', 'scale_ang', 'group')}
  meta = []  # per group: (dof, names, free_dofs or None)
  for gi, (dof, v) in enumerate(groups):
    if dof not in (1, 2, 3):
      raise RuntimeError(f'invalid number of joint limits: {dof}')
    jtype = REVOLUTE if dof == 1 else SPHERICAL
    free = v['free_dofs'] if dof == 3 else None
    meta.append((dof, [j.name for j in v['joint']], free))
    for k, j in enumerate(v['joint']):
      J['type'].append(jtype)
      J['dof'].append(dof)
      J['free_dofs'].append(free[k] if free is not None else -1)
      J['body_p'].append(index[j.parent])
      J['body_c'].append(index[j.child])
      off_p, off_c, axis_p, axis_c = _joint_geometry(j)
      J['off_p'].append(off_p)
      J['off_c'].append(off_c)
      J['axis_c'].append(axis_c)
      J['axis_p'].append(axis_p)
      lim = np.zeros((3, 2))
      lim[:dof] = np.array([[i.min, i.max] for i in j.angle_limit]) / 180.0 * np.pi
      J['limit'].append(lim)
      J['damping'].append(j.angular_damping)
      J['scale_pos'].append(scale_pos)
      J['scale_ang'].append(scale_ang)
      J['group'].append(gi)
  return _joint_arrays(J), meta


def _actuators(config, jmeta):
  """Actuator groups (`actuators.py:115-164`)."""
  groups = {}
  current = 0
  gbase = np.cumsum([0] + [len(m[1]) for m in jmeta])
  for actuator in config.actuators:
    gi = [i for i, m in enumerate(jmeta) if actuator.joint in m[1]]
    if not gi:
      raise RuntimeError(f'joint not found: {actuator.joint}')
    gi = gi[0]
    dof, names, free = jmeta[gi]
    jidx = names.index(actuator.joint)
    if free is not None:
      fd = free[jidx]
      act_index = tuple(i if i - current < fd else -1
                        for i in range(current, current + dof))
      current += fd
    else:
      act_index = tuple(range(current, current + dof))
      current += dof
    kind = actuator.WhichOneof('type')
    if kind not in ('torque', 'angle'):
      raise RuntimeError(f'unknown actuator type: {kind}')
    key = (kind, dof, gi)
    groups.setdefault(key, []).append((actuator, act_index, gbase[gi] + jidx))
  groups = sorted(groups.items(), key=lambda kv: kv[0][:2])
  A = {k: [] for k in ('type', 'joint', 'strength', 'index', 'group')}
  for g, ((kind, dof, _), items) in enumerate(groups):
    for act, idx, jglob in items:
      A['type'].append(TORQUE if kind == 'torque' else ANGLE)
      A['joint'].append(jglob)
      A['strength'].append(act.strength)
      ii = -np.ones(3, np.int64)
      ii[:dof] = idx
      A['index'].append(ii)
      A['group'].append(g)
  d = {'act_type': np.asarray(A['type'], np.int32),
       'act_joint': np.asarray(A['joint'], np.int32),
       'act_strength': np.asarray(A['strength'], np.float64),
       'act_index': np.asarray(A['index'], np.int32).reshape(-1, 3),
       'act_group': np.asarray(A['group'], np.int32)}
  return d, current


def _forces(config, index):
  """Thruster/Twister groups (`forces.py:110-138`).

  Action indices continue after the ACTUATORS' dofs, counted on the joints as
  they stand after sphericalisation (`forces.py:114-116`; joints.get has
  already mutated the config), and are assigned in config order; the groups
  then apply Thrusters first, Twisters second (`forces.py:130-136`)."""
  dofs = {j.name: len(j.angle_limit) for j in config.joints}
  cur = sum(dofs[a.joint] for a in config.actuators)
  start = cur
  items = {'thruster': [], 'twister': []}
  for f in config.forces:
    kind = f.WhichOneof('type')
    if kind not in items:
      raise ValueError(f'unknown force type: {kind}')
    if f.body not in index:
      raise KeyError(f.body)
    items[kind].append((f, [cur, cur + 1, cur + 2]))
    cur += 3
  F = {'type': [], 'body': [], 'strength': [], 'index': []}
  for kind, code in (('thruster', THRUSTER), ('twister', TWISTER)):
    for f, idx in items[kind]:
      F['type'].append(code)
      F['body'].append(index[f.body])
      F['strength'].append(f.strength)
      F['index'].append(idx)
  # num_forces_dof = sum(f.act_index.shape[-1] for f in forces) (system.py:72)
  # counts 3 per force GROUP, not per force: with several Thrusters the
  # action is shorter than their index range and the tail clips (jp.take)
  n_dof = 3 * sum(1 for kind in items if items[kind])
  return {'force_type': np.asarray(F['type'], np.int32),
          'force_body': np.asarray(F['body'], np.int32),
          'force_strength': np.asarray(F['strength'], np.float64),
          'force_index': np.asarray(F['index'], np.int32).reshape(-1, 3)}, n_dof


def compile_system(config):
  """Returns (validated config, descriptor dict, metadata dict)."""
  config = validate_config(config)
  num_joint_dof = sum(len(j.angle_limit) for j in config.joints)
  mass, inv_inertia, index = _bodies(config)
  d = {}
  d['n_bodies'] = np.int32(len(config.bodies))
  d['body_mass'] = mass
  d['body_inv_inertia'] = inv_inertia
  d['pos_mask'], d['rot_mask'], d['quat_mask'] = _integrator(config)
  d['h'] = np.float64(config.dt / config.substeps)
  d['dt'] = np.float64(config.dt)
  d['substeps'] = np.int32(config.substeps)
  d['gravity'] = vec(config.gravity)
  d['velocity_damping'] = np.float64(config.velocity_damping)
  d['angular_damping'] = np.float64(config.angular_damping)
  d['dynamics_mode'] = np.int32(DYN_LEGACY_SPRING if config.dynamics_mode == 'legacy_spring'
                                else DYN_PBD)
  d.update(_colliders(config, index))
  jd, jmeta = _joints(config, mass, inv_inertia, index)
  d.update(jd)
  ad, _ = _actuators(config, jmeta)
  d.update(ad)
  fd, n_force_dof = _forces(config, index)
  d.update(fd)
  d['num_joint_dof'] = np.int32(num_joint_dof)
  d['action_size'] = np.int32(num_joint_dof + n_force_dof)
  meta = dict(num_joint_dof=num_joint_dof, num_forces_dof=n_force_dof,
              body_index=index, joint_groups=jmeta,
              action_size=num_joint_dof + n_force_dof)
  return config, d, meta


# --------------------------------------------------------------------------
# reset (System.default_angle / default_qp / bodies.min_z)
# --------------------------------------------------------------------------

def default_angle(config, default_index=0):
  """`System.default_angle` (system.py:86-110), float64."""
  if not config.joints:
    return np.zeros(0)
  dofs = {j.name: sum([l.min != 0 or l.max != 0 for l in j.angle_limit])
          for j in config.joints}
  angles = {}
  if default_index < len(config.defaults):
    for ja in config.defaults[default_index].angles:
      angles[ja.name] = vec(ja.angle)[:dofs[ja.name]] * np.pi / 180
  for joint in config.joints:
    if joint.name not in angles:
      dof = dofs[joint.name]
      angles[joint.name] = np.array(
          [(l.min + l.max) * np.pi / 360 for l in joint.angle_limit][:dof])
  return np.concatenate([angles[j.name] for j in config.joints])




def compile_reset(config, index, default_index=0):
  """Reset descriptor for `System.default_qp` (system.py:112-242).

  `config` must be the validated config AFTER joints.get padded it (the
  reference's System.config is that same mutated object)."""
  N = len(config.bodies)
  base = np.zeros((N, 13))
  base[:, 3] = 1.0
  default = None
  if default_index < len(config.defaults):
    default = config.defaults[default_index]
    for dqp in default.qps:
      i = index[dqp.name]
      base[i, 0:3] = vec(dqp.pos)
      base[i, 3:7] = euler_to_quat(vec(dqp.rot))
      base[i, 7:10] = vec(dqp.vel)
      base[i, 10:13] = vec(dqp.ang)
  joint_idxs = []
  for j in config.joints:
    beg = joint_idxs[-1][1][1] if joint_idxs else 0
    dof = sum([l.min != 0 or l.max != 0 for l in j.angle_limit])
    joint_idxs.append((j, (beg, beg + dof)))
  lineage = {j.child: j.parent for j in config.joints}
  depth = {}
  for child, parent in lineage.items():
    depth[child] = 1
    while parent in lineage:
      parent = lineage[parent]
      depth[child] += 1
  joint_idxs = sorted(joint_idxs, key=lambda x: depth.get(x[0].parent, 0))
  joints = [j for j, _ in joint_idxs]
  r = {k: [] for k in ('fk_body_p', 'fk_body_c', 'fk_dof_index', 'fk_rot',
                       'fk_ref', 'fk_off_p', 'fk_off_c')}
  for j, (beg, end) in joint_idxs:
    r['fk_body_p'].append(index[j.parent])
    r['fk_body_c'].append(index[j.child])
    ix = list(range(beg, end)) + [-1] * (3 - (end - beg))
    r['fk_dof_index'].append(ix[:3])
    r['fk_rot'].append(euler_to_quat(vec(j.rotation)))
    r['fk_ref'].append(euler_to_quat(vec(j.reference_rotation)))
    r['fk_off_p'].append(vec(j.parent_offset))
    r['fk_off_c'].append(vec(j.child_offset))
  out = {
      'fk_body_p': np.asarray(r['fk_body_p'], np.int32),
      'fk_body_c': np.asarray(r['fk_body_c'], np.int32),
      'fk_dof_index': np.asarray(r['fk_dof_index'], np.int32).reshape(-1, 3),
      'fk_rot': np.asarray(r['fk_rot'], np.float64).reshape(-1, 4),
      'fk_ref': np.asarray(r['fk_ref'], np.float64).reshape(-1, 4),
      'fk_off_p': np.asarray(r['fk_off_p'], np.float64).reshape(-1, 3),
      'fk_off_c': np.asarray(r['fk_off_c'], np.float64).reshape(-1, 3),
      'base_qp': base,
  }
  # root trees lifted above the plane (system.py:213-240)
  fixed = {j.child for j in joints}
  if default:
    fixed |= {q.name for q in default.qps}
  root_idx = {b.name: [i] for i, b in enumerate(config.bodies)
              if b.name not in fixed}
  for j in joints:
    parent = j.parent
    while parent in lineage:
      parent = lineage[parent]
    if parent in root_idx:
      root_idx[parent].append(index[j.child])
  group = -np.ones(N, np.int32)
  for gi, members in enumerate(root_idx.values()):
    for b in members:
      group[b] = gi
  out['body_root_group'] = group
  out['n_root_groups'] = np.int32(len(root_idx))
  # bodies.min_z candidates (bodies.py:62-98)
  zb, zl, zr = [], [], []
  zero = np.zeros(N, np.int32)
  for bi, b in enumerate(config.bodies):
    if not b.colliders:
      zero[bi] = 1
    for col in b.colliders:
      kind = col.WhichOneof('type')
      if kind == 'sphere':
        zb.append(bi); zl.append(vec(col.position)); zr.append(col.sphere.radius)
      elif kind == 'capsule':
        axis = rotate(np.array([0., 0., 1.]), euler_to_quat(vec(col.rotation)))
        length = col.capsule.length / 2 - col.capsule.radius
        for e in (-1, 1):
          zb.append(bi)
          zl.append(vec(col.position) + e * axis * length)
          zr.append(col.capsule.radius)
      elif kind == 'box':
        q = euler_to_quat(vec(col.rotation))
        for corner in _BOX_CORNERS:
          c = rotate(corner * vec(col.box.halfsize), q) + vec(col.position)
          zb.append(bi); zl.append(c); zr.append(0.0)
      else:
        zero[bi] = 1
  out['zpt_body'] = np.asarray(zb, np.int32)
  out['zpt_local'] = np.asarray(zl, np.float64).reshape(-1, 3)
  out['zpt_radius'] = np.asarray(zr, np.float64)
  out['body_zero_cand'] = zero
  out['default_angle'] = default_angle(config, default_index)
  return out
