"""`brax.Config` without protobuf: a schema-driven text-format reader.

Mirrors the message schema of `brax/physics/config.proto:6-309` (the reference's
System description) so configs written for the reference parse unchanged:

  cfg = brax_amd.Config.from_text(text)          # == text_format.Parse
  cfg.bodies[0].colliders[0].capsule.radius      # attribute access
  cfg.bodies[0].colliders[0].WhichOneof('type')  # oneof query
  cfg.HasField('frozen'), cfg.joints.add(), obj.CopyFrom(other)

Every `float` field of the proto is an IEEE fp32, so values are rounded to fp32
on assignment (`dt: 0.05` reads back as 0.05000000074505806);
derived constants are then computed in Python double like the reference does.
"""
import copy as _copy
import re

import numpy as np

# --------------------------------------------------------------------------
# schema: message -> {field: (kind, type, repeated)}; kind in scalar|msg
# --------------------------------------------------------------------------

_F, _I, _B, _S = 'float', 'int32', 'bool', 'string'

_SCHEMA = {
    'Vector3': {'x': _F, 'y': _F, 'z': _F},
    'Frozen': {'position': 'Vector3', 'rotation': 'Vector3', 'all': _B},
    'Body': {'name': _S, 'colliders': ['Collider'], 'inertia': 'Vector3',
             'mass': _F, 'frozen': 'Frozen'},
    'Material': {'elasticity': _F, 'friction': _F},
    'Box': {'halfsize': 'Vector3'},
    'Plane': {},
    'ClippedPlane': {'halfsize_x': _F, 'halfsize_y': _F},
    'Sphere': {'radius': _F},
    'Capsule': {'radius': _F, 'length': _F, 'end': _I},
    'HeightMap': {'size': _F, 'data': [_F]},
    'MeshRef': {'name': _S, 'scale': _F},
    'Collider': {'position': 'Vector3', 'rotation': 'Vector3', 'box': 'Box',
                 'plane': 'Plane', 'sphere': 'Sphere', 'capsule': 'Capsule',
                 'heightMap': 'HeightMap', 'material': 'Material',
                 'mesh': 'MeshRef', 'color': _S, 'hidden': _B,
                 'no_contact': _B, 'clipped_plane': 'ClippedPlane'},
    'Range': {'min': _F, 'max': _F},
    'Joint': {'name': _S, 'stiffness': _F, 'parent': _S, 'child': _S,
              'parent_offset': 'Vector3', 'child_offset': 'Vector3',
              'rotation': 'Vector3', 'angular_damping': _F,
              'angle_limit': ['Range'], 'limit_strength': _F,
              'spring_damping': _F, 'reference_rotation': 'Vector3'},
    'Empty': {},
    'Actuator': {'name': _S, 'joint': _S, 'strength': _F, 'torque': 'Empty',
                 'angle': 'Empty'},
    'Force': {'name': _S, 'body': _S, 'strength': _F, 'thruster': 'Empty',
              'twister': 'Empty'},
    'JointAngle': {'name': _S, 'angle': 'Vector3'},
    'DefaultQP': {'name': _S, 'pos': 'Vector3', 'rot': 'Vector3',
                  'vel': 'Vector3', 'ang': 'Vector3'},
    'DefaultState': {'angles': ['JointAngle'], 'qps': ['DefaultQP']},
    'MeshGeometry': {'name': _S, 'path': _S, 'vertices': ['Vector3'],
                     'faces': [_I], 'vertex_normals': ['Vector3'],
                     'face_normals': ['Vector3']},
    'NamePair': {'first': _S, 'second': _S},
    'Config': {'bodies': ['Body'], 'joints': ['Joint'],
               'actuators': ['Actuator'], 'forces': ['Force'],
               'elasticity': _F, 'friction': _F, 'gravity': 'Vector3',
               'velocity_damping': _F, 'angular_damping': _F,
               'baumgarte_erp': _F, 'collide_include': ['NamePair'],
               'dt': _F, 'substeps': _I, 'frozen': 'Frozen',
               'defaults': ['DefaultState'], 'collider_cutoff': _I,
               'mesh_geometries': ['MeshGeometry'], 'dynamics_mode': _S,
               'solver_scale_pos': _F, 'solver_scale_ang': _F,
               'solver_scale_collide': _F},
}

# proto3 oneof groups (config.proto Collider.type, Actuator.type, Force.type)
_ONEOF = {
    'Collider': ('box', 'plane', 'sphere', 'capsule', 'heightMap', 'mesh',
                 'clipped_plane'),
    'Actuator': ('torque', 'angle'),
    'Force': ('thruster', 'twister'),
}
# `optional` scalar fields whose presence is tracked (config.proto:244-245,305-308)
_OPTIONAL = {('Joint', 'limit_strength'), ('Joint', 'spring_damping'),
             ('Config', 'solver_scale_pos'), ('Config', 'solver_scale_ang'),
             ('Config', 'solver_scale_collide')}

_SCALAR_DEFAULT = {_F: 0.0, _I: 0, _B: False, _S: ''}


def _short(x):
  """Shortest decimal that rounds back to the same fp32."""
  for p in range(1, 18):
    t = f'{x:.{p}g}'
    if np.float32(float(t)) == np.float32(x):
      if 'e+' in t:
        t = str(float(t))
      return t[:-2] if t.endswith('.0') else t
  return repr(x)


def f32(x):
  """Rounds a Python number to the nearest fp32, returned as a Python float."""
  return float(np.float32(x))


def _coerce(kind, v):
  if kind == _F:
    return f32(v)
  if kind == _I:
    return int(v)
  if kind == _B:
    return bool(v)
  return str(v)


class RepeatedField(list):
  """List of messages/scalars with proto-style `add()`."""

  def __init__(self, mtype, items=()):
    super().__init__(items)
    self._mtype = mtype

  def add(self, **kwargs):
    if isinstance(self._mtype, str) and self._mtype in _SCHEMA:
      m = Message(self._mtype, **kwargs)
      self.append(m)
      return m
    raise TypeError('add() only for repeated message fields')

  def __deepcopy__(self, memo):
    return RepeatedField(self._mtype, [_copy.deepcopy(x, memo) for x in self])


class Message:
  """A proto3 message instance for one `_SCHEMA` type."""

  def __init__(self, mtype, **kwargs):
    object.__setattr__(self, '_type', mtype)
    object.__setattr__(self, '_vals', {})
    for k, v in kwargs.items():
      setattr(self, k, v)

  # -- access ---------------------------------------------------------------
  def _spec(self, name):
    try:
      return _SCHEMA[self._type][name]
    except KeyError:
      raise AttributeError(f'{self._type} has no field {name!r}') from None

  def __getattr__(self, name):
    if name.startswith('_'):
      raise AttributeError(name)
    spec = self._spec(name)
    vals = self._vals
    if name in vals:
      return vals[name]
    if isinstance(spec, list):
      r = RepeatedField(spec[0])
      vals[name] = r
      return r
    if spec in _SCHEMA:
      m = Message(spec)
      # sub-messages materialise on first write, like protobuf: reading an
      # unset sub-message returns a default instance linked to its parent.
      object.__setattr__(m, '_parent', (self, name))
      return m
    return _SCALAR_DEFAULT[spec]

  def __setattr__(self, name, value):
    spec = self._spec(name)
    if isinstance(spec, list):
      r = RepeatedField(spec[0])
      for v in value:
        r.append(v if isinstance(v, Message) else _coerce(spec[0], v))
      self._vals[name] = r
    elif spec in _SCHEMA:
      if not isinstance(value, Message):
        raise TypeError(f'{name} expects a {spec} message')
      self._vals[name] = value
    else:
      self._vals[name] = _coerce(spec, value)
    self._touch()
    if self._type in _ONEOF and name in _ONEOF[self._type]:
      for other in _ONEOF[self._type]:
        if other != name:
          self._vals.pop(other, None)

  def _touch(self):
    """Attaches a lazily-created sub-message to its parent once written."""
    parent = self.__dict__.get('_parent')
    if parent is not None:
      p, name = parent
      if name not in p._vals:
        p._vals[name] = self
        if p._type in _ONEOF and name in _ONEOF[p._type]:
          for other in _ONEOF[p._type]:
            if other != name:
              p._vals.pop(other, None)
        p._touch()
      del self.__dict__['_parent']

  # -- proto-ish API --------------------------------------------------------
  def HasField(self, name):  # pylint: disable=invalid-name
    self._spec(name)
    return name in self._vals

  def WhichOneof(self, group):  # pylint: disable=invalid-name
    del group
    for name in _ONEOF.get(self._type, ()):
      if name in self._vals:
        return name
    return None

  def ClearField(self, name):  # pylint: disable=invalid-name
    self._vals.pop(name, None)

  def CopyFrom(self, other):  # pylint: disable=invalid-name
    object.__setattr__(self, '_vals', _copy.deepcopy(other._vals))
    self._touch()

  def __deepcopy__(self, memo):
    m = Message(self._type)
    object.__setattr__(m, '_vals', _copy.deepcopy(self._vals, memo))
    return m

  def __repr__(self):
    return f'{self._type}({self._vals!r})'

  def to_compact(self):
    """One-line text-format rendering (round-trips through `parse`)."""
    out = []
    for k, v in self._vals.items():
      spec = _SCHEMA[self._type][k]
      items = v if isinstance(spec, list) else [v]
      for it in items:
        if isinstance(it, Message):
          out.append(f'{k} {{ {it.to_compact()} }}')
        elif isinstance(it, str):
          out.append(f'{k}: "{it}"')
        elif isinstance(it, bool):
          out.append(f'{k}: {"true" if it else "false"}')
        elif isinstance(it, float):
          out.append(f'{k}: {_short(it)}')
        else:
          out.append(f'{k}: {it}')
    return ' '.join(out)

  def to_text(self, indent=0):
    pad = '  ' * indent
    out = []
    for k, v in self._vals.items():
      spec = _SCHEMA[self._type][k]
      items = v if isinstance(spec, list) else [v]
      for it in items:
        if isinstance(it, Message):
          out.append(f'{pad}{k} {{\n{it.to_text(indent + 1)}{pad}}}\n')
        elif isinstance(it, str):
          out.append(f'{pad}{k}: "{it}"\n')
        elif isinstance(it, bool):
          out.append(f'{pad}{k}: {"true" if it else "false"}\n')
        else:
          out.append(f'{pad}{k}: {it!r}\n')
    return ''.join(out)


# --------------------------------------------------------------------------
# text-format tokenizer / parser
# --------------------------------------------------------------------------

_TOKEN = re.compile(r'''
    \s+ | \#[^\n]* |
    (?P<str>"(?:[^"\\]|\\.)*"|'(?:[^'\\]|\\.)*') |
    (?P<punct>[{}:\[\],;<>]) |
    (?P<word>[A-Za-z0-9_.+\-]+)
''', re.VERBOSE)


def _tokens(text):
  pos = 0
  n = len(text)
  while pos < n:
    m = _TOKEN.match(text, pos)
    if not m:
      raise ValueError(f'config parse error near: {text[pos:pos + 40]!r}')
    pos = m.end()
    if m.lastgroup:
      yield m.lastgroup, m.group(m.lastgroup)


def _scalar(kind, tok_kind, tok):
  if kind == _S:
    if tok_kind != 'str':
      raise ValueError(f'expected string, got {tok!r}')
    return bytes(tok[1:-1], 'utf-8').decode('unicode_escape')
  if kind == _B:
    return tok in ('true', 'True', '1', 't')
  if kind == _I:
    return int(tok)
  t = tok.lower().rstrip('f') if not tok.lower().startswith(('inf', '-inf')) else tok
  return float(t)


def _parse_msg(msg, toks, closing):
  while True:
    try:
      kind, tok = next(toks)
    except StopIteration:
      if closing is None:
        return
      raise ValueError('unterminated message') from None
    if kind == 'punct' and tok in ('}', '>'):
      if closing is None:
        raise ValueError('unbalanced }')
      return
    if kind == 'punct' and tok in (',', ';'):
      continue
    if kind != 'word':
      raise ValueError(f'unexpected token {tok!r}')
    name = tok
    spec = msg._spec(name)  # pylint: disable=protected-access
    base = spec[0] if isinstance(spec, list) else spec
    kind, tok = next(toks)
    if kind == 'punct' and tok == ':':
      kind, tok = next(toks)
    if base in _SCHEMA:
      if not (kind == 'punct' and tok in ('{', '<')):
        raise ValueError(f'expected {{ after {name}')
      sub = Message(base)
      _parse_msg(sub, toks, '}')
      if isinstance(spec, list):
        getattr(msg, name).append(sub)
      else:
        if name in msg._vals:  # pylint: disable=protected-access
          # repeated occurrences of a singular message merge (text_format)
          _merge(msg._vals[name], sub)  # pylint: disable=protected-access
        else:
          setattr(msg, name, sub)
    else:
      if kind == 'punct' and tok == '[':
        vals = []
        while True:
          kind, tok = next(toks)
          if kind == 'punct' and tok == ']':
            break
          if kind == 'punct' and tok == ',':
            continue
          vals.append(_scalar(base, kind, tok))
        for v in vals:
          getattr(msg, name).append(_coerce(base, v))
      else:
        v = _scalar(base, kind, tok)
        if isinstance(spec, list):
          getattr(msg, name).append(_coerce(base, v))
        else:
          setattr(msg, name, v)


def _merge(dst, src):
  for k, v in src._vals.items():  # pylint: disable=protected-access
    spec = _SCHEMA[dst._type][k]  # pylint: disable=protected-access
    if isinstance(spec, list):
      getattr(dst, k).extend(v)
    elif isinstance(v, Message) and k in dst._vals:  # pylint: disable=protected-access
      _merge(dst._vals[k], v)  # pylint: disable=protected-access
    else:
      setattr(dst, k, v)


def parse(text: str) -> Message:
  """Parses a brax text-format config (as `text_format.Parse(text, Config())`)."""
  cfg = Message('Config')
  _parse_msg(cfg, iter(_tokens(text)), None)
  return cfg


def Config(**kwargs) -> Message:  # pylint: disable=invalid-name
  return Message('Config', **kwargs)


Config.from_text = parse
