"""Minimal pytree utilities (flatten/unflatten/map) over None, tuple, list,
dict, namedtuple and registered classes."""

_REGISTRY = {}


def register_pytree_node(cls, flatten, unflatten):
  _REGISTRY[cls] = (flatten, unflatten)


def _is_namedtuple(x):
  return isinstance(x, tuple) and hasattr(x, '_fields')


def tree_flatten(tree):
  leaves = []

  def rec(x):
    if x is None:
      return ('none',)
    t = type(x)
    if t in _REGISTRY:
      children, aux = _REGISTRY[t][0](x)
      return ('reg', t, aux, [rec(c) for c in children])
    if _is_namedtuple(x):
      return ('nt', t, [rec(c) for c in x])
    if isinstance(x, (tuple, list)):
      return ('seq', t, [rec(c) for c in x])
    if isinstance(x, dict):
      keys = sorted(x.keys())
      return ('dict', keys, [rec(x[k]) for k in keys])
    leaves.append(x)
    return ('leaf',)

  return leaves, rec(tree)


def tree_unflatten(treedef, leaves):
  it = iter(leaves)

  def rec(d):
    kind = d[0]
    if kind == 'none':
      return None
    if kind == 'leaf':
      return next(it)
    if kind == 'reg':
      _, t, aux, ch = d
      return _REGISTRY[t][1](aux, [rec(c) for c in ch])
    if kind == 'nt':
      return d[1](*[rec(c) for c in d[2]])
    if kind == 'seq':
      return d[1](rec(c) for c in d[2])
    if kind == 'dict':
      return {k: rec(c) for k, c in zip(d[1], d[2])}
    raise ValueError(kind)

  return rec(treedef)


def tree_leaves(tree):
  return tree_flatten(tree)[0]


def tree_map(f, tree, *rest):
  leaves, td = tree_flatten(tree)
  others = [tree_flatten(r)[0] for r in rest]
  return tree_unflatten(td, [f(*xs) for xs in zip(leaves, *others)])


def tree_reduce(f, tree, initializer=None):
  leaves = tree_leaves(tree)
  if initializer is None:
    acc, leaves = leaves[0], leaves[1:]
  else:
    acc = initializer
  for x in leaves:
    acc = f(acc, x)
  return acc
