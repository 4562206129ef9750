"""Stand-in for flax.struct: frozen dataclass + .replace + pytree registration."""
import dataclasses

from jax import tree_util


def field(pytree_node=True, **kwargs):
  return dataclasses.field(metadata={'pytree_node': pytree_node}, **kwargs)


def dataclass(cls):
  cls = dataclasses.dataclass(frozen=True)(cls)
  names = [f.name for f in dataclasses.fields(cls)]

  def flatten(obj):
    return [getattr(obj, n) for n in names], None

  def unflatten(_, children):
    return cls(*children)

  tree_util.register_pytree_node(cls, flatten, unflatten)
  cls.replace = lambda self, **kw: dataclasses.replace(self, **kw)
  return cls
