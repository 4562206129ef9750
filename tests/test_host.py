"""Host-side containers of the fast step path (no GPU): the lazily viewed
packed QP and the lazily sliced metrics behave as the QP dataclass and the
metrics dict of the reference's State (`brax/physics/base.py:75-133`,
`brax/envs/env.py:28-36`)."""
import dataclasses

import torch

from brax_amd.base import PackedQP, QP, packed_buffer, packed_view
from brax_amd.envs.env import _Metrics


def _buf(B=4, N=3):
  b = torch.arange(B * N * 16, dtype=torch.float32).view(B, N, 16)
  return b


def test_packed_qp_fields_are_views_of_the_buffer():
  b = _buf()
  q = packed_view(b)
  assert type(q) is PackedQP and isinstance(q, QP)
  assert '_f' not in q.__dict__  # no views until a field is read
  assert q.shape == (4, 3)
  assert torch.equal(q.pos, b[..., 0:3]) and torch.equal(q.rot, b[..., 3:7])
  assert torch.equal(q.vel, b[..., 7:10]) and torch.equal(q.ang, b[..., 10:13])
  assert q.pos.data_ptr() == b.data_ptr() and q.ang.data_ptr() == b.data_ptr() + 40
  assert packed_buffer(q) is b


def test_packed_qp_replace_and_dataclass_ops():
  b = _buf()
  q = packed_view(b)
  v = torch.ones(4, 3, 3)
  for r in (q.replace(vel=v), dataclasses.replace(q, vel=v)):
    assert type(r) is QP
    assert torch.equal(r.vel, v) and torch.equal(r.pos, q.pos)
  assert q == q
  assert torch.equal(q[1].pos, b[1, :, 0:3])
  s = q + q
  assert torch.equal(s.rot, 2 * b[..., 3:7])


def test_metrics_mapping():
  m = torch.arange(8, dtype=torch.float32).view(4, 2)
  mt = _Metrics(m, ('a', 'b'), {'carried': 7})
  d = dict(mt)
  assert set(d) == {'a', 'b', 'carried'} and d['carried'] == 7
  assert torch.equal(d['b'], m[:, 1]) and len(mt) == 3 and 'a' in mt
  # a next step rewrites the kernel's keys and carries the rest
  assert _Metrics(m, ('a', 'b'), {'carried': 7}).carried(('a', 'b')) == {'carried': 7}
  mt['reward'] = 1.0  # as EvalWrapper adds it
  assert mt.carried(('a', 'b')) == {'carried': 7, 'reward': 1.0}
  # a kernel key set by hand is overwritten by the next step's column
  assert 'a' not in _Metrics(m, ('a', 'b'), {}).carried(('a', 'b'))
