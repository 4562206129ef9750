"""Parity margins: every GPU gate records (test, field, measured, tol).

A GPU run writes the worst ratio per (test, field) to
gpurun_out/parity_margins.json (committed per round under profiles/), so drift
toward a gate is visible before it fails. Imported as `tests.margins` by the
tests and by conftest's session hook (one module, one list)."""
import json
import os

_MARGINS = []


def record_margin(field, measured, tol, **extra):
  """`extra`: e.g. `n`, the samples the gate covered."""
  test = os.environ.get('PYTEST_CURRENT_TEST', '?').split(' ')[0]
  _MARGINS.append({'test': test, 'field': field, 'measured': measured, 'tol': tol,
                   'ratio': measured / tol if tol > 0 else None, **extra})


def write(path):
  if not _MARGINS:
    return
  worst = {}
  for m in _MARGINS:
    k = (m['test'], m['field'])
    if k not in worst or (m['ratio'] or 0) > (worst[k]['ratio'] or 0):
      worst[k] = m
  rows = sorted(worst.values(), key=lambda m: -(m['ratio'] or 0))
  os.makedirs(os.path.dirname(path), exist_ok=True)
  with open(path, 'w') as f:
    # the binding gates whose bound exceeds 1e-2 (the reset-lift obs, where
    # any env may flip); the ill-conditioned groups' envelope bounds (Brax's
    # own fp32 off by > 5e-3 there, role 'envelope') are listed apart: those
    # envs' binding gate is `:illcond_nearest` (<= 1e-2 by construction)
    wide = [m for m in rows if m['tol'] > 1e-2 and m.get('role') != 'envelope']
    env = [m for m in rows if m.get('role') == 'envelope']
    json.dump({'n_gates': len(_MARGINS), 'n_wide_gates': len(wide), 'wide_gates': wide,
               'envelope_gates': env, 'worst_per_test_field': rows}, f, indent=1)
