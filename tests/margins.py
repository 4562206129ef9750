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
    # the gates whose bound exceeds 1e-2 (Brax's own fp32 off by > 5e-3 on
    # their samples): the ill-conditioned groups and the reset-lift obs
    wide = [m for m in rows if m['tol'] > 1e-2]
    json.dump({'n_gates': len(_MARGINS), 'n_wide_gates': len(wide), 'wide_gates': wide,
               'worst_per_test_field': rows}, f, indent=1)
