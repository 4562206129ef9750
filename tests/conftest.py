import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
  sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
  config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI)')


def golden(name):
  return np.load(os.path.join(GOLDEN, name + '.npz'))


@pytest.fixture(scope='session')
def oracle_lib():
  from oracle import oracle  # test infrastructure
  oracle.build()
  return oracle


def pytest_sessionfinish(session, exitstatus):
  # the parity margins recorded by the GPU gates (tests/margins.py)
  from tests import margins
  margins.write(os.path.join(ROOT, 'gpurun_out', 'parity_margins.json'))
