"""The C-ABI library builds, loads without a GPU and exports every symbol
declared in include/brax_amd.h (no compute calls here)."""
import ctypes
import os
import re

from brax_amd import _native
from brax_amd import abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
  src = open(os.path.join(ROOT, 'include', 'brax_amd.h')).read()
  return sorted(set(re.findall(r'^\s*(?:int|const char\*)\s+(bx_\w+)\s*\(', src, re.M)))


def test_header_declares_the_boundary():
  names = _declared()
  for n in ('bx_system_create', 'bx_system_step', 'bx_env_step', 'bx_system_default_qp',
            'bx_system_info', 'bx_last_error'):
    assert n in names


def test_library_exports_every_declared_symbol():
  if not os.path.exists(_native.LIB_PATH):
    _native.build()
  lib = ctypes.CDLL(_native.LIB_PATH)
  for n in _declared():
    assert hasattr(lib, n), n
  assert set(_native.EXPORTS) == set(_declared())


def test_abi_version_and_error_path():
  lib = _native.lib()
  assert lib.bx_abi_version() == abi.ABI_VERSION
  # a null descriptor fails at create with a message, no GPU touched
  h = ctypes.c_void_p()
  rc = lib.bx_system_create(None, None, 0, ctypes.byref(h))
  assert rc != 0 and b'null' in lib.bx_last_error()


def test_missing_library_fails_loudly(tmp_path):
  """No CPU fallback: with the HIP library absent, the product path raises
  NativeError at its first native call instead of computing anything."""
  import subprocess
  import sys
  code = ('import brax_amd, sys\n'
          'from brax_amd._native import NativeError\n'
          'from brax_amd.system import System\n'
          'from tests.helpers import config_for\n'
          'try:\n'
          '  System.plan(config_for("ant"))\n'
          'except NativeError as e:\n'
          '  print("raised", e)\n'
          '  sys.exit(0)\n'
          'sys.exit(3)\n')
  env = dict(os.environ, BRAX_AMD_LIB=str(tmp_path / 'absent' / 'libbrax_amd.so'))
  r = subprocess.run([sys.executable, '-c', code], cwd=ROOT, env=env, capture_output=True,
                     text=True, timeout=120)
  assert r.returncode == 0, r.stdout + r.stderr
  assert 'raised' in r.stdout
