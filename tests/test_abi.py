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
