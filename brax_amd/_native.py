"""Loader of the in-tree HIP library `brax_amd/_lib/libbrax_amd.so`.

There is no CPU fallback: if the library or a GPU is missing, every device
entry point raises. Build with `python -c "import __graft_entry__ as g; g.build()"`
or `make -C brax_amd/csrc`.
"""
import ctypes as C
import os
import subprocess

from brax_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('BRAX_AMD_LIB') or os.path.join(HERE, '_lib', 'libbrax_amd.so')
CSRC = os.path.join(HERE, 'csrc')


class NativeError(RuntimeError):
  pass


def build(arch='gfx950', jobs=4):
  subprocess.run(['make', '-s', f'-j{jobs}', '-C', CSRC, f'ARCH={arch}'], check=True)


_lib = None

_SIGS = {
    'bx_abi_version': ([], C.c_int),
    'bx_last_error': ([], C.c_char_p),
    'bx_device_count': ([C.POINTER(C.c_int)], C.c_int),
    'bx_system_create': ([C.POINTER(abi.BxDesc), C.POINTER(abi.BxResetDesc), C.c_int,
                          C.POINTER(C.c_void_p)], C.c_int),
    'bx_system_destroy': ([C.c_void_p], C.c_int),
    'bx_system_lanes': ([C.c_void_p], C.c_int),
    'bx_system_env_lanes': ([C.c_void_p], C.c_int),
    'bx_system_lds_bytes': ([C.c_void_p], C.c_int),
    'bx_system_plan': ([C.c_void_p, C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                        C.POINTER(C.c_int32)], C.c_int),
    'bx_system_set_single': ([C.c_void_p, C.c_int], C.c_int),
    'bx_system_set_variant': ([C.c_void_p, C.c_int, C.c_int], C.c_int),
    'bx_system_set_block': ([C.c_void_p, C.c_int], C.c_int),
    'bx_system_step': ([C.c_void_p, C.c_int64, C.POINTER(abi.BxQP), C.c_void_p, C.c_int64,
                        C.c_int64, C.POINTER(abi.BxQP), C.POINTER(abi.BxInfo), C.c_void_p],
                       C.c_int),
    'bx_env_step': ([C.c_void_p, C.POINTER(abi.BxEnvParams), C.c_int64,
                     C.POINTER(abi.BxEnvState), C.c_void_p, C.c_int64, C.c_int64,
                     C.POINTER(abi.BxEnvState), C.c_void_p], C.c_int),
    'bx_env_step_packed': ([C.c_void_p, C.POINTER(abi.BxEnvParams), C.c_int64, C.c_void_p,
                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_int64,
                            C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    'bx_env_rollout_packed': ([C.c_void_p, C.POINTER(abi.BxEnvParams), C.c_int64, C.c_int32,
                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                               C.c_int64, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                               C.c_void_p], C.c_int),
    'bx_env_rollout_random': ([C.c_void_p, C.POINTER(abi.BxEnvParams), C.c_int64, C.c_int32,
                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                               C.c_uint64, C.c_uint64, C.c_float, C.c_float, C.c_int64,
                               C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p], C.c_int),
    'bx_env_sizes': ([C.c_void_p, C.POINTER(abi.BxEnvParams), C.POINTER(C.c_int32),
                      C.POINTER(C.c_int32)], C.c_int),
    'bx_env_reset': ([C.c_void_p, C.POINTER(abi.BxEnvParams), C.c_int64, C.c_uint64, C.c_int64,
                      C.c_void_p, C.c_float, C.POINTER(abi.BxEnvState), C.c_void_p], C.c_int),
    'bx_system_default_qp': ([C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p,
                              C.POINTER(abi.BxQP), C.c_void_p], C.c_int),
    'bx_system_info': ([C.c_void_p, C.c_int64, C.POINTER(abi.BxQP), C.POINTER(abi.BxInfo),
                        C.c_void_p], C.c_int),
    'bx_env_observe': ([C.c_void_p, C.POINTER(abi.BxEnvParams), C.c_int64,
                        C.POINTER(abi.BxQP), C.c_void_p, C.c_int64, C.c_int64, C.c_void_p,
                        C.c_void_p], C.c_int),
    'bx_system_joint_angles': ([C.c_void_p, C.c_int64, C.POINTER(abi.BxQP), C.c_void_p,
                                C.c_void_p, C.c_void_p], C.c_int),
    'bx_phase': ([C.c_void_p, C.c_int, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                  C.c_void_p, C.c_int64, C.c_void_p], C.c_int),
    'bx_phase_capsule_plane': ([C.c_void_p, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p,
                                C.c_int64, C.c_void_p], C.c_int),
    'bx_debug_stamps': ([C.POINTER(C.c_ulonglong), C.c_int], C.c_int),
    'bx_debug_partner': ([C.c_void_p, C.c_int, C.c_void_p], C.c_int),
    'bx_uniform': ([C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_float, C.c_float,
                    C.c_void_p], C.c_int),
    'bx_uniform_epoch': ([C.c_void_p, C.c_int64, C.c_uint64, C.c_uint64, C.c_void_p,
                          C.c_uint64, C.c_float, C.c_float, C.c_void_p], C.c_int),
    'bx_uniform_slabs': ([C.c_void_p, C.c_int64, C.c_int64, C.c_uint64, C.c_uint64, C.c_uint64,
                          C.c_void_p, C.c_uint64, C.c_float, C.c_float, C.c_void_p], C.c_int),
}

EXPORTS = tuple(_SIGS)


def lib():
  """Returns the loaded library; raises NativeError if it is not built."""
  global _lib
  if _lib is None:
    if not os.path.exists(LIB_PATH):
      raise NativeError(
          f'{LIB_PATH} is missing: the MI355X kernels are not built '
          '(run __graft_entry__.build() or make -C brax_amd/csrc). '
          'brax_amd has no CPU fallback.')
    l = C.CDLL(LIB_PATH)
    for name, (args, res) in _SIGS.items():
      f = getattr(l, name)
      f.argtypes = args
      f.restype = res
    if l.bx_abi_version() != abi.ABI_VERSION:
      raise NativeError('libbrax_amd ABI version mismatch')
    _lib = l
  return _lib


def check(rc):
  if rc != 0:
    raise NativeError(lib().bx_last_error().decode())
