"""ctypes binding of the C-ABI library libdrpo_hip.so (declared in include/drpo_hip.h).

The product path has NO CPU fallback: every compute entry point goes through this
library and raises if it is missing or if tensors are not on a HIP device.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('DRPO_LIB_OVERRIDE') or os.path.join(_HERE, 'libdrpo_hip.so')   # override: profiling builds only
_lib = None

c_int, c_i64, c_u64, c_f32, c_sz, c_vp = (ctypes.c_int, ctypes.c_int64, ctypes.c_uint64, ctypes.c_float,
                                          ctypes.c_size_t, ctypes.c_void_p)


class DrpoError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise DrpoError(f'{LIB_PATH} is missing: build it with __graft_entry__.build() '
                            '(the HIP path has no CPU fallback)')
        lib_ = ctypes.CDLL(LIB_PATH)
        from . import _abi, build_lib
        _abi.declare(lib_)
        got, want = lib_.drpo_build_digest().decode(), build_lib.source_digest()
        if got != want:
            raise DrpoError(f'{LIB_PATH} was built from other sources (library digest {got[:16]}, '
                            f'csrc/include digest {want[:16]}): rebuild it with __graft_entry__.build()')
        _lib = lib_
    return _lib


def build_digest():
    """Source digest compiled into the loaded library (== build_lib.source_digest())."""
    return lib().drpo_build_digest().decode()


def check(rc, what=''):
    if rc != 0:
        msg = lib().drpo_last_error().decode()
        raise DrpoError(f'{what}: {msg}' if what else msg)


def require_device(*tensors):
    for t in tensors:
        if t is not None and t.device.type != 'cuda':
            raise DrpoError('drpo_amd compute path requires tensors on a HIP (cuda) device; '
                            f'got {t.device} (there is no CPU fallback)')


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
