"""ctypes binding of ``libkompressor_hip.so`` (the C-ABI in ``include/kompressor_hip.h``).

The shared library is built in-tree by ``kompressor_amd._build`` (``__graft_entry__.build()``).
Importing this module never falls back to anything: a missing library raises ``ImportError``
and a missing / non-gfx950 GPU raises ``RuntimeError`` at the first compute call.
"""

import ctypes
import os

import numpy as np
# torch must be imported BEFORE the CDLL below: torch ships its own libamdhip64.so (SONAME
# libamdhip64.so.7); loaded first, our library's NEEDED libamdhip64.so.7 binds to that same
# runtime, so torch's allocations, streams and events and our launches share ONE HIP runtime.
# Loaded the other way round the process would carry two runtimes and the second to initialise
# sees no GPU.
import torch  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
# KMP_DEBUG=1 loads the variant with device bounds checks (kompressor_amd/_build.py --debug)
_DEFAULT_LIB = 'libkompressor_hip_debug.so' if os.environ.get('KMP_DEBUG', '0') != '0' else 'libkompressor_hip.so'
LIB_PATH = os.environ.get('KOMPRESSOR_HIP_LIB', os.path.join(HERE, _DEFAULT_LIB))

if not os.path.exists(LIB_PATH):
    raise ImportError(f'kompressor_amd: {LIB_PATH} is missing -- build it with '
                      f'`python -m kompressor_amd._build` (hipcc --offload-arch=gfx950)')

lib = ctypes.CDLL(LIB_PATH)

# enums (include/kompressor_hip.h)
KMP_OK, KMP_ERR_ARG, KMP_ERR_UNSUPPORTED, KMP_ERR_LAUNCH = 0, -1, -2, -3
U8, U16, I32, F32, U32 = 0, 1, 2, 3, 4
CODER_RAW, CODER_U8, CODER_U16, CODER_U32 = 0, 1, 2, 3
ENCODE, DECODE = 0, 1
PRED_MEAN, PRED_LINEAR, PRED_LINEAR_MFMA = 0, 1, 2

_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_i64p = ctypes.POINTER(ctypes.c_int64)
_i32p = ctypes.POINTER(ctypes.c_int32)
_vpp = ctypes.POINTER(ctypes.c_void_p)
_fp = ctypes.POINTER(ctypes.c_float)


class Predictor(ctypes.Structure):
    _fields_ = [('kind', ctypes.c_int32), ('padding', ctypes.c_int32),
                ('weights', ctypes.c_void_p), ('bias', ctypes.c_void_p)]


class RiceArray(ctypes.Structure):  # kmp_rice_array (include/kompressor_hip.h)
    _fields_ = [('samples', ctypes.c_void_p), ('n', ctypes.c_int64), ('side_off', ctypes.c_int64),
                ('toff_off', ctypes.c_int64), ('rec_off', ctypes.c_int64)]


class Region(ctypes.Structure):
    _fields_ = [('begin', ctypes.c_int64 * 3), ('end', ctypes.c_int64 * 3)]


_PROTOS = {
    'kmp_version': (ctypes.c_char_p, []),
    'kmp_last_error': (ctypes.c_char_p, []),
    'kmp_last_launch': (ctypes.c_char_p, []),
    'kmp_device_ok': (ctypes.c_int, []),
    'kmp_set_option': (ctypes.c_int, [ctypes.c_char_p, ctypes.c_int]),
    'kmp_clear_option': (ctypes.c_int, [ctypes.c_char_p]),
    'kmp_get_option': (ctypes.c_int, [ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]),
    'kmp_host_device_pointer': (ctypes.c_int, [_vp, _vpp]),
    'kmp_volume_encode': (ctypes.c_int, [_i32, _vp, _i64, _i64, _i64, _i64, _i64, ctypes.POINTER(Predictor), _i32,
                                         _vp, _vpp, _i32p, ctypes.POINTER(Region), _vp, ctypes.c_size_t, _vp]),
    'kmp_volume_decode': (ctypes.c_int, [_i32, _vp, _vpp, _i64, _i64, _i64, _i64, _i64, _i32p,
                                         ctypes.POINTER(Predictor), _i32, _vp, ctypes.POINTER(Region), _vp,
                                         ctypes.c_size_t, _vp]),
    'kmp_volume_workspace_bytes': (ctypes.c_int64, [_i32, _i64, _i64, _i64, _i64, _i64, ctypes.POINTER(Predictor)]),
    'kmp_image_encode': (ctypes.c_int, [_i32, _vp, _i64, _i64, _i64, _i64, ctypes.POINTER(Predictor), _i32,
                                        _vp, _vpp, _i32p, ctypes.POINTER(Region), _vp, ctypes.c_size_t, _vp]),
    'kmp_image_decode': (ctypes.c_int, [_i32, _vp, _vpp, _i64, _i64, _i64, _i64, _i32p,
                                        ctypes.POINTER(Predictor), _i32, _vp, ctypes.POINTER(Region), _vp,
                                        ctypes.c_size_t, _vp]),
    'kmp_image_workspace_bytes': (ctypes.c_int64, [_i32, _i64, _i64, _i64, _i64, ctypes.POINTER(Predictor)]),
    'kmp_lowres_from_highres': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _vp, _vp]),
    'kmp_maps_from_highres': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _vpp, _vp]),
    'kmp_targets_from_highres': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _vp, _vp]),
    'kmp_highres_from_lowres_and_maps': (ctypes.c_int, [_i32, _i32, _vp, _vpp, _i64, _i64p, _i64, _vp, _vp]),
    'kmp_features_from_lowres': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _i32, _vp, _vp]),
    'kmp_maps_from_predictions': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _vpp, _vp]),
    'kmp_mean_predict_maps': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _i32, _vpp, _vp]),
    'kmp_mean_predict_maps_typed': (ctypes.c_int, [_i32, _i32, _i32, _vp, _i64, _i64p, _i64, _i32, _vpp, _vp]),
    'kmp_linear_predict': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    'kmp_linear_predict_mfma': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _i32, _vp, _vp, _vp, _vp, _vp]),
    'kmp_pad': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _i64p, _i64p, _i32, _vp, _vp]),
    'kmp_copy_box': (ctypes.c_int, [_i32, _i32, _vp, _i64p, _i64p, _i32, _vp, _i64p, _i64p, _i64, _i64, _i64p,
                                    _vp]),
    'kmp_code': (ctypes.c_int, [_i32, _i32, _i32, _vp, _i32, _vp, _i64, _vp, _vp]),
    'kmp_categorical': (ctypes.c_int, [_i32, _vp, _i64, _i64, _i32, _vp, _vp, _vp]),
    'kmp_tiles': (ctypes.c_int, [_i32, _i32, _i32, _vp, _i64p, _i64, _i64p, _vp, _vp]),
    'kmp_window_from_highres': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _i32, _vp, _vp]),
    'kmp_window_from_lowres': (ctypes.c_int, [_i32, _i32, _vp, _i64, _i64p, _i64, _i32p, _i32, _vp, _vp]),
    'kmp_encode_with_predictions': (ctypes.c_int, [_i32, _i32, _i32, _vp, _i64, _i64p, _i64, _vpp, _vp, _vpp,
                                                   _vp]),
    'kmp_pack_blocks': (ctypes.c_int64, [_i64]),
    'kmp_pack_workspace_bytes': (ctypes.c_int64, [_i64]),
    'kmp_pack_total_offset': (ctypes.c_int64, [_i64]),
    'kmp_pack_plan': (ctypes.c_int, [_i32, _vp, _i64, _vp, _vp, _vp]),
    'kmp_pack': (ctypes.c_int, [_i32, _vp, _i64, _vp, _vp, _vp, _vp]),
    'kmp_pack_header': (ctypes.c_int, [_vp, ctypes.c_char_p, _i32, _i64, _i64, _vp, _i64, _i64, _vp]),
    'kmp_unpack_plan': (ctypes.c_int, [_vp, _i64, _vp, _vp]),
    'kmp_unpack': (ctypes.c_int, [_i32, _vp, _i64, _vp, _vp, _vp, _vp]),
    'kmp_unpack_check': (ctypes.c_int, [_i32, _i32, _vp, _vp, _i64, _vp, _vp]),
    'kmp_rice_tiles': (ctypes.c_int64, [_i64]),
    'kmp_rice_bundle_workspace_bytes': (ctypes.c_int64, [_i64]),
    'kmp_rice_bundle_encode': (ctypes.c_int, [_i32, _vp, _i32, _i64, _i64, _vp, _i64, _vp, _vp]),
    'kmp_rice_bundle_decode': (ctypes.c_int, [_i32, _vp, _i32, _i64, _vp, _i64, ctypes.c_uint64, _vp, _vp]),
    'kmp_crc32': (ctypes.c_int, [_vp, _i64, _vp, _vp, _vp]),
    'kmp_decode_with_predictions': (ctypes.c_int, [_i32, _i32, _i32, _vp, _vpp, _i64, _i64p, _i64, _i32p, _vpp,
                                                   _vp, _vp]),
    'kmp_encode_with_predictions_typed': (ctypes.c_int, [_i32, _i32, _i32, _i32, _vp, _i64, _i64p, _i64, _vpp, _vp,
                                                         _vpp, _vp]),
    'kmp_decode_with_predictions_typed': (ctypes.c_int, [_i32, _i32, _i32, _i32, _vp, _vpp, _i64, _i64p, _i64,
                                                         _i32p, _vpp, _vp, _vp]),
}

for _name, (_res, _args) in _PROTOS.items():
    _fn = getattr(lib, _name)  # AttributeError here == the library does not export the C-ABI
    _fn.restype = _res
    _fn.argtypes = _args

EXPORTED = tuple(_PROTOS)


class KompressorHipError(RuntimeError):
    pass


def check(status, what):
    if status != KMP_OK:
        msg = lib.kmp_last_error().decode(errors='replace')
        raise KompressorHipError(f'{what} failed ({status}): {msg}')


def version():
    return lib.kmp_version().decode()


def get_option(name):
    """A dispatch option's value, or None while it is unset."""
    v = ctypes.c_int()
    r = lib.kmp_get_option(name.encode(), ctypes.byref(v))
    if r < 0:
        check(r, 'kmp_get_option')
    return v.value if r == 1 else None


def set_option(name, value):
    """Set a dispatch option (``None`` returns it to the kernel's own default)."""
    if value is None:
        check(lib.kmp_clear_option(name.encode()), 'kmp_clear_option')
    else:
        check(lib.kmp_set_option(name.encode(), int(value)), 'kmp_set_option')


class option:
    """``with option('KMP_DISABLE_FAST', 1): ...`` -- set a dispatch option for a block, restoring
    its previous state after (the library reads its environment variable only once, at load)."""

    def __init__(self, name, value):
        self.name, self.value = name, value

    def __enter__(self):
        self.prev = get_option(self.name)
        set_option(self.name, self.value)
        return self

    def __exit__(self, *exc):
        set_option(self.name, self.prev)
        return False


# ---------------------------------------------------------------------------------------------
# small ctypes helpers
# ---------------------------------------------------------------------------------------------

def i64x3(vals):
    vals = list(vals) + [0] * (3 - len(vals))
    return (ctypes.c_int64 * 3)(*vals)


def i32xn(vals):
    vals = list(vals)
    return (ctypes.c_int32 * max(3, len(vals)))(*(vals + [0] * (3 - len(vals))))


def ptrs(tensors, n=7):
    arr = (ctypes.c_void_p * n)()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr() if t is not None else None
    return arr


_NP_TO_CODE = {np.dtype(np.uint8): U8, np.dtype(np.uint16): U16, np.dtype(np.int32): I32,
               np.dtype(np.float32): F32, np.dtype(np.uint32): U32}
