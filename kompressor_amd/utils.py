"""Residual coders, chunk enumerator and padding validator -- ``src/kompressor/utils.py`` of the
reference, running on the HIP engine.

Each coder is a plain function ``coder(pred, value)`` like the reference's; it additionally
carries a ``_kmp_coder`` tag so ``encode`` / ``decode`` can recognise it and run the fused
one-pass kernel instead of one launch per map.
"""

from . import _lib
from ._nd import d_categorical, d_code, validate_padding, yield_chunks  # noqa: F401
from . import _device as dev


def _coder(direction, coder, name, doc):
    def fn(pred, x):
        kind = 'torch' if dev.is_torch(x) else 'numpy'
        return dev.from_device(d_code(direction, coder, pred, x), kind)
    fn.__name__ = fn.__qualname__ = name
    fn.__doc__ = doc
    fn._kmp_coder = (coder, direction)
    return fn


encode_values_raw = _coder(_lib.ENCODE, _lib.CODER_RAW, 'encode_values_raw',
                           'utils.py:28-30 -- int32(gt) - int32(pred) (int32 wrap-around).')
decode_values_raw = _coder(_lib.DECODE, _lib.CODER_RAW, 'decode_values_raw',
                           'utils.py:33-35 -- int32(pred) + int32(encoded).')
encode_values_uint8 = _coder(_lib.ENCODE, _lib.CODER_U8, 'encode_values_uint8',
                             'utils.py:38-40 -- uint8(((int32(gt) - int32(pred)) + 256) % 256).')
decode_values_uint8 = _coder(_lib.DECODE, _lib.CODER_U8, 'decode_values_uint8',
                             'utils.py:43-45 -- uint8(((int32(pred) + int32(encoded)) + 256) % 256).')
encode_values_uint16 = _coder(_lib.ENCODE, _lib.CODER_U16, 'encode_values_uint16',
                              'utils.py:48-50 -- uint16(((int32(gt) - int32(pred)) + 65536) % 65536).')
decode_values_uint16 = _coder(_lib.DECODE, _lib.CODER_U16, 'decode_values_uint16',
                              'utils.py:53-55 -- uint16(((int32(pred) + int32(encoded)) + 65536) % 65536).')
# Build extension (no reference counterpart): lossless mod-2^32 coder for float32 volumes
# bit-cast to uint32.
encode_values_uint32 = _coder(_lib.ENCODE, _lib.CODER_U32, 'encode_values_uint32',
                              'uint32(gt - pred) modulo 2^32 (build extension for bit-cast float32).')
decode_values_uint32 = _coder(_lib.DECODE, _lib.CODER_U32, 'decode_values_uint32',
                              'uint32(pred + encoded) modulo 2^32 (build extension for bit-cast float32).')


def encode_categorical(pred, gt):
    """utils.py:58-83 -- rank of ``gt`` in the descending (reversed stable) order of the logits."""
    kind = 'torch' if dev.is_torch(gt) else 'numpy'
    return dev.from_device(d_categorical(_lib.ENCODE, pred, gt), kind)


def decode_categorical(pred, encoded):
    """utils.py:86-111 -- the class at rank ``encoded`` of the descending order of the logits."""
    kind = 'torch' if dev.is_torch(encoded) else 'numpy'
    return dev.from_device(d_categorical(_lib.DECODE, pred, encoded), kind)
