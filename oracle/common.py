"""Oracle (test infrastructure only): residual coders, chunk enumerator, padding validator.

Restates ``src/kompressor/utils.py`` of the reference (file:line cited per function) in numpy.
See ``oracle/__init__.py`` for the parity status of this restatement.
"""

import numpy as np


# ---------------------------------------------------------------------------------------------
# Residual coders -- utils.py:28-55.  x64 is off in the reference, so all arithmetic is int32.
# ---------------------------------------------------------------------------------------------

def as_int32(x):
    """``jnp.int32(x)``: integers wrap into int32, floats truncate toward zero (saturating)."""
    x = np.asarray(x)
    if np.issubdtype(x.dtype, np.floating):
        return cast_from_f32(x.astype(np.float32), np.int32)
    return x.astype(np.int32)


def encode_values_raw(pred, gt):
    """utils.py:28-30 -- ``int32(gt) - int32(pred)`` (int32 wrap-around)."""
    return as_int32(gt) - as_int32(pred)


def decode_values_raw(pred, encoded):
    """utils.py:33-35 -- ``int32(pred) + int32(encoded)``."""
    return as_int32(pred) + as_int32(encoded)


def _modular(a, m, dtype):
    # ((a) + m) % m with int32 arithmetic, then the narrowing cast (values are already in range).
    return ((a + np.int32(m)) % np.int32(m)).astype(dtype)


def encode_values_uint8(pred, gt):
    """utils.py:38-40 -- ``uint8(((int32(gt) - int32(pred)) + 256) % 256)``."""
    return _modular(as_int32(gt) - as_int32(pred), 256, np.uint8)


def decode_values_uint8(pred, encoded):
    """utils.py:43-45 -- ``uint8(((int32(pred) + int32(encoded)) + 256) % 256)``."""
    return _modular(as_int32(pred) + as_int32(encoded), 256, np.uint8)


def encode_values_uint16(pred, gt):
    """utils.py:48-50 -- ``uint16(((int32(gt) - int32(pred)) + 65536) % 65536)``."""
    return _modular(as_int32(gt) - as_int32(pred), 65536, np.uint16)


def decode_values_uint16(pred, encoded):
    """utils.py:53-55 -- ``uint16(((int32(pred) + int32(encoded)) + 65536) % 65536)``."""
    return _modular(as_int32(pred) + as_int32(encoded), 65536, np.uint16)


def encode_values_uint32(pred, gt):
    """Build extension (no reference counterpart): the mod-2^16 coder of
    utils.py:48-50 widened to 2^32 for bit-cast float32 samples, ``uint32(gt - pred) mod 2^32``."""
    return ((np.asarray(gt).astype(np.int64) - np.asarray(pred).astype(np.int64)) % (1 << 32)).astype(np.uint32)


def decode_values_uint32(pred, encoded):
    """Inverse of :func:`encode_values_uint32` (the utils.py:53-55 analogue)."""
    return ((np.asarray(pred).astype(np.int64) + np.asarray(encoded).astype(np.int64)) % (1 << 32)).astype(np.uint32)


# ---------------------------------------------------------------------------------------------
# Categorical rank coder -- utils.py:58-111
# ---------------------------------------------------------------------------------------------

def _descending_ranks(pred, dtype):
    # utils.py:66 / :94 -- stable ascending argsort, cast to the value dtype (integer narrowing
    # wraps), then reversed along the class axis.
    order = np.argsort(np.asarray(pred), axis=-1, kind='stable')
    return order.astype(dtype)[..., ::-1]


def encode_categorical(pred, gt):
    """utils.py:58-83 -- index of the first rank equal to ``gt`` (``argmax`` of the match; 0 if none)."""
    gt = np.asarray(gt)
    ranks = _descending_ranks(pred, gt.dtype)
    return np.argmax(ranks == gt[..., None], axis=-1).astype(gt.dtype)


def decode_categorical(pred, encoded):
    """utils.py:86-111 -- ``ranks[encoded]`` per element (out-of-range indices clamp, as XLA gathers do)."""
    encoded = np.asarray(encoded)
    ranks = _descending_ranks(pred, encoded.dtype)
    idx = np.clip(encoded.astype(np.int64), 0, ranks.shape[-1] - 1)
    return np.take_along_axis(ranks, idx[..., None], axis=-1)[..., 0]


# ---------------------------------------------------------------------------------------------
# Chunk enumerator and padding validator -- utils.py:114-161
# ---------------------------------------------------------------------------------------------

def yield_chunks(max_value, chunk):
    """utils.py:114-155 -- constant-size windows over ``max_value`` lowres nodes.

    Windows start every ``chunk - 3`` nodes and cover ``chunk - 2`` nodes; the last one is
    pulled back to end at the edge.  Each yields ``(i0, i1), (p0, p1)`` with a one-sided halo
    ``p0 + p1 == 2`` so every window (nodes plus halo) has exactly ``chunk`` entries.
    """
    assert max_value > 0
    assert chunk > 3
    if chunk >= max_value:
        yield (0, max_value), (0, 0)
        return
    step, span = chunk - 3, chunk - 2
    start = 0
    while start < max_value:
        i1 = min(max_value, start + span)
        last = i1 == max_value
        i0 = max(0, i1 - span) if last else start
        first = i0 == 0
        assert not (first and last)
        p0 = 0 if first else (2 if last else 1)
        p1 = 0 if last else (2 if first else 1)
        assert p0 + p1 == 2
        yield (i0, i1), (p0, p1)
        if last:
            return
        start += step


def validate_padding(padding):
    """utils.py:158-161."""
    assert isinstance(padding, int)
    assert padding >= 0


# ---------------------------------------------------------------------------------------------
# XLA-style float32 -> dtype conversion
# ---------------------------------------------------------------------------------------------

def cast_from_f32(x, dtype):
    """``astype(dtype)`` of float32 values as XLA does it: identity for floats; for integers
    truncation toward zero, saturating at the dtype's range, NaN -> 0.  In-range values (the only
    ones the reference's tests produce) are plain truncation."""
    dtype = np.dtype(dtype)
    x = np.asarray(x, dtype=np.float32)
    if np.issubdtype(dtype, np.floating):
        return x.astype(dtype)
    info = np.iinfo(dtype)
    t = np.trunc(x.astype(np.float64))
    t = np.nan_to_num(t, nan=0.0, posinf=info.max, neginf=info.min)
    return np.clip(t, info.min, info.max).astype(dtype)


def sym_index(i, n):
    """numpy/jnp ``mode='symmetric'`` source index for a (possibly far) out-of-range index."""
    m = i % (2 * n)
    return m if m < n else 2 * n - 1 - m
