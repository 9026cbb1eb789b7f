"""Training losses -- ``src/kompressor/losses.py:29-41`` (off the encode/decode hot path).

Kept import-compatible with the reference; computed with plain torch
reductions on whatever device the inputs live on (numpy inputs run on the CPU).  They return
0-d float32 values.
"""

import numpy as np
import torch


def _f32(x):
    if isinstance(x, torch.Tensor):
        return x.to(torch.float32) if x.dtype != torch.uint16 else x.to(torch.int32).to(torch.float32)
    return torch.from_numpy(np.asarray(x).astype(np.float32))


def _out(value, like):
    return value if isinstance(like, torch.Tensor) else np.float32(value.item())


def mean_squared_error(pred, gt):
    """losses.py:29-31."""
    return _out(torch.mean(torch.square(_f32(gt) - _f32(pred))), gt)


def mean_abs_error(pred, gt):
    """losses.py:34-36."""
    return _out(torch.mean(torch.abs(_f32(gt) - _f32(pred))), gt)


def mean_charbonnier_error(pred, gt, eps):
    """losses.py:39-41."""
    d = _f32(gt) - _f32(pred)
    return _out(torch.mean(torch.sqrt(torch.square(d) + np.float32(eps) ** 2)), gt)


_WRAP_BITS = {torch.uint8: 8, torch.uint16: 16, torch.int8: 8, torch.int16: 16, torch.int32: 32}
_SIGNED = {torch.int8, torch.int16, torch.int32}


def _as_tensor(x):
    return x if isinstance(x, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(x)))


def _diff_mean(t, axis):
    """Mean of the signed forward difference along ``axis`` computed in the input dtype, as
    ``input[1:] - input[:-1]`` does under jnp (integer types wrap modulo 2^bits), then averaged in
    float32 -- on the device ``t`` lives on (no host round trip)."""
    n = t.shape[axis]
    hi, lo = t.narrow(axis, 1, n - 1), t.narrow(axis, 0, n - 1)
    bits = _WRAP_BITS.get(t.dtype)
    if bits is None:  # floating point: the difference in the input dtype
        d = (hi - lo).to(torch.float32)
    else:             # integers: exact difference in int64, wrapped to the dtype's range
        d = hi.to(torch.int32).to(torch.int64) - lo.to(torch.int32).to(torch.int64) if t.dtype == torch.uint16 \
            else hi.to(torch.int64) - lo.to(torch.int64)
        d = torch.remainder(d, 1 << bits)
        if t.dtype in _SIGNED:
            d = torch.where(d >= (1 << (bits - 1)), d - (1 << bits), d)
        d = d.to(torch.float32)
    return torch.mean(d)


def total_variation(inputs, axes):
    """Mean over ``axes`` of the mean signed forward difference (volume/losses.py:30-35,
    image/losses.py:30-34): ``(mean(dz) + mean(dy) + mean(dx)) / 3`` in 3D, ``/ 2`` in 2D."""
    t = _as_tensor(inputs)
    terms = [_diff_mean(t, a) for a in axes]
    value = (sum(terms[1:], terms[0]) / np.float32(len(axes))).to(torch.float32)
    return _out(value, inputs)
