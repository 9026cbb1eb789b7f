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


def _diff_mean(x, axis):
    """Mean of the signed forward difference along ``axis`` in the input dtype (unsigned wraps)."""
    if isinstance(x, torch.Tensor):
        a = x.detach().cpu().numpy()
    else:
        a = np.asarray(x)
    return np.float32(np.mean(np.diff(a, axis=axis).astype(np.float32), dtype=np.float32))


def total_variation(inputs, axes):
    terms = [_diff_mean(inputs, a) for a in axes]
    value = np.float32(sum(terms, np.float32(0)) / np.float32(len(axes)))
    if isinstance(inputs, torch.Tensor):
        return torch.tensor(value, dtype=torch.float32)
    return value
