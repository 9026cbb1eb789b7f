"""Oracle (test infrastructure only): the reference path on multithreaded torch-CPU ops.

The multithreaded comparator SURVEY.md §8d / BASELINE.md §2 ask for beside the 1-thread numpy
restatement: the same op sequence as ``oracle.volume`` / ``oracle.image`` (itself an op-for-op
restatement of ``src/kompressor/{volume,image}/encode_decode.py:30-85`` with the reference
tests' mean predictor, ``tests/volume/test_encode_decode.py:43-55``), keeping the reference's
materialised intermediates -- reflect-padded highres, strided lowres / ground-truth maps, the
``(2p+2)^d``-feature stack, the f32 mean, the 19- (5-) way repeat, the f32 scatter-add
aggregation -- but every op a torch CPU kernel that runs on ``torch.get_num_threads()`` threads
(the way XLA's CPU backend would spread the reference's ops over the host cores).

Samples are carried as int32 (int64 for uint32; torch's CPU arithmetic on uint16 / uint32 is incomplete); casts
apply the reference's truncation into the sample dtype's range, so every value is the
reference's.  uint32 (the build's bit-cast float32 extension, config C5) sums the features in
the build's fixed order like ``oracle.predictors.mean_predictions_fn``.  Used
only by ``bench.py``'s ``cpu_baseline`` leg and checked bit-exact against ``oracle.volume`` /
``oracle.image`` by ``tests/test_oracle_torch_cpu.py``.
"""

import numpy as np
import torch

_PARITY = {3: ((1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1), (1, 0, 0), (0, 1, 0), (0, 0, 1)),  # volume/utils.py:161-169
           2: ((1, 0), (0, 1), (1, 1))}                                                       # image/utils.py:92-94
_RANGE = {np.dtype(np.uint8): (0, 255), np.dtype(np.uint16): (0, 65535), np.dtype(np.uint32): (0, (1 << 32) - 1)}


def _sym(i, n):
    """numpy mode='symmetric' source index (period 2n)."""
    m = np.mod(i, 2 * n)
    return np.where(m < n, m, 2 * n - 1 - m)


def _refl(i, n):
    """numpy mode='reflect' source index (period 2n - 2)."""
    m = np.mod(i, 2 * n - 2)
    return np.where(m < n, m, 2 * n - 2 - m)


def _pad(x, nsp, lo, hi, mode):
    """jnp.pad of the spatial axes (volume/utils.py:213-244): one index_select per axis."""
    for a in range(nsp):
        n = x.shape[1 + a]
        if lo[a] == 0 and hi[a] == 0:
            continue
        idx = np.arange(-lo[a], n + hi[a])
        idx = _sym(idx, n) if mode == 'symmetric' else _refl(idx, n)
        x = x.index_select(1 + a, torch.from_numpy(idx.astype(np.int64)))
    return x


def _carrier(hi):
    return np.int32 if hi < (1 << 24) else np.int64


def _sl(p):
    return slice(1, None, 2) if p else slice(None, None, 2)


def _cast(f, lo, hi):
    """astype(dtype) of an f32 array (XLA: truncate toward zero, saturate, NaN -> 0), carried
    as int64 (f32 -> f64 is exact, so the clamp at 2^32 - 1 saturates exactly)."""
    if hi < (1 << 24):  # 8 / 16-bit: every f32 in range is exact, int32 carries it
        return torch.clamp(torch.trunc(torch.nan_to_num(f, nan=0.0)), lo, hi).to(torch.int32)
    d = torch.nan_to_num(f.to(torch.float64), nan=0.0)
    return torch.clamp(torch.trunc(d), lo, hi).to(torch.int64)


def _features(lowres, padding, nsp):
    """volume/utils.py:199-210 / image/utils.py:120-129: stack of the shifted windows."""
    k = 2 * padding + 2
    cells = [s - 2 * padding - 1 for s in lowres.shape[1:1 + nsp]]
    wins = []
    for off in np.ndindex(*(k,) * nsp):
        wins.append(lowres[(slice(None),) + tuple(slice(o, o + c) for o, c in zip(off, cells))])
    return torch.stack(wins, dim=1 + nsp)


def _maps_from_predictions(f, nsp, lo, hi):
    """volume/utils.py:83-155 / image/utils.py:58-86: f32 scatter-add in the reference's order,
    its x0.5 / x0.25 normalisation, then the truncating cast."""
    S = slice(None)
    if nsp == 2:
        B, ph, pw = f.shape[:3]
        ch = f.shape[4:]
        lr = torch.zeros((B, ph, pw + 1, *ch))
        lr[S, S, :-1] += f[:, :, :, 0]
        lr[S, S, 1:] += f[:, :, :, 1]
        lr[S, S, 1:-1] *= 0.5
        ud = torch.zeros((B, ph + 1, pw, *ch))
        ud[S, :-1] += f[:, :, :, 2]
        ud[S, 1:] += f[:, :, :, 3]
        ud[S, 1:-1] *= 0.5
        return _cast(lr, lo, hi), _cast(ud, lo, hi), _cast(f[:, :, :, 4], lo, hi)
    B, pd, ph, pw = f.shape[:4]
    ch = f.shape[5:]

    def two_way(shape, ax, a, b):
        m = torch.zeros(shape)
        i0 = (S,) * ax + (slice(None, -1),)
        i1 = (S,) * ax + (slice(1, None),)
        mid = (S,) * ax + (slice(1, -1),)
        m[i0] += f[:, :, :, :, a]
        m[i1] += f[:, :, :, :, b]
        m[mid] *= 0.5
        return _cast(m, lo, hi)

    lr = two_way((B, pd, ph, pw + 1, *ch), 3, 0, 1)
    ud = two_way((B, pd, ph + 1, pw, *ch), 2, 2, 3)
    fb = two_way((B, pd + 1, ph, pw, *ch), 1, 4, 5)
    c = _cast(f[:, :, :, :, 6], lo, hi)
    a_, b_, mid = slice(None, -1), slice(1, None), slice(1, -1)
    z = torch.zeros((B, pd, ph + 1, pw + 1, *ch))
    z[S, S, a_, a_] += f[:, :, :, :, 7]
    z[S, S, a_, b_] += f[:, :, :, :, 8]
    z[S, S, b_, b_] += f[:, :, :, :, 9]
    z[S, S, b_, a_] += f[:, :, :, :, 10]
    z[S, S, mid, mid] *= 0.25
    z[S, S, mid, ::pw] *= 0.5
    z[S, S, ::ph, mid] *= 0.5
    y = torch.zeros((B, pd + 1, ph, pw + 1, *ch))
    y[S, a_, S, a_] += f[:, :, :, :, 11]
    y[S, a_, S, b_] += f[:, :, :, :, 12]
    y[S, b_, S, b_] += f[:, :, :, :, 13]
    y[S, b_, S, a_] += f[:, :, :, :, 14]
    y[S, mid, S, mid] *= 0.25
    y[S, mid, S, ::pw] *= 0.5
    y[S, ::pd, S, mid] *= 0.5
    x = torch.zeros((B, pd + 1, ph + 1, pw, *ch))
    x[S, a_, a_, S] += f[:, :, :, :, 15]
    x[S, a_, b_, S] += f[:, :, :, :, 16]
    x[S, b_, b_, S] += f[:, :, :, :, 17]
    x[S, b_, a_, S] += f[:, :, :, :, 18]
    x[S, mid, mid, S] *= 0.25
    x[S, mid, ::ph, S] *= 0.5
    x[S, ::pd, mid, S] *= 0.5
    return lr, ud, fb, c, _cast(z, lo, hi), _cast(y, lo, hi), _cast(x, lo, hi)


def _mean_predictions(padded_lowres, padding, nsp, lo, hi):
    """tests/volume/test_encode_decode.py:46-53: f32 mean of the features, cast, repeat, aggregate."""
    feats = _features(padded_lowres, padding, nsp)
    if hi < (1 << 24):  # 8 / 16-bit samples: the f32 sum is exact, any order
        mean = torch.mean(feats.to(torch.float32), dim=1 + nsp, keepdim=True)
    else:               # 32-bit samples: the build's fixed feature order, one rounding per add
        acc = torch.zeros(feats.select(1 + nsp, 0).shape, dtype=torch.float32)
        for n in range(feats.shape[1 + nsp]):
            acc += feats.select(1 + nsp, n).to(torch.float32)
        mean = (acc / np.float32(feats.shape[1 + nsp])).unsqueeze(1 + nsp)
    pred = _cast(mean, lo, hi).to(torch.float32)
    pred = pred.repeat_interleave(19 if nsp == 3 else 5, dim=1 + nsp)
    return _maps_from_predictions(pred, nsp, lo, hi)


def _trim(x, nsp, dims):
    return x[(slice(None),) + tuple(slice(0, x.shape[1 + a] - dims[a]) for a in range(nsp))]


def _map_dims(dims, nsp):
    return [tuple(d if p == 0 else 0 for d, p in zip(dims, par)) for par in _PARITY[nsp]]


def encode(highres, padding, nsp):
    """volume/encode_decode.py:30-56 (image/encode_decode.py:30-56) with the mean predictor and
    the mod-2^k coder (utils.py:38-55; mod 2^32 for uint32) for the sample dtype; numpy in ->
    numpy out."""
    dt = highres.dtype
    lo, hi = _RANGE[dt]
    x = torch.from_numpy(highres.astype(_carrier(hi)))
    dims = tuple((s + 1) % 2 for s in highres.shape[1:1 + nsp])
    x = _pad(x, nsp, (0,) * nsp, dims, 'reflect')
    lowres = x[(slice(None),) + (slice(None, None, 2),) * nsp]
    gt = [x[(slice(None),) + tuple(_sl(p) for p in par)] for par in _PARITY[nsp]]
    preds = _mean_predictions(_pad(lowres, nsp, (padding,) * nsp, (padding,) * nsp, 'symmetric'), padding, nsp, lo, hi)
    enc = [torch.bitwise_and(g - p, hi) for g, p in zip(gt, preds)]
    enc = [_trim(m, nsp, md) for m, md in zip(enc, _map_dims(dims, nsp))]
    return _trim(lowres, nsp, dims).numpy().astype(dt), ([m.numpy().astype(dt) for m in enc], dims)


def decode(lowres, encoded, padding, nsp):
    """volume/encode_decode.py:59-85 (image/encode_decode.py:59-85)."""
    maps, dims = encoded
    dt = lowres.dtype
    lo, hi = _RANGE[dt]
    lr = _pad(torch.from_numpy(lowres.astype(_carrier(hi))), nsp, (0,) * nsp, dims, 'symmetric')
    enc = [_pad(torch.from_numpy(m.astype(_carrier(hi))), nsp, (0,) * nsp, md, 'symmetric')
           for m, md in zip(maps, _map_dims(dims, nsp))]
    preds = _mean_predictions(_pad(lr, nsp, (padding,) * nsp, (padding,) * nsp, 'symmetric'), padding, nsp, lo, hi)
    dec = [torch.bitwise_and(p + e, hi) for p, e in zip(preds, enc)]
    out = torch.zeros((lr.shape[0], *[2 * s - 1 for s in lr.shape[1:1 + nsp]], *lr.shape[1 + nsp:]), dtype=lr.dtype)
    out[(slice(None),) + (slice(None, None, 2),) * nsp] = lr
    for par, m in zip(_PARITY[nsp], dec):
        out[(slice(None),) + tuple(_sl(p) for p in par)] = m
    return _trim(out, nsp, dims).numpy().astype(dt)
