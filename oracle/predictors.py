"""Oracle (test infrastructure only): the reference tests' predictor doubles, restated in numpy.

* ``mean_predictions_fn`` -- tests/volume/test_encode_decode.py:43-55 and
  tests/image/test_encode_decode.py:43-55: mean of the (2p+2)^d neighbourhood in float32,
  cast to the input dtype, repeated 19x (5x), then ``maps_from_predictions``.
* ``categorical_predictions_fn`` -- tests/volume/test_encode_decode.py:57-75 and
  tests/image/test_encode_decode.py:57-74: one constant logit vector tiled everywhere, then
  ``maps_from_predictions`` and a softmax.  The reference draws the logits with
  ``jax.random.PRNGKey(1234)``; JAX is absent, so a seeded numpy uniform draw stands in (the
  reference test checks losslessness and chunk invariance only, which hold for any logits).
* ``linear_predictions_fn`` -- the build-defined LinearPredictor (no reference counterpart;
  SURVEY.md §8a row a9'): ``pred[cell, k] = sum_n feat[cell, n] * W[n, k] + b[k]`` in float,
  cast to the input dtype, then ``maps_from_predictions``.
"""

import numpy as np

from . import volume as _vol, image as _img
from .common import cast_from_f32


def _ns(ndim):
    return _vol if ndim == 3 else _img


def mean_predictions_fn(padding, ndim=3):
    ns = _ns(ndim)
    k = 19 if ndim == 3 else 5

    def predictions_fn(lowres):
        lowres = np.asarray(lowres)
        features = ns.features_from_lowres(lowres, padding)
        axis = ndim + 1
        if features.dtype.itemsize < 4:
            pred = np.mean(features.astype(np.float32), axis=axis, keepdims=True, dtype=np.float32)
        else:
            # 32-bit samples: the f32 sum is inexact, so its order matters.  XLA's reduce order is
            # not pinned by the reference (its tests only use values < 2^24, where every order is
            # exact); the build fixes the feature order (z-major, y, x), one rounding per add.
            pred = np.zeros(features.shape[:axis] + (1,) + features.shape[axis + 1:], np.float32)
            for n in range(features.shape[axis]):
                pred += np.take(features, [n], axis=axis).astype(np.float32)
            pred = pred / np.float32(features.shape[axis])
        pred = cast_from_f32(pred, lowres.dtype)
        pred = np.repeat(pred, k, axis=axis)
        return ns.maps_from_predictions(pred)

    return predictions_fn


def categorical_logits(ndim, channels, classes, seed=1234):
    k = 19 if ndim == 3 else 5
    rng = np.random.default_rng(seed)
    return rng.uniform(size=(k, *channels, classes)).astype(np.float32)


def categorical_predictions_fn(padding, classes, ndim=3, seed=1234):
    ns = _ns(ndim)

    def predictions_fn(lowres):
        lowres = np.asarray(lowres)
        ch = lowres.shape[ndim + 1:]
        logits = categorical_logits(ndim, ch, classes, seed)
        cells = tuple(s - 1 - 2 * padding for s in lowres.shape[1:ndim + 1])
        pred = np.broadcast_to(logits, (lowres.shape[0], *cells, *logits.shape)).copy()
        maps = ns.maps_from_predictions(pred)
        out = []
        for m in maps:
            e = np.exp(m - m.max(axis=-1, keepdims=True))
            out.append((e / e.sum(axis=-1, keepdims=True)).astype(np.float32))
        return out

    return predictions_fn


def linear_predictions(features, weights, bias, dtype):
    """Per-cell linear predictor on ``features [.., N, C]`` -> ``[.., K, C]`` (float64 math, then the
    XLA-style cast).  Used as the 1e-5 tolerance reference for the HIP MFMA predictor."""
    f = features.astype(np.float64)
    w = np.asarray(weights, np.float64)
    b = np.asarray(bias, np.float64)
    n_axis = f.ndim - 2
    pred = np.moveaxis(np.tensordot(np.moveaxis(f, n_axis, -1), w, axes=([-1], [0])), -1, n_axis)
    pred = pred + b.reshape((-1, 1))
    return pred, cast_from_f32(pred.astype(np.float32), dtype)


def fma_f32(a, b, c):
    """Correctly rounded float32 fused multiply-add, vectorised: the exact a*b + c rounded once.

    a*b of two float32 is exact in float64; TwoSum gives s + e == a*b + c exactly; rounding s to
    float32 equals rounding the exact value unless s sits exactly on a float32 midpoint (the
    only double-rounding case, since float64 rounding is monotone and midpoints are float64
    representable), where the sign of e decides."""
    a = np.asarray(a, np.float32).astype(np.float64)
    b = np.asarray(b, np.float32).astype(np.float64)
    c = np.asarray(c, np.float32).astype(np.float64)
    p = a * b                          # exact
    s = p + c                          # TwoSum: s + e == p + c exactly
    bb = s - p
    e = (p - (s - bb)) + (c - bb)
    r = s.astype(np.float32)           # round half to even
    r64 = r.astype(np.float64)
    with np.errstate(invalid='ignore'):
        nb = np.nextafter(r, np.where(s > r64, np.float32(np.inf), np.float32(-np.inf)).astype(np.float32))
        gap = np.abs(nb.astype(np.float64) - r64)
        tie = (s != r64) & (2 * np.abs(s - r64) == gap)
        # on a tie r is the even neighbour; the exact value lies beyond the midpoint iff e points
        # the same way as s - r
        away = tie & (e != 0) & (np.sign(e) == np.sign(s - r64))
    return np.where(away, nb, r).astype(np.float32)


def linear_fma_chain(features, weights, bias):
    """The build's LinearPredictor arithmetic, bit for bit: acc = b[k]; acc = fma(f[n], W[n, k], acc)
    for n = 0..N-1 (what the f32 MFMA computes, kmp_linear.hip).  ``features [.., N, C]`` ->
    float32 ``[.., K, C]``."""
    f = np.asarray(features).astype(np.float32)
    w = np.asarray(weights, np.float32)
    b = np.asarray(bias, np.float32)
    n_axis = f.ndim - 2
    f = np.moveaxis(f, n_axis, -1)  # [.., C, N]
    acc = np.broadcast_to(b, f.shape[:-1] + b.shape).astype(np.float32).copy()  # [.., C, K]
    for n in range(w.shape[0]):
        acc = fma_f32(f[..., n:n + 1], w[n], acc)
    return np.moveaxis(acc, -1, n_axis)  # [.., K, C]


def linear_predictions_fn(padding, weights, bias, ndim=3):
    """LinearPredictor as a predictions_fn: the exact fma chain, cast to the dtype, aggregated."""
    ns = _ns(ndim)

    def predictions_fn(lowres):
        lowres = np.asarray(lowres)
        features = ns.features_from_lowres(lowres, padding)
        pred = cast_from_f32(linear_fma_chain(features, weights, bias), lowres.dtype)
        return ns.maps_from_predictions(pred)

    return predictions_fn


def bf16_rne(x):
    """float32 -> bfloat16 (round to nearest even), returned as float32 values (the bf16 set)."""
    u = np.asarray(x, np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7fff + ((u >> 16) & 1)) & 0xffff0000
    return u.astype(np.uint32).view(np.float32)


def bf16x2_weights(weights):
    """The two bf16 terms of the build's matrix-core LinearPredictor arithmetic (kmp_bf16x2.h):
    w1 = bf16(w), w2 = bf16(w - w1), so |w - w1 - w2| <= 2^-18 |w|."""
    w = np.asarray(weights, np.float32)
    w1 = bf16_rne(w)
    w2 = bf16_rne((w - w1).astype(np.float32))
    return w1, w2


def linear_bf16x2_split(features, weights, bias):
    """float64 value of what the bf16x2 MFMAs multiply: sum_n f_n (w1 + w2)[n, k] + b[k], each
    product exact (features are u8 / u16, split into two exact bytes, and 256 * w_i is exact) -- the
    kernel's float32 result differs from this only by the rounding of its f32 accumulation."""
    w1, w2 = bf16x2_weights(weights)
    return linear_predictions(features, w1.astype(np.float64) + w2.astype(np.float64), bias, np.float32)[0]
