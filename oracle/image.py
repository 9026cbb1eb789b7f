"""Oracle (test infrastructure only): the 2D image path, op for op.

Restates ``src/kompressor/image/utils.py``, ``image/encode_decode.py`` and
``image/encode_decode_chunk.py`` of the reference in numpy (file:line cited per function).
Arrays are channels-last ``[B, H, W, C...]``.  See ``oracle/__init__.py`` for the parity status.
"""

from itertools import product

import numpy as np

from .common import (cast_from_f32, validate_padding, yield_chunks,  # noqa: F401
                     encode_values_raw, decode_values_raw, encode_values_uint8, decode_values_uint8,
                     encode_values_uint16, decode_values_uint16, encode_categorical, decode_categorical,
                     encode_values_uint32, decode_values_uint32)

MAP_NAMES = ('lr', 'ud', 'c')
# Parity along (y, x): image/utils.py:92-94
MAP_PARITY = ((1, 0), (0, 1), (1, 1))


def _par(p):
    return slice(1, None, 2) if p else slice(None, None, 2)


def targets_from_highres(highres):
    """image/utils.py:37-49 -- the 5 per-cell targets in L,R,U,D,C order."""
    h = np.asarray(highres)
    o, lo, hi = slice(1, None, 2), slice(None, -1, 2), slice(2, None, 2)
    return np.stack([h[:, o, lo], h[:, o, hi], h[:, lo, o], h[:, hi, o], h[:, o, o]], axis=3)


def lowres_from_highres(highres):
    """image/utils.py:52-55."""
    return np.asarray(highres)[:, ::2, ::2]


def maps_from_predictions(predictions):
    """image/utils.py:58-86 -- float32 scatter-add of the 5 per-cell predictions, normalise, cast."""
    predictions = np.asarray(predictions)
    dtype = predictions.dtype
    B, ph, pw = predictions.shape[:3]
    ch = predictions.shape[4:]
    f = predictions.astype(np.float32)
    half = np.float32(0.5)
    S = slice(None)

    lr = np.zeros((B, ph, pw + 1, *ch), np.float32)
    lr[S, S, slice(None, -1)] += f[:, :, :, 0]
    lr[S, S, slice(1, None)] += f[:, :, :, 1]
    lr[S, S, slice(1, -1)] *= half

    ud = np.zeros((B, ph + 1, pw, *ch), np.float32)
    ud[S, slice(None, -1)] += f[:, :, :, 2]
    ud[S, slice(1, None)] += f[:, :, :, 3]
    ud[S, slice(1, -1)] *= half

    return cast_from_f32(lr, dtype), cast_from_f32(ud, dtype), predictions[:, :, :, 4]


def maps_from_highres(highres):
    """image/utils.py:89-96."""
    h = np.asarray(highres)
    return tuple(h[:, _par(py), _par(px)] for py, px in MAP_PARITY)


def highres_from_lowres_and_maps(lowres, maps):
    """image/utils.py:99-116."""
    lowres = np.asarray(lowres)
    B, lh, lw = lowres.shape[:3]
    out = np.zeros((B, 2 * lh - 1, 2 * lw - 1, *lowres.shape[3:]), lowres.dtype)
    out[:, ::2, ::2] = lowres
    for (py, px), m in zip(MAP_PARITY, maps):
        out[:, _par(py), _par(px)] = m
    return out


def features_from_lowres(lowres, padding):
    """image/utils.py:120-129 -- stack of the (2p+2)^2 shifted windows (y-major, then x)."""
    lowres = np.asarray(lowres)
    k = 2 * padding + 2
    ph, pw = (s - 2 * padding - 1 for s in lowres.shape[1:3])
    return np.stack([lowres[:, y:y + ph, x:x + pw] for y in range(k) for x in range(k)], axis=3)


def _pad(x, spatial, mode):
    x = np.asarray(x)
    return np.pad(x, ((0, 0), *spatial, *(((0, 0),) * (x.ndim - 3))), mode=mode)


def pad_neighborhood(lowres, padding):
    """image/utils.py:132-137."""
    return _pad(lowres, ((padding, padding),) * 2, 'symmetric')


def pad_highres(highres):
    """image/utils.py:145-156."""
    d = tuple((s + 1) % 2 for s in np.asarray(highres).shape[1:3])
    return _pad(highres, tuple((0, p) for p in d), 'reflect'), d


def pad_lowres(lowres, padding):
    """image/utils.py:159-163."""
    return _pad(lowres, tuple((0, p) for p in padding), 'symmetric')


def pad_map(inputs, padding):
    """image/utils.py:166-170."""
    return _pad(inputs, tuple((0, p) for p in padding), 'symmetric')


def _per_map_dims(dims):
    return [tuple(dim if par == 0 else 0 for dim, par in zip(dims, parity)) for parity in MAP_PARITY]


def pad_maps(maps, padding):
    """image/utils.py:173-178."""
    return tuple(m if pm == (0, 0) else pad_map(m, pm) for m, pm in zip(maps, _per_map_dims(padding)))


def trim(inputs, padding):
    """image/utils.py:181-185."""
    h, w = inputs.shape[1:3]
    ph, pw = padding
    return inputs[:, :h - ph, :w - pw]


def trim_maps(maps, padding):
    """image/utils.py:188-193."""
    return tuple(trim(m, pm) for m, pm in zip(maps, _per_map_dims(padding)))


def validate_highres(highres):
    """image/utils.py:201-208."""
    assert highres.ndim >= 4
    assert np.prod(highres.shape) > 0
    hh, hw = highres.shape[1:3]
    for s in (hh, hw):
        assert s > 2 and s % 2 != 0
    return hh, hw


def validate_lowres(lowres):
    """image/utils.py:211-218."""
    assert lowres.ndim >= 4
    assert np.prod(lowres.shape) > 0
    lh, lw = lowres.shape[1:3]
    assert lh >= 2 and lw >= 2
    return lh, lw


def validate_chunk(chunk):
    """image/utils.py:221-232."""
    if isinstance(chunk, int):
        assert chunk > 3
        return (chunk,) * 2
    if isinstance(chunk, tuple):
        ch, cw = chunk
        assert ch > 3 and cw > 3
        return ch, cw
    raise AssertionError('chunk must be int or tuple(int, int)')


def encode(predictions_fn, encode_fn, highres, padding=0):
    """image/encode_decode.py:30-56."""
    validate_padding(padding)
    highres, dims = pad_highres(highres)
    validate_highres(highres)
    lowres = lowres_from_highres(highres)
    validate_lowres(lowres)
    gt_maps = maps_from_highres(highres)
    pred_maps = predictions_fn(pad_neighborhood(lowres, padding))
    encoded = trim_maps([encode_fn(p, g) for p, g in zip(pred_maps, gt_maps)], dims)
    return trim(lowres, dims), (encoded, dims)


def decode(predictions_fn, decode_fn, lowres, encoded, padding=0):
    """image/encode_decode.py:59-85."""
    encoded_maps, dims = encoded
    validate_padding(padding)
    validate_lowres(lowres)
    lowres = pad_lowres(lowres, dims)
    encoded_maps = pad_maps(encoded_maps, dims)
    pred_maps = predictions_fn(pad_neighborhood(lowres, padding))
    decoded = [decode_fn(p, e) for p, e in zip(pred_maps, encoded_maps)]
    return trim(highres_from_lowres_and_maps(lowres, decoded), dims)


def process_chunks(predictions_fn, code_fn, lowres, reference_maps, chunk, padding, progress_fn):
    """image/encode_decode_chunk.py:77-115."""
    validate_padding(padding)
    ch, cw = validate_chunk(chunk)
    lh, lw = validate_lowres(lowres)
    padded = pad_neighborhood(lowres, padding)
    coded = [np.zeros_like(r) for r in reference_maps]
    chunks = product(yield_chunks(lh, ch), yield_chunks(lw, cw))
    if progress_fn is not None:
        chunks = progress_fn(list(chunks))
    p2 = 2 * padding
    for ((y0, y1), (py0, py1)), ((x0, x1), (px0, px1)) in chunks:
        window = padded[:, y0 - py0:y1 + py1 + p2, x0 - px0:x1 + px1 + p2]
        preds = predictions_fn(window)
        for i, (pm, ref) in enumerate(zip(preds, reference_maps)):
            nh, nw = pm.shape[1] - (py0 + py1), pm.shape[2] - (px0 + px1)
            region = (slice(None), slice(y0, y0 + nh), slice(x0, x0 + nw))
            value = code_fn(pm[:, py0:py0 + nh, px0:px0 + nw], ref[region])
            coded[i][region] = np.asarray(value).astype(coded[i].dtype, casting='unsafe')
    return coded


def encode_chunks(predictions_fn, encode_fn, highres, chunk=32, padding=0, progress_fn=None):
    """image/encode_decode_chunk.py:33-53."""
    highres, dims = pad_highres(highres)
    validate_highres(highres)
    lowres = lowres_from_highres(highres)
    gt_maps = maps_from_highres(highres)
    coded = process_chunks(predictions_fn, encode_fn, lowres, gt_maps, chunk, padding, progress_fn)
    return trim(lowres, dims), (trim_maps(coded, dims), dims)


def decode_chunks(predictions_fn, decode_fn, lowres, encoded, chunk=32, padding=0, progress_fn=None):
    """image/encode_decode_chunk.py:56-74."""
    encoded_maps, dims = encoded
    lowres = pad_lowres(lowres, dims)
    encoded_maps = pad_maps(encoded_maps, dims)
    decoded = process_chunks(predictions_fn, decode_fn, lowres, encoded_maps, chunk, padding, progress_fn)
    return trim(highres_from_lowres_and_maps(lowres, decoded), dims)


# Losses -- src/kompressor/losses.py:29-41, image/losses.py:30-34 (off the hot path)
from .volume import mean_squared_error, mean_abs_error, mean_charbonnier_error  # noqa: E402,F401


def mean_total_variation(inputs):
    """image/losses.py:30-34."""
    x = np.asarray(inputs)
    terms = [np.mean(np.diff(x, axis=a).astype(np.float32), dtype=np.float32) for a in (1, 2)]
    return np.float32((terms[0] + terms[1]) / np.float32(2.0))
