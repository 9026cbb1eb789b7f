"""Oracle (test infrastructure only): the 3D volume path, op for op.

Restates ``src/kompressor/volume/utils.py``, ``volume/encode_decode.py`` and
``volume/encode_decode_chunk.py`` of the reference in numpy (file:line cited per function),
keeping the reference's materialised intermediates.  Arrays are channels-last
``[B, D, H, W, C...]``.  See ``oracle/__init__.py`` for the parity status.
"""

from itertools import product

import numpy as np

from .common import (cast_from_f32, validate_padding, yield_chunks,  # noqa: F401
                     encode_values_raw, decode_values_raw, encode_values_uint8, decode_values_uint8,
                     encode_values_uint16, decode_values_uint16, encode_categorical, decode_categorical,
                     encode_values_uint32, decode_values_uint32)

MAP_NAMES = ('lr', 'ud', 'fb', 'c', 'z', 'y', 'x')

# Parity of each map along (z, y, x): 1 = odd highres index (cell lattice), 0 = even (node lattice).
# volume/utils.py:161-169
MAP_PARITY = ((1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1), (1, 0, 0), (0, 1, 0), (0, 0, 1))


def _par(p):
    return slice(1, None, 2) if p else slice(None, None, 2)


def targets_from_highres(highres):
    """volume/utils.py:37-74 -- the 19 per-cell targets in L,R,U,D,F,B,C,z0..z3,y0..y3,x0..x3 order."""
    h = np.asarray(highres)
    o, e, lo, hi = slice(1, None, 2), slice(None, None, 2), slice(None, -1, 2), slice(2, None, 2)
    del e
    parts = [
        h[:, o, o, lo], h[:, o, o, hi],            # L, R
        h[:, o, lo, o], h[:, o, hi, o],            # U, D
        h[:, lo, o, o], h[:, hi, o, o],            # F, B
        h[:, o, o, o],                             # C
        h[:, o, lo, lo], h[:, o, lo, hi], h[:, o, hi, hi], h[:, o, hi, lo],   # z0..z3
        h[:, lo, o, lo], h[:, lo, o, hi], h[:, hi, o, hi], h[:, hi, o, lo],   # y0..y3
        h[:, lo, lo, o], h[:, lo, hi, o], h[:, hi, hi, o], h[:, hi, lo, o],   # x0..x3
    ]
    return np.stack(parts, axis=4)


def lowres_from_highres(highres):
    """volume/utils.py:77-80 -- skip sampling ``x[:, ::2, ::2, ::2]``."""
    return np.asarray(highres)[:, ::2, ::2, ::2]


def maps_from_predictions(predictions):
    """volume/utils.py:83-155 -- float32 scatter-add of 19 per-cell predictions onto the 7
    lattices, the reference's normalisation, then the truncating cast back to the input dtype.
    The additions happen in the reference's order (XLA does not reassociate float adds)."""
    predictions = np.asarray(predictions)
    dtype = predictions.dtype
    B, pd, ph, pw = predictions.shape[:4]
    ch = predictions.shape[5:]
    f = predictions.astype(np.float32)
    half, quarter = np.float32(0.5), np.float32(0.25)

    def two_way(shape, a_idx, a, b_idx, b, interior):
        m = np.zeros(shape, np.float32)
        m[a_idx] += f[:, :, :, :, a]
        m[b_idx] += f[:, :, :, :, b]
        m[interior] *= half
        return cast_from_f32(m, dtype)

    S = slice(None)
    lr = two_way((B, pd, ph, pw + 1, *ch), (S, S, S, slice(None, -1)), 0, (S, S, S, slice(1, None)), 1,
                 (S, S, S, slice(1, -1)))
    ud = two_way((B, pd, ph + 1, pw, *ch), (S, S, slice(None, -1)), 2, (S, S, slice(1, None)), 3,
                 (S, S, slice(1, -1)))
    fb = two_way((B, pd + 1, ph, pw, *ch), (S, slice(None, -1)), 4, (S, slice(1, None)), 5,
                 (S, slice(1, -1)))
    c = predictions[:, :, :, :, 6]

    lo, up, mid = slice(None, -1), slice(1, None), slice(1, -1)

    # z map: corners of the central z plane (volume/utils.py:119-129)
    z = np.zeros((B, pd, ph + 1, pw + 1, *ch), np.float32)
    z[S, S, lo, lo] += f[:, :, :, :, 7]
    z[S, S, lo, up] += f[:, :, :, :, 8]
    z[S, S, up, up] += f[:, :, :, :, 9]
    z[S, S, up, lo] += f[:, :, :, :, 10]
    z[S, S, mid, mid] *= quarter
    z[S, S, mid, slice(None, None, pw)] *= half
    z[S, S, slice(None, None, ph), mid] *= half
    z = cast_from_f32(z, dtype)

    # y map (volume/utils.py:131-141)
    y = np.zeros((B, pd + 1, ph, pw + 1, *ch), np.float32)
    y[S, lo, S, lo] += f[:, :, :, :, 11]
    y[S, lo, S, up] += f[:, :, :, :, 12]
    y[S, up, S, up] += f[:, :, :, :, 13]
    y[S, up, S, lo] += f[:, :, :, :, 14]
    y[S, mid, S, mid] *= quarter
    y[S, mid, S, slice(None, None, pw)] *= half
    y[S, slice(None, None, pd), S, mid] *= half
    y = cast_from_f32(y, dtype)

    # x map (volume/utils.py:143-153)
    x = np.zeros((B, pd + 1, ph + 1, pw, *ch), np.float32)
    x[S, lo, lo, S] += f[:, :, :, :, 15]
    x[S, lo, up, S] += f[:, :, :, :, 16]
    x[S, up, up, S] += f[:, :, :, :, 17]
    x[S, up, lo, S] += f[:, :, :, :, 18]
    x[S, mid, mid, S] *= quarter
    x[S, mid, slice(None, None, ph), S] *= half
    x[S, slice(None, None, pd), mid, S] *= half
    x = cast_from_f32(x, dtype)

    return lr, ud, fb, c, z, y, x


def maps_from_highres(highres):
    """volume/utils.py:158-171 -- the 7 ground-truth maps by parity class."""
    h = np.asarray(highres)
    return tuple(h[:, _par(pz), _par(py), _par(px)] for pz, py, px in MAP_PARITY)


def highres_from_lowres_and_maps(lowres, maps):
    """volume/utils.py:174-195 -- interleave lowres and the 7 maps into the full grid."""
    lowres = np.asarray(lowres)
    B, ld, lh, lw = lowres.shape[:4]
    out = np.zeros((B, 2 * ld - 1, 2 * lh - 1, 2 * lw - 1, *lowres.shape[4:]), lowres.dtype)
    out[:, ::2, ::2, ::2] = lowres
    for (pz, py, px), m in zip(MAP_PARITY, maps):
        out[:, _par(pz), _par(py), _par(px)] = m
    return out


def features_from_lowres(lowres, padding):
    """volume/utils.py:199-210 -- stack of the (2p+2)^3 shifted windows (z-major, then y, x)."""
    lowres = np.asarray(lowres)
    k = 2 * padding + 2
    pd, ph, pw = (s - 2 * padding - 1 for s in lowres.shape[1:4])
    return np.stack([lowres[:, z:z + pd, y:y + ph, x:x + pw]
                     for z in range(k) for y in range(k) for x in range(k)], axis=4)


def _pad(x, spatial, mode):
    x = np.asarray(x)
    return np.pad(x, ((0, 0), *spatial, *(((0, 0),) * (x.ndim - 4))), mode=mode)


def pad_neighborhood(lowres, padding):
    """volume/utils.py:213-218 -- symmetric pad of the 3 spatial axes by ``padding``."""
    return _pad(lowres, ((padding, padding),) * 3, 'symmetric')


def pad_highres(highres):
    """volume/utils.py:226-237 -- reflect-pad each even spatial dim by one at the far end."""
    d = tuple((s + 1) % 2 for s in np.asarray(highres).shape[1:4])
    return _pad(highres, tuple((0, p) for p in d), 'reflect'), d


def pad_lowres(lowres, padding):
    """volume/utils.py:240-244 -- symmetric pad at the far end by ``dims``."""
    return _pad(lowres, tuple((0, p) for p in padding), 'symmetric')


def pad_map(inputs, padding):
    """volume/utils.py:247-251."""
    return _pad(inputs, tuple((0, p) for p in padding), 'symmetric')


def _per_map_dims(dims):
    pd, ph, pw = dims
    # A map is padded/trimmed on the axes where it lies on the node lattice (volume/utils.py:258-276).
    return [tuple(dim if par == 0 else 0 for dim, par in zip((pd, ph, pw), parity)) for parity in MAP_PARITY]


def pad_maps(maps, padding):
    """volume/utils.py:254-260."""
    return tuple(m if pm == (0, 0, 0) else pad_map(m, pm) for m, pm in zip(maps, _per_map_dims(padding)))


def trim(inputs, padding):
    """volume/utils.py:263-267."""
    d, h, w = inputs.shape[1:4]
    pd, ph, pw = padding
    return inputs[:, :d - pd, :h - ph, :w - pw]


def trim_maps(maps, padding):
    """volume/utils.py:270-276."""
    return tuple(trim(m, pm) for m, pm in zip(maps, _per_map_dims(padding)))


def validate_highres(highres):
    """volume/utils.py:284-292."""
    assert highres.ndim >= 5
    assert np.prod(highres.shape) > 0
    hd, hh, hw = highres.shape[1:4]
    for s in (hd, hh, hw):
        assert s > 2 and s % 2 != 0
    return hd, hh, hw


def validate_lowres(lowres):
    """volume/utils.py:295-303."""
    assert lowres.ndim >= 5
    assert np.prod(lowres.shape) > 0
    ld, lh, lw = lowres.shape[1:4]
    for s in (ld, lh, lw):
        assert s >= 2
    return ld, lh, lw


def validate_chunk(chunk):
    """volume/utils.py:306-318."""
    if isinstance(chunk, int):
        assert chunk > 3
        return (chunk,) * 3
    if isinstance(chunk, tuple):
        cd, ch, cw = chunk
        assert cd > 3 and ch > 3 and cw > 3
        return cd, ch, cw
    raise AssertionError('chunk must be int or tuple(int, int, int)')


def encode(predictions_fn, encode_fn, highres, padding=0):
    """volume/encode_decode.py:30-56."""
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
    """volume/encode_decode.py:59-85."""
    encoded_maps, dims = encoded
    validate_padding(padding)
    validate_lowres(lowres)
    lowres = pad_lowres(lowres, dims)
    encoded_maps = pad_maps(encoded_maps, dims)
    pred_maps = predictions_fn(pad_neighborhood(lowres, padding))
    decoded = [decode_fn(p, e) for p, e in zip(pred_maps, encoded_maps)]
    return trim(highres_from_lowres_and_maps(lowres, decoded), dims)


def process_chunks(predictions_fn, code_fn, lowres, reference_maps, chunk, padding, progress_fn):
    """volume/encode_decode_chunk.py:77-117."""
    validate_padding(padding)
    cd, ch, cw = validate_chunk(chunk)
    ld, lh, lw = validate_lowres(lowres)
    padded = pad_neighborhood(lowres, padding)
    coded = [np.zeros_like(r) for r in reference_maps]
    chunks = product(yield_chunks(ld, cd), yield_chunks(lh, ch), yield_chunks(lw, cw))
    if progress_fn is not None:
        chunks = progress_fn(list(chunks))
    p2 = 2 * padding
    for ((z0, z1), (pz0, pz1)), ((y0, y1), (py0, py1)), ((x0, x1), (px0, px1)) in chunks:
        window = padded[:, z0 - pz0:z1 + pz1 + p2, y0 - py0:y1 + py1 + p2, x0 - px0:x1 + px1 + p2]
        preds = predictions_fn(window)
        for i, (pm, ref) in enumerate(zip(preds, reference_maps)):
            nd, nh, nw = pm.shape[1] - (pz0 + pz1), pm.shape[2] - (py0 + py1), pm.shape[3] - (px0 + px1)
            region = (slice(None), slice(z0, z0 + nd), slice(y0, y0 + nh), slice(x0, x0 + nw))
            value = code_fn(pm[:, pz0:pz0 + nd, py0:py0 + nh, px0:px0 + nw], ref[region])
            coded[i][region] = np.asarray(value).astype(coded[i].dtype, casting='unsafe')
    return coded


def encode_chunks(predictions_fn, encode_fn, highres, chunk=32, padding=0, progress_fn=None):
    """volume/encode_decode_chunk.py:33-53."""
    highres, dims = pad_highres(highres)
    validate_highres(highres)
    lowres = lowres_from_highres(highres)
    gt_maps = maps_from_highres(highres)
    coded = process_chunks(predictions_fn, encode_fn, lowres, gt_maps, chunk, padding, progress_fn)
    return trim(lowres, dims), (trim_maps(coded, dims), dims)


def decode_chunks(predictions_fn, decode_fn, lowres, encoded, chunk=32, padding=0, progress_fn=None):
    """volume/encode_decode_chunk.py:56-74."""
    encoded_maps, dims = encoded
    lowres = pad_lowres(lowres, dims)
    encoded_maps = pad_maps(encoded_maps, dims)
    decoded = process_chunks(predictions_fn, decode_fn, lowres, encoded_maps, chunk, padding, progress_fn)
    return trim(highres_from_lowres_and_maps(lowres, decoded), dims)


# Losses -- src/kompressor/losses.py:29-41, volume/losses.py:30-35 (off the hot path)

def mean_squared_error(pred, gt):
    return np.float32(np.mean(np.square(np.float32(gt) - np.float32(pred)), dtype=np.float32))


def mean_abs_error(pred, gt):
    return np.float32(np.mean(np.abs(np.float32(gt) - np.float32(pred)), dtype=np.float32))


def mean_charbonnier_error(pred, gt, eps):
    d = np.float32(gt) - np.float32(pred)
    return np.float32(np.mean(np.sqrt(np.square(d) + np.float32(eps) ** 2), dtype=np.float32))


def mean_total_variation(inputs):
    """volume/losses.py:30-35 -- signed forward differences in the input dtype (unsigned wraps),
    each averaged as float32."""
    x = np.asarray(inputs)
    terms = [np.mean(np.diff(x, axis=a).astype(np.float32), dtype=np.float32) for a in (1, 2, 3)]
    return np.float32((terms[0] + terms[1] + terms[2]) / np.float32(3.0))
