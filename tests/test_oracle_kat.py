"""Known-answer tests derived in closed form from the reference arithmetic, the numpy-vs-loops
cross-check of the two oracle restatements, and the oracle against the committed fixtures."""

import numpy as np
import pytest

from oracle import volume as V, image as I, predictors as P, loops, common
from conftest import golden_names, load_golden, golden_maps, ramp


def test_affine_ramp_known_answers_volume():
    """on an affine ramp (no wrap) with the p=0 mean predictor, the C map
    residuals are all 0, LR is 0 in the interior with -1 (65535) at x=0 and +1 at x=last, and
    the corner Z map is 0 inside with its edge values in a small closed set."""
    hi = ramp((2, 17, 17, 17, 1), 65536, np.uint16)
    lo, (maps, dims) = V.encode(P.mean_predictions_fn(0, 3), V.encode_values_uint16, hi)
    lr, ud, fb, c, z, y, x = maps
    assert dims == (0, 0, 0)
    assert np.all(c == 0)
    assert np.all(lr[:, :, :, 1:-1] == 0)
    assert np.all(lr[:, :, :, 0] == 65535) and np.all(lr[:, :, :, -1] == 1)
    assert np.all(z[:, :, 1:-1, 1:-1] == 0)
    assert set(np.unique(z).tolist()) <= {0, 1, 16, 17, 18, 65518, 65519, 65520, 65535}


def test_constant_input_has_zero_residuals():
    for ns, ndim, shape, dt in ((V, 3, (1, 9, 8, 7, 2), np.uint16), (I, 2, (2, 10, 9, 3), np.uint8)):
        for p in (0, 1, 2):
            hi = np.full(shape, 200, dt)
            lo, (maps, dims) = ns.encode(P.mean_predictions_fn(p, ndim),
                                         V.encode_values_uint16 if dt == np.uint16 else V.encode_values_uint8,
                                         hi, padding=p)
            assert np.all(lo == 200)
            assert all(np.all(m == 0) for m in maps)


def test_mean_predictor_is_integer_floor():
    """§8a a9: for p <= 2 on uint16 the reference's f32 mean equals floor(sum / N)."""
    rng = np.random.default_rng(3)
    for p in (0, 1, 2):
        lo = rng.integers(0, 65536, size=(2, 2 * p + 4, 2 * p + 5, 2 * p + 3, 1)).astype(np.uint16)
        f = V.features_from_lowres(lo, p)
        want = f.astype(np.int64).sum(axis=4) // f.shape[4]
        got = common.cast_from_f32(np.mean(f.astype(np.float32), axis=4, dtype=np.float32), np.uint16)
        assert np.array_equal(got, want)


def test_maps_from_predictions_normalisation():
    """volume/utils.py:119-129: four-way lattice = quarter inside, half on edges, raw corners."""
    pred = np.zeros((1, 2, 2, 2, 19, 1), np.float32)
    pred[..., 7:11, :] = 4.0
    z = V.maps_from_predictions(pred)[4][0, :, :, :, 0]
    assert np.all(z == 4.0)  # every entry is a mean of 4.0's


@pytest.mark.parametrize('ndim,shape,dtype,p', [(3, (2, 7, 8, 9, 1), np.uint16, 0), (3, (1, 8, 8, 8, 2), np.uint16, 1),
                                                (3, (1, 5, 6, 7, 1), np.uint16, 2), (3, (1, 6, 5, 4, 1), np.uint8, 1),
                                                (2, (2, 9, 10, 3), np.uint8, 0), (2, (1, 16, 16, 1), np.uint8, 1),
                                                (2, (1, 7, 12, 2), np.uint16, 2), (2, (1, 3, 4, 1), np.uint8, 3)])
def test_two_restatements_agree(ndim, shape, dtype, p):
    ns = V if ndim == 3 else I
    rng = np.random.default_rng(sum(shape) + p)
    hi = rng.integers(0, np.iinfo(dtype).max + 1, size=shape).astype(dtype)
    enc = V.encode_values_uint16 if dtype == np.uint16 else V.encode_values_uint8
    dec = V.decode_values_uint16 if dtype == np.uint16 else V.decode_values_uint8
    pf = P.mean_predictions_fn(p, ndim)
    lo, (maps, dims) = ns.encode(pf, enc, hi, padding=p)
    lo2, maps2, dims2 = loops.encode_mean(hi, p, ndim)
    assert tuple(dims) == dims2 and np.array_equal(lo, lo2)
    for a, b in zip(maps, maps2):
        assert np.array_equal(a, b)
    assert np.array_equal(ns.decode(pf, dec, lo, (maps, dims), padding=p), hi)
    assert np.array_equal(loops.decode_mean(lo, maps, dims, p, ndim), hi)


@pytest.mark.parametrize('name', [n for n in golden_names() if n.startswith(('vol_', 'img_'))
                                  and 'categorical' not in n])
def test_oracle_reproduces_golden(name):
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns = V if ndim == 3 else I
    coder = str(g['coder'])
    enc = {'uint8': common.encode_values_uint8, 'uint16': common.encode_values_uint16,
           'raw': common.encode_values_raw}[coder]
    lo, (maps, dims) = ns.encode(P.mean_predictions_fn(p, ndim), enc, g['highres'], padding=p)
    assert tuple(dims) == tuple(g['dims']) and np.array_equal(lo, g['lowres'])
    for a, b in zip(maps, golden_maps(g, ndim)):
        assert a.dtype == b.dtype and np.array_equal(a, b)


@pytest.mark.parametrize('name', golden_names('mfp_'))
def test_oracle_maps_from_predictions_golden(name):
    g = load_golden(name)
    ns = V if int(g['ndim']) == 3 else I
    for i, m in enumerate(ns.maps_from_predictions(g['predictions'])):
        assert np.array_equal(m, g[f'map{i}'])


def test_categorical_rank_coder_semantics():
    """utils.py:58-111: rank in the reversed stable argsort; ties -> the higher index first."""
    logits = np.array([[0.1, 0.5, 0.5, 0.2]], np.float32)
    order = [2, 1, 3, 0]  # descending, tie 1/2 resolved higher index first by the reversal
    for rank, cls in enumerate(order):
        assert common.encode_categorical(logits, np.array([cls], np.uint8))[0] == rank
        assert common.decode_categorical(logits, np.array([rank], np.uint8))[0] == cls
