"""Row kernels of the geometry primitives (kmp_primitives.hip ``rows_*``: C == 1, 16-byte chunks
of a row, unaligned vectors on interior chunks, per-element edges) vs the oracle / numpy, at row
lengths around every chunk boundary for each sample size."""

import numpy as np
import pytest
import torch

import oracle
from kompressor_amd import _nd

pytestmark = pytest.mark.gpu

DTYPES = [np.uint8, np.uint16, np.int32, np.float32]
WIDTHS = [3, 7, 9, 15, 16, 17, 31, 33, 47, 63, 64, 65, 66, 97]


def _rand(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    if dtype == np.float32:
        return rng.standard_normal(shape).astype(np.float32)
    info = np.iinfo(dtype)
    return rng.integers(info.min, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


def _np(t):
    return t.cpu().numpy()


@pytest.mark.parametrize('dtype', DTYPES)
@pytest.mark.parametrize('w', WIDTHS)
@pytest.mark.parametrize('nsp', [3, 2])
def test_rows_deinterleave_interleave(kom, dtype, w, nsp):
    shape = (2, 5, 6, w, 1) if nsp == 3 else (3, 7, w, 1)
    hi = _rand(shape, dtype, w)
    ons = oracle.volume if nsp == 3 else oracle.image
    h = torch.from_numpy(hi).cuda()
    assert np.array_equal(_np(_nd.d_lowres_from_highres(h, nsp)), ons.lowres_from_highres(hi))
    for a, b in zip(_nd.d_maps_from_highres(h, nsp), ons.maps_from_highres(hi)):
        assert np.array_equal(_np(a), b)
    # merge: an odd-extent highres rebuilt from its lowres + maps
    odd = tuple(s | 1 for s in shape[1:1 + nsp])
    ho = _rand((2, *odd, 1), dtype, w + 1)
    lo, maps = ons.lowres_from_highres(ho), ons.maps_from_highres(ho)
    rec = _nd.d_highres_from_lowres_and_maps(torch.from_numpy(lo).cuda(),
                                             [torch.from_numpy(m).cuda() for m in maps], nsp)
    assert np.array_equal(_np(rec), ho)


@pytest.mark.parametrize('dtype', DTYPES)
@pytest.mark.parametrize('w', WIDTHS)
@pytest.mark.parametrize('mode', [0, 1])
@pytest.mark.parametrize('pads', [((0, 0, 0), (1, 1, 1)), ((2, 1, 3), (2, 0, 5)), ((1, 2, 17), (0, 3, 9)),
                                  ((0, -1, -2), (1, 0, -3))])
def test_rows_pad(kom, dtype, w, mode, pads):
    lo, hi_ = pads
    x = _rand((2, 6, 5, w, 1), dtype, w)
    if w + lo[2] + hi_[2] <= 0 or (mode == 1 and max(lo[2], hi_[2]) >= w):
        pytest.skip('pad wider than numpy allows for this row')
    got = _np(_nd.d_pad(torch.from_numpy(x).cuda(), lo, hi_, mode, 3))
    # numpy pads first, then crops negative pads
    pos = [(max(a, 0), max(b, 0)) for a, b in zip(lo, hi_)]
    ref = np.pad(x, [(0, 0), *pos, (0, 0)], mode='symmetric' if mode == 0 else 'reflect')
    sl = [slice(None)] + [slice(-min(a, 0), ref.shape[i + 1] + min(b, 0)) for i, (a, b) in enumerate(zip(lo, hi_))]
    assert np.array_equal(got, ref[tuple(sl)])


@pytest.mark.parametrize('dtype', DTYPES)
@pytest.mark.parametrize('w', WIDTHS)
def test_rows_copy_box(kom, dtype, w):
    src = _rand((2, 7, 6, w, 1), dtype, w)
    dst = _rand((2, 9, 8, w + 5, 1), dtype, w + 2)
    s, d = torch.from_numpy(src).cuda(), torch.from_numpy(dst).cuda()
    ext = (5, 4, max(w - 2, 1))
    _nd.d_copy_box(s, (1, 2, min(2, w - ext[2])), ext, d, (3, 1, 4), 3)
    ref = dst.copy()
    x0 = min(2, w - ext[2])
    ref[:, 3:8, 1:5, 4:4 + ext[2]] = src[:, 1:6, 2:6, x0:x0 + ext[2]]
    assert np.array_equal(_np(d), ref)


@pytest.mark.parametrize('dtype', DTYPES + [np.uint32])
@pytest.mark.parametrize('w', [1, 2, 7, 31, 32, 33, 63, 64, 65, 130])
@pytest.mark.parametrize('nsp', [3, 2])
def test_maps_from_predictions_lds(kom, dtype, w, nsp):
    """The LDS-staged aggregation (x tiles of 64 frame columns, 8 / 4 frame rows per workgroup)
    vs the oracle, including ragged last tiles and one-cell axes."""
    K = 19 if nsp == 3 else 5
    cells = (2, 3, 9, w) if nsp == 3 else (2, 11, w)
    preds = _rand((*cells, K, 1), dtype, w)
    if dtype == np.float32:
        preds = (preds * 3000).astype(np.float32)
    ons = oracle.volume if nsp == 3 else oracle.image
    got = _nd.d_maps_from_predictions(torch.from_numpy(preds).cuda(), nsp)
    for a, b in zip(got, ons.maps_from_predictions(preds)):
        assert np.array_equal(_np(a), b)


@pytest.mark.parametrize('dtype', [np.uint8, np.uint16])
@pytest.mark.parametrize('w', [5, 16, 17, 33, 34, 50, 65, 97])
@pytest.mark.parametrize('nsp,p', [(3, 0), (3, 1), (3, 2), (2, 0), (2, 1), (2, 2)])
def test_rows_window_and_mean_predictor(kom, dtype, w, nsp, p):
    """The callback path's window gathers (from highres and from lowres + dims) and the mean
    predictor's two row passes, against the oracle's composition, across chunk boundaries."""
    ons = oracle.volume if nsp == 3 else oracle.image
    shape = (2, 7, 9, w, 1) if nsp == 3 else (3, 9, w, 1)
    hi = _rand(shape, dtype, w + p)
    hp, dims = ons.pad_highres(hi)
    want = ons.pad_neighborhood(ons.lowres_from_highres(hp), p)
    got = _nd.d_window_from_highres(torch.from_numpy(hi).cuda(), p, nsp)
    assert np.array_equal(_np(got), want)
    lo = ons.trim(ons.lowres_from_highres(hp), dims)
    got_lo = _nd.d_window_from_lowres(torch.from_numpy(lo).cuda(), tuple(dims), p, nsp)
    assert np.array_equal(_np(got_lo), ons.pad_neighborhood(ons.pad_lowres(lo, tuple(dims)), p))
    maps = kom.MeanPredictor(p, nsp)(got)
    for a, b in zip(maps, oracle.predictors.mean_predictions_fn(p, nsp)(want)):
        assert np.array_equal(_np(a), b)
