"""The reference's own test assertions (tests/{volume,image}/test_*.py), re-expressed against the
CPU oracle.  This is what pins the oracle to the reference: shapes, dtypes, lossless round trips,
chunk invariance and validator behaviour."""

from functools import partial
from itertools import product

import numpy as np
import pytest

from oracle import volume as V, image as I, predictors as P, common
from conftest import ramp

SPEC = {
    3: dict(ns=V, odd=(2, 17, 17, 17, 1), even=(2, 16, 16, 16, 1), max=65536, dtype=np.uint16,
            enc=V.encode_values_uint16, dec=V.decode_values_uint16, chunks=[6, 11, (6, 11, 11)], K=19),
    2: dict(ns=I, odd=(2, 17, 17, 3), even=(2, 16, 16, 3), max=256, dtype=np.uint8,
            enc=I.encode_values_uint8, dec=I.decode_values_uint8, chunks=[6, 11, (6, 11)], K=5),
}


def expected_map_shapes(hshape, ndim):
    # tests/volume/test_encode_decode.py:107-175 (odd input): cells (h-1)//2, nodes (h-1)//2 + 1
    par = V.MAP_PARITY if ndim == 3 else I.MAP_PARITY
    b, sp, ch = hshape[0], hshape[1:1 + ndim], hshape[1 + ndim:]
    return [(b, *[((s - 1) // 2 + (0 if p else 1)) for s, p in zip(sp, pa)], *ch) for pa in par]


@pytest.mark.parametrize('ndim', [3, 2])
@pytest.mark.parametrize('padding', [0, 1])
def test_encode_decode(ndim, padding):
    # tests/volume/test_encode_decode.py:77-215, tests/image/test_encode_decode.py:76-178
    s = SPEC[ndim]
    ns, pf = s['ns'], P.mean_predictions_fn(padding, ndim)
    hi = ramp(s['odd'], s['max'], s['dtype'])
    lowres, (maps, dims) = ns.encode(pf, s['enc'], hi, padding=padding)
    assert tuple(dims) == (0,) * ndim
    for m, shape in zip(maps, expected_map_shapes(hi.shape, ndim)):
        assert m.dtype == hi.dtype and m.ndim == hi.ndim and m.shape == shape
    rec = ns.decode(pf, s['dec'], lowres, (maps, dims), padding=padding)
    assert rec.dtype == hi.dtype and np.array_equal(rec, hi)
    hi = ramp(s['even'], s['max'], s['dtype'])
    lowres, (maps, dims) = ns.encode(pf, s['enc'], hi, padding=padding)
    assert tuple(dims) == (1,) * ndim
    assert np.array_equal(ns.decode(pf, s['dec'], lowres, (maps, dims), padding=padding), hi)


@pytest.mark.parametrize('ndim', [3, 2])
@pytest.mark.parametrize('padding', [0, 1])
def test_encode_decode_categorical(ndim, padding):
    # tests/volume/test_encode_decode.py:217-356 (uint8 volumes, 256-class rank coder)
    s = SPEC[ndim]
    ns, pf = s['ns'], P.categorical_predictions_fn(padding, 256, ndim)
    for shape, dims_want in ((s['odd'], 0), (s['even'], 1)):
        hi = ramp(shape, 256, np.uint8)
        lowres, (maps, dims) = ns.encode(pf, common.encode_categorical, hi, padding=padding)
        assert tuple(dims) == (dims_want,) * ndim
        if dims_want == 0:
            for m, es in zip(maps, expected_map_shapes(hi.shape, ndim)):
                assert m.dtype == np.uint8 and m.shape == es
        assert np.array_equal(ns.decode(pf, common.decode_categorical, lowres, (maps, dims), padding=padding), hi)


@pytest.mark.parametrize('ndim', [3, 2])
def test_encode_decode_raw(ndim):
    # tests/volume/test_encode_decode.py:358-464: int32 input, raw int32 coder, padding 0
    s = SPEC[ndim]
    ns, pf = s['ns'], P.mean_predictions_fn(0, ndim)
    hi = ramp(s['odd'], s['max'], np.uint16 if ndim == 3 else np.uint8).astype(np.int32)
    lowres, (maps, dims) = ns.encode(pf, common.encode_values_raw, hi)
    for m, es in zip(maps, expected_map_shapes(hi.shape, ndim)):
        assert m.dtype == np.int32 and m.shape == es
    assert np.array_equal(ns.decode(pf, common.decode_values_raw, lowres, (maps, dims)), hi)


@pytest.mark.parametrize('ndim', [3, 2])
@pytest.mark.parametrize('padding', [0, 1])
@pytest.mark.parametrize('categorical', [False, True])
def test_encode_chunks_and_decode_chunks(ndim, padding, categorical):
    # tests/volume/test_encode_decode.py:466-841: chunk invariance + lossless, odd and even dims
    s = SPEC[ndim]
    ns = s['ns']
    if categorical:
        pf = P.categorical_predictions_fn(padding, 256, ndim)
        enc, dec, mx, dt = common.encode_categorical, common.decode_categorical, 256, np.uint8
    else:
        pf = P.mean_predictions_fn(padding, ndim)
        enc, dec, mx, dt = s['enc'], s['dec'], s['max'], s['dtype']
    for shape, chunks in ((s['odd'], s['chunks']), (s['even'], s['chunks'][:2])):
        hi = ramp(shape, mx, dt)
        full_lo, (full_maps, full_dims) = ns.encode(pf, enc, hi, padding=padding)
        for chunk in chunks:
            calls = []

            def progress(c):
                calls.append(len(c))
                return c

            lo, (maps, dims) = ns.encode_chunks(pf, enc, hi, chunk=chunk, padding=padding, progress_fn=progress)
            assert calls and tuple(dims) == tuple(full_dims)
            assert np.array_equal(lo, full_lo)
            for a, b in zip(maps, full_maps):
                assert np.array_equal(a, b)
            assert np.array_equal(ns.decode(pf, dec, lo, (maps, dims), padding=padding), hi)
            rec = ns.decode_chunks(pf, dec, full_lo, (full_maps, full_dims), chunk=chunk, padding=padding)
            assert np.array_equal(rec, hi)


@pytest.mark.parametrize('ndim', [3, 2])
def test_utils_shapes(ndim):
    # tests/volume/test_utils.py:40-252 (targets, lowres, maps_from_predictions, maps_from_highres)
    s = SPEC[ndim]
    ns = s['ns']
    hi = ramp(s['odd'], s['max'], s['dtype'])
    sp, ch = hi.shape[1:1 + ndim], hi.shape[1 + ndim:]
    t = ns.targets_from_highres(hi)
    assert t.dtype == hi.dtype and t.shape == (hi.shape[0], *[(x - 1) // 2 for x in sp], s['K'], *ch)
    lo = ns.lowres_from_highres(hi)
    assert lo.shape == (hi.shape[0], *[(x - 1) // 2 + 1 for x in sp], *ch)
    for m, es in zip(ns.maps_from_predictions(t), expected_map_shapes(hi.shape, ndim)):
        assert m.dtype == t.dtype and m.shape == es
    for m, es in zip(ns.maps_from_highres(hi), expected_map_shapes(hi.shape, ndim)):
        assert m.dtype == hi.dtype and m.shape == es


@pytest.mark.parametrize('ndim', [3, 2])
def test_reconstruction_identities(ndim):
    # tests/volume/test_utils.py:253-291
    s = SPEC[ndim]
    ns = s['ns']
    hi = ramp(s['odd'], s['max'], s['dtype'])
    lo = ns.lowres_from_highres(hi)
    assert np.array_equal(ns.highres_from_lowres_and_maps(lo, ns.maps_from_highres(hi)), hi)
    assert np.array_equal(ns.highres_from_lowres_and_maps(lo, ns.maps_from_predictions(ns.targets_from_highres(hi))),
                          hi)


@pytest.mark.parametrize('ndim', [3, 2])
@pytest.mark.parametrize('padding', range(4))
def test_features_and_pad_shapes(ndim, padding):
    # tests/volume/test_utils.py:293-345
    s = SPEC[ndim]
    ns = s['ns']
    lo = ns.lowres_from_highres(ramp(s['odd'], s['max'], s['dtype']))
    padded = ns.pad_neighborhood(lo, padding)
    assert padded.dtype == lo.dtype
    assert padded.shape == (lo.shape[0], *[x + 2 * padding for x in lo.shape[1:1 + ndim]], *lo.shape[1 + ndim:])
    f = ns.features_from_lowres(padded, padding)
    assert f.shape == (lo.shape[0], *[x - 1 for x in lo.shape[1:1 + ndim]], (2 * padding + 2) ** ndim,
                       *lo.shape[1 + ndim:])


def test_validators():
    # tests/volume/test_utils.py:347-444 (any Exception passes there)
    z = lambda s: np.zeros(s, np.uint16)  # noqa: E731
    for bad in [z((2, 3, 3, 3)), z((0, 3, 3, 3, 1)), z((2, 2, 2, 2, 3)), z((2, 4, 4, 4, 3))]:
        with pytest.raises(Exception):
            V.validate_highres(bad)
    assert V.validate_highres(z((2, 3, 5, 3, 3))) == (3, 5, 3)
    for bad in [z((2, 1, 1, 2, 3)), z((2, 2, 1, 1, 3))]:
        with pytest.raises(Exception):
            V.validate_lowres(bad)
    for p in [None, -1]:
        with pytest.raises(Exception):
            common.validate_padding(p)
    for c in [(4,), (4, 4), None, (None, 4, 4), 3, (4, 4, 3)]:
        with pytest.raises(Exception):
            V.validate_chunk(c)
    assert V.validate_chunk((4, 5, 4)) == (4, 5, 4)
    with pytest.raises(Exception):
        I.validate_chunk((4, 4, 4))


def test_losses():
    # tests/{volume,image}/test_losses.py
    for ns, shape, mx, dt in ((V, (2, 4, 4, 4, 1), 65536, np.uint16), (I, (2, 4, 4, 3), 256, np.uint8)):
        d = ramp(shape, mx, dt)
        for fn in (ns.mean_squared_error, ns.mean_abs_error, partial(ns.mean_charbonnier_error, eps=1e-3)):
            loss = fn(d + 1, d)
            assert np.asarray(loss).dtype == np.float32 and np.asarray(loss).ndim == 0 and np.isclose(loss, 1.0)
        tv = ns.mean_total_variation(np.ones_like(d))
        assert np.asarray(tv).dtype == np.float32 and tv == 0.0
