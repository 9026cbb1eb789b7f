"""LinearPredictor parity.  arith='f32': float32 intermediates bit-exact to the oracle's fma chain
and within the north star's 1e-5 of a float64 reference; residual maps bit-exact; lossless.
arith='bf16x2' (the matrix cores) and 'auto' (the default, one of the two by configuration): see
the sections at the end."""

import numpy as np
import pytest
import torch

import oracle
from oracle import predictors as OP

pytestmark = pytest.mark.gpu


def _weights(ndim, padding, seed, dtype):
    n, k = (2 * padding + 2) ** ndim, 19 if ndim == 3 else 5
    rng = np.random.default_rng(seed)
    w = (1.0 / n + rng.standard_normal((n, k)) * (0.3 / n)).astype(np.float32)  # ~ a noisy mean
    b = (rng.standard_normal(k) * (3.0 if dtype == np.uint8 else 50.0)).astype(np.float32)
    return w, b


CASES = [(3, 0, (2, 9, 10, 12, 1), np.uint16), (3, 1, (2, 8, 9, 7, 1), np.uint16), (3, 0, (1, 9, 8, 16, 2), np.uint8),
         (3, 0, (4, 64, 64, 64, 1), np.uint16), (2, 0, (3, 33, 20, 1), np.uint8), (2, 1, (2, 30, 31, 2), np.uint16),
         (2, 2, (2, 17, 17, 1), np.uint8),
         # fused 2D wave kernel (LinearPredictor p = 0): multi-row waves, odd height, one-row waves
         (2, 0, (3, 64, 64, 1), np.uint16), (2, 0, (2, 37, 128, 1), np.uint8), (2, 0, (2, 9, 1024, 1), np.uint8),
         (2, 0, (3, 10, 512, 1), np.uint16), (2, 0, (8, 30, 256, 1), np.uint16)]


def _data(shape, dtype, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)


@pytest.mark.parametrize('kernel', ['valu', 'mfma'])
@pytest.mark.parametrize('ndim,p,shape,dtype', CASES)
def test_linear_cell_predictions(kom, ndim, p, shape, dtype, kernel):
    """Both f32 kernels (kmp_linear.hip: the per-thread fma chain, the default, and the f32 MFMA
    under KMP_LINEAR_F32_MFMA=1) are the oracle's k-ordered chain, bit for bit."""
    ons = oracle.volume if ndim == 3 else oracle.image
    hi = _data(shape, dtype, 1)
    w, b = _weights(ndim, p, 2, dtype)
    window = ons.pad_neighborhood(ons.lowres_from_highres(ons.pad_highres(hi)[0]), p)
    pred = kom.LinearPredictor(w, b, p, ndim, arith='f32')
    with kom._lib.option('KMP_LINEAR_F32_MFMA', int(kernel == 'mfma')):
        cells_t, cells_f = pred.predict_cells(window, with_f32=True)
        assert kom._lib.lib.kmp_last_launch().decode() == 'linear_' + kernel
    feats = ons.features_from_lowres(window, p)
    exact = OP.linear_fma_chain(feats, w, b)
    assert cells_f.dtype == np.float32 and cells_f.shape == exact.shape
    assert np.array_equal(cells_f.view(np.uint32), exact.view(np.uint32)), f'f32 {kernel} != k-ordered fma chain'
    f64, _ = OP.linear_predictions(feats, w, b, dtype)
    scale = np.tensordot(np.abs(np.moveaxis(feats.astype(np.float64), ndim + 1, -1)), np.abs(w), axes=([-1], [0]))
    scale = np.moveaxis(scale, -1, ndim + 1) + np.abs(b).reshape(-1, 1)
    assert np.all(np.abs(cells_f - f64) <= 1e-5 * scale + 1e-6), 'north-star 1e-5 tolerance'
    assert np.array_equal(cells_t, oracle.common.cast_from_f32(exact, dtype))


@pytest.mark.parametrize('ndim,p,shape,dtype', CASES)
def test_linear_codec(kom, ndim, p, shape, dtype):
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    hi = _data(shape, dtype, 3)
    w, b = _weights(ndim, p, 4, dtype)
    pred = kom.LinearPredictor(w, b, p, ndim, arith='f32')
    enc, dec = (ns.encode_values_uint16, ns.decode_values_uint16) if dtype == np.uint16 else \
               (ns.encode_values_uint8, ns.decode_values_uint8)
    oenc = ons.encode_values_uint16 if dtype == np.uint16 else ons.encode_values_uint8
    want_lo, (want_maps, want_dims) = ons.encode(OP.linear_predictions_fn(p, w, b, ndim), oenc, hi, padding=p)
    for fn in (pred, lambda x: pred(x)):  # fused kernels, then the callback path
        lo, (maps, dims) = ns.encode(fn, enc, hi, padding=p)
        assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
        for a, c in zip(maps, want_maps):
            assert np.array_equal(a, c)
        assert np.array_equal(ns.decode(fn, dec, lo, (maps, dims), padding=p), hi)


def test_linear_chunks(kom):
    hi = _data((2, 17, 16, 15, 1), np.uint16, 5)
    w, b = _weights(3, 1, 6, np.uint16)
    pred = kom.LinearPredictor(w, b, 1, 3, arith='f32')
    lo, (maps, dims) = kom.volume.encode(pred, kom.volume.encode_values_uint16, hi, padding=1)
    for chunk in (6, (6, 11, 7)):
        lo2, (maps2, dims2) = kom.volume.encode_chunks(pred, kom.volume.encode_values_uint16, hi, chunk=chunk, padding=1)
        assert np.array_equal(lo, lo2) and all(np.array_equal(a, c) for a, c in zip(maps, maps2))
        rec = kom.volume.decode_chunks(pred, kom.volume.decode_values_uint16, lo, (maps, dims), chunk=chunk, padding=1)
        assert np.array_equal(rec, hi)


@pytest.mark.parametrize('dtype', [np.uint16, np.uint8])
@pytest.mark.parametrize('shape', [(8, 64, 64, 64, 1), (2, 17, 30, 16, 1), (1, 9, 14, 128, 1), (2, 12, 33, 32, 1),
                                   (1, 6, 8, 8, 1), (1, 10, 40, 32, 1), (2, 9, 32, 128, 1)])
def test_linear_fused_p1(kom, shape, dtype):
    """The fused LinearPredictor p = 1 volume kernel (kmp_codec_linear3dp.hip, packed-FMA chain; 8-bit
    samples since round 6): residuals and lowres bit-exact to the oracle's fma chain + aggregation,
    lossless, z-region (chunked) launches, over lowres widths 4 .. 64 and partial last waves."""
    hi = _data(shape, dtype, 7)
    w, b = _weights(3, 1, 8, dtype)
    pred = kom.LinearPredictor(w, b, 1, 3, arith='f32')
    V, OV = kom.volume, oracle.volume
    enc, dec, oenc = ((V.encode_values_uint16, V.decode_values_uint16, OV.encode_values_uint16) if dtype == np.uint16
                      else (V.encode_values_uint8, V.decode_values_uint8, OV.encode_values_uint8))
    want_lo, (want_maps, want_dims) = OV.encode(OP.linear_predictions_fn(1, w, b, 3), oenc, hi, padding=1)
    lo, (maps, dims) = V.encode(pred, enc, hi, padding=1)
    assert kom._lib.lib.kmp_last_launch().decode() == 'linear3dp_encode'
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for i, (a, c) in enumerate(zip(maps, want_maps)):
        bad = np.argwhere(a != c)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'
    assert np.array_equal(V.decode(pred, dec, lo, (maps, dims), padding=1), hi)
    assert kom._lib.lib.kmp_last_launch().decode() == 'linear3dp_decode'
    lo2, (maps2, _) = V.encode_chunks(pred, enc, hi, chunk=5, padding=1)
    assert np.array_equal(lo2, want_lo) and all(np.array_equal(a, c) for a, c in zip(maps2, want_maps))


@pytest.mark.parametrize('shape,dtype,kernel', [
    # the y-rolling kernel (FULL tiles whose rows split into 1, 2, 4 or 8 wave steps)
    ((4, 64, 64, 64, 1), np.uint16, 'linear3y'), ((1, 7, 64, 64, 1), np.uint16, 'linear3y'),
    ((2, 6, 32, 32, 1), np.uint16, 'linear3y'), ((1, 4, 128, 64, 1), np.uint16, 'linear3y'),
    ((1, 6, 64, 32, 1), np.uint16, 'linear3y'), ((2, 8, 32, 64, 1), np.uint8, 'linear3y'),
    ((1, 9, 64, 64, 1), np.uint8, 'linear3y'), ((1, 4, 64, 128, 1), np.uint8, 'linear3y'),
    # the plane-block kernel: FULL rows that do not split into wave steps, and odd heights
    ((2, 17, 30, 16, 1), np.uint16, 'linear3d'), ((2, 12, 33, 32, 1), np.uint16, 'linear3d'),
    ((1, 9, 14, 128, 1), np.uint8, 'linear3d'), ((3, 10, 9, 64, 1), np.uint8, 'linear3d')])
def test_linear_fused_p0(kom, shape, dtype, kernel):
    """The fused LinearPredictor p = 0 volume kernels (kmp_codec_linear3d.hip: weights in scalar
    registers; the y-rolling kernel for FULL tiles -- one wave per output plane, row steps with the
    next step's loads in flight, row neighbours by lane rotations; the plane-block kernel's FULL body
    -- only row-0 / lane-0 masks, missing z planes through zero weights -- and its general body for
    odd heights): residuals and lowres bit-exact to the oracle's fma chain + aggregation, lossless,
    chunked.  The shapes cover FULL with an odd depth (the last output plane has no cell plane c),
    1 / 2 / 4 / 8 row steps for both sample sizes, and the general body."""
    hi = _data(shape, dtype, 9)
    w, b = _weights(3, 0, 10, dtype)
    pred = kom.LinearPredictor(w, b, 0, 3, arith='f32')
    V, OV = kom.volume, oracle.volume
    enc, dec, oenc = ((V.encode_values_uint16, V.decode_values_uint16, OV.encode_values_uint16) if dtype == np.uint16
                      else (V.encode_values_uint8, V.decode_values_uint8, OV.encode_values_uint8))
    want_lo, (want_maps, want_dims) = OV.encode(OP.linear_predictions_fn(0, w, b, 3), oenc, hi, padding=0)
    lo, (maps, dims) = V.encode(pred, enc, hi, padding=0)
    assert kom._lib.lib.kmp_last_launch().decode() == kernel + '_encode'
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for i, (a, c) in enumerate(zip(maps, want_maps)):
        assert np.array_equal(a, c), f'map {i}'
    assert np.array_equal(V.decode(pred, dec, lo, (maps, dims), padding=0), hi)
    assert kom._lib.lib.kmp_last_launch().decode() == kernel + '_decode'
    rec = V.decode_chunks(pred, dec, lo, (maps, dims), chunk=6, padding=0)
    assert np.array_equal(rec, hi)


# ---------------------------------------------------------------------------------------------
# arith='bf16x2': the matrix-core arithmetic (kmp_bf16x2.h).  Not equal to the f32 fma chain by
# design; pinned by (1) the float32 channel values within the north star's 1e-5 of float64 (and
# within f32 accumulation rounding of the exactly split products), (2) every path -- fused
# linear3m kernel, the callable / callback path, the generic codec -- producing the same bits,
# (3) the residuals equal to the oracle's coder applied to the kernel's own prediction maps, and
# (4) lossless round trips, including across paths.
# ---------------------------------------------------------------------------------------------

BF_CASES = [(3, 0, (4, 64, 64, 64, 1), np.uint16), (3, 0, (2, 16, 32, 32, 1), np.uint16),
            (3, 0, (1, 7, 32, 64, 1), np.uint16), (3, 0, (2, 9, 10, 12, 1), np.uint16),
            (3, 0, (2, 8, 32, 64, 1), np.uint8), (3, 0, (1, 9, 64, 32, 1), np.uint8),
            (3, 1, (2, 8, 9, 7, 1), np.uint16), (2, 0, (3, 33, 20, 1), np.uint8), (2, 1, (2, 30, 31, 2), np.uint16),
            # p = 1 on the fused matrix-core kernel (linear3pm): 32 / 16-wide rows and planes
            (3, 1, (2, 12, 64, 64, 1), np.uint16), (3, 1, (1, 10, 32, 32, 1), np.uint16),
            (3, 1, (1, 8, 32, 64, 1), np.uint16), (3, 1, (1, 7, 64, 32, 1), np.uint16),
            (3, 1, (1, 8, 32, 64, 1), np.uint8),
            (3, 1, (1, 6, 32, 32, 1), np.uint16),  # a small volume: the workspace still holds the fragments
            # p = 1 u8 on linear3pm (round 6): every row width / plane height, C3 tiles, an odd depth
            (3, 1, (2, 12, 64, 64, 1), np.uint8), (3, 1, (1, 10, 32, 32, 1), np.uint8),
            (3, 1, (1, 7, 64, 32, 1), np.uint8), (3, 1, (4, 64, 64, 64, 1), np.uint8)]


@pytest.mark.parametrize('ndim,p,shape,dtype', BF_CASES)
def test_linear_bf16x2_cells_within_tolerance(kom, ndim, p, shape, dtype):
    ons = oracle.volume if ndim == 3 else oracle.image
    hi = _data(shape, dtype, 11)
    w, b = _weights(ndim, p, 12, dtype)
    window = ons.pad_neighborhood(ons.lowres_from_highres(ons.pad_highres(hi)[0]), p)
    pred = kom.LinearPredictor(w, b, p, ndim, arith='bf16x2')
    cells, cells_f = pred.predict_cells(window, with_f32=True)
    feats = ons.features_from_lowres(window, p)
    exact, _ = OP.linear_predictions(feats, w, b, dtype)
    split = OP.linear_bf16x2_split(feats, w, b)
    n_axis = feats.ndim - 2
    scale = np.tensordot(np.moveaxis(np.abs(feats.astype(np.float64)), n_axis, -1), np.abs(w.astype(np.float64)),
                         axes=([-1], [0]))
    scale = np.moveaxis(scale, -1, ndim + 1) + np.abs(b).reshape(-1, 1)
    assert cells_f.shape == exact.shape
    assert np.all(np.abs(cells_f - exact) <= 1e-5 * scale), np.max(np.abs(cells_f - exact) / scale)
    assert np.all(np.abs(cells_f - split) <= 2e-6 * scale), np.max(np.abs(cells_f - split) / scale)
    assert np.array_equal(cells, OP.cast_from_f32(cells_f, dtype))


@pytest.mark.parametrize('ndim,p,shape,dtype', BF_CASES)
def test_linear_bf16x2_codec_paths_agree(kom, ndim, p, shape, dtype):
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    hi = _data(shape, dtype, 13)
    w, b = _weights(ndim, p, 14, dtype)
    pred = kom.LinearPredictor(w, b, p, ndim, arith='bf16x2')
    enc, dec = (ns.encode_values_uint16, ns.decode_values_uint16) if dtype == np.uint16 else \
               (ns.encode_values_uint8, ns.decode_values_uint8)
    oenc = ons.encode_values_uint16 if dtype == np.uint16 else ons.encode_values_uint8
    lo, (maps, dims) = ns.encode(pred, enc, hi, padding=p)
    # the fused matrix-core kernel serves FULL volumes whose 16 / 32-wide rows split into 1, 2 or 4
    # wave steps; the rest runs the generic codec on the same arithmetic
    ex, ey, vx = shape[3] // 2, shape[2] // 2, 8 // np.dtype(dtype).itemsize
    rows = 64 // max(1, ex // vx)
    fused = (ndim == 3 and p == 0 and shape[2] % 2 == 0 and shape[3] % 2 == 0 and ex in (16, 32)
             and ey % rows == 0 and ey // rows in (1, 2, 4))
    # p = 1: u8 / u16 FULL volumes with 16 / 32-wide rows and 16 / 32 rows a plane
    fused1 = (ndim == 3 and p == 1 and shape[2] % 2 == 0 and shape[3] % 2 == 0
              and ex in (16, 32) and ey in (16, 32))
    want_kernel = 'linear3m_encode' if fused else 'linear3pm_encode' if fused1 else 'encode_generic'
    assert kom._lib.lib.kmp_last_launch().decode() == want_kernel
    # (3) residuals == the oracle's coder on the kernel's own predictions (the callable's maps)
    padded = ons.pad_highres(hi)[0]
    pmaps = pred(ons.pad_neighborhood(ons.lowres_from_highres(padded), p))
    want = ons.trim_maps([oenc(pm, g) for pm, g in zip(pmaps, ons.maps_from_highres(padded))], dims)
    for i, (a, c) in enumerate(zip(maps, want)):
        assert np.array_equal(a, c), f'map {i}: {np.count_nonzero(a != c)} mismatches'
    # (2) the callback path (opaque predictions_fn = the same predictor) gives the same bits
    lo2, (maps2, _) = ns.encode(lambda x: pred(x), enc, hi, padding=p)
    assert np.array_equal(lo2, lo) and all(np.array_equal(a, c) for a, c in zip(maps2, maps))
    # (4) lossless, fused and across paths, and chunked
    assert np.array_equal(ns.decode(pred, dec, lo, (maps, dims), padding=p), hi)
    assert np.array_equal(ns.decode(lambda x: pred(x), dec, lo, (maps, dims), padding=p), hi)
    assert np.array_equal(ns.decode_chunks(pred, dec, lo, (maps, dims), chunk=6, padding=p), hi)
    lo3, (maps3, _) = ns.encode_chunks(pred, enc, hi, chunk=6, padding=p)
    assert np.array_equal(lo3, lo) and all(np.array_equal(a, c) for a, c in zip(maps3, maps))


def test_linear_bf16x2_rejects_32bit_samples(kom):
    """The byte split is exact only for 8 / 16-bit samples: 32-bit samples raise, never round."""
    hi = _data((1, 9, 9, 9, 1), np.uint16, 1).astype(np.int32)
    w, b = _weights(3, 0, 2, np.uint16)
    pred = kom.LinearPredictor(w, b, 0, 3, arith='bf16x2')
    with pytest.raises(Exception):
        kom.volume.encode(pred, kom.volume.encode_values_raw, hi)


@pytest.mark.parametrize('dtype', [np.uint16, np.uint8])
def test_linear_bf16x2_p1_fused_sweep(kom, dtype):
    """Seeded sweep of fused-eligible p = 1 volumes (u8 / u16, 16 / 32-wide rows and planes, any depth,
    batch sizes that do and do not take the XCD order, smooth and full-range data, chunked regions):
    linear3pm's lowres + maps equal the generic bf16x2 path's bit for bit (KMP_DISABLE_LINEAR_FUSED),
    and the round trip is lossless."""
    V = kom.volume
    rng = np.random.default_rng(2024)
    for case in range(10):
        B = int(rng.choice([1, 2, 3, 8]))
        D = int(rng.integers(6, 24))
        H, W = int(rng.choice([32, 64])), int(rng.choice([32, 64]))
        hi = _data((B, D, H, W, 1), dtype, 100 + case)
        if case % 2:  # smooth data: small residuals, the predictor's realistic regime
            z, y, x = np.meshgrid(np.arange(D), np.arange(H), np.arange(W), indexing='ij')
            sc = 1 if dtype == np.uint16 else 0.1
            hi = ((1000 + 40 * z + 25 * y + 10 * x)[None, ..., None] * sc + rng.integers(0, 9, (B, D, H, W, 1))
                  ).astype(np.int64) % (np.iinfo(dtype).max + 1)
            hi = hi.astype(dtype)
        w, b = _weights(3, 1, 200 + case, dtype)
        pred = kom.LinearPredictor(w, b, 1, 3, arith='bf16x2')
        hi_t = torch.from_numpy(hi).cuda()
        enc, dec = ((V.encode_values_uint16, V.decode_values_uint16) if dtype == np.uint16
                    else (V.encode_values_uint8, V.decode_values_uint8))
        lo, (maps, dims) = V.encode(pred, enc, hi_t, padding=1)
        assert kom._lib.lib.kmp_last_launch().decode() == 'linear3pm_encode', (B, D, H, W)
        chunk = int(rng.integers(4, 12))
        lo_c, (maps_c, _) = V.encode_chunks(pred, enc, hi_t, chunk=chunk, padding=1)
        with kom._lib.option('KMP_DISABLE_LINEAR_FUSED', 1):
            lo_g, (maps_g, _) = V.encode(pred, enc, hi_t, padding=1)
            assert kom._lib.lib.kmp_last_launch().decode() == 'encode_generic'
        assert torch.equal(lo, lo_g) and torch.equal(lo_c, lo_g)
        for i, (a, c, g) in enumerate(zip(maps, maps_c, maps_g)):
            assert torch.equal(a, g), f'case {case} map {i}: {int((a != g).sum())} mismatches'
            assert torch.equal(c, g), f'case {case} chunked map {i}'
        rec = V.decode(pred, dec, lo, (maps, dims), padding=1)
        assert kom._lib.lib.kmp_last_launch().decode() == 'linear3pm_decode'
        assert torch.equal(rec, hi_t)
        rec_c = V.decode_chunks(pred, dec, lo, (maps, dims), chunk=chunk, padding=1)
        assert torch.equal(rec_c, hi_t)


# ---- arith='auto' (the default) ----

AUTO_CASES = [(3, 1, (2, 32, 32, 32, 1), np.uint16, 'bf16x2'), (3, 1, (1, 17, 30, 16, 1), np.uint16, 'bf16x2'),
              (3, 0, (2, 32, 32, 32, 1), np.uint16, 'f32'), (3, 1, (2, 32, 32, 32, 1), np.uint8, 'bf16x2'),
              (3, 1, (1, 13, 22, 32, 1), np.uint8, 'bf16x2'), (3, 0, (1, 16, 32, 32, 1), np.uint8, 'f32'),
              (2, 1, (2, 64, 64, 1), np.uint16, 'f32')]


@pytest.mark.parametrize('ndim,p,shape,dtype,want', AUTO_CASES)
def test_linear_auto_arith(kom, tmp_path, ndim, p, shape, dtype, want):
    """arith='auto' evaluates with the matrix cores for volumes with padding 1 and uint16 samples and
    with the f32 chain elsewhere: the same maps and lowres as the explicit arithmetic (fused kernels
    and the callback path), lossless, chunk-invariant, and a file records the resolved arithmetic,
    so a reader holding an explicit predictor of it decodes the file."""
    hi = _data(shape, dtype, 11)
    w, b = _weights(ndim, p, 12, dtype)
    auto = kom.LinearPredictor(w, b, p, ndim)
    explicit = kom.LinearPredictor(w, b, p, ndim, arith=want)
    tdt = torch.uint16 if dtype == np.uint16 else torch.uint8
    assert auto.arith == 'auto' and auto.arith_for(tdt) == want
    ns = kom.volume if ndim == 3 else kom.image
    enc, dec = (ns.encode_values_uint16, ns.decode_values_uint16) if dtype == np.uint16 else \
               (ns.encode_values_uint8, ns.decode_values_uint8)
    want_lo, (want_maps, want_dims) = ns.encode(explicit, enc, hi, padding=p)
    for fn in (auto, lambda x: auto(x)):
        lo, (maps, dims) = ns.encode(fn, enc, hi, padding=p)
        assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
        assert all(np.array_equal(a, c) for a, c in zip(maps, want_maps))
        assert np.array_equal(ns.decode(fn, dec, lo, (maps, dims), padding=p), hi)
    if ndim == 3:
        lo2, (maps2, _) = ns.encode_chunks(auto, enc, hi, chunk=7, padding=p)
        assert np.array_equal(lo2, want_lo) and all(np.array_equal(a, c) for a, c in zip(maps2, want_maps))
        path = str(tmp_path / 'auto.kmp')
        kom.container.compress(path, hi, auto)
        assert kom.container.load(path)[2]['predictor']['arith'] == want
        assert np.array_equal(kom.container.decompress(path), hi)
        assert np.array_equal(kom.container.decompress(path, predictor=explicit), hi)
        other = 'f32' if want == 'bf16x2' else 'bf16x2'
        if dtype == np.uint16:
            with pytest.raises(AssertionError):
                kom.container.decompress(path, predictor=kom.LinearPredictor(w, b, p, ndim, arith=other))


# ---- the default p = 1 arithmetic against the f32 oracle: flip-bounded ----

def _smooth_c3(n, seed):
    """C3-geometry u16 tiles of smooth data (planes + noise): the predictor's realistic regime."""
    rng = np.random.default_rng(seed)
    z, y, x = np.meshgrid(np.arange(64), np.arange(64), np.arange(64), indexing='ij')
    hi = np.empty((n, 64, 64, 64, 1), np.uint16)
    for t in range(n):
        a = rng.uniform(-60, 60, 3)
        hi[t, ..., 0] = np.clip(30000 + a[0] * z + a[1] * y + a[2] * x + rng.normal(0, 30, z.shape), 0, 65535)
    return hi


FLIP_CASES = ['golden:vol_tile64_p1', 'smooth_c3', 'golden:vol_ramp_even_p1', 'golden:vol_rand_mixed_p1',
              'golden:vol_tile_small_p1', 'golden:vol_ramp_odd_p1',
              # uint8 volumes (the default is bf16x2 there too since round 6)
              'golden:vol_fast_u8_p1', 'golden:vol_rand_u8_c3_p1', 'smooth_c3_u8', 'rand_c3_u8']


@pytest.mark.parametrize('case', FLIP_CASES)
def test_linear_auto_p1_flips_vs_f32_oracle(kom, case):
    """The default arithmetic for u8 / u16 volumes at padding 1 (arith='auto' -> bf16x2, the matrix
    cores) against the oracle's f32 fma chain, on C3 tiles and the golden p = 1 inputs:
      * a cell prediction differs only by +-1, and only where the float64 value lies within the north
        star's 1e-5 (relative to sum|f w| + |b|) of the integer boundary the two truncations straddle;
      * a residual differs from the oracle's f32 residual only by +-1 mod 2^bits, and only at a position
        whose aggregation (maps_from_predictions) takes a flipped cell;
      * the mismatch rates are printed (run with -s), and the round trip is lossless."""
    from conftest import GOLDEN
    V, OV = kom.volume, oracle.volume
    if case.startswith('golden:'):
        hi = np.load(f'{GOLDEN}/{case[7:]}.npz')['highres']
    elif case == 'smooth_c3':
        hi = _smooth_c3(2, 31)
    elif case == 'smooth_c3_u8':
        hi = (_smooth_c3(2, 32) >> 8).astype(np.uint8)
    else:
        hi = _data((2, 64, 64, 64, 1), np.uint8, 33)
    dt = hi.dtype.type
    mod = np.iinfo(dt).max + 1
    w, b = _weights(3, 1, 21, dt)
    auto = kom.LinearPredictor(w, b, 1, 3)
    assert auto.arith_for(torch.from_numpy(hi[:0]).dtype) == 'bf16x2'
    enc, dec, oenc = ((V.encode_values_uint16, V.decode_values_uint16, OV.encode_values_uint16) if dt == np.uint16
                      else (V.encode_values_uint8, V.decode_values_uint8, OV.encode_values_uint8))
    lo, (maps, dims) = V.encode(auto, enc, hi, padding=1)
    if hi.shape[1:] == (64, 64, 64, 1):
        assert kom._lib.lib.kmp_last_launch().decode() == 'linear3pm_encode'
    want_lo, (want_maps, want_dims) = OV.encode(OP.linear_predictions_fn(1, w, b, 3), oenc, hi, padding=1)
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    # cells
    window = OV.pad_neighborhood(OV.lowres_from_highres(OV.pad_highres(hi)[0]), 1)
    feats = OV.features_from_lowres(window, 1)
    o_cells = OP.cast_from_f32(OP.linear_fma_chain(feats, w, b), dt)
    h_cells, h_f32 = auto.predict_cells(window, with_f32=True)
    f64, _ = OP.linear_predictions(feats, w, b, dt)
    scale = np.tensordot(np.moveaxis(np.abs(feats.astype(np.float64)), 4, -1), np.abs(w.astype(np.float64)),
                         axes=([-1], [0]))
    scale = np.moveaxis(scale, -1, 4) + np.abs(b).reshape(-1, 1)
    flips = h_cells != o_cells
    d = h_cells.astype(np.int64) - o_cells.astype(np.int64)
    assert np.all(np.abs(d[flips]) == 1), np.unique(d[flips])
    boundary = np.maximum(h_cells, o_cells).astype(np.float64)
    dist = np.abs(f64 - boundary)
    assert np.all(dist[flips] <= 1e-5 * scale[flips]), np.max(dist[flips] / scale[flips]) if flips.any() else 0
    # residuals
    touched = OV.trim_maps(OV.maps_from_predictions(flips.astype(np.float32)), dims)
    nbad = ntot = 0
    for i, (a, c, t) in enumerate(zip(maps, want_maps, touched)):
        bad = a != c
        dd = (a.astype(np.int64) - c.astype(np.int64)) % mod
        assert np.all((dd[bad] == 1) | (dd[bad] == mod - 1)), f'map {i}: {np.unique(dd[bad])}'
        assert np.all(t[bad] > 0), f'map {i}: a residual mismatch with no flipped cell in its aggregation'
        nbad += int(bad.sum())
        ntot += bad.size
    print(f'\n[flip-rate {case}] cells {int(flips.sum())} / {flips.size} = {flips.mean():.3e}; '
          f'residuals {nbad} / {ntot} = {nbad / ntot:.3e}')
    assert np.array_equal(V.decode(auto, dec, lo, (maps, dims), padding=1), hi)


def test_linear_bf16x2_golden(kom):
    """The bf16x2 arithmetic's exact bits at the current revision (predictors.ARITH_REV), pinned by
    GPU-generated fixtures (tests/golden/make_bf16x2_golden.py): any change of how the products are
    grouped into MFMAs changes maps / cell values and fails here, so it must come with a revision
    bump (files record the revision and refuse a mismatch)."""
    import importlib.util
    from conftest import GOLDEN
    from kompressor_amd.predictors import ARITH_REV
    spec = importlib.util.spec_from_file_location('make_bf16x2_golden', f'{GOLDEN}/make_bf16x2_golden.py')
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    rev = ARITH_REV['bf16x2']
    with np.load(f'{GOLDEN}/bf16x2_r{rev}.npz', allow_pickle=False) as g:
        assert int(g['arith_rev']) == rev
        for i, (name, ndim, p, shape, dtype) in enumerate(mk.CASES):
            # the default dispatch (fused kernels where they apply) and the generic MFMA kernel
            for generic in (0, 1):
                with kom._lib.option('KMP_DISABLE_LINEAR_FUSED', generic):
                    dims, maps, sha, launch = mk.run_case(kom, ndim, p, shape, dtype, 500 + i)
                assert np.array_equal(dims, g[f'{name}/dims'])
                for j, m in enumerate(maps):
                    want = g[f'{name}/map{j}']
                    assert np.array_equal(m, want), f'{name} ({launch}) map {j}: {np.count_nonzero(m != want)} mismatches'
                assert sha == str(g[f'{name}/cells_sha256']), f'{name}: f32 cell values changed'
