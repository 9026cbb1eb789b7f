"""HIP codec parity: fused one-pass kernels, the generic two-pass kernels and the reference-style
callback path, all bit-exact against the oracle's golden fixtures (tests/golden/)."""

import os

import numpy as np
import pytest
import torch

from conftest import golden_names, load_golden, golden_maps

pytestmark = pytest.mark.gpu

CODEC_CASES = [n for n in golden_names() if n.startswith(('vol_', 'img_')) and 'categorical' not in n]


def _ns(kom, ndim):
    return kom.volume if ndim == 3 else kom.image


def _coders(ns, coder):
    return {'uint8': (ns.encode_values_uint8, ns.decode_values_uint8),
            'uint16': (ns.encode_values_uint16, ns.decode_values_uint16),
            'raw': (ns.encode_values_raw, ns.decode_values_raw)}[str(coder)]


def _assert_encoded(g, lowres, maps, dims, ndim):
    assert tuple(int(d) for d in dims) == tuple(int(d) for d in g['dims'])
    lowres = lowres.cpu().numpy() if isinstance(lowres, torch.Tensor) else lowres
    assert lowres.dtype == g['lowres'].dtype and np.array_equal(lowres, g['lowres'])
    for i, (m, ref) in enumerate(zip(maps, golden_maps(g, ndim))):
        m = m.cpu().numpy() if isinstance(m, torch.Tensor) else m
        assert m.shape == ref.shape, (i, m.shape, ref.shape)
        assert m.dtype == ref.dtype, (i, m.dtype, ref.dtype)
        bad = np.argwhere(m != ref)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'


@pytest.fixture(params=['fast', 'generic'])
def kernel_mode(request, kmp_opt):
    # 'fast' lets the C layer pick the one-pass kernel where eligible; 'generic' forces the
    # two-pass kernels (kmp_codec_generic.hip) for every shape.
    kmp_opt('KMP_DISABLE_FAST', 1 if request.param == 'generic' else None)
    return request.param


@pytest.mark.parametrize('name', CODEC_CASES)
def test_fused_codec_matches_golden(kom, name, kernel_mode):
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns = _ns(kom, ndim)
    enc, dec = _coders(ns, g['coder'])
    pred = kom.MeanPredictor(p, ndim)
    lowres, (maps, dims) = ns.encode(pred, enc, g['highres'], padding=p)
    _assert_encoded(g, lowres, maps, dims, ndim)
    rec = ns.decode(pred, dec, g['lowres'], (golden_maps(g, ndim), tuple(g['dims'])), padding=p)
    assert rec.dtype == g['highres'].dtype and np.array_equal(rec, g['highres'])


@pytest.mark.parametrize('name', [n for n in CODEC_CASES if 'tile64' not in n and 'tile256' not in n])
@pytest.mark.parametrize('coders', ['builtin', 'opaque'])
def test_callback_path_matches_golden(kom, name, coders):
    """Callback path: the predictor is an opaque callable (no fused kernel).  With the built-in
    coder the steps around it run as the fused window / coder kernels (kmp_callback.hip); with an
    opaque coder too, exactly the reference's step sequence on HIP primitives."""
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns = _ns(kom, ndim)
    enc, dec = _coders(ns, g['coder'])
    if coders == 'opaque':
        enc0, dec0 = enc, dec
        enc = lambda a, b: enc0(a, b)  # noqa: E731
        dec = lambda a, b: dec0(a, b)  # noqa: E731
    mean = kom.MeanPredictor(p, ndim)
    opaque = lambda lowres: mean(lowres)  # noqa: E731
    lowres, (maps, dims) = ns.encode(opaque, enc, g['highres'], padding=p)
    last = kom._lib.lib.kmp_last_launch().decode()
    assert (last == 'encode_with_predictions') == (coders == 'builtin'), last
    _assert_encoded(g, lowres, maps, dims, ndim)
    rec = ns.decode(opaque, dec, lowres, (maps, dims), padding=p)
    assert np.array_equal(rec, g['highres'])


@pytest.mark.parametrize('name', ['vol_rand_mixed_p1', 'img_rand_p2', 'vol_ramp_odd_p0', 'img_ramp_even_p1'])
def test_callback_window_is_the_reference_window(kom, name):
    """predictions_fn receives exactly pad_neighborhood(lowres_from_highres(pad_highres(h)), p) on
    encode and pad_neighborhood(pad_lowres(lowres, dims), p) on decode (the fused windows)."""
    import oracle
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns, ons = _ns(kom, ndim), (oracle.volume if ndim == 3 else oracle.image)
    enc, dec = _coders(ns, g['coder'])
    mean = kom.MeanPredictor(p, ndim)
    seen = []

    def fn(window):
        seen.append(window.cpu().numpy())
        return mean(window)

    lowres, (maps, dims) = ns.encode(fn, enc, torch.from_numpy(g['highres']).cuda(), padding=p)
    hp, _ = ons.pad_highres(g['highres'])
    assert np.array_equal(seen[0], ons.pad_neighborhood(ons.lowres_from_highres(hp), p))
    ns.decode(fn, dec, lowres, (maps, dims), padding=p)
    assert np.array_equal(seen[1], ons.pad_neighborhood(ons.pad_lowres(g['lowres'], tuple(g['dims'])), p))


def reference_style_predictions_fn(kom, padding, ndim):
    """The reference test's dummy predictor (tests/volume/test_encode_decode.py:43-55) written
    against kompressor_amd + torch: features -> f32 mean -> cast -> repeat -> maps."""
    ns = _ns(kom, ndim)
    k = 19 if ndim == 3 else 5

    def fn(lowres):
        features = ns.features_from_lowres(lowres, padding)
        mean = torch.mean(features.to(torch.int32).to(torch.float32), dim=ndim + 1, keepdim=True)
        pred = mean.to(torch.int32).repeat_interleave(k, dim=ndim + 1)
        pred = kom._nd.d_cast(pred.contiguous(), lowres.dtype, ndim)
        return ns.maps_from_predictions(pred)

    return fn


@pytest.mark.parametrize('name', ['vol_ramp_odd_p0', 'vol_ramp_even_p1', 'vol_rand_mixed_p1', 'img_ramp_odd_p1',
                                  'img_rand_p0', 'vol_ramp_i32_raw_p0'])
def test_reference_style_predictor(kom, name):
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns = _ns(kom, ndim)
    enc, dec = _coders(ns, g['coder'])
    fn = reference_style_predictions_fn(kom, p, ndim)
    hi = torch.from_numpy(g['highres']).cuda()
    lowres, (maps, dims) = ns.encode(fn, enc, hi, padding=p)
    assert isinstance(lowres, torch.Tensor) and lowres.is_cuda
    _assert_encoded(g, lowres, maps, dims, ndim)
    rec = ns.decode(fn, dec, lowres, (maps, dims), padding=p)
    assert torch.equal(rec.cpu(), hi.cpu())


def float_predictions_fn(kom, padding, ndim, seen, special=True):
    """A network-like predictor: float32 maps that are not integers -- fractional, negative, past
    the sample range, and (``special``) a few +-inf / NaN / beyond-int32 entries placed by flat
    index, so not translation-invariant -- recorded in ``seen``."""
    ns = _ns(kom, ndim)
    k = 19 if ndim == 3 else 5

    def fn(lowres):
        features = ns.features_from_lowres(lowres, padding).to(torch.float32)
        pred = torch.mean(features, dim=ndim + 1, keepdim=True) * 1.37 - 40.25
        pred = pred.repeat_interleave(k, dim=ndim + 1)
        pred = pred + torch.linspace(-3.7, 2.9, k, device=pred.device).reshape(
            *([1] * (ndim + 1)), k, *([1] * (pred.dim() - ndim - 2)))
        if special:
            flat = pred.view(-1)
            flat[::97] = float('nan')
            flat[5::131] = float('inf')
            flat[7::151] = -float('inf')
            flat[11::173] = 3.5e9
            flat[13::179] = -3.5e9
        maps = ns.maps_from_predictions(pred.contiguous())
        seen.append([m.cpu().numpy() for m in maps])
        return maps

    return fn


@pytest.mark.parametrize('name', ['vol_rand_mixed_p1', 'vol_ramp_odd_p0', 'vol_rand_u8_c3_p1', 'vol_ramp_i32_raw_p0',
                                  'img_rand_p2', 'img_ramp_even_p1', 'img_rand_u16_c2_p1', 'vol_tile_small_p0'])
@pytest.mark.parametrize('rows', ['1', '0'])
def test_callback_float32_predictions(kom, name, rows, kmp_opt):
    """A predictions_fn returning float32 maps (what a trained network gives) with the built-in coder
    stays on the fused callback coder (kmp_*_with_predictions_typed): residuals bit-exact to the
    oracle's step sequence on the same maps (the coder reads jnp.int32(pred): truncating, saturating,
    NaN -> 0), and lossless.  rows=0: the per-element kernel instead of the 16-byte row kernel."""
    import oracle
    kmp_opt('KMP_DISABLE_ROWS', 1 if rows == '0' else None)
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns, ons = _ns(kom, ndim), (oracle.volume if ndim == 3 else oracle.image)
    enc, dec = _coders(ns, g['coder'])
    oenc = getattr(oracle.common, f"encode_values_{g['coder']}")
    odec = getattr(oracle.common, f"decode_values_{g['coder']}")
    seen = []
    fn = float_predictions_fn(kom, p, ndim, seen)
    hi = torch.from_numpy(g['highres']).cuda()
    lowres, (maps, dims) = ns.encode(fn, enc, hi, padding=p)
    assert kom._lib.lib.kmp_last_launch().decode() == 'encode_with_predictions'
    assert seen[0][0].dtype == np.float32
    want_lo, (want_maps, want_dims) = ons.encode(lambda w: seen[0], oenc, g['highres'], padding=p)
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lowres.cpu().numpy(), want_lo)
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        a = a.cpu().numpy()
        assert a.dtype == b.dtype and a.shape == b.shape, i
        bad = np.argwhere(a != b)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'
    rec = ns.decode(fn, dec, lowres, (maps, dims), padding=p)
    assert kom._lib.lib.kmp_last_launch().decode() == 'decode_with_predictions'
    assert torch.equal(rec.cpu(), hi.cpu())
    orec = ons.decode(lambda w: seen[1], odec, want_lo, (want_maps, want_dims), padding=p)
    assert np.array_equal(orec, g['highres'])
    # the chunked drivers call predictions_fn per chunk window: chunk invariance needs a predictor of
    # the neighbourhood alone, so the one without the index-placed special values
    local = float_predictions_fn(kom, p, ndim, [], special=False)
    lo1, (maps1, dims1) = ns.encode(local, enc, hi, padding=p)
    lo2, (maps2, _) = ns.encode_chunks(local, enc, hi, chunk=5, padding=p)
    assert torch.equal(lo2, lo1)
    for i, (a, b) in enumerate(zip(maps2, maps1)):
        assert torch.equal(a, b), f'chunked map {i}'
    assert torch.equal(ns.decode_chunks(local, dec, lo1, (maps1, dims1), chunk=(6, 7) if ndim == 2 else 6,
                                        padding=p), hi)


@pytest.mark.parametrize('name,chunk', [('vol_ramp_odd_p0', 6), ('vol_ramp_odd_p1', 11), ('vol_ramp_odd_p1', (6, 11, 11)),
                                        ('vol_ramp_even_p0', 6), ('vol_rand_mixed_p2', 7), ('vol_tile64_p0', 12),
                                        ('img_ramp_odd_p0', (6, 11)), ('img_ramp_even_p1', 6), ('img_rand_p2', 9)])
@pytest.mark.parametrize('fused', [True, False])
def test_chunks_match_golden(kom, name, chunk, fused):
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns = _ns(kom, ndim)
    enc, dec = _coders(ns, g['coder'])
    mean = kom.MeanPredictor(p, ndim)
    pred = mean if fused else (lambda x: mean(x))
    seen = []

    def progress(chunks):
        seen.append(len(chunks))
        return chunks

    lowres, (maps, dims) = ns.encode_chunks(pred, enc, g['highres'], chunk=chunk, padding=p, progress_fn=progress)
    _assert_encoded(g, lowres, maps, dims, ndim)
    rec = ns.decode_chunks(pred, dec, lowres, (maps, dims), chunk=chunk, padding=p, progress_fn=progress)
    assert np.array_equal(rec, g['highres'])
    assert len(seen) == 2 and seen[0] == seen[1] > 0


def test_metric_volume_round_trip_full_size(kom):
    """BASELINE config C3 at full size: 512^3 uint16 as 512 tiles of 64^3, encode -> decode is
    lossless, and a 4-tile slice matches the oracle bit for bit."""
    import oracle
    from oracle import predictors as OP
    rng = np.random.default_rng(0)
    vol = torch.from_numpy(rng.integers(0, 65536, size=(512, 64, 64, 64, 1), dtype=np.int64).astype(np.uint16)).cuda()
    pred = kom.MeanPredictor(0, 3)
    lowres, (maps, dims) = kom.volume.encode(pred, kom.volume.encode_values_uint16, vol)
    assert dims == (1, 1, 1) and tuple(lowres.shape) == (512, 32, 32, 32, 1)
    rec = kom.volume.decode(pred, kom.volume.decode_values_uint16, lowres, (maps, dims))
    assert torch.equal(rec, vol)
    sl = slice(100, 104)
    ref_lo, (ref_maps, _) = oracle.volume.encode(OP.mean_predictions_fn(0, 3), oracle.volume.encode_values_uint16,
                                                 vol[sl].cpu().numpy())
    assert np.array_equal(lowres[sl].cpu().numpy(), ref_lo)
    for m, r in zip(maps, ref_maps):
        assert np.array_equal(m[sl].cpu().numpy(), r)


def test_image_batch_round_trip_full_size(kom):
    """BASELINE config C2 at full size: 1024 x 256^2 uint8 tiles round-trip losslessly."""
    rng = np.random.default_rng(0)
    img = torch.from_numpy(rng.integers(0, 256, size=(1024, 256, 256, 1), dtype=np.int64).astype(np.uint8)).cuda()
    pred = kom.MeanPredictor(0, 2)
    lowres, (maps, dims) = kom.image.encode(pred, kom.image.encode_values_uint8, img)
    rec = kom.image.decode(pred, kom.image.decode_values_uint8, lowres, (maps, dims))
    assert torch.equal(rec, img)


@pytest.mark.parametrize('ndim,padding', [(3, 0), (3, 1), (2, 0), (2, 2)])
def test_empty_batch_is_rejected_like_the_reference(kom, ndim, padding):
    """A batch of zero tiles: the reference's validators reject it (``assert np.prod(shape) > 0``,
    volume/utils.py:284-303, image/utils.py:201-218) and so does every path here -- fused and
    callback, encode and decode, numpy and CUDA inputs -- with AssertionError, before any launch."""
    import oracle
    from oracle import predictors as OP
    ns, ons = _ns(kom, ndim), (oracle.volume if ndim == 3 else oracle.image)
    shape = (0, 9, 13, 17, 1) if ndim == 3 else (0, 13, 17, 1)
    lo_shape = (0, 5, 7, 9, 1) if ndim == 3 else (0, 7, 9, 1)
    x = np.zeros(shape, np.uint16)
    with pytest.raises(AssertionError):
        ons.encode(OP.mean_predictions_fn(padding, ndim), ons.encode_values_uint16, x, padding=padding)
    mean = kom.MeanPredictor(padding, ndim)
    for pred in (mean, lambda w: mean(w)):
        for arr in (x, torch.from_numpy(x).cuda()):
            with pytest.raises(AssertionError):
                ns.encode(pred, ns.encode_values_uint16, arr, padding=padding)
        lo = torch.zeros(lo_shape, dtype=torch.uint16, device='cuda')
        with pytest.raises(AssertionError):
            ns.decode(pred, ns.decode_values_uint16, lo, ([lo] * (7 if ndim == 3 else 3), (0,) * ndim),
                      padding=padding)


@pytest.mark.parametrize('ndim', [3, 2])
@pytest.mark.parametrize('path', ['fused', 'callback'])
def test_batch_past_int32_elements(kom, ndim, path):
    """More than 2^31 samples in one call (17 tiles of 512^3 uint16; 33 000 images of 256^2 uint8):
    the batch offsets are 64-bit, on the fused kernels and on the callback path (window gather, an
    opaque predictions_fn, the coder kernels' 64-bit form).  Lossless, and the last tile -- past
    element 2^31 -- codes exactly as it does alone (single tiles are pinned to the oracle by the
    golden tests)."""
    ns = _ns(kom, ndim)
    if ndim == 3:
        B, tile, dt, enc, dec = 17, (512, 512, 512, 1), torch.uint16, ns.encode_values_uint16, ns.decode_values_uint16
        hi = 65536
    else:
        B, tile, dt, enc, dec = 33000, (256, 256, 1), torch.uint8, ns.encode_values_uint8, ns.decode_values_uint8
        hi = 256
    x = torch.empty((B, *tile), dtype=dt, device='cuda')
    g = torch.Generator(device='cuda').manual_seed(7)
    step = 1 if ndim == 3 else 4096
    for i in range(0, B, step):  # int32 draws a chunk at a time (the uint16 / uint8 batch is 4.6 / 2.2 GB)
        x[i:i + step] = torch.randint(0, hi, (min(step, B - i), *tile), generator=g, dtype=torch.int32,
                                      device='cuda').to(dt)
    assert x.numel() > (1 << 31)
    mean = kom.MeanPredictor(0, ndim)
    pred = mean if path == 'fused' else (lambda w: mean(w))
    lo, (maps, dims) = ns.encode(pred, enc, x)
    assert (kom._lib.lib.kmp_last_launch().decode() == 'encode_with_predictions') == (path == 'callback')
    lo1, (maps1, dims1) = ns.encode(pred, enc, x[B - 1:].clone())
    assert tuple(dims) == tuple(dims1) and torch.equal(lo[B - 1:], lo1)
    for m, m1 in zip(maps, maps1):
        assert torch.equal(m[B - 1:], m1)
    del lo1, maps1
    rec = ns.decode(pred, dec, lo, (maps, dims))
    assert torch.equal(rec, x)


def categorical_predictions_fn(kom, logits, padding, ndim):
    """tests/volume/test_encode_decode.py:57-75 with the fixture's logits: constant logits tiled
    over every cell, maps_from_predictions (HIP, float32), softmax (torch)."""
    ns = _ns(kom, ndim)
    lg = torch.from_numpy(logits).cuda()

    def fn(lowres):
        cells = [s - 1 - 2 * padding for s in lowres.shape[1:1 + ndim]]
        pred = lg.expand(lowres.shape[0], *cells, *lg.shape).contiguous()
        return [torch.softmax(m, dim=-1).contiguous() for m in ns.maps_from_predictions(pred)]

    return fn


@pytest.mark.parametrize('name', ['vol_categorical_p0', 'img_categorical_p1'])
@pytest.mark.parametrize('chunk', [None, 6])
def test_categorical_matches_golden(kom, name, chunk):
    g = load_golden(name)
    ndim, p = int(g['ndim']), int(g['padding'])
    ns = _ns(kom, ndim)
    fn = categorical_predictions_fn(kom, g['logits'], p, ndim)
    hi = torch.from_numpy(g['highres']).cuda()
    if chunk is None:
        lowres, (maps, dims) = ns.encode(fn, ns.encode_categorical, hi, padding=p)
    else:
        lowres, (maps, dims) = ns.encode_chunks(fn, ns.encode_categorical, hi, chunk=chunk, padding=p)
    _assert_encoded(g, lowres, maps, dims, ndim)
    rec = ns.decode(fn, ns.decode_categorical, lowres, (maps, dims), padding=p)
    assert torch.equal(rec, hi)
    rec = ns.decode_chunks(fn, ns.decode_categorical, lowres, (maps, dims), chunk=6, padding=p)
    assert torch.equal(rec, hi)


@pytest.mark.parametrize('vec', ['1', '0'])
def test_categorical_coder_vs_oracle(kom, vec):
    """Rank coder vs the oracle's stable argsort.  vec='1': 16-byte-aligned logits, so L % 4 == 0,
    L <= 512 runs the vector kernels and the other L the scalar ones; vec='0': the logits start 4
    bytes past a 16-byte boundary, which sends every L to the scalar kernels."""
    import oracle
    rng = np.random.default_rng(7)
    for L, dt in ((256, np.uint8), (300, np.uint8), (17, np.uint16), (2000, np.uint16), (5, np.int32),
                  (64, np.uint8), (128, np.uint16), (512, np.uint16), (1, np.uint8), (2, np.uint8),
                  (65, np.uint8), (511, np.uint16), (-200, np.uint8), (-500, np.uint16), (4, np.uint32),
                  (260, np.uint8), (8, np.uint8), (256, np.int32)):
        heavy_ties = L < 0  # few distinct values: long runs of equal keys ordered by class index
        L = abs(L)
        logits = rng.standard_normal((513, L)).astype(np.float32)
        if heavy_ties:
            logits = rng.integers(0, 3, size=(513, L)).astype(np.float32)
        if L > 3:
            logits[::7, 3] = logits[::7, 1]  # ties
        if L > 4:
            logits[5, :] = 0.5          # an all-tie row
            logits[6, :4] = [np.nan, -0.0, 0.0, np.nan]      # NaN after every number, -0 == +0
            logits[7, :4] = [np.inf, -np.inf, np.nan, np.inf]
        x = rng.integers(0, min(L + 3, np.iinfo(dt).max), size=513).astype(dt)
        x[::3] = rng.integers(0, min(L, 10), size=x[::3].size)  # small ranks / classes (the peel)
        lg = torch.from_numpy(logits).cuda()
        if vec == '0':
            buf = torch.empty(logits.size + 4, dtype=torch.float32, device='cuda')
            lg = buf[1:1 + logits.size].view(logits.shape)
            lg.copy_(torch.from_numpy(logits))
            assert lg.data_ptr() % 16 == 4
        xg = torch.from_numpy(x).cuda()
        got = kom.utils.encode_categorical(lg, xg).cpu().numpy()
        want = oracle.common.encode_categorical(logits, x)
        assert np.array_equal(got, want), L
        got = kom.utils.decode_categorical(lg, xg).cpu().numpy()
        want = oracle.common.decode_categorical(logits, x)
        assert np.array_equal(got, want), L
    # non-negative logits (softmax output: the decode's raw-bits key path), with +0, +inf, ties, and
    # rows that fall back to the order key (-0, a negative, NaN)
    for L, dt in ((256, np.uint8), (512, np.uint16), (64, np.uint8), (300, np.uint16), (4, np.uint8),
                  (260, np.uint8), (252, np.uint8)):
        logits = rng.random((513, L)).astype(np.float32)
        logits[::5] = np.exp(logits[::5] * 8) / np.exp(logits[::5] * 8).sum(axis=1, keepdims=True)
        logits[1, :2] = [0.0, np.inf]
        logits[2, :] = 0.0
        logits[3, :3] = [-0.0, 0.0, 0.25]
        logits[4, 1] = -1.0
        logits[8, 2] = np.nan
        logits[::9, L // 2] = logits[::9, 0]  # ties
        x = rng.integers(0, min(L + 3, np.iinfo(dt).max), size=513).astype(dt)
        x[::3] = rng.integers(0, min(L, 10), size=x[::3].size)
        lg, xg = torch.from_numpy(logits).cuda(), torch.from_numpy(x).cuda()
        if vec == '0':
            buf = torch.empty(logits.size + 4, dtype=torch.float32, device='cuda')
            lg = buf[1:1 + logits.size].view(logits.shape)
            lg.copy_(torch.from_numpy(logits))
        assert np.array_equal(kom.utils.encode_categorical(lg, xg).cpu().numpy(),
                              oracle.common.encode_categorical(logits, x)), L
        assert np.array_equal(kom.utils.decode_categorical(lg, xg).cpu().numpy(),
                              oracle.common.decode_categorical(logits, x)), L


@pytest.mark.parametrize('dt', [np.uint8, np.uint16])
@pytest.mark.parametrize('off', [1, 2, 3])
def test_categorical_value_offsets(kom, dt, off):
    """Values (classes / ranks) that start off elements past an aligned address and end at their
    buffer's last element: the vector kernels read each value as the aligned dword that holds it
    and shift it out (cat_xval), so every byte position inside the dword is exercised, on both
    directions and on the peel and radix paths of the decode."""
    import oracle
    n, L = 2053, 256
    rng = np.random.default_rng(19 + off)
    logits = rng.random((n, L)).astype(np.float32)
    logits[::4] = rng.standard_normal((logits[::4].shape[0], L)).astype(np.float32)
    x = rng.integers(0, L, n).astype(dt)
    x[::2] = rng.integers(0, 4, x[::2].size)  # small ranks: the peel
    lg = torch.from_numpy(logits).cuda()
    # the values end at the buffer's last element (the kernels read the aligned dword around each one)
    buf = torch.zeros(off + n, dtype=torch.uint8 if dt == np.uint8 else torch.int16, device='cuda')
    xg = buf[off:]
    xg.copy_(torch.from_numpy(x.view(np.int16) if dt == np.uint16 else x))
    if dt == np.uint16:
        xg = xg.view(torch.uint16)
    assert np.array_equal(kom.utils.encode_categorical(lg, xg).cpu().numpy().astype(dt),
                          oracle.common.encode_categorical(logits, x))
    assert np.array_equal(kom.utils.decode_categorical(lg, xg).cpu().numpy().astype(dt),
                          oracle.common.decode_categorical(logits, x))


@pytest.mark.parametrize('L,dt,rows', [(8, np.uint8, None), (8, np.uint16, None), (12, np.int32, None),
                                       (260, np.uint16, 3000), (256, np.uint8, 3000)])
def test_categorical_long_ranges(kom, L, dt, rows):
    """Enough elements that every wave of the vector kernels codes a long contiguous range (8 192
    waves x 139 elements, the last range ragged): whole batches of 64 values and codes, whole
    prefetch rounds, and a tail of 3.  Small L: every element vs the oracle; large L: all elements
    through the round trip and `rows` sampled elements (with every range's first and last) vs the
    oracle."""
    import oracle
    n = 8192 * 139 - 5
    rng = np.random.default_rng(11)
    lg = torch.rand((n, L), device='cuda')
    lg[::11, 1] = lg[::11, 0]  # ties
    lg[::13] = torch.softmax(lg[::13] * 8, dim=1)
    xh = rng.integers(0, L, n).astype(dt)
    xg = torch.from_numpy(xh).cuda()
    enc = kom.utils.encode_categorical(lg, xg)
    dec = kom.utils.decode_categorical(lg, enc).cpu().numpy()
    assert np.array_equal(dec, xh)  # every x < L <= 2^bits: decode inverts encode
    if rows is None:
        idx = np.arange(n)
    else:
        ends = np.arange(0, n, 139)
        idx = np.unique(np.concatenate([ends, np.minimum(ends + 138, n - 1), rng.integers(0, n, rows)]))
    lh = lg[torch.from_numpy(idx).cuda()].cpu().numpy()
    assert np.array_equal(enc.cpu().numpy()[idx], oracle.common.encode_categorical(lh, xh[idx]))
    r = rng.integers(0, L, n).astype(dt)  # uniform ranks
    rd = kom.utils.decode_categorical(lg, torch.from_numpy(r).cuda()).cpu().numpy()
    assert np.array_equal(rd[idx], oracle.common.decode_categorical(lh, r[idx]))


@pytest.mark.parametrize('shape,dtype,p', [
    ((1, 6, 8, 512, 1), np.uint16, 0),    # 64 lanes per output row: one-row waves (both halos)
    ((2, 7, 5, 512, 1), np.uint16, 0),    # odd depth / height
    ((1, 5, 6, 1024, 1), np.uint8, 0),
    ((1, 9, 9, 512, 1), np.uint16, 1),    # p = 1 on a wide row (fast3d / generic)
    ((2, 9, 1024, 1), np.uint8, 0),       # images, one-row waves
    ((3, 10, 512, 1), np.uint16, 0),
    ((2, 11, 512, 1), np.uint16, 0),
])
def test_wide_rows_match_oracle(kom, shape, dtype, p):
    """Wide volumes / images (a whole 512^3 volume as ONE array has 256 outputs per row)."""
    import oracle
    from oracle import predictors as OP
    ndim = len(shape) - 2
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    enc, dec, oenc = (ns.encode_values_uint16, ns.decode_values_uint16, ons.encode_values_uint16) \
        if dtype == np.uint16 else (ns.encode_values_uint8, ns.decode_values_uint8, ons.encode_values_uint8)
    x = np.random.default_rng(5).integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)
    want_lo, (want_maps, want_dims) = ons.encode(OP.mean_predictions_fn(p, ndim), oenc, x, padding=p)
    pred = kom.MeanPredictor(p, ndim)
    lo, (maps, dims) = ns.encode(pred, enc, x, padding=p)
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for a, b in zip(maps, want_maps):
        assert np.array_equal(a, b)
    assert np.array_equal(ns.decode(pred, dec, lo, (maps, dims), padding=p), x)


@pytest.mark.parametrize('ndim,shape,dtype,levels,p', [
    (3, (2, 33, 40, 36, 1), np.uint16, 3, 0),
    (3, (1, 64, 64, 64, 1), np.uint16, 2, 1),
    (2, (3, 130, 96, 1), np.uint8, 4, 0),
])
def test_pyramid_matches_oracle_composition(kom, ndim, shape, dtype, levels, p):
    """Multi-level pyramid (f-4): each level equals the oracle's encode of the previous lowres."""
    import oracle
    from oracle import predictors as OP
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    enc, dec, oenc = (ns.encode_values_uint16, ns.decode_values_uint16, ons.encode_values_uint16) \
        if dtype == np.uint16 else (ns.encode_values_uint8, ns.decode_values_uint8, ons.encode_values_uint8)
    x = np.random.default_rng(8).integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)
    pred = kom.MeanPredictor(p, ndim)
    lo, levels_out = ns.encode_pyramid(pred, enc, x, levels, padding=p)
    assert len(levels_out) == levels
    cur = x
    for maps, dims in levels_out:
        want_lo, (want_maps, want_dims) = ons.encode(OP.mean_predictions_fn(p, ndim), oenc, cur, padding=p)
        assert tuple(dims) == tuple(want_dims)
        for a, b in zip(maps, want_maps):
            assert np.array_equal(a, b)
        cur = want_lo
    assert np.array_equal(lo, cur)
    assert np.array_equal(ns.decode_pyramid(pred, dec, lo, levels_out, padding=p), x)


def _last_launch(kom):
    return kom._lib.lib.kmp_last_launch().decode()


@pytest.mark.parametrize('shape,dtype,p', [
    ((8, 12, 14, 64, 1), np.uint16, 1),    # Ey = 7 < rows: idle rows read mirrored rows
    ((8, 12, 14, 64, 1), np.uint16, 2),
    ((2, 17, 34, 32, 1), np.uint16, 2),    # odd depth, 16 rows per wave, Ey = 17
    ((3, 9, 40, 128, 1), np.uint16, 1),    # 16 lanes per row, 4 rows per wave
    ((8, 10, 20, 64, 1), np.uint8, 2),     # u8: 8 outputs per lane
    ((1, 6, 66, 16, 1), np.uint8, 1),      # one lane per row, 64 rows per wave, Ey = 33
    ((2, 7, 5, 32, 1), np.uint16, 2),      # odd height, rows beyond the volume
    ((1, 64, 64, 64, 1), np.uint16, 2),
])
@pytest.mark.parametrize('pl', [None, '1', '2'])
def test_wave_p12_matches_oracle(kom, shape, dtype, p, pl, kmp_opt):
    """The p = 1, 2 wave kernels (kmp_codec_wave3dp.hip) against the oracle, encode and decode, and
    chunked (z-region) launches: the default kernel per (p, dtype) -- the z-rolling kernel (runs of
    8 planes) for p = 2 with 16-bit samples, else the plane-block kernel -- and the plane-block
    kernel's two planes-per-workgroup forms (KMP_W3P_PL, where it serves); asserts the kernel served
    the call."""
    kernel = 'wave3dr' if p == 2 and dtype == np.uint16 else 'wave3dp'  # the default per (p, dtype)
    if pl is not None:
        if kernel == 'wave3dr':
            pytest.skip('KMP_W3P_PL applies to the plane-block kernel')
        kmp_opt('KMP_W3P_PL', int(pl))
    import oracle
    from oracle import predictors as OP
    ns, ons = kom.volume, oracle.volume
    enc, dec, oenc = (ns.encode_values_uint16, ns.decode_values_uint16, ons.encode_values_uint16) \
        if dtype == np.uint16 else (ns.encode_values_uint8, ns.decode_values_uint8, ons.encode_values_uint8)
    x = np.random.default_rng(11).integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)
    want_lo, (want_maps, want_dims) = ons.encode(OP.mean_predictions_fn(p, 3), oenc, x, padding=p)
    pred = kom.MeanPredictor(p, 3)
    lo, (maps, dims) = ns.encode(pred, enc, x, padding=p)
    assert _last_launch(kom) == kernel + '_encode'
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'
    assert np.array_equal(ns.decode(pred, dec, lo, (maps, dims), padding=p), x)
    assert _last_launch(kom) == kernel + '_decode'
    lo2, (maps2, _) = ns.encode_chunks(pred, enc, x, chunk=5, padding=p)
    assert np.array_equal(lo2, want_lo) and all(np.array_equal(a, b) for a, b in zip(maps2, want_maps))
    assert np.array_equal(ns.decode_chunks(pred, dec, lo, (maps, dims), chunk=(5, 7, 9), padding=p), x)


def _W2P_DEFAULT(p, dtype):
    """The image p = 1, 2 kernel the dispatcher picks without overrides."""
    return 'wave2dr'


@pytest.mark.parametrize('shape,dtype,p', [
    ((8, 256, 256, 1), np.uint8, 1),     # C2 geometry: 16 lanes per row, 4 rows per wave
    ((8, 256, 256, 1), np.uint8, 2),     # rows (4) < 2p+2: a lane holds both halo rows
    ((3, 33, 64, 1), np.uint8, 2),       # odd height, 16 rows per wave
    ((2, 30, 32, 1), np.uint16, 1),
    ((2, 31, 48, 1), np.uint16, 2),      # 6 lanes per row is not a power of two: the LDS kernel
    ((1, 20, 256, 1), np.uint16, 1),     # 2 rows per wave
    ((2, 9, 16, 1), np.uint8, 2),        # one lane per row, Ey = 5 < rows
    ((2, 67, 256, 1), np.uint8, 1),      # odd height, a partial last run; Ly < run + rows: the step loop
    ((2, 67, 256, 1), np.uint8, 2),
    ((2, 70, 128, 1), np.uint16, 2),
    ((2, 141, 256, 1), np.uint8, 1),     # runs of 8 unrolled steps (Ly >= run + rows), the last one partial
    ((2, 141, 256, 1), np.uint8, 2),
    ((2, 142, 128, 1), np.uint16, 1),    # 16-bit, 4 rows per wave, unrolled, partial last run
])
def test_wave2d_p12_matches_oracle(kom, shape, dtype, p):
    """The p = 1, 2 image wave kernel (kmp_codec_wave2dp.hip: y-rolling, runs of 32 rows per wave,
    the unrolled form where the run is 8 steps) against the oracle, whole-image and row-region
    (chunked) launches; asserts which kernel served the call."""
    import oracle
    from oracle import predictors as OP
    ns, ons = kom.image, oracle.image
    enc, dec, oenc = (ns.encode_values_uint16, ns.decode_values_uint16, ons.encode_values_uint16) \
        if dtype == np.uint16 else (ns.encode_values_uint8, ns.decode_values_uint8, ons.encode_values_uint8)
    x = np.random.default_rng(12).integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)
    want_lo, (want_maps, want_dims) = ons.encode(OP.mean_predictions_fn(p, 2), oenc, x, padding=p)
    pred = kom.MeanPredictor(p, 2)
    lo, (maps, dims) = ns.encode(pred, enc, x, padding=p)
    wave = (shape[2] // 2 // (8 // np.dtype(dtype).itemsize)) in (1, 2, 4, 8, 16, 32, 64)
    kern = _W2P_DEFAULT(p, dtype)
    assert _last_launch(kom) == (kern + '_encode' if wave else 'fast2d_encode')
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'
    assert np.array_equal(ns.decode(pred, dec, lo, (maps, dims), padding=p), x)
    assert _last_launch(kom) == (kern + '_decode' if wave else 'fast2d_decode')
    lo2, (maps2, _) = ns.encode_chunks(pred, enc, x, chunk=5, padding=p)
    assert np.array_equal(lo2, want_lo) and all(np.array_equal(a, b) for a, b in zip(maps2, want_maps))
    assert np.array_equal(ns.decode_chunks(pred, dec, lo, (maps, dims), chunk=(7, 9), padding=p), x)


@pytest.mark.parametrize('shape', [
    (8, 256, 256, 1),      # C2 geometry: 16 lanes per row, 4 rows per wave
    (3, 35, 64, 1),        # odd height: the last cell row is missing, Ey = 18, 16 rows per wave
    (2, 31, 128, 1),       # odd height, 8 lanes per row
    (4, 18, 32, 1),        # 2 lanes per row, Ey = 9 < 32 rows per wave
    (2, 9, 16, 1),         # one lane per row, Ey = 5 < rows
    (1, 40, 1024, 1),      # 64 lanes per row: the one-row wave (generic kernel only)
])
@pytest.mark.parametrize('mode', ['swar_dec', 'generic'])
def test_wave2d_u8_p0_matches_oracle(kom, shape, mode, kmp_opt):
    """The p = 0 uint8 image kernels of kmp_codec_wave2d.hip -- the SWAR decode (the default) and
    the generic per-cell form (KMP_DISABLE_SWAR) -- against the oracle, whole-image and chunked."""
    if mode == 'generic':
        kmp_opt('KMP_DISABLE_SWAR', 1)
    import oracle
    from oracle import predictors as OP
    ns, ons = kom.image, oracle.image
    x = np.random.default_rng(13).integers(0, 256, size=shape, dtype=np.int64).astype(np.uint8)
    want_lo, (want_maps, want_dims) = ons.encode(OP.mean_predictions_fn(0, 2), ons.encode_values_uint8, x)
    pred = kom.MeanPredictor(0, 2)
    lo, (maps, dims) = ns.encode(pred, ns.encode_values_uint8, x)
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'
    assert np.array_equal(ns.decode(pred, ns.decode_values_uint8, lo, (maps, dims)), x)
    lo2, (maps2, _) = ns.encode_chunks(pred, ns.encode_values_uint8, x, chunk=5)
    assert np.array_equal(lo2, want_lo) and all(np.array_equal(a, b) for a, b in zip(maps2, want_maps))
    assert np.array_equal(ns.decode_chunks(pred, ns.decode_values_uint8, lo, (maps, dims), chunk=(7, 9)), x)


@pytest.mark.parametrize('shape,dtype', [
    ((4, 16, 16, 16, 1), np.uint32),
    ((8, 9, 10, 32, 1), np.uint32),        # odd depth, 8 rows per wave
    ((1, 24, 28, 128, 1), np.uint32),      # 2 rows per wave (the C5 chunk geometry)
    ((3, 12, 14, 64, 1), np.int32),        # raw coder, negative samples
    ((8, 6, 7, 8, 1), np.int32),           # 2 lanes per row, odd height
])
def test_wave32_matches_oracle(kom, shape, dtype):
    """The 32-bit-sample wave kernel (kmp_codec_wave3d32.hip): float32 cell means and map
    aggregation in the reference's order are NOT exact for full-range 32-bit samples, so this pins
    the order against the oracle bit for bit; float32 bit patterns (C5) included."""
    import oracle
    from oracle import predictors as OP
    ns, ons = kom.volume, oracle.volume
    rng = np.random.default_rng(13)
    if dtype == np.uint32:
        x = rng.integers(0, 1 << 32, size=shape, dtype=np.uint64).astype(np.uint32)
        flat = x.reshape(-1)
        k = flat[::7].size
        flat[::7] = (rng.standard_normal(k) * 1e3).astype(np.float32).view(np.uint32)  # float32 bit patterns
        enc, dec, oenc = ns.encode_values_uint32, ns.decode_values_uint32, ons.encode_values_uint32
    else:
        x = rng.integers(-(1 << 31), 1 << 31, size=shape, dtype=np.int64).astype(np.int32)
        enc, dec, oenc = ns.encode_values_raw, ns.decode_values_raw, ons.encode_values_raw
    want_lo, (want_maps, want_dims) = ons.encode(OP.mean_predictions_fn(0, 3), oenc, x)
    pred = kom.MeanPredictor(0, 3)
    lo, (maps, dims) = ns.encode(pred, enc, x)
    assert _last_launch(kom) == 'wave3d32_encode'
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'
    assert np.array_equal(ns.decode(pred, dec, lo, (maps, dims)), x)
    assert _last_launch(kom) == 'wave3d32_decode'


def test_trace_ranges_do_not_change_results(kom, monkeypatch):
    """KMP_TRACE's roctx ranges wrap the same calls (SURVEY.md §5 tracing)."""
    monkeypatch.setattr(kom._trace, 'ENABLED', True)
    x = torch.randint(0, 65536, (2, 16, 16, 16, 1), dtype=torch.int32, device='cuda').to(torch.uint16)
    pred = kom.MeanPredictor(1, 3)
    cb = lambda w: pred(w)  # noqa: E731
    lo, enc = kom.volume.encode(cb, kom.volume.encode_values_uint16, x, padding=1)
    assert torch.equal(kom.volume.decode(cb, kom.volume.decode_values_uint16, lo, enc, padding=1), x)
    lo2, enc2 = kom.volume.encode_chunks(pred, kom.volume.encode_values_uint16, x, chunk=6, padding=1)
    assert torch.equal(lo2, lo)


@pytest.mark.parametrize('case', [
    ('KMP_W3_ST_ENC', (2, 64, 64, 64, 1), np.uint16, 0, 'wave3d'),   # the metric kernel
    ('KMP_W2_ST_ENC', (3, 256, 256, 1), np.uint8, 0, 'wave2d'),
    ('KMP_W3P_ST_ENC', (2, 20, 24, 32, 1), np.uint16, 1, 'wave3d'),  # wave3dp / wave3dr
    ('KMP_W3P_ST_ENC', (2, 20, 24, 32, 1), np.uint16, 2, 'wave3d'),
    ('KMP_W2P_ST_ENC', (3, 40, 128, 1), np.uint8, 1, 'wave2d'),      # wave2dp / wave2dr
    ('KMP_W2P_ST_ENC', (3, 40, 128, 1), np.uint16, 2, 'wave2d'),
])
@pytest.mark.parametrize('cached', ['0', '1'])
def test_encode_store_policy_is_output_neutral(kom, case, cached, kmp_opt):
    """The encode kernels' lowres / map stores are cached (MALL-allocating) or non-temporal
    (KMP_*_ST_ENC = 1 / 0, INTEGRATION.md knobs; the defaults per kernel and padding were chosen on
    the pipeline rows): both policies give the oracle's bytes and a lossless decode, and
    the wave kernel family served the call."""
    knob, shape, dtype, p, family = case
    kmp_opt(knob, int(cached))
    import oracle
    from oracle import predictors as OP
    ndim = len(shape) - 2
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    coder = 'uint16' if dtype == np.uint16 else 'uint8'
    enc, dec = getattr(ns, f'encode_values_{coder}'), getattr(ns, f'decode_values_{coder}')
    x = np.random.default_rng(29).integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)
    want_lo, (want_maps, _) = ons.encode(OP.mean_predictions_fn(p, ndim), getattr(oracle.common, f'encode_values_{coder}'),
                                         x, padding=p)
    pred = kom.MeanPredictor(p, ndim)
    lo, (maps, dims) = ns.encode(pred, enc, x, padding=p)
    assert _last_launch(kom).startswith(family) and _last_launch(kom).endswith('_encode'), _last_launch(kom)
    assert np.array_equal(lo, want_lo)
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        assert np.array_equal(a, b), (knob, cached, i)
    assert np.array_equal(ns.decode(pred, dec, lo, (maps, dims), padding=p), x)


@pytest.mark.parametrize('ndim,shape,dtype,p,top', [
    # u16 at p = 3 takes the in-order float kernel; values < 2^14 keep its sums exact, because past
    # 2^24 the sum's order matters and the reference does not pin it (XLA's reduce; the oracle's
    # np.mean) -- see oracle/predictors.py mean_predictions_fn
    (3, (2, 21, 18, 23, 1), np.uint16, 3, 1 << 14),
    (3, (1, 30, 26, 34, 1), np.uint8, 3, None),    # exact integer sums
    (3, (2, 19, 27, 33, 1), np.uint16, 2, None),
    (3, (2, 17, 15, 31, 2), np.uint16, 1, None),   # two channels
    (2, (3, 45, 38, 1), np.uint16, 3, None),
    (2, (2, 61, 77, 3), np.uint8, 2, None),        # RGB
])
def test_generic_mean_cells_match_oracle(kom, ndim, shape, dtype, p, top):
    """The generic path's cell means (kmp_codec_generic.hip cell_mean_row_kernel: 4 cells of a row
    per thread, exact integer sums or the reference's in-order float sum) on shapes the one-pass
    kernels do not take, paddings up to 3, against the oracle, encode and decode."""
    import oracle
    from oracle import predictors as OP
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    enc, dec, oenc = (ns.encode_values_uint16, ns.decode_values_uint16, ons.encode_values_uint16) \
        if dtype == np.uint16 else (ns.encode_values_uint8, ns.decode_values_uint8, ons.encode_values_uint8)
    x = np.random.default_rng(21).integers(0, top or np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)
    want_lo, (want_maps, want_dims) = ons.encode(OP.mean_predictions_fn(p, ndim), oenc, x, padding=p)
    pred = kom.MeanPredictor(p, ndim)
    lo, (maps, dims) = ns.encode(pred, enc, x, padding=p)
    assert _last_launch(kom) == 'encode_generic'
    assert tuple(dims) == tuple(want_dims) and np.array_equal(lo, want_lo)
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        bad = np.argwhere(a != b)
        assert bad.size == 0, f'map {i}: {len(bad)} mismatches, first at {bad[:3].tolist()}'
    assert np.array_equal(ns.decode(pred, dec, lo, (maps, dims), padding=p), x)
