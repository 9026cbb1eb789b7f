"""HIP geometry primitives and coders vs the CPU oracle (bit-exact), volume and image."""

import numpy as np
import pytest
import torch

import oracle
from conftest import load_golden, ramp

pytestmark = pytest.mark.gpu

SHAPES3 = [(2, 17, 17, 17, 1), (2, 16, 16, 16, 1), (1, 9, 10, 12, 3), (2, 5, 4, 7, 2, 2)]
SHAPES2 = [(2, 17, 17, 3), (2, 16, 16, 3), (1, 33, 20, 1), (3, 7, 4, 2, 2)]


def _pair(kom, ndim):
    return (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)


def _rand(shape, dtype, seed=0):
    info = np.iinfo(dtype)
    return np.random.default_rng(seed).integers(info.min, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


def _eq(a, b):
    a = a.cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (a.shape, b.shape)
    assert a.dtype == b.dtype, (a.dtype, b.dtype)
    assert np.array_equal(a, b)


@pytest.mark.parametrize('ndim,shape', [(3, s) for s in SHAPES3] + [(2, s) for s in SHAPES2])
@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.int32])
def test_gathers_and_scatter(kom, ndim, shape, dtype):
    ns, ons = _pair(kom, ndim)
    hi = _rand(shape, dtype)
    _eq(ns.lowres_from_highres(hi), ons.lowres_from_highres(hi))
    for a, b in zip(ns.maps_from_highres(hi), ons.maps_from_highres(hi)):
        _eq(a, b)
    if all(s % 2 == 1 for s in shape[1:1 + ndim]):
        _eq(ns.targets_from_highres(hi), ons.targets_from_highres(hi))
        lo, maps = ons.lowres_from_highres(hi), ons.maps_from_highres(hi)
        _eq(ns.highres_from_lowres_and_maps(lo, maps), hi)


@pytest.mark.parametrize('ndim', [3, 2])
@pytest.mark.parametrize('padding', [0, 1, 2, 3])
def test_features_and_pads(kom, ndim, padding):
    ns, ons = _pair(kom, ndim)
    hi = ramp((2, 17, 17, 17, 1) if ndim == 3 else (2, 17, 17, 3), 65536 if ndim == 3 else 256,
              np.uint16 if ndim == 3 else np.uint8)
    lo = ons.lowres_from_highres(hi)
    padded = ons.pad_neighborhood(lo, padding)
    _eq(ns.pad_neighborhood(lo, padding), padded)
    _eq(ns.features_from_lowres(padded, padding), ons.features_from_lowres(padded, padding))


@pytest.mark.parametrize('ndim,shape', [(3, (2, 16, 15, 14, 1)), (3, (1, 6, 6, 6, 2)), (2, (2, 16, 15, 3)),
                                        (2, (1, 4, 6, 1))])
def test_even_pad_and_trim(kom, ndim, shape):
    ns, ons = _pair(kom, ndim)
    hi = _rand(shape, np.uint16)
    (a, da), (b, db) = ns.utils.pad_highres(hi), ons.pad_highres(hi)
    assert tuple(da) == tuple(db)
    _eq(a, b)
    lo = ons.lowres_from_highres(b)
    trimmed = ons.trim(lo, db)
    _eq(ns.utils.trim(lo, db), trimmed)
    _eq(ns.utils.pad_lowres(trimmed, db), ons.pad_lowres(trimmed, db))
    maps = ons.trim_maps(ons.maps_from_highres(b), db)
    for x, y in zip(ns.utils.pad_maps(maps, db), ons.pad_maps(maps, db)):
        _eq(x, y)
    for x, y in zip(ns.utils.trim_maps(ons.maps_from_highres(b), db), maps):
        _eq(x, y)


@pytest.mark.parametrize('name', ['mfp_vol_f32', 'mfp_vol_i32', 'mfp_vol_u16', 'mfp_img_f32', 'mfp_img_u8'])
def test_maps_from_predictions_golden(kom, name):
    g = load_golden(name)
    ns = kom.volume if int(g['ndim']) == 3 else kom.image
    out = ns.maps_from_predictions(g['predictions'])
    for i, m in enumerate(out):
        _eq(m, g[f'map{i}'])


@pytest.mark.parametrize('ndim', [3, 2])
def test_maps_from_predictions_targets_identity(kom, ndim):
    # tests/volume/test_utils.py:275-291: targets -> maps_from_predictions -> reconstruction
    ns, ons = _pair(kom, ndim)
    hi = ramp((2, 17, 17, 17, 1) if ndim == 3 else (2, 17, 17, 3), 65536, np.uint16)
    lo = ns.lowres_from_highres(hi)
    maps = ns.maps_from_predictions(ns.targets_from_highres(hi))
    _eq(ns.highres_from_lowres_and_maps(lo, maps), hi)


CODER_DTYPES = [np.uint8, np.uint16, np.int32]


@pytest.mark.parametrize('coder', ['raw', 'uint8', 'uint16'])
@pytest.mark.parametrize('pdt', CODER_DTYPES + [np.float32])
@pytest.mark.parametrize('xdt', CODER_DTYPES)
def test_coders(kom, coder, pdt, xdt):
    n = 4097
    if pdt == np.float32:
        pred = (np.random.default_rng(1).standard_normal(n) * 300).astype(np.float32)
    else:
        pred = _rand((n,), pdt, 1)
    x = _rand((n,), xdt, 2)
    enc = getattr(kom.utils, f'encode_values_{coder}')
    dec = getattr(kom.utils, f'decode_values_{coder}')
    _eq(enc(pred, x), getattr(oracle.common, f'encode_values_{coder}')(pred, x))
    _eq(dec(pred, x), getattr(oracle.common, f'decode_values_{coder}')(pred, x))


def test_coders_keep_torch(kom):
    x = torch.arange(100, dtype=torch.int32, device='cuda').to(torch.uint8)
    out = kom.utils.encode_values_uint8(x, x)
    assert isinstance(out, torch.Tensor) and out.is_cuda and out.dtype == torch.uint8
    assert int(out.to(torch.int32).sum()) == 0


def _mp_lds_bytes(window_shape, itemsize, padding, q):
    """The LDS of the per-plane mean predictor kernel with q output planes per workgroup
    (kmp_primitives.hip, kmp_mean_predict_maps): which variant a window gets."""
    S1, S2 = window_shape[2], window_shape[3]
    c1, c2 = S1 - 2 * padding - 1, S2 - 2 * padding - 1
    nb = 16 * (-(-(2 * padding + 2 + q) * S1 * S2 * itemsize // 16) + 1)
    xs = 4 * (2 * padding + 2 + q) * S1 * c2 if padding else 0
    return nb + xs + 4 * (q + 1) * c1 * c2 + 8 * 4 * ((c2 + 4) // 4)


@pytest.mark.parametrize('shape,dtype', [((2, 64, 64, 64, 1), np.uint16), ((3, 17, 9, 22, 1), np.uint8),
                                         ((1, 5, 41, 7, 1), np.uint16),
                                         ((8, 30, 16, 16, 1), np.uint16),   # B % 8 == 0 (XCD order), even plane count
                                         ((16, 17, 12, 32, 1), np.uint8)])  # B % 8 == 0, odd plane count
@pytest.mark.parametrize('padding', [0, 1, 2])
def test_mean_predictor_plane_kernel(kom, shape, dtype, padding):
    """The LDS-staged mean predictor (3D, C == 1): two output planes per workgroup where the LDS
    fits ('mean_predict_plane2'), else one ('mean_predict_plane': e.g. the C3 window at p = 2), on
    C3 tiles, ragged windows, and batches that take the XCD-contiguous block order with an even and
    an odd output-plane count (the last group then holds one plane), against the oracle."""
    hi = _rand(shape, dtype, 11)
    lo = oracle.volume.lowres_from_highres(oracle.volume.pad_highres(hi)[0])
    window = oracle.volume.pad_neighborhood(lo, padding)
    want = oracle.predictors.mean_predictions_fn(padding, 3)(window)
    two = _mp_lds_bytes(window.shape, window.itemsize, padding, 2) <= 64 * 1024
    x8 = padding == 0 and (window.shape[3] - 1) % 8 == 0  # p = 0, cell rows of 8k: mean_predict_p0x8
    runs = {'default': kom.MeanPredictor(padding, 3)(torch.from_numpy(window).cuda())}
    assert kom._lib.lib.kmp_last_launch().decode() == (
        'mean_predict_p0x8' if x8 else 'mean_predict_plane2' if two else 'mean_predict_plane')
    for key, got in runs.items():
        for a, b in zip(got, want):
            _eq(a, b)


@pytest.mark.parametrize('wshape,dtype', [((2, 33, 33, 33, 1), np.uint16),  # the C3 callback window
                                          ((3, 9, 17, 9, 1), np.uint8),
                                          ((8, 5, 3, 17, 1), np.uint16),    # B % 8 == 0, last group of 2 planes
                                          ((1, 2, 2, 9, 1), np.uint16),     # one cell
                                          ((16, 4, 9, 25, 1), np.uint8)])
@pytest.mark.parametrize('fill', ['rand', 'max'])
def test_mean_predictor_p0x8_kernel(kom, wshape, dtype, fill):
    """p = 0 windows whose cell rows are a multiple of 8 long take the eight-positions-per-lane kernel
    ('mean_predict_p0x8'); its maps, in the sample dtype and as float32, equal the oracle's."""
    window = _rand(wshape, dtype, 3) if fill == 'rand' else np.full(wshape, np.iinfo(dtype).max, dtype)
    want = oracle.predictors.mean_predictions_fn(0, 3)(window)
    got = kom.MeanPredictor(0, 3)(torch.from_numpy(window).cuda())
    assert kom._lib.lib.kmp_last_launch().decode() == 'mean_predict_p0x8'
    for a, b in zip(got, want):
        _eq(a, b)
    got = kom.MeanPredictor(0, 3, maps_dtype=torch.float32)(torch.from_numpy(window).cuda())
    assert kom._lib.lib.kmp_last_launch().decode() == 'mean_predict_p0x8'
    for a, b in zip(got, want):
        _eq(a, b.astype(np.float32))


@pytest.mark.parametrize('ndim,padding', [(3, 1), (3, 2), (2, 0), (2, 1)])
def test_mean_predictor_float32_maps(kom, ndim, padding):
    """maps_dtype=float32 on the per-plane kernel (3D, p >= 1: the kernel writes float32) and on
    image windows (converted on the device): the sample-dtype maps' values as float32."""
    ns, ons = _pair(kom, ndim)
    hi = _rand((2, 20, 18, 22, 1) if ndim == 3 else (2, 20, 18, 1), np.uint16, 9)
    window = ons.pad_neighborhood(ons.lowres_from_highres(ons.pad_highres(hi)[0]), padding)
    want = oracle.predictors.mean_predictions_fn(padding, ndim)(window)
    got = kom.MeanPredictor(padding, ndim, maps_dtype=np.float32)(torch.from_numpy(window).cuda())
    if ndim == 3:
        assert kom._lib.lib.kmp_last_launch().decode().startswith('mean_predict_plane')
    for a, b in zip(got, want):
        assert a.dtype == torch.float32
        _eq(a, b.astype(np.float32))


@pytest.mark.parametrize('ndim', [3, 2])
@pytest.mark.parametrize('padding', [0, 1, 2])
def test_mean_predictor_callable(kom, ndim, padding):
    ns, ons = _pair(kom, ndim)
    hi = _rand((2, 13, 12, 11, 1) if ndim == 3 else (2, 13, 12, 2), np.uint16, 5)
    lo = ons.lowres_from_highres(ons.pad_highres(hi)[0])
    window = ons.pad_neighborhood(lo, padding)
    got = kom.MeanPredictor(padding, ndim)(window)
    want = oracle.predictors.mean_predictions_fn(padding, ndim)(window)
    for a, b in zip(got, want):
        _eq(a, b)


@pytest.mark.gpu
def test_zero_width_pads_and_trims_return_fresh_tensors(kom):
    """SURVEY.md §8b "Ownership": every output is a new array, as under JAX -- a zero-width pad or
    trim of a CUDA tensor must not hand the caller's own tensor back (writing the output would
    silently change the input)."""
    import torch
    for ns, shape in ((kom.volume, (2, 5, 6, 7, 1)), (kom.image, (2, 6, 7, 1))):
        n = len(shape) - 2
        x = torch.arange(int(np.prod(shape)), dtype=torch.int32).reshape(shape).to(torch.uint16).cuda()
        keep = x.clone()
        outs = [ns.pad_neighborhood(x, 0), ns.utils.trim(x, (0,) * n), ns.utils.pad_lowres(x, (0,) * n),
                ns.utils.pad_map(x, (0,) * n)]
        outs += list(ns.utils.pad_maps([x, x], (0,) * n)) + list(ns.utils.trim_maps([x, x], (0,) * n))
        for o in outs:
            assert torch.equal(o, keep)
            assert o.untyped_storage().data_ptr() != x.untyped_storage().data_ptr()
            o.view(torch.int16).fill_(7)
            assert torch.equal(x, keep), 'writing an output changed the input'


def test_stream_handle_follows_torch_current_stream(kom):
    """_device.stream() (the raw handle every C-ABI call gets) is torch's current stream, on the
    default stream and inside a torch.cuda.stream context, and work launched there is ordered on it."""
    from kompressor_amd import _device as dev
    assert dev.stream() == torch.cuda.current_stream().cuda_stream
    side = torch.cuda.Stream()
    x = torch.from_numpy(np.random.default_rng(5).integers(0, 65536, (4, 16, 16, 16, 1), dtype=np.int64)
                         .astype(np.uint16)).cuda()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        assert dev.stream() == side.cuda_stream == torch.cuda.current_stream().cuda_stream
        pred = kom.MeanPredictor(0, 3)
        lo, enc = kom.volume.encode(pred, kom.volume.encode_values_uint16, x)
        rec = kom.volume.decode(pred, kom.volume.decode_values_uint16, lo, enc)
    torch.cuda.current_stream().wait_stream(side)
    assert torch.equal(rec, x)
    assert dev.stream() == torch.cuda.current_stream().cuda_stream
