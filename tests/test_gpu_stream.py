"""Pinned-host streaming codec (kompressor_amd.stream.TileStream; BASELINE config C5 and the
north star's end-to-end H<->D rate): identical results to the device-resident fused calls,
lossless round trips, and the float32-as-uint32 extension bit-exact against the oracle."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _pinned_from(a):
    t = torch.empty(a.shape, dtype=torch.from_numpy(a[:0].copy()).dtype, pin_memory=True)
    t.copy_(torch.from_numpy(a))
    return t


@pytest.mark.parametrize('zero_copy', [False, True])
@pytest.mark.parametrize('ndim,shape,dtype,chunk,slots', [
    (3, (10, 16, 16, 16, 1), np.uint16, 3, 2),     # ragged last chunk
    (3, (8, 64, 64, 64, 1), np.uint16, 2, 3),      # metric tile
    (2, (9, 64, 32, 1), np.uint8, 4, 3),
])
def test_stream_equals_device_resident(kom, ndim, shape, dtype, chunk, slots, zero_copy):
    rng = np.random.default_rng(11)
    host = rng.integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)
    ns = kom.volume if ndim == 3 else kom.image
    pred = kom.MeanPredictor(0, ndim)
    enc, dec = (ns.encode_values_uint16, ns.decode_values_uint16) if dtype == np.uint16 else \
               (ns.encode_values_uint8, ns.decode_values_uint8)
    ref_lo, (ref_maps, dims) = ns.encode(pred, enc, torch.from_numpy(host).cuda())
    ts = kom.stream.TileStream(pred, shape[1:], torch.from_numpy(host[:0]).dtype, chunk, slots, ndim,
                               zero_copy=zero_copy)
    src = _pinned_from(host)
    lo, maps = ts.alloc_encoded(shape[0])
    ts.encode(src, lo, maps)
    ts.synchronize()
    assert torch.equal(lo, ref_lo.cpu()) and all(torch.equal(a, b.cpu()) for a, b in zip(maps, ref_maps))
    out = torch.empty_like(src).pin_memory()
    ts.decode(lo, maps, out)
    ts.synchronize()
    assert torch.equal(out, src)


def test_float32_stream_bit_exact_vs_oracle(kom):
    """C5 semantics on a small batch: float32 bit-cast to uint32, MeanPredictor (f32 mean in
    feature order), mod-2^32 coder; every bit pattern round-trips (NaN, -0, inf included)."""
    import oracle
    from oracle import predictors as OP
    rng = np.random.default_rng(2)
    x = rng.standard_normal((5, 18, 16, 20, 1)).astype(np.float32) * 1000
    flat = x.reshape(-1)
    flat[:4] = [np.nan, -0.0, np.inf, -np.inf]
    bits = x.view(np.uint32)
    ref_lo, (ref_maps, ref_dims) = oracle.volume.encode(OP.mean_predictions_fn(0, 3), oracle.volume.encode_values_uint32,
                                                        bits)
    pred = kom.MeanPredictor(0, 3)
    ts = kom.stream.TileStream(pred, x.shape[1:], torch.float32, 2, 2, 3)
    src = _pinned_from(x)
    lo, maps = ts.alloc_encoded(x.shape[0])
    ts.encode(src, lo, maps)
    ts.synchronize()
    assert np.array_equal(lo.numpy(), ref_lo)
    for m, r in zip(maps, ref_maps):
        assert np.array_equal(m.numpy(), r)
    out = torch.empty_like(src).pin_memory()
    ts.decode(lo, maps, out)
    ts.synchronize()
    assert np.array_equal(out.numpy().view(np.uint32), bits)


@pytest.mark.parametrize('p', [0, 1])
def test_uint32_fused_codec_vs_oracle(kom, p):
    import oracle
    from oracle import predictors as OP
    rng = np.random.default_rng(7 + p)
    x = rng.integers(0, 1 << 32, size=(2, 11, 14, 9, 1), dtype=np.int64).astype(np.uint32)
    ref_lo, (ref_maps, _) = oracle.volume.encode(OP.mean_predictions_fn(p, 3), oracle.volume.encode_values_uint32, x,
                                                 padding=p)
    pred = kom.MeanPredictor(p, 3)
    lo, (maps, dims) = kom.volume.encode(pred, kom.volume.encode_values_uint32, x, padding=p)
    assert np.array_equal(lo, ref_lo)
    for m, r in zip(maps, ref_maps):
        assert np.array_equal(m, r)
    assert np.array_equal(kom.volume.decode(pred, kom.volume.decode_values_uint32, lo, (maps, dims), padding=p), x)
