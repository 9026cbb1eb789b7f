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


@pytest.mark.parametrize('zero_copy', [True, False])
def test_c5_chunk_shape_float32(kom, zero_copy):
    """BASELINE config C5 at its real chunk geometry: a handful of 128^3 float32 chunks streamed
    through TileStream (zero-copy and the 3-stream copy pipeline), chunk 1 bit-exact against the
    oracle's uint32 restatement (volume/encode_decode.py:30-85 with the mod-2^32 coder), every
    chunk round-tripping bit for bit -- NaN / +-0 / +-inf / denormals included."""
    import oracle
    from oracle import predictors as OP
    n = 5
    rng = np.random.default_rng(128)
    x = (rng.standard_normal((n, 128, 128, 128, 1), dtype=np.float32) * 100).astype(np.float32)
    flat = x.reshape(-1)
    flat[:6] = [np.nan, -0.0, 0.0, np.inf, -np.inf, np.float32(1e-40)]
    ts = kom.stream.TileStream(kom.MeanPredictor(0, 3), x.shape[1:], torch.float32, 2, 3, 3, zero_copy=zero_copy)
    assert ts.zero_copy == zero_copy
    src = _pinned_from(x)
    lo, maps = ts.alloc_encoded(n)
    ts.encode(src, lo, maps)
    ts.synchronize()
    bits = x[1:2].view(np.uint32)
    ref_lo, (ref_maps, _) = oracle.volume.encode(OP.mean_predictions_fn(0, 3), oracle.volume.encode_values_uint32, bits)
    assert np.array_equal(lo[1:2].numpy(), ref_lo)
    for m, r in zip(maps, ref_maps):
        assert np.array_equal(m[1:2].numpy(), r)
    out = torch.empty_like(src).pin_memory()
    ts.decode(lo, maps, out)
    ts.synchronize()
    assert np.array_equal(out.numpy().view(np.uint32), x.view(np.uint32))


def test_stream_rejects_mismatched_host_buffers(kom):
    """on the zero-copy path the kernel writes the caller's pinned buffers
    directly, so buffers that do not match the stream's shapes raise before any launch."""
    shape = (4, 16, 16, 16, 1)
    ts = kom.stream.TileStream(kom.MeanPredictor(0, 3), shape[1:], torch.uint16, 2, 2, 3, zero_copy=True)
    src = _pinned_from(np.zeros(shape, np.uint16))
    lo, maps = ts.alloc_encoded(shape[0])
    short_lo, short_maps = ts.alloc_encoded(shape[0] - 1)
    with pytest.raises(AssertionError):
        ts.encode(src, short_lo, maps)
    with pytest.raises(AssertionError):
        ts.encode(src, lo, short_maps)
    with pytest.raises(AssertionError):
        ts.encode(src, lo, maps[:-1])
    out_bad = torch.empty((shape[0], 16, 16, 15, 1), dtype=torch.uint16, pin_memory=True)
    ts.encode(src, lo, maps)
    ts.synchronize()
    with pytest.raises(AssertionError):
        ts.decode(lo, maps, out_bad)
