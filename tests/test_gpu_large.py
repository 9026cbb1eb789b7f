"""Maximum sizes: arrays past 2^31 elements, where every 32-bit index would wrap.  Inputs are
generated on the device (no host copies of GBs); parity is by size-independent properties --
lossless round trips, tile independence (tile i of a batch encodes exactly like tile i alone),
chunk invariance -- plus an oracle spot check of tiles beyond the 2^31 boundary."""

import numpy as np
import pytest
import torch

import oracle
from oracle import predictors as OP

pytestmark = pytest.mark.gpu

G2 = 1 << 31


def _rand_u16(shape, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    return torch.randint(-32768, 32768, shape, dtype=torch.int16, device='cuda', generator=g).view(torch.uint16)


def _rand_u8(shape, seed):
    g = torch.Generator(device='cuda').manual_seed(seed)
    return torch.randint(0, 256, shape, dtype=torch.uint8, device='cuda', generator=g)


def test_tile_batch_past_2g_elements(kom):
    """8200 tiles of 64^3 uint16 (2.15 G voxels, 4.3 GB): the fused wave kernels with 64-bit batch
    offsets.  Round trip, and the last tiles equal their own single-tile encode and the oracle."""
    V = kom.volume
    B = 8200
    assert B * 64 ** 3 > G2
    hi = _rand_u16((B, 64, 64, 64, 1), 11)
    pred = kom.MeanPredictor(0, 3)
    lo, (maps, dims) = V.encode(pred, V.encode_values_uint16, hi)
    rec = V.decode(pred, V.decode_values_uint16, lo, (maps, dims))
    assert torch.equal(rec, hi)
    del rec
    for t in (0, B // 2, B - 1):
        lo1, (maps1, _) = V.encode(pred, V.encode_values_uint16, hi[t:t + 1].contiguous())
        assert torch.equal(lo1, lo[t:t + 1])
        for a, b in zip(maps1, maps):
            assert torch.equal(a, b[t:t + 1])
    x = hi[B - 1:].cpu().numpy()
    olo, (omaps, _) = oracle.volume.encode(OP.mean_predictions_fn(0, 3), oracle.volume.encode_values_uint16, x)
    assert np.array_equal(lo[B - 1:].cpu().numpy(), olo)
    for a, b in zip(maps, omaps):
        assert np.array_equal(a[B - 1:].cpu().numpy(), b)


@pytest.mark.parametrize('p', [0, 1])
def test_single_volume_past_2g_elements(kom, p):
    """ONE 1292^3 uint8 volume (2.16 G voxels): one array past 2^31 elements goes to the 64-bit
    kernels.  Lossless, and equal to the chunked driver (chunk invariance at this size)."""
    V = kom.volume
    n = 1292
    assert n ** 3 > G2
    hi = _rand_u8((1, n, n, n, 1), 12 + p)
    pred = kom.MeanPredictor(p, 3)
    lo, (maps, dims) = V.encode(pred, V.encode_values_uint8, hi, padding=p)
    rec = V.decode(pred, V.decode_values_uint8, lo, (maps, dims), padding=p)
    assert torch.equal(rec, hi)
    del rec
    clo, (cmaps, cdims) = V.encode_chunks(pred, V.encode_values_uint8, hi, chunk=400, padding=p)
    assert tuple(cdims) == tuple(dims) and torch.equal(clo, lo)
    for a, b in zip(cmaps, maps):
        assert torch.equal(a, b)


def test_image_batch_past_2g_elements(kom):
    """33000 images of 256^2 uint8 (2.16 G pixels) through the fused image kernels."""
    I = kom.image
    B = 33000
    assert B * 256 * 256 > G2
    hi = _rand_u8((B, 256, 256, 1), 13)
    pred = kom.MeanPredictor(0, 2)
    lo, (maps, dims) = I.encode(pred, I.encode_values_uint8, hi)
    rec = I.decode(pred, I.decode_values_uint8, lo, (maps, dims))
    assert torch.equal(rec, hi)
    x = hi[B - 2:].cpu().numpy()
    olo, (omaps, _) = oracle.image.encode(OP.mean_predictions_fn(0, 2), oracle.image.encode_values_uint8, x)
    assert np.array_equal(lo[B - 2:].cpu().numpy(), olo)
    for a, b in zip(maps, omaps):
        assert np.array_equal(a[B - 2:].cpu().numpy(), b)
