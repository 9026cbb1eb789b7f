"""Tile split / reassembly (kmp_tiles) and the sharded codec driver on one GPU (BASELINE
configs C3/C4): bit-exact against numpy's reshape/transpose, and the full 512^3 volume
round trip volume -> tiles -> encode -> decode -> volume."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def np_tiles(vol, tile):
    nsp = len(tile)
    sp, ch = vol.shape[:nsp], vol.shape[nsp:]
    split = []
    for s, t in zip(sp, tile):
        split += [s // t, t]
    x = vol.reshape(*split, *ch)
    order = [2 * a for a in range(nsp)] + [2 * a + 1 for a in range(nsp)] + list(range(2 * nsp, 2 * nsp + len(ch)))
    return x.transpose(order).reshape(-1, *tile, *ch)


@pytest.mark.parametrize('shape,tile,dtype', [
    ((64, 64, 64, 1), (16, 16, 16), np.uint16),     # 16-B rows: vector path
    ((12, 10, 15, 2), (4, 5, 5), np.uint8),         # odd rows: element path
    ((8, 8, 8, 3), (8, 4, 2), np.int32),
    ((48, 40, 1), (16, 8), np.uint8),               # image
    ((6, 6, 6, 1), (6, 6, 6), np.float32),          # one tile
])
def test_tiles_match_numpy(kom, shape, tile, dtype):
    rng = np.random.default_rng(3)
    vol = rng.integers(0, 200, size=shape).astype(dtype)
    ndim = len(tile)
    t = kom.tiles.volume_to_tiles(vol, tile, ndim)
    assert np.array_equal(t, np_tiles(vol, tile))
    back = kom.tiles.tiles_to_volume(t, shape[:ndim], ndim)
    assert np.array_equal(back, vol)


def test_tiles_reject_bad_shapes(kom):
    with pytest.raises(AssertionError):
        kom.tiles.volume_to_tiles(np.zeros((10, 10, 10, 1), np.uint16), 4)
    with pytest.raises(AssertionError):
        kom.tiles.tiles_to_volume(np.zeros((3, 4, 4, 4, 1), np.uint16), (8, 8, 8))


def test_encode_shard_single_process_equals_encode(kom):
    rng = np.random.default_rng(5)
    tiles = torch.from_numpy(rng.integers(0, 65536, size=(6, 16, 16, 16, 1)).astype(np.uint16)).cuda()
    pred = kom.MeanPredictor(0, 3)
    (b, e), (lo, (maps, dims)) = kom.shard.encode_shard(pred, kom.volume.encode_values_uint16, tiles)
    assert (b, e) == (0, 6)
    lo2, (maps2, _) = kom.volume.encode(pred, kom.volume.encode_values_uint16, tiles)
    assert torch.equal(lo, lo2) and all(torch.equal(x, y) for x, y in zip(maps, maps2))
    rec = kom.shard.decode_shard(pred, kom.volume.decode_values_uint16, lo, (maps, dims))
    assert torch.equal(kom.shard.all_gather_tiles(rec, 6), tiles)


def test_metric_volume_tiled_round_trip(kom):
    """C3 end to end on the device: one 512^3 uint16 volume -> 512 tiles of 64^3 -> fused
    encode -> fused decode -> reassembled volume, lossless; tile 77 equals the oracle's
    encode of the same sub-volume cut with numpy."""
    import oracle
    from oracle import predictors as OP
    rng = np.random.default_rng(0)
    host = rng.integers(0, 65536, size=(512, 512, 512, 1), dtype=np.int64).astype(np.uint16)
    vol = torch.from_numpy(host).cuda()
    tiles = kom.tiles.volume_to_tiles(vol, 64)
    assert tuple(tiles.shape) == (512, 64, 64, 64, 1)
    pred = kom.MeanPredictor(0, 3)
    lo, (maps, dims) = kom.volume.encode(pred, kom.volume.encode_values_uint16, tiles)
    rec = kom.volume.decode(pred, kom.volume.decode_values_uint16, lo, (maps, dims))
    assert torch.equal(kom.tiles.tiles_to_volume(rec, (512, 512, 512)), vol)
    t = 77
    tz, ty, tx = t // 64, (t // 8) % 8, t % 8
    sub = host[tz * 64:(tz + 1) * 64, ty * 64:(ty + 1) * 64, tx * 64:(tx + 1) * 64][None]
    ref_lo, (ref_maps, _) = oracle.volume.encode(OP.mean_predictions_fn(0, 3), oracle.volume.encode_values_uint16, sub)
    assert np.array_equal(lo[t:t + 1].cpu().numpy(), ref_lo)
    for m, r in zip(maps, ref_maps):
        assert np.array_equal(m[t:t + 1].cpu().numpy(), r)
