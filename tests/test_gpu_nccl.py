"""The RCCL (torch.distributed "nccl") branches of the multi-GPU code, one process per GPU
(SURVEY.md §8e): the C4 tile all-gather (``shard.all_gather_tiles``: byte-slab
``all_gather_into_tensor``) and global-volume mode's P2P halo exchange + plane all-gather
(``slabs.encode_global`` / ``decode_global``), each bit-exact against the single-process call.
Needs >= 2 visible GPUs and skips otherwise (the driver's round-end GPU box has one; the 8-GPU
node runs bench.py's N > 1 lines, whose "c4" leg runs the same all-gather)."""

import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _vol(shape, seed):
    return np.random.default_rng(seed).integers(0, 65536, size=shape, dtype=np.int64).astype(np.uint16)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(rank)
    dist.init_process_group('nccl', rank=rank, world_size=world, device_id=torch.device('cuda', rank))
    try:
        import kompressor_amd as kom
        assert dist.get_backend() == 'nccl'
        ok = []
        # C4: tiles sharded over the ranks, coded locally, reassembled by one RCCL all-gather
        for n in (8, 7):  # even and ragged shards
            tiles = torch.from_numpy(_vol((n, 32, 32, 32, 1), 5)).cuda()
            pred = kom.MeanPredictor(0, 3)
            (b, e), (lo, enc) = kom.shard.encode_shard(pred, kom.volume.encode_values_uint16, tiles)
            rec = kom.shard.decode_shard(pred, kom.volume.decode_values_uint16, lo, enc)
            ok.append(torch.equal(rec, tiles[b:e]))
            ok.append(torch.equal(kom.shard.all_gather_tiles(rec, n), tiles))
            ok.append(torch.equal(kom.shard.all_gather_tiles(lo, n), kom.volume.encode(
                pred, kom.volume.encode_values_uint16, tiles)[0]))
        # global-volume mode: D-slabs, P2P halo exchange over RCCL, plane all-gather
        for shape, p in [((1, 64, 32, 32, 1), 0), ((1, 45, 20, 24, 1), 1)]:
            vol = torch.from_numpy(_vol(shape, 4)).cuda()
            depth = shape[1]
            pred = kom.MeanPredictor(p, 3)
            S = kom.slabs
            (z0, z1), (h0, h1) = S.slab_planes(depth, rank, world)
            lo, (maps, dims) = S.encode_global(pred, kom.volume.encode_values_uint16, vol[:, h0:h1], depth, p)
            ref_lo, (ref_maps, ref_dims) = kom.volume.encode(pred, kom.volume.encode_values_uint16, vol, padding=p)
            ok.append(tuple(dims) == tuple(ref_dims))
            ok.append(torch.equal(S.gather_planes(lo, (depth + 1) // 2), ref_lo))
            rec = S.decode_global(pred, kom.volume.decode_values_uint16, lo, (maps, dims), depth, p)
            ok.append(torch.equal(S.gather_planes(rec, depth), vol))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_rccl_tiles_and_slabs():
    if torch.cuda.device_count() < WORLD:
        pytest.skip(f'needs {WORLD} GPUs (one process per GPU over RCCL); {torch.cuda.device_count()} visible')
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(all(v) for v in res.values()), res
