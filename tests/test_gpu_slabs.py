"""Global-volume mode on the GPU (kompressor_amd.slabs): the per-rank D-slab
results, computed from each rank's local array with its halo, are exactly that rank's planes of
the whole-volume encode / decode -- emulated rank by rank in one process for 1-5 ranks, and for
real with 2 processes on cuda:0 over gloo (P2P halo exchange + plane all-gather)."""

import os
import socket

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _vol(shape, dtype, seed):
    info = np.iinfo(dtype)
    return np.random.default_rng(seed).integers(0, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)


def _predictor(kom, kind, p):
    if kind == 'mean':
        return kom.MeanPredictor(p, 3)
    if kind == 'callback':
        inner = kom.MeanPredictor(p, 3)
        return lambda lowres: inner(lowres)
    n = (2 * p + 2) ** 3
    rng = np.random.default_rng(9)
    return kom.LinearPredictor((1.0 / n + rng.standard_normal((n, 19)) * 0.02).astype(np.float32),
                               (rng.standard_normal(19) * 20).astype(np.float32), p, 3)


CASES = [((1, 64, 32, 32, 1), np.uint16, 0, 'mean'),
         ((1, 65, 32, 32, 1), np.uint16, 0, 'mean'),
         ((1, 33, 18, 20, 1), np.uint16, 1, 'mean'),
         ((2, 30, 16, 16, 1), np.uint8, 2, 'mean'),
         ((1, 40, 32, 32, 1), np.uint16, 0, 'linear'),
         ((1, 21, 12, 10, 1), np.uint16, 1, 'callback')]


@pytest.mark.parametrize('shape,dtype,p,kind', CASES)
@pytest.mark.parametrize('world', [1, 2, 3, 5])
def test_slabs_equal_whole_volume(kom, shape, dtype, p, kind, world):
    S = kom.slabs
    vol = torch.from_numpy(_vol(shape, dtype, 3)).cuda()
    depth = shape[1]
    if world > 1 and (depth + 1) // 2 // world < 2 + p:
        pytest.skip('slabs thinner than the halo')
    pred = _predictor(kom, kind, p)
    enc, dec = (kom.volume.encode_values_uint16, kom.volume.decode_values_uint16) if dtype == np.uint16 else \
               (kom.volume.encode_values_uint8, kom.volume.decode_values_uint8)
    ref_lo, (ref_maps, ref_dims) = kom.volume.encode(pred, enc, vol, padding=p)
    los, maps_r, recs = [], [], []
    for r in range(world):
        (z0, z1), _ = S.slab_planes(depth, r, world)
        a, b = S.encode_halo(depth, z0, z1, p)
        lo, (maps, dims) = S.encode_local(pred, enc, vol[:, a:b], a, (z0, z1), p)
        los.append(lo)
        maps_r.append(maps)
    assert torch.equal(torch.cat(los, 1), ref_lo)
    for k in range(7):
        assert torch.equal(torch.cat([m[k] for m in maps_r], 1), ref_maps[k]), k
    ez = (depth + 1) // 2
    for r in range(world):
        (z0, z1), (h0, h1) = S.slab_planes(depth, r, world)
        la, lb = S.decode_halo(ez, z0, z1, p)
        rec = S.decode_local(pred, dec, ref_lo[:, la:lb], maps_r[r], la, (z0, z1), ref_dims, p, at_top=(lb == ez))
        recs.append(rec)
        assert torch.equal(rec, vol[:, h0:h1]), r
    assert torch.equal(torch.cat(recs, 1), vol)


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import kompressor_amd as kom
        S = kom.slabs
        ok = []
        for shape, p in [((1, 64, 32, 32, 1), 0), ((1, 45, 20, 24, 1), 1)]:
            vol = torch.from_numpy(_vol(shape, np.uint16, 4)).cuda()
            depth = shape[1]
            pred = kom.MeanPredictor(p, 3)
            (z0, z1), (h0, h1) = S.slab_planes(depth, rank, world)
            lo, (maps, dims) = S.encode_global(pred, kom.volume.encode_values_uint16, vol[:, h0:h1], depth, p)
            ref_lo, (ref_maps, ref_dims) = kom.volume.encode(pred, kom.volume.encode_values_uint16, vol, padding=p)
            ok.append(tuple(dims) == tuple(ref_dims))
            ok.append(torch.equal(S.gather_planes(lo, (depth + 1) // 2), ref_lo))
            rec = S.decode_global(pred, kom.volume.decode_values_uint16, lo, (maps, dims), depth, p)
            ok.append(torch.equal(rec, vol[:, h0:h1]))
            ok.append(torch.equal(S.gather_planes(rec, depth), vol))
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_slabs_two_processes_gloo(kom):
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert all(res[0]) and all(res[1]), res
