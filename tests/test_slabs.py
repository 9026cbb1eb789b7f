"""Global-volume mode (kompressor_amd.slabs) host logic: the D-slab partition
and halo geometry, and the point-to-point halo exchange over gloo with world sizes 2 and 3
(CPU tensors): every rank ends up with exactly the planes its outputs depend on."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kompressor_amd import slabs


@pytest.mark.parametrize('depth,world,p', [(64, 2, 0), (65, 3, 0), (64, 4, 1), (33, 3, 2), (16, 1, 0), (9, 4, 0)])
def test_partition_and_halo(depth, world, p):
    ez = (depth + 1) // 2
    planes = []
    for r in range(world):
        (z0, z1), (h0, h1) = slabs.slab_planes(depth, r, world)
        planes.append((h0, h1))
        a, b = slabs.encode_halo(depth, z0, z1, p)
        if z1 > z0:
            # node planes z0-1-p .. z1+p (clipped) == highres planes 2*(z0-1-p) .. 2*(z1+p)
            assert a == 2 * max(0, z0 - 1 - p) and b == min(depth, 2 * (z1 + p) + 1)
            assert a <= h0 and b >= h1
        la, lb = slabs.decode_halo(ez, z0, z1, p)
        assert la == max(0, z0 - 1 - p) and lb == min(ez, z1 + p + 1)
    # the highres slabs tile the volume
    assert planes[0][0] == 0 and planes[-1][1] == depth
    assert all(a[1] == b[0] for a, b in zip(planes, planes[1:]))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, cases, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ok = []
        for depth, p in cases:
            vol = (torch.arange(depth * 6 * 4, dtype=torch.int32) * 2654435761 % 65521).reshape(1, depth, 6, 4, 1)
            vol = vol.to(torch.uint16)
            (z0, z1), (h0, h1) = slabs.slab_planes(depth, rank, world)
            local, (a, b) = slabs.encode_halo_exchange(vol[:, h0:h1].clone(), depth, p)
            ok.append(torch.equal(local, vol[:, a:b]))
            ez = (depth + 1) // 2
            lo = vol[:, ::2][:, :ez].contiguous()  # any array with ez planes
            llocal, (la, lb) = slabs.decode_halo_exchange(lo[:, z0:z1].clone(), depth, p)
            ok.append(torch.equal(llocal, lo[:, la:lb]))
            # reassembly of the per-rank planes
            ok.append(torch.equal(slabs.gather_planes(vol[:, h0:h1].clone(), depth), vol))
        # a slab thinner than the halo makes EVERY rank raise (none is left blocked in
        # a send): depth 13 -> 7 node planes, one or two per rank, against a (1 + p) = 3-plane halo
        depth = 13
        vol = torch.zeros((1, depth, 6, 4, 1), dtype=torch.uint16)
        (z0, z1), (h0, h1) = slabs.slab_planes(depth, rank, world)
        try:
            slabs.encode_halo_exchange(vol[:, h0:h1].clone(), depth, 2)
            ok.append(world < 3)  # with 2 ranks the slabs are thick enough
        except AssertionError:
            ok.append(world >= 3)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 3])
def test_halo_exchange_gloo(world):
    cases = [(64, 0), (65, 0), (40, 1), (31, 2)]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cases, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        assert all(res[r]), (r, res[r])
