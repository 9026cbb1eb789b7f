"""Multi-process (world_size 2, gloo on CPU) tests of the tile-sharding layer:
the partition covers every tile exactly once and the reassembly all-gather rebuilds the
batch bit-exactly, for even and ragged shards and any dtype (byte-slab transport)."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from kompressor_amd.shard import shard_range, all_gather_tiles, local_shard, world_and_rank


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('n,world', [(0, 1), (1, 1), (7, 1), (5, 2), (512, 8), (3, 4), (513, 8)])
def test_shard_range_partitions(n, world):
    ranges = [shard_range(n, r, world) for r in range(world)]
    assert ranges[0][0] == 0 and ranges[-1][1] == n
    for (b0, e0), (b1, e1) in zip(ranges, ranges[1:]):
        assert e0 == b1
    sizes = [e - b for b, e in ranges]
    assert max(sizes) - min(sizes) <= 1 and all(s >= 0 for s in sizes)


def test_shard_range_rejects_bad_requests():
    for args in [(4, 2, 2), (4, -1, 2), (4, 0, 0), (-1, 0, 1)]:
        with pytest.raises(AssertionError):
            shard_range(*args)


def test_single_process_is_identity():
    x = torch.arange(24, dtype=torch.int32).reshape(6, 2, 2)
    assert world_and_rank() == (1, 0)
    assert local_shard(x).data_ptr() == x.data_ptr()
    y = all_gather_tiles(x, 6)
    assert torch.equal(y, x) and y.data_ptr() != x.data_ptr()   # a new tensor, never an alias


def _worker(rank, world, port, cases, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        ok = []
        for n, shape, dtype in cases:
            full = (torch.arange(n * int(np.prod(shape)), dtype=torch.int64) * 7919 % 65521).reshape(n, *shape)
            full = full.to(dtype)
            local = local_shard(full).clone()
            b, e = shard_range(n, rank, world)
            assert local.shape[0] == e - b
            got = all_gather_tiles(local, n)
            ok.append(bool(torch.equal(got, full)) and got.dtype == full.dtype)
        q.put((rank, ok))
    finally:
        dist.destroy_process_group()


def test_all_gather_tiles_gloo_world2():
    cases = [(4, (3, 5, 5, 1), torch.uint16),      # even shards, uint16 (no RCCL dtype: byte slabs)
             (5, (2, 4, 4, 1), torch.uint16),      # ragged: 3 + 2
             (3, (6, 6, 1), torch.uint8),          # images
             (1, (2, 2, 2, 1), torch.int32)]       # one rank holds nothing
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cases, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert results[r] == [True] * len(cases), (r, results[r])
