"""Multi-GPU tile sharding (BASELINE config C4).

One process per GPU (``torch.distributed``; backend ``nccl`` is RCCL over xGMI on ROCm).
Tiles are independent -- every reference primitive is ``[:, ...]``-parallel
(``volume/utils.py:80,161-169``) and each tile gets its own padding and boundary handling -- so
the codec itself needs NO collective: rank r codes the contiguous tile range
:func:`shard_range` gives it (weak scaling).  The only exchange is the optional reassembly of
the decoded volume (or of the encoded maps) on every rank, one all-gather of per-rank byte
slabs: :func:`all_gather_tiles`.
"""

import torch

from . import _nd


def _dist():
    import torch.distributed as dist
    return dist


def world_and_rank(group=None):
    dist = _dist()
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def shard_range(n_units, rank, world):
    """Contiguous, balanced ``[begin, end)`` of ``n_units`` for ``rank`` of ``world`` (the first
    ``n_units % world`` ranks take one extra unit)."""
    if world < 1 or not 0 <= rank < world or n_units < 0:
        raise AssertionError(f'bad shard request: {n_units} units, rank {rank} of {world}')
    base, extra = divmod(n_units, world)
    begin = rank * base + min(rank, extra)
    return begin, begin + base + (1 if rank < extra else 0)


def local_shard(tiles, group=None):
    """This rank's tiles of the batch ``tiles`` (a view; no copy)."""
    world, rank = world_and_rank(group)
    b, e = shard_range(int(tiles.shape[0]), rank, world)
    return tiles[b:e]


def encode_shard(predictions_fn, encode_fn, tiles, padding=0, ndim=3, group=None):
    """``encode`` of this rank's shard of the tile batch -> ``(begin, end), (lowres, (maps, dims))``."""
    world, rank = world_and_rank(group)
    b, e = shard_range(int(tiles.shape[0]), rank, world)
    ns = _nd
    return (b, e), ns.encode(predictions_fn, encode_fn, tiles[b:e], padding, ndim)


def decode_shard(predictions_fn, decode_fn, lowres, encoded, padding=0, ndim=3):
    """``decode`` of this rank's encoded shard (as returned by :func:`encode_shard`)."""
    return _nd.decode(predictions_fn, decode_fn, lowres, encoded, padding, ndim)


def all_gather_tiles(local, n_units, group=None):
    """Reassemble the full ``[n_units, ...]`` batch on every rank from each rank's
    :func:`shard_range` slice ``local``, as a new tensor (never an alias of ``local``).  Byte
    views travel, so any dtype does (RCCL has no uint16).  Equal shards: one
    ``all_gather_into_tensor`` straight into the result (the list form over gloo).  Uneven shards:
    padded to the largest, gathered the same way, the padding dropped."""
    world, rank = world_and_rank(group)
    if world == 1:
        return local.clone()
    dist = _dist()
    b, e = shard_range(n_units, rank, world)
    if local.shape[0] != e - b:
        raise AssertionError(f'rank {rank} holds {local.shape[0]} units, its shard is {e - b}')
    per = -(-n_units // world)
    row = tuple(local.shape[1:])
    send = local.contiguous()
    sb = send.view(torch.uint8).reshape(-1)
    nccl = dist.get_backend(group) == 'nccl'
    if n_units == per * world:
        out = torch.empty((n_units, *row), dtype=local.dtype, device=local.device)
        ob = out.view(torch.uint8).reshape(-1)
        if nccl:
            dist.all_gather_into_tensor(ob, sb, group=group)
        else:
            dist.all_gather(list(ob.chunk(world)), sb, group=group)
        return out
    # uneven shards (including ranks with none): equal-size padded slabs -- one
    # all_gather_into_tensor over RCCL, the list form over gloo -- and the padding dropped.  (The
    # RCCL list form with exact-size receive views would save the padding but has never run on a
    # multi-GPU box here, so it is not used.)
    pad = torch.empty((per, *row), dtype=local.dtype, device=local.device)
    pad[:send.shape[0]].copy_(send)
    full = torch.empty((per * world, *row), dtype=local.dtype, device=local.device)
    fb, pb = full.view(torch.uint8).reshape(-1), pad.view(torch.uint8).reshape(-1)
    if nccl:
        dist.all_gather_into_tensor(fb, pb, group=group)
    else:
        dist.all_gather(list(fb.chunk(world)), pb, group=group)
    parts = []
    for r in range(world):
        rb, re_ = shard_range(n_units, r, world)
        parts.append(full[r * per: r * per + (re_ - rb)])
    return torch.cat(parts, 0)
