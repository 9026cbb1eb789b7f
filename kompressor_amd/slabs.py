"""Global-volume mode across GPUs: one volume split into D-slabs with a halo exchange
(SURVEY.md §8e "global-volume mode", §8f row f-1).

The tile mode (``kompressor_amd.shard``) codes independent tiles.  This mode codes ONE volume
``[1, D, H, W, C...]`` exactly as a single ``encode`` / ``decode`` of the whole array would
(``volume/encode_decode.py:30-85``; chunk invariance, ``tests/volume/test_encode_decode.py:
466-548``, is the same property across chunks), with the output planes split over the ranks:

* rank r owns output (lowres) planes ``[Z0, Z1) = shard_range(ceil(D / 2), r, world)`` and the
  highres planes ``[2*Z0, min(2*Z1, D))`` (:func:`slab_planes`);
* its outputs depend on node planes ``Z0-1-p .. Z1+p`` only, so it first receives that halo --
  the last highres planes of rank r-1 and the first of rank r+1 (decode: lowres planes) -- by
  point-to-point send / recv (RCCL over xGMI for ``nccl``; host-staged for ``gloo``), the one
  real exchange step of this path;
* it then runs the fused kernel on its local array with a z-region (``kmp_region``): inside
  the local array every node the region needs is a real node, and the local array's edges are
  the global edges exactly where the reference pads (even-dim reflect, neighbourhood symmetric).

The per-rank results are the rank's planes of the whole-array result, bit for bit
(``tests/test_gpu_slabs.py``); :func:`gather_planes` reassembles them.
"""

import torch

from . import _device as dev
from . import _nd
from .shard import shard_range, world_and_rank, _dist  # noqa: F401

_N = 3


def slab_planes(depth, rank, world):
    """``((Z0, Z1), (h0, h1))``: the output planes rank owns and the highres planes it holds."""
    ez = (depth + 1) // 2
    z0, z1 = shard_range(ez, rank, world)
    return (z0, z1), (min(2 * z0, depth), min(2 * z1, depth))


def encode_halo(depth, z0, z1, padding):
    """Highres planes ``[a, b)`` rank's outputs ``[z0, z1)`` depend on (node planes
    ``z0-1-p .. z1+p``; node j is highres plane 2j)."""
    n0 = max(0, z0 - 1 - padding)
    return 2 * n0, min(depth, 2 * (z1 + padding) + 1)


def decode_halo(ez, z0, z1, padding):
    """Lowres planes ``[a, b)`` rank's output planes ``[z0, z1)`` depend on."""
    return max(0, z0 - 1 - padding), min(ez, z1 + padding + 1)


# ---------------------------------------------------------------------------------------------
# local compute (one rank's share, given its local array with halo)
# ---------------------------------------------------------------------------------------------

def _map_z_extent(k, E, L):
    return L - 1 if _nd.PARITY[_N][k][0] else E


def encode_local(predictions_fn, encode_fn, local, local_z0, region, padding=0):
    """Encode output planes ``region = (z0, z1)`` (global indices) from ``local`` = highres planes
    ``[local_z0, ...)`` of the volume (with halo).  Returns this rank's planes of the global
    ``(lowres, (maps, dims))``; ``dims`` is the local array's z padding at the global top."""
    t = _nd._dev(local)
    r0, r1 = region[0] - local_z0 // 2, region[1] - local_z0 // 2
    plan = _nd.fused_plan(predictions_fn, encode_fn, padding, t.dtype, _N, 0)
    if plan is not None:
        predictor, coder = plan
        lowres, maps, dims = _nd._alloc_encoded(t, coder, _N)
        E = _nd._sp(lowres.shape, _N)
        _nd.fused_encode_into(t, predictor, coder, lowres, maps, _N,
                              region=[(r0, r1), (0, E[1]), (0, E[2])])
    else:  # any predictions_fn / coder: the whole local array, then this rank's planes
        lowres, (maps, dims) = _nd.encode(predictions_fn, encode_fn, t, padding, _N)
    E0 = int(lowres.shape[1])
    L0 = E0 + int(dims[0])
    lo = lowres[:, r0:r1]
    out_maps = tuple(m[:, r0:min(r1, _map_z_extent(k, E0, L0))] for k, m in enumerate(maps))
    return lo, (out_maps, tuple(dims))


def decode_local(predictions_fn, decode_fn, lowres_local, maps_region, local_z0, region, dims, padding=0,
                 at_top=True):
    """Decode output planes ``region`` from ``lowres_local`` = lowres planes ``[local_z0, ...)``
    (with halo) and this rank's encoded map planes.  Returns highres planes ``[2*z0, ...)`` of
    the global result (up to the volume's last plane on the top rank)."""
    lo = _nd._dev(lowres_local)
    maps_region = [_nd._dev(m) for m in maps_region]
    ldims = (int(dims[0]) if at_top else 0, int(dims[1]), int(dims[2]))
    r0, r1 = region[0] - local_z0, region[1] - local_z0
    E = _nd._sp(lo.shape, _N)
    L = [e + d for e, d in zip(E, ldims)]
    maps = []  # local-shape maps: this rank's planes at [r0, ...), the halo planes are never read
    for k, (par, m) in enumerate(zip(_nd.PARITY[_N], maps_region)):
        shape = (lo.shape[0], *[(l - 1 if p else e) for l, e, p in zip(L, E, par)], *lo.shape[1 + _N:])
        full = _nd._zeros(shape, m.dtype)
        full[:, r0:r0 + m.shape[1]] = m
        maps.append(full)
    plan = _nd.fused_plan(predictions_fn, decode_fn, padding, lo.dtype, _N, 1)
    out_planes = [2 * r0, min(2 * r1, 2 * E[0] - 1 + ldims[0])]
    if plan is not None and all(m.dtype == _nd.CODER_DTYPE[plan[1]] for m in maps):
        predictor, coder = plan
        out = dev.empty((lo.shape[0], *[2 * e - 1 + d for e, d in zip(E, ldims)], *lo.shape[1 + _N:]), lo.dtype)
        _nd.fused_decode_into(lo, maps, ldims, predictor, coder, out, _N, region=[(r0, r1), (0, E[1]), (0, E[2])])
    else:
        out = _nd.decode(predictions_fn, decode_fn, lo, (maps, ldims), padding, _N)
    return out[:, out_planes[0]:out_planes[1]]


# ---------------------------------------------------------------------------------------------
# exchange + drivers
# ---------------------------------------------------------------------------------------------

def _p2p(dist, group, sends, recvs):
    """Point-to-point exchange.  ``sends`` / ``recvs``: lists of ``(peer, tensor view)``.  nccl
    (RCCL over xGMI) moves device buffers directly; gloo stages them through host memory."""
    if not sends and not recvs:
        return
    nccl = dist.get_backend(group) == 'nccl'
    ops, landing = [], []
    for peer, t in sends:
        buf = t.contiguous() if nccl else t.detach().cpu().contiguous()
        ops.append(dist.P2POp(dist.isend, buf.view(torch.uint8).reshape(-1), peer, group))
    for peer, t in recvs:
        buf = torch.empty(t.shape, dtype=t.dtype, device=t.device if nccl else 'cpu')
        landing.append((t, buf))
        ops.append(dist.P2POp(dist.irecv, buf.view(torch.uint8).reshape(-1), peer, group))
    for req in dist.batch_isend_irecv(ops):
        req.wait()
    for t, buf in landing:
        t.copy_(buf)


def _exchange(slab, own, need, world, rank, group, ranges):
    """Assemble planes ``need = [a, b)`` around this rank's ``slab`` (= planes ``own``) from the
    neighbours' slabs; ``ranges[r]`` = planes rank r holds."""
    dist = _dist()
    a, b = need
    below = own[0] - a
    above = b - own[1]
    out = torch.empty((slab.shape[0], b - a, *slab.shape[2:]), dtype=slab.dtype, device=slab.device)
    out[:, below:below + slab.shape[1]] = slab
    sends, recvs = [], []
    if rank > 0 and below > 0:
        if ranges[rank - 1][1] - ranges[rank - 1][0] < below:
            raise AssertionError('slab thinner than the halo: use fewer ranks')
        recvs.append((rank - 1, out[:, :below]))
    if rank < world - 1 and above > 0:
        if ranges[rank + 1][1] - ranges[rank + 1][0] < above:
            raise AssertionError('slab thinner than the halo: use fewer ranks')
        recvs.append((rank + 1, out[:, below + slab.shape[1]:]))
    return out, sends, recvs


def _with_halo(x, own, need, ranges, needs, group):
    """This rank's planes ``x`` (= ``own``) extended to ``need`` with the neighbours' planes:
    ``ranges[r]`` / ``needs[r]`` = planes rank r holds / needs."""
    world, rank = world_and_rank(group)
    if world == 1:
        return x
    # every rank evaluates the same global decision before any p2p call, so a slab thinner than
    # a neighbour's halo makes ALL ranks raise together instead of one raising while its
    # neighbour blocks forever in a send nobody receives
    for r in range(world):
        lo_need = ranges[r][0] - needs[r][0]
        hi_need = needs[r][1] - ranges[r][1]
        if r > 0 and lo_need > ranges[r - 1][1] - ranges[r - 1][0]:
            thin = r - 1   # the lower neighbour cannot supply the planes above rank r
        elif r < world - 1 and hi_need > ranges[r + 1][1] - ranges[r + 1][0]:
            thin = r + 1   # the upper neighbour cannot supply the planes below rank r
        else:
            continue
        raise AssertionError(f'slab of rank {thin} is thinner than the halo rank {r} needs: use fewer ranks')
    local, sends, recvs = _exchange(x, own, need, world, rank, group, ranges)
    if rank > 0:  # rank r-1 needs my first planes above its own
        n_up = needs[rank - 1][1] - ranges[rank - 1][1]
        if n_up > 0:
            sends.append((rank - 1, x[:, :n_up]))
    if rank < world - 1:  # rank r+1 needs my last planes below its own
        n_dn = ranges[rank + 1][0] - needs[rank + 1][0]
        if n_dn > 0:
            sends.append((rank + 1, x[:, x.shape[1] - n_dn:]))
    _p2p(_dist(), group, sends, recvs)
    return local


def encode_halo_exchange(slab, depth, padding=0, group=None):
    """``(local, need)``: this rank's highres slab extended by the halo planes its outputs need."""
    world, rank = world_and_rank(group)
    (z0, z1), own = slab_planes(depth, rank, world)
    if slab.shape[1] != own[1] - own[0]:
        raise AssertionError(f'rank {rank} must hold highres planes {own}, got {slab.shape[1]} planes')
    need = encode_halo(depth, z0, z1, padding)
    ranges = [slab_planes(depth, r, world)[1] for r in range(world)]
    needs = [encode_halo(depth, *slab_planes(depth, r, world)[0], padding) for r in range(world)]
    return _with_halo(slab, own, need, ranges, needs, group), need


def decode_halo_exchange(lowres, depth, padding=0, group=None):
    """``(local, need)``: this rank's lowres planes extended by the halo planes its outputs need."""
    world, rank = world_and_rank(group)
    ez = (depth + 1) // 2
    (z0, z1), _ = slab_planes(depth, rank, world)
    if lowres.shape[1] != z1 - z0:
        raise AssertionError(f'rank {rank} must hold lowres planes {(z0, z1)}, got {lowres.shape[1]} planes')
    need = decode_halo(ez, z0, z1, padding)
    ranges = [slab_planes(depth, r, world)[0] for r in range(world)]
    needs = [decode_halo(ez, *ranges[r], padding) for r in range(world)]
    return _with_halo(lowres, (z0, z1), need, ranges, needs, group), need


def encode_global(predictions_fn, encode_fn, slab, depth, padding=0, group=None):
    """Encode ONE volume held as D-slabs: ``slab`` = this rank's highres planes (``slab_planes``)
    of ``[B, depth, H, W, C...]``.  Returns this rank's planes of the whole-volume
    ``(lowres, (maps, dims))``."""
    world, rank = world_and_rank(group)
    (z0, z1), _ = slab_planes(depth, rank, world)
    local, need = encode_halo_exchange(_nd._dev(slab), depth, padding, group)
    lo, (maps, dims) = encode_local(predictions_fn, encode_fn, local, need[0], (z0, z1), padding)
    return lo, (maps, ((depth + 1) % 2, *dims[1:]))  # the volume's dims, not the local array's


def decode_global(predictions_fn, decode_fn, lowres, encoded, depth, padding=0, group=None):
    """Inverse of :func:`encode_global`: ``lowres`` / ``encoded`` are this rank's planes; returns
    this rank's highres planes (``slab_planes``) of the whole decoded volume."""
    world, rank = world_and_rank(group)
    maps, dims = encoded
    ez = (depth + 1) // 2
    (z0, z1), _ = slab_planes(depth, rank, world)
    local, need = decode_halo_exchange(_nd._dev(lowres), depth, padding, group)
    return decode_local(predictions_fn, decode_fn, local, maps, need[0], (z0, z1), dims, padding,
                        at_top=(need[1] == ez))


def gather_planes(local, total, group=None):
    """Reassemble ``[B, total, ...]`` from each rank's contiguous planes along axis 1: one
    all-gather of equal-size (padded) byte slabs."""
    world, rank = world_and_rank(group)
    if world == 1:
        return local
    dist = _dist()
    x = local.movedim(1, 0).contiguous()  # planes first
    sizes = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    allsz = [torch.zeros_like(sizes) for _ in range(world)]
    dist.all_gather(allsz, sizes, group=group)
    counts = [int(t.item()) for t in allsz]
    biggest = max(counts)
    pad = torch.empty((biggest, *x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[:x.shape[0]] = x
    gathered = torch.empty((biggest * world, *x.shape[1:]), dtype=x.dtype, device=x.device)
    gb, sb = gathered.view(torch.uint8).reshape(-1), pad.view(torch.uint8).reshape(-1)
    if dist.get_backend(group) == 'nccl':
        dist.all_gather_into_tensor(gb, sb, group=group)
    else:
        dist.all_gather(list(gb.chunk(world)), sb, group=group)
    out = torch.cat([gathered[r * biggest: r * biggest + counts[r]] for r in range(world)], 0)
    if out.shape[0] != total:
        raise AssertionError(f'gathered {out.shape[0]} planes, expected {total}')
    return out.movedim(0, 1).contiguous()
