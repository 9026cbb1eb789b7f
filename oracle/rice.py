"""Oracle (test infrastructure only): the build's block-adaptive Rice coding of coded maps, in numpy.

SURVEY.md §8f row f-3 (on-disk format + entropy coding).  The reference has no entropy stage --
encode returns the residual arrays (volume/encode_decode.py:56) -- so this module IS the
specification of the build's entropy-coded payload ("parity unpinned" by the reference); the HIP
kernels (kompressor_amd/csrc/kmp_rice.hip) are pinned to it byte for byte.

Why Rice: a good predictor leaves residuals with a roughly two-sided geometric (Laplacian)
distribution, for which Golomb-Rice codes are within a few percent of the entropy.  The
parameter k adapts per block of 64 samples, so smooth regions and edges each get their own.

Format of one array of n W-bit samples (W = 8, 16, 32):
  * zigzag: the sample's signed W-bit reading s -> z = (s << 1) ^ (s >> (W-1)), masked to W bits
    (0, -1, 1, -2 ... -> 0, 1, 2, 3 ...);
  * blocks of 64 consecutive samples (the last padded with z = 0);
  * per block: S_k = sum_i (z_i >> k) and words(k) = 2k + ceil((64 + S_k) / 32) for k = 0 .. W;
    an all-zero block has param 0 and no payload; otherwise k* = the smallest k minimising
    words(k), param = k* + 1, and the block's payload is words(k*) 32-bit words:
      - k* low bit-planes: plane b (b < k*) is the 64-bit word whose bit i is bit b of z_i,
        stored as two 32-bit words (samples 0-31, then 32-63);
      - the unary part: for i = 0 .. 63, q_i = z_i >> k* zero bits then a one bit; stream bit t
        is bit (t & 31) of unary word t >> 5; zero padded to ceil((64 + S_k*) / 32) words;
  * side information per block: ``params`` (uint8: k* + 1, 0 = all-zero block) and ``bw``
    (uint8: the block's payload words, 2k* + unary words <= 2W + 2);
  * payload: the blocks' words in block order (uint32).
"""

import numpy as np

from .packing import BLOCK, _blocks, sample_bits, unzigzag, zigzag


def plan(x):
    """``(params uint8[nb], bw uint8[nb])`` of the flat array ``x``."""
    x = np.asarray(x)
    W = sample_bits(x.dtype)
    zb = _blocks(zigzag(x.reshape(-1), W))  # [nb, 64] uint64
    nb = zb.shape[0]
    if nb == 0:
        return np.zeros(0, np.uint8), np.zeros(0, np.uint8)
    ks = np.arange(W + 1)
    S = np.stack([(zb >> np.uint64(k)).sum(axis=1) for k in ks], axis=1).astype(np.int64)  # [nb, W+1]
    words = 2 * ks[None, :] + (64 + S + 31) // 32
    kstar = np.argmin(words, axis=1)                       # first minimum: the smallest k
    zero = (zb == 0).all(axis=1)
    params = np.where(zero, 0, kstar + 1).astype(np.uint8)
    bw = np.where(zero, 0, words[np.arange(nb), kstar]).astype(np.uint8)
    return params, bw


def pack(x):
    """``(params, bw, payload uint32[sum(bw)])`` of the flat array ``x``."""
    x = np.asarray(x)
    W = sample_bits(x.dtype)
    params, bw = plan(x)
    zb = _blocks(zigzag(x.reshape(-1), W))
    nb = zb.shape[0]
    off = np.zeros(nb + 1, np.int64)
    np.cumsum(bw.astype(np.int64), out=off[1:])
    payload = np.zeros(int(off[-1]), np.uint32)
    lanes = np.arange(BLOCK, dtype=np.uint64)
    for blk in np.nonzero(params)[0]:
        k = int(params[blk]) - 1
        z = zb[blk]
        o = int(off[blk])
        for b in range(k):
            plane = int(np.bitwise_or.reduce(((z >> np.uint64(b)) & np.uint64(1)) << lanes))
            payload[o + 2 * b] = plane & 0xffffffff
            payload[o + 2 * b + 1] = plane >> 32
        q = (z >> np.uint64(k)).astype(np.int64)
        pos = np.cumsum(q + 1) - 1                          # the terminators' stream positions
        u = o + 2 * k
        np.bitwise_or.at(payload, u + (pos >> 5), (np.uint32(1) << (pos & 31).astype(np.uint32)))
    return params, bw, payload


def unpack(params, bw, payload, n, dtype):
    W = sample_bits(dtype)
    params = np.asarray(params).astype(np.int64)
    bw = np.asarray(bw).astype(np.int64)
    payload = np.asarray(payload, np.uint32)
    nb = len(params)
    off = np.zeros(nb + 1, np.int64)
    np.cumsum(bw, out=off[1:])
    z = np.zeros((nb, BLOCK), np.uint64)
    lanes = np.arange(BLOCK, dtype=np.uint64)
    for blk in np.nonzero(params)[0]:
        k = int(params[blk]) - 1
        o = int(off[blk])
        low = np.zeros(BLOCK, np.uint64)
        for b in range(k):
            plane = np.uint64(int(payload[o + 2 * b]) | (int(payload[o + 2 * b + 1]) << 32))
            low |= ((plane >> lanes) & np.uint64(1)) << np.uint64(b)
        words = payload[o + 2 * k: int(off[blk + 1])]
        bits = ((words[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1).reshape(-1)
        pos = np.nonzero(bits)[0][:BLOCK]                  # the 64 terminators
        q = np.diff(np.concatenate([[-1], pos])) - 1
        z[blk] = (q.astype(np.uint64) << np.uint64(k)) | low
    return unzigzag(z.reshape(-1)[:n], W).view(np.dtype(dtype))


# ---------------------------------------------------------------------------------------------
# Bundle format v2 (kompressor_amd.packing, kmp_rice.hip rice_bundle_*): the byte layout of a
# Rice bundle of several arrays, restated here as the specification the GPU bundle is compared
# against byte for byte (tests/test_packing.py).  Little-endian throughout.
#
#   0   'KMPB'  u16 version = 2  u16 count  u32 nsp  u32 0
#   16  i32 dims[8] (nsp used, the rest 0)
#   48  u64 payload_off  u64 payload_words  u64 bundle_bytes  u64 0
#   80  count records of 128 bytes: u32 dtype code, u32 ndim, i64 shape[8] (zero-padded),
#       i64 n, i64 nb, i64 ntile, i64 side_off, i64 toff_off, u64 first word, u64 end word
#   then for each array params[nb] and bw[nb], each zero-padded to 8 bytes (at side_off);
#   then for each array its tile offsets: u64 word offset of every tile of 256 blocks (at toff_off);
#   then, 8-aligned at payload_off, the payload: every array's blocks in order (array after
#   array), the Rice block payload of ``pack`` above; bundle_bytes = payload_off + the payload
#   zero-padded to 8 bytes.  An empty array (n = 0) has first = end = 0.
# ---------------------------------------------------------------------------------------------

TILE_BLOCKS = 256
DTYPE_CODE = {np.dtype(np.uint8): 0, np.dtype(np.uint16): 1, np.dtype(np.int32): 2, np.dtype(np.float32): 3,
              np.dtype(np.uint32): 4}
CODE_DTYPE = {v: k for k, v in DTYPE_CODE.items()}


def _pad8(n):
    return (n + 7) // 8 * 8


def bundle_layout(ns):
    """``(header bytes, [(side_off, toff_off)], payload_off)`` for arrays of ``ns`` samples."""
    head = 80 + 128 * len(ns)
    off, sides, tofs = head, [], []
    for n in ns:
        nb = -(-n // BLOCK)
        sides.append(off)
        off += 2 * _pad8(nb)
    for n in ns:
        nb = -(-n // BLOCK)
        tofs.append(off)
        off += 8 * (-(-nb // TILE_BLOCKS))
    return head, list(zip(sides, tofs)), _pad8(off)


def pack_bundle(arrays, dims=()):
    """The v2 bundle bytes (numpy uint8) of ``arrays`` (numpy, any shape) and the even-size dims."""
    import struct
    arrays = [np.ascontiguousarray(a) for a in arrays]
    ns = [a.size for a in arrays]
    head, offs, poff = bundle_layout(ns)
    words, recs, parts = 0, [], []
    for a in arrays:
        params, bw, payload = pack(a.reshape(-1))
        nb = len(params)
        boff = np.zeros(nb + 1, np.int64)
        np.cumsum(bw.astype(np.int64), out=boff[1:])
        tiles = (words + boff[:-1][::TILE_BLOCKS]).astype(np.uint64) if nb else np.zeros(0, np.uint64)
        first, end = (words, words + int(boff[-1])) if nb else (0, 0)
        recs.append((params, bw, tiles, first, end))
        parts.append(payload)
        words += int(boff[-1]) if nb else 0
    total = poff + _pad8(4 * words)
    out = np.zeros(total, np.uint8)
    hdr = struct.pack('<4sHHII', b'KMPB', 2, len(arrays), len(dims), 0)
    hdr += struct.pack('<8i', *(list(int(d) for d in dims) + [0] * (8 - len(dims))))
    hdr += struct.pack('<4Q', poff, words, total, 0)
    for a, (side, toff), (params, bw, tiles, first, end) in zip(arrays, offs, recs):
        nb = len(params)
        shape = list(a.shape) + [0] * (8 - a.ndim)
        hdr += struct.pack('<II8q', DTYPE_CODE[a.dtype], a.ndim, *shape)
        hdr += struct.pack('<5q2Q', a.size, nb, len(tiles), side, toff, first, end)
        out[side:side + nb] = params
        out[side + _pad8(nb):side + _pad8(nb) + nb] = bw
        out[toff:toff + 8 * len(tiles)] = tiles.view(np.uint8)
    out[:head] = np.frombuffer(hdr, np.uint8)
    if words:
        out[poff:poff + 4 * words] = np.concatenate(parts).astype(np.uint32).view(np.uint8)
    return out


def unpack_bundle(blob):
    """``(arrays, dims)`` of a v2 bundle (numpy)."""
    import struct
    b = np.asarray(blob, np.uint8).tobytes()
    magic, version, count, nsp, _ = struct.unpack('<4sHHII', b[:16])
    assert magic == b'KMPB' and version == 2
    dims = struct.unpack('<8i', b[16:48])[:nsp]
    poff, words, _, _ = struct.unpack('<4Q', b[48:80])
    payload = np.frombuffer(b, np.uint32, count=words, offset=poff)
    arrays = []
    for i in range(count):
        r = b[80 + 128 * i:80 + 128 * (i + 1)]
        code, ndim = struct.unpack('<II', r[:8])
        shape = struct.unpack('<8q', r[8:72])[:ndim]
        n, nb, ntile, side, toff, first, end = struct.unpack('<5q2Q', r[72:128])
        params = np.frombuffer(b, np.uint8, count=nb, offset=side)
        bw = np.frombuffer(b, np.uint8, count=nb, offset=side + _pad8(nb))
        dt = CODE_DTYPE[code]
        x = unpack(params, bw, payload[first:end], n, np.dtype(dt.str.replace('f', 'u')) if dt.kind == 'f' else dt)
        arrays.append(x.view(dt).reshape(shape))
    return arrays, tuple(dims)
