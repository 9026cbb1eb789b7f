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
