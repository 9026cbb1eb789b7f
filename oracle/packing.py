"""Oracle (test infrastructure only): the build's bit-plane packing of coded maps, in numpy.

SURVEY.md §8f row f-3.  The reference has NO container or entropy stage -- encode returns the
residual arrays themselves (volume/encode_decode.py:56) -- so there is nothing of the reference's
to restate: this module IS the specification of the build's payload format, and parity of the
HIP kernels (kompressor_amd/csrc/kmp_pack.hip) is pinned to it ("parity unpinned" by the
reference).

Format of one array of n W-bit samples (W = 8, 16, 32):
  * zigzag: the sample's signed W-bit reading s -> (s << 1) ^ (s >> (W-1)), masked to W bits;
  * blocks of 64 consecutive samples (the last zero-padded); width[b] = bit length of the
    block's largest zigzag value (0 .. W);
  * payload: for each block in order, width[b] 64-bit words; word i has bit l set iff bit i of
    sample l's zigzag value is set (bit-plane i of the block).
"""

import numpy as np

BLOCK = 64
_SIGNED = {8: np.int8, 16: np.int16, 32: np.int32}
_UNSIGNED = {8: np.uint8, 16: np.uint16, 32: np.uint32}


def sample_bits(dtype):
    return np.dtype(dtype).itemsize * 8


def zigzag(x, W):
    s = np.ascontiguousarray(x).view(_SIGNED[W]).astype(np.int64)
    return (((s << 1) ^ (s >> (W - 1))) & ((1 << W) - 1)).astype(np.uint64)


def unzigzag(z, W):
    z = z.astype(np.uint64)
    v = (z >> np.uint64(1)) ^ (np.uint64(0) - (z & np.uint64(1)))
    return (v & np.uint64((1 << W) - 1)).astype(_UNSIGNED[W])


def _blocks(z):
    nb = -(-z.size // BLOCK)
    zb = np.zeros(nb * BLOCK, np.uint64)
    zb[:z.size] = z
    return zb.reshape(nb, BLOCK)


def widths(x):
    """Bit length of each block's largest zigzag value."""
    x = np.asarray(x)
    zb = _blocks(zigzag(x.reshape(-1), sample_bits(x.dtype)))
    out = np.zeros(zb.shape[0], np.uint8)
    if zb.shape[0]:
        m = zb.max(axis=1)
        for i in range(33):
            out += (m >= np.uint64(1 << i)).astype(np.uint8)
    return out


def pack(x):
    """``(widths uint8[nb], payload uint64[sum(widths)])`` of the flat array ``x``."""
    x = np.asarray(x)
    W = sample_bits(x.dtype)
    zb = _blocks(zigzag(x.reshape(-1), W))                     # [nb, 64]
    w = widths(x)
    lanes = np.arange(BLOCK, dtype=np.uint64)
    planes = np.stack([np.bitwise_or.reduce(((zb >> np.uint64(i)) & np.uint64(1)) << lanes, axis=1)
                       for i in range(W)], axis=1) if zb.shape[0] else np.zeros((0, W), np.uint64)
    keep = np.arange(W)[None, :] < w[:, None].astype(np.int64)  # planes 0 .. width-1 of each block
    return w, planes[keep].astype(np.uint64)                     # block-major, then plane


def unpack(w, payload, n, dtype):
    W = sample_bits(dtype)
    w = np.asarray(w).astype(np.int64)
    nb = len(w)
    planes = np.zeros((nb, W), np.uint64)
    planes[np.arange(W)[None, :] < w[:, None]] = np.asarray(payload, np.uint64)
    lanes = np.arange(BLOCK, dtype=np.uint64)
    z = np.zeros((nb, BLOCK), np.uint64)
    for i in range(W):
        z |= ((planes[:, i:i + 1] >> lanes) & np.uint64(1)) << np.uint64(i)
    return unzigzag(z.reshape(-1)[:n], W).view(np.dtype(dtype))
