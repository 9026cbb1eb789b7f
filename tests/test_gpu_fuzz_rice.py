"""Randomised parity sweep of the Rice bundle (spec oracle/rice.py): seeded
random bundles -- 1-6 arrays of mixed sample dtypes (uint8 / uint16 / int32 / uint32 / float32),
ragged sizes around the block (64) and tile (16 384 samples) boundaries, and residual
distributions that reach every path of the kernels: small Laplacian residuals (32-bit unary masks,
short streams), wide spreads (large k), single spikes and lopsided lanes (a lane's 8 codes past 32
and 64 bits, unary streams past 8 words: the word-walk fallbacks), all-zero blocks and runs.  Each
bundle is packed by the HIP kernels (one single-pass launch per run of same-dtype arrays), compared
byte for byte with the numpy specification, and unpacked losslessly.  120 cases by default
(KMP_FUZZ_RICE_CASES, first seed KMP_FUZZ_SEED0)."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DTYPES = [np.uint8, np.uint16, np.int32, np.uint32, np.float32]
EDGE_SIZES = [0, 1, 63, 64, 65, 511, 16383, 16384, 16385, 2 * 16384 + 7]


def _segment(rng, n, dtype):
    """n samples of one residual regime, as the dtype's bit pattern."""
    W = 8 * np.dtype(dtype).itemsize
    kind = rng.choice(['laplace', 'wide', 'spikes', 'lopsided', 'zeros', 'uniform'],
                      p=[0.35, 0.15, 0.15, 0.15, 0.1, 0.1])
    if kind == 'laplace':
        v = np.round(rng.laplace(0, rng.choice([0.3, 1.0, 4.0, 30.0]), n))
    elif kind == 'wide':
        v = np.round(rng.laplace(0, 2.0 ** rng.integers(2, W - 2), n))
    elif kind == 'spikes':
        v = np.round(rng.laplace(0, 1.0, n))
        hit = rng.random(n) < 0.02
        v[hit] = rng.integers(-(1 << (W - 2)), 1 << (W - 2), int(hit.sum()))
    elif kind == 'lopsided':  # whole lanes (8 consecutive samples) large, the rest small
        v = np.round(rng.laplace(0, 0.5, n))
        lanes = rng.random(-(-n // 8)) < 0.1
        big = np.repeat(lanes, 8)[:n]
        v[big] = rng.integers(1 << min(W - 3, 10), 1 << (W - 2), int(big.sum()))
    elif kind == 'zeros':
        v = np.zeros(n)
    else:
        return rng.integers(0, 1 << W, n, dtype=np.uint64).astype(np.dtype(f'u{W // 8}'))
    return np.mod(v.astype(np.int64), 1 << W).astype(np.dtype(f'u{W // 8}'))


def _array(rng, dtype):
    n = int(rng.choice(EDGE_SIZES)) if rng.random() < 0.35 else int(rng.integers(0, 70000))
    parts, left = [], n
    while left > 0:
        m = min(left, int(rng.integers(1, 20000)))
        parts.append(_segment(rng, m, dtype))
        left -= m
    bits = np.concatenate(parts) if parts else np.zeros(0, np.dtype(f'u{np.dtype(dtype).itemsize}'))
    x = bits.view(dtype)
    if n and n % 4 == 0 and rng.random() < 0.5:
        x = x.reshape(4, n // 4)
    return x


_SEED0 = int(os.environ.get('KMP_FUZZ_SEED0', '0'))


@pytest.mark.parametrize('seed', range(_SEED0, _SEED0 + int(os.environ.get('KMP_FUZZ_RICE_CASES', '120'))))
def test_random_bundle_matches_spec(kom, seed):
    from oracle import rice as ORC
    rng = np.random.default_rng(5000 + seed)
    count = int(rng.integers(1, 7))
    same = rng.random() < 0.5
    d0 = DTYPES[int(rng.integers(0, len(DTYPES)))]
    arrays = [_array(rng, d0 if same else DTYPES[int(rng.integers(0, len(DTYPES)))]) for _ in range(count)]
    dims = tuple(int(d) for d in rng.integers(0, 2, int(rng.integers(0, 4))))
    want = ORC.pack_bundle(arrays, dims)
    dev = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrays]
    blob = kom.packing.pack_encoded(dev[0], (tuple(dev[1:]), dims))
    got = blob.cpu().numpy()
    assert got.size == want.size, (seed, got.size, want.size)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f'seed {seed}: {bad.size} bytes differ from the spec, first at {bad[:5].tolist()}'
    lo, (maps, dims2) = kom.packing.unpack_encoded(blob)
    assert tuple(dims2) == dims
    for a, b in zip(arrays, (lo, *maps)):
        b = b.cpu().numpy()
        assert b.dtype == a.dtype and b.shape == a.shape
        assert np.array_equal(b.view(np.uint8), a.view(np.uint8)), seed
