"""How good is the entropy stage (VERDICT r2 "give f-3 a ratio bar")?  On the
residual maps of a smooth, noisy C3-like volume (the bench field of tools/bench_rows.py, native
scale, 2 x 2 x 2 tiles of 64^3, MeanPredictor(0) maps through the oracle), compare the Rice payload
(oracle/rice.py, the bytes the GPU writes) with the order-0 empirical entropy of the same residuals,
zlib level 6 and lzma preset 6 on the same bytes.  The reference has no entropy stage
(volume/encode_decode.py:56), so this is the build's own bar ("parity unpinned").

Measured (bits per residual sample; noise = the Gaussian noise std added to the field):

    noise  H0     rice   ideal  zlib   lzma
    1      3.91   4.86   4.36   4.23   3.24
    2      4.28   5.04   4.55   5.21   4.17
    4      4.89   5.46   4.96   6.30   5.10
    16     6.36   6.88   6.38   8.43   6.95

(``ideal`` = the per-block Rice cost without side information or word padding.)  The gap to H0 is
0.5-0.95 bit: 16 bits of side information per 64-sample block (0.25 bit/sample) plus the unary
part padded to a 32-bit word (0.25 on average), the price of decoding every block independently;
the rest is Rice's own redundancy on narrow distributions.  Rice beats zlib from noise 2 up; at
noise 1 the residual is dominated by the field's curvature, a smooth deterministic pattern that
LZ77 matches (and lzma better still) but no memoryless per-sample code can.
"""

import lzma
import zlib

import numpy as np
import pytest

from oracle import predictors as OP
from oracle import rice as ORC
from oracle import volume as OV
from oracle.packing import _blocks, zigzag


def field_volume(n, noise, seed=0, off=(180, 250, 150)):
    zz, yy, xx = np.meshgrid(*[np.arange(o, o + n, dtype=np.float32) for o in off], indexing='ij')
    f = (np.sin(xx / 41.0) * np.cos(yy / 29.0) + np.sin(zz / 53.0 + xx / 97.0)
         + 1.5 * np.exp(-((xx - 200) ** 2 + (yy - 300) ** 2 + (zz - 250) ** 2) / (2 * 90.0 ** 2)))
    f = 4000 + 9000 * (f + 2) / 4.5
    v = np.clip(np.round(f + noise * np.random.default_rng(seed).standard_normal(f.shape)), 0, 65535).astype(np.uint16)
    t = n // 64
    return v.reshape(t, 64, t, 64, t, 64).transpose(0, 2, 4, 1, 3, 5).reshape(-1, 64, 64, 64, 1)


def ratio_row(noise):
    x = field_volume(128, noise)
    _, (maps, _) = OV.encode(OP.mean_predictions_fn(0, 3), OV.encode_values_uint16, x)
    res = np.concatenate([m.reshape(-1) for m in maps])
    n = res.size
    p = np.bincount(res.astype(np.int64), minlength=65536)
    p = p[p > 0] / n
    h0 = float(-(p * np.log2(p)).sum())
    rice = sum(ORC.pack(m.reshape(-1))[2].size * 32 + 16 * -(-m.size // 64) for m in maps) / n
    ideal = 0
    for m in maps:
        z = _blocks(zigzag(m.reshape(-1), 16)).astype(np.int64)
        ideal += int(np.min(np.stack([64 * k + 64 + (z >> k).sum(1) for k in range(17)], 1), 1).sum())
    return {'H0': h0, 'rice': rice, 'ideal': ideal / n, 'zlib': 8 * len(zlib.compress(res.tobytes(), 6)) / n,
            'lzma': 8 * len(lzma.compress(res.tobytes(), preset=6)) / n}


@pytest.mark.parametrize('noise', [1.0, 2.0, 4.0, 16.0])
def test_rice_within_a_stated_gap_of_the_entropy(noise):
    r = ratio_row(noise)
    print(noise, {k: round(v, 3) for k, v in r.items()})
    assert r['rice'] - r['H0'] < 1.0, r                 # the stated gap
    assert r['rice'] - r['ideal'] < 0.55, r             # side information + word padding, at most
    if noise >= 2:
        assert r['rice'] < r['zlib'], r                 # beats a general-purpose coder on real noise
