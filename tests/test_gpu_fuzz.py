"""Randomised parity sweep: seeded random configurations -- 2D / 3D, every sample dtype with its
built-in coder, padding 0-2, MeanPredictor or LinearPredictor, ragged and kernel-friendly shapes,
1-2 channels -- each coded by the dispatching C layer (whatever one-pass or generic kernel it picks)
and compared bit for bit with the oracle's restatement of the reference step sequence
(volume/encode_decode.py:30-85, image/encode_decode.py:30-85, the chunked drivers of
*/encode_decode_chunk.py), decoded losslessly, and re-coded through the chunked drivers and the
callback path.  200 cases by default (KMP_FUZZ_CASES; 1 000 passed on the GPU in round 2)."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DTYPES = [(np.uint8, 'uint8'), (np.uint16, 'uint16'), (np.int32, 'raw'), (np.uint32, 'uint32')]
FRIENDLY = [16, 32, 48, 64, 128]  # row lengths the one-pass kernels take


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    ndim = 3 if seed % 2 == 0 else 2
    dtype, coder = DTYPES[int(rng.integers(0, 4))]
    padding = int(rng.integers(0, 3))
    linear = bool(rng.random() < 0.3) and dtype in (np.uint8, np.uint16)
    C = 2 if rng.random() < 0.15 else 1
    hi_dim = 40 if ndim == 3 else 140
    dims = []
    for a in range(ndim):
        if a == ndim - 1 and rng.random() < 0.5:
            dims.append(int(rng.choice(FRIENDLY[:3] if ndim == 3 else FRIENDLY)))
        else:
            dims.append(int(rng.integers(3, hi_dim)))
    B = int(rng.integers(1, 4))
    return ndim, dtype, coder, padding, linear, (B, *dims, C), rng


def _data(rng, shape, dtype):
    if np.issubdtype(dtype, np.unsignedinteger):
        hi = np.iinfo(dtype).max
        if rng.random() < 0.5:  # smooth field + noise: small residuals, structured predictions
            grid = np.indices(shape[1:-1]).sum(axis=0).astype(np.float64)
            base = (np.sin(grid / 7.0) + 1) * (hi / 3)
            x = base[None, ..., None] + rng.normal(0, hi / 200, size=shape)
            return np.clip(x, 0, hi).astype(dtype)
        return rng.integers(0, hi + 1, size=shape, dtype=np.uint64).astype(dtype)
    return rng.integers(-(1 << 31), 1 << 31, size=shape, dtype=np.int64).astype(dtype)


_SEED0 = int(os.environ.get('KMP_FUZZ_SEED0', '0'))  # first case (later sweeps draw new cases)


@pytest.mark.parametrize('seed', range(_SEED0, _SEED0 + int(os.environ.get('KMP_FUZZ_CASES', '200'))))
def test_random_configuration_matches_oracle(kom, seed):
    import oracle
    from oracle import predictors as OP
    ndim, dtype, coder, padding, linear, shape, rng = _case(seed)
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    x = _data(rng, shape, dtype)
    if linear:
        n, k = (2 * padding + 2) ** ndim, 19 if ndim == 3 else 5
        w = (1.0 / n + rng.standard_normal((n, k)) * (0.3 / n)).astype(np.float32)
        b = (rng.standard_normal(k) * 2).astype(np.float32)
        pred, opf = kom.LinearPredictor(w, b, padding, ndim, arith='f32'), OP.linear_predictions_fn(padding, w, b, ndim)
    else:
        pred, opf = kom.MeanPredictor(padding, ndim), OP.mean_predictions_fn(padding, ndim)
    enc, dec = getattr(ns, f'encode_values_{coder}'), getattr(ns, f'decode_values_{coder}')
    oenc, odec = getattr(oracle.common, f'encode_values_{coder}'), getattr(oracle.common, f'decode_values_{coder}')
    info = f'ndim={ndim} dtype={np.dtype(dtype).name} padding={padding} linear={linear} shape={shape}'

    want_lo, (want_maps, want_dims) = ons.encode(opf, oenc, x, padding=padding)
    lo, (maps, dims) = ns.encode(pred, enc, x, padding=padding)
    assert tuple(dims) == tuple(want_dims), info
    assert lo.dtype == want_lo.dtype and np.array_equal(lo, want_lo), info
    for i, (m, r) in enumerate(zip(maps, want_maps)):
        assert m.shape == r.shape and m.dtype == r.dtype, (info, i)
        bad = np.argwhere(m != r)
        assert bad.size == 0, f'{info}: map {i}, {len(bad)} mismatches, first at {bad[:3].tolist()}'
    rec = ns.decode(pred, dec, lo, (maps, dims), padding=padding)
    assert rec.dtype == x.dtype and np.array_equal(rec, x), info

    # the chunked drivers: chunk invariance (encode_decode_chunk.py) against the same result
    chunk = int(rng.integers(4, 12))
    lo2, (maps2, _) = ns.encode_chunks(pred, enc, x, chunk=chunk, padding=padding)
    assert np.array_equal(lo2, want_lo), (info, chunk)
    for i, (m, r) in enumerate(zip(maps2, want_maps)):
        assert np.array_equal(m, r), (info, chunk, i)
    rec2 = ns.decode_chunks(pred, dec, lo, (maps, dims), chunk=chunk, padding=padding)
    assert np.array_equal(rec2, x), (info, chunk)

    # the same volume as a CUDA tensor through an opaque callable (the callback path)
    xt = torch.from_numpy(x).cuda()
    lo3, (maps3, _) = ns.encode(lambda wdw: pred(wdw), enc, xt, padding=padding)
    assert np.array_equal(lo3.cpu().numpy(), want_lo), info
    for i, (m, r) in enumerate(zip(maps3, want_maps)):
        assert np.array_equal(m.cpu().numpy(), r), (info, i)
