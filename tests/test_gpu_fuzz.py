"""Seeded random sweep over the dispatch space: random ndim, batch,
odd / even extents (rows around the wave kernels' eligibility limits), channels, dtype + coder,
padding 0..2, Mean / Linear predictor, whole-array or chunked driver -- the fused HIP path
bit-exact against the oracle's reference step sequence, and lossless.  Each case is small
enough for the numpy oracle; which kernel family serves a case is the dispatcher's choice, so
the sweep crosses the wave / fast / linear / generic boundaries."""

import numpy as np
import pytest
import torch

import oracle
from oracle import predictors as OP

pytestmark = pytest.mark.gpu

CODERS = {  # dtype -> (coder name, value range)
    np.uint8: ('uint8', 256), np.uint16: ('uint16', 65536), np.int32: ('raw', 1 << 20),
    np.uint32: ('uint32', 1 << 32)}


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    ndim = int(rng.choice([2, 3]))
    dtype = [np.uint8, np.uint16, np.int32, np.uint32][int(rng.integers(4))]
    linear = bool(rng.random() < 0.3) and dtype in (np.uint8, np.uint16)
    p = int(rng.integers(0, 3)) if not linear else int(rng.integers(0, 2))
    C = 1 if rng.random() < 0.75 else int(rng.integers(2, 4))
    B = int(rng.integers(1, 4))
    lo_ext = 2 * p + 3
    if ndim == 3:
        sp = [int(rng.integers(lo_ext, 24)), int(rng.integers(lo_ext, 24)), int(rng.choice([8, 16, 17, 31, 32, 64, 65, 128]))]
    else:
        sp = [int(rng.integers(lo_ext, 60)), int(rng.choice([16, 17, 32, 63, 64, 128, 256, 257]))]
    chunk = None if rng.random() < 0.6 else int(rng.integers(4, 12))
    return ndim, dtype, linear, p, C, B, sp, chunk, rng


@pytest.mark.parametrize('seed', range(160))
def test_random_case_matches_oracle(kom, seed):
    ndim, dtype, linear, p, C, B, sp, chunk, rng = _case(seed)
    ns, ons = (kom.volume, oracle.volume) if ndim == 3 else (kom.image, oracle.image)
    cname, vmax = CODERS[dtype]
    enc = getattr(ns, f'encode_values_{cname}')
    dec = getattr(ns, f'decode_values_{cname}')
    oenc = getattr(ons, f'encode_values_{cname}') if hasattr(ons, f'encode_values_{cname}') \
        else getattr(oracle.common, f'encode_values_{cname}')
    x = rng.integers(0, vmax, size=(B, *sp, C), dtype=np.int64).astype(dtype)
    if linear:
        n, k = (2 * p + 2) ** ndim, 19 if ndim == 3 else 5
        w = (rng.standard_normal((n, k)) / n).astype(np.float32)
        bias = rng.standard_normal(k).astype(np.float32)
        pred, opred = kom.LinearPredictor(w, bias, p, ndim), OP.linear_predictions_fn(p, w, bias, ndim)
    else:
        pred, opred = kom.MeanPredictor(p, ndim), OP.mean_predictions_fn(p, ndim)
    want_lo, (want_maps, want_dims) = ons.encode(opred, oenc, x, padding=p)
    xt = torch.from_numpy(x).cuda()
    if chunk is None:
        lo, (maps, dims) = ns.encode(pred, enc, xt, padding=p)
    else:
        lo, (maps, dims) = ns.encode_chunks(pred, enc, xt, chunk=chunk, padding=p)
    case = f'ndim={ndim} {np.dtype(dtype).name} linear={linear} p={p} C={C} shape={(B, *sp, C)} chunk={chunk}'
    assert tuple(int(d) for d in dims) == tuple(int(d) for d in want_dims), case
    assert np.array_equal(lo.cpu().numpy(), want_lo), case
    for i, (a, b) in enumerate(zip(maps, want_maps)):
        a = a.cpu().numpy()
        assert a.dtype == b.dtype and a.shape == b.shape, (case, i)
        assert np.array_equal(a, b), (case, i, int((a != b).sum()))
    rec = ns.decode(pred, dec, lo, (maps, dims), padding=p) if chunk is None else \
        ns.decode_chunks(pred, dec, lo, (maps, dims), chunk=chunk, padding=p)
    assert torch.equal(rec, xt), case
