"""The multithreaded torch-CPU restatement of the reference path (oracle/torch_cpu.py, bench.py's
multithreaded CPU comparator) is bit-exact to the numpy op-for-op oracle: lowres, every residual
map, dims, and the decoded output, 2D and 3D, odd / even extents, p = 0, 1, 2, uint8 / uint16 / uint32 (float32 bit patterns, config C5)."""

import numpy as np
import pytest

import oracle
from oracle import predictors as OP
from oracle import torch_cpu as TC


@pytest.mark.parametrize('ndim,shape,dt,p', [
    (3, (2, 17, 17, 17, 1), np.uint16, 0),
    (3, (2, 16, 14, 18, 1), np.uint16, 1),
    (3, (1, 12, 11, 10, 2), np.uint8, 2),
    (3, (3, 16, 16, 16, 1), np.uint8, 0),
    (2, (2, 17, 17, 3), np.uint8, 0),
    (2, (2, 16, 20, 1), np.uint16, 1),
    (2, (1, 14, 13, 1), np.uint8, 2),
    (3, (2, 11, 14, 9, 1), np.uint32, 0),
    (3, (1, 10, 12, 8, 1), np.uint32, 1),
])
def test_torch_cpu_matches_numpy_oracle(ndim, shape, dt, p):
    rng = np.random.default_rng(sum(shape) + p)
    x = rng.integers(0, np.iinfo(dt).max + 1, size=shape, dtype=np.int64).astype(dt)
    if dt == np.uint32:  # float32 bit patterns, NaN / inf / -0 included
        x = (rng.standard_normal(shape).astype(np.float32) * 1000).view(np.uint32)
        x.reshape(-1)[:3] = np.array([np.nan, np.inf, -0.0], np.float32).view(np.uint32)
    ns = oracle.volume if ndim == 3 else oracle.image
    enc, dec = {np.uint16: (ns.encode_values_uint16, ns.decode_values_uint16),
                np.uint8: (ns.encode_values_uint8, ns.decode_values_uint8),
                np.uint32: (ns.encode_values_uint32, ns.decode_values_uint32)}[dt]
    pf = OP.mean_predictions_fn(p, ndim)
    lo, (maps, dims) = ns.encode(pf, enc, x, padding=p)
    tlo, (tmaps, tdims) = TC.encode(x, p, ndim)
    assert tuple(int(d) for d in dims) == tuple(tdims)
    assert tlo.dtype == lo.dtype and np.array_equal(tlo, lo)
    for a, b in zip(tmaps, maps):
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a, b)
    back = TC.decode(tlo, (tmaps, tdims), p, ndim)
    assert back.dtype == x.dtype and np.array_equal(back, x)
