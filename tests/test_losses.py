"""The product losses (``kompressor_amd.{volume,image}.losses``) against the reference's own loss
spec, ``tests/volume/test_losses.py:39-100`` and ``tests/image/test_losses.py:39-101``: on a ramp
map, MSE / MAE / Charbonnier of ``x + 1`` vs ``x`` are 1.0, the TV of ones is 0.0, and every loss
is a 0-d float32.  numpy and CPU-tensor inputs run here; CUDA tensors (device-resident, no host
round trip) under ``-m gpu``."""

import numpy as np
import pytest
import torch

from conftest import ramp

CASES = [
    ('volume', (2, 4, 4, 4, 1), 65536, np.uint16),   # tests/volume/test_losses.py:36-37
    ('image', (2, 4, 4, 3), 256, np.uint8),          # tests/image/test_losses.py:36-37
]


def _mod(name):
    import kompressor_amd as kom
    return getattr(kom, name).losses


def _check(loss, value, torch_kind):
    if torch_kind:
        assert isinstance(loss, torch.Tensor) and loss.dtype == torch.float32 and loss.dim() == 0
        loss = loss.item()
    else:
        assert np.asarray(loss).dtype == np.float32 and np.asarray(loss).ndim == 0
    assert np.isclose(value, loss), (value, loss)


def _inputs(shape, mx, dt, kind):
    x = ramp(shape, mx, dt)
    # x + 1 in the input dtype, like ``dummy + 1`` on a jnp array (the ramp never reaches the max)
    x1 = (x.astype(np.int64) + 1).astype(dt)
    if kind == 'numpy':
        return x1, x
    if kind == 'cpu':
        return torch.from_numpy(x1), torch.from_numpy(x)
    return torch.from_numpy(x1).cuda(), torch.from_numpy(x).cuda()


def _run_spec(name, shape, mx, dt, kind):
    L = _mod(name)
    x1, x = _inputs(shape, mx, dt, kind)
    t = kind != 'numpy'
    _check(L.mean_squared_error(x1, x), 1.0, t)
    _check(L.mean_abs_error(x1, x), 1.0, t)
    _check(L.mean_charbonnier_error(x1, x, 1e-3), 1.0, t)
    ones = np.ones(shape, dt)
    ones = ones if kind == 'numpy' else (torch.from_numpy(ones) if kind == 'cpu' else torch.from_numpy(ones).cuda())
    tv = L.mean_total_variation(ones)
    _check(tv, 0.0, t)
    if kind == 'cuda':
        assert tv.is_cuda, 'total variation left the device'


@pytest.mark.parametrize('name,shape,mx,dt', CASES)
@pytest.mark.parametrize('kind', ['numpy', 'cpu'])
def test_losses_reference_spec(name, shape, mx, dt, kind):
    _run_spec(name, shape, mx, dt, kind)


@pytest.mark.parametrize('name,shape,mx,dt', CASES)
def test_total_variation_matches_oracle(name, shape, mx, dt):
    """TV of a non-trivial input (random, so unsigned differences wrap) equals the oracle's
    restatement of volume/losses.py:30-35 / image/losses.py:30-34."""
    import oracle
    x = np.random.default_rng(3).integers(0, mx, size=shape, dtype=np.int64).astype(dt)
    got = _mod(name).mean_total_variation(x)
    want = getattr(oracle, name).mean_total_variation(x)
    assert np.isclose(got, want, rtol=1e-6), (got, want)


@pytest.mark.gpu
@pytest.mark.parametrize('name,shape,mx,dt', CASES)
def test_losses_reference_spec_on_device(kom, name, shape, mx, dt):
    _run_spec(name, shape, mx, dt, 'cuda')
    x = np.random.default_rng(3).integers(0, mx, size=shape, dtype=np.int64).astype(dt)
    L = _mod(name)
    a, b = L.mean_total_variation(torch.from_numpy(x).cuda()), L.mean_total_variation(x)
    assert a.is_cuda and np.isclose(a.item(), b, rtol=1e-6)
