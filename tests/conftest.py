"""Shared test helpers.  ``-m gpu`` tests need an MI355X; everything else runs on the CPU."""

import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), '..'))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def pytest_configure(config):
    # the product library is built in-tree (git-ignored); build it once if this checkout lacks it
    if not os.path.exists(os.path.join(ROOT, 'kompressor_amd', 'libkompressor_hip.so')):
        import __graft_entry__
        __graft_entry__._load_builder().build(verbose=False)
    config.addinivalue_line('markers', 'gpu: needs an MI355X (gfx950) GPU and the built libkompressor_hip.so')


def golden_names(prefix=''):
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.endswith('.npz') and f.startswith(prefix))


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_maps(g, ndim):
    return [g[f'map{i}'] for i in range(7 if ndim == 3 else 3)]


@pytest.fixture(scope='session')
def kom():
    """The product package, on a GPU box (skips nothing: gpu tests fail loudly without it)."""
    import kompressor_amd
    kompressor_amd._device.require_gpu()
    return kompressor_amd


def ramp(shape, max_value, dtype):
    # tests/volume/test_encode_decode.py:39-41
    return (np.arange(np.prod(shape)).reshape(shape) % max_value).astype(dtype)


@pytest.fixture
def kmp_opt(kom):
    """``kmp_opt('KMP_DISABLE_FAST', 1)``: set a library dispatch option for this test (the library
    reads its environment once, at load; ``None`` = the kernel's default); restored after."""
    from kompressor_amd import _lib
    saved = {}

    def set_(name, value):
        if name not in saved:
            saved[name] = _lib.get_option(name)
        _lib.set_option(name, value)

    yield set_
    for name, value in saved.items():
        _lib.set_option(name, value)
