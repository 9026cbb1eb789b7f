"""The C-ABI from a plain C++ host (tools/capi_example.cpp, built by kompressor_amd/_build.py):
no Python layer, no torch -- hipMalloc'd buffers, kmp_volume_encode / kmp_volume_decode on a
stream, round trip + a C-map value checked against the reference arithmetic in the program."""

import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

EXE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools', 'capi_example')


@pytest.mark.parametrize('tiles', [1, 512])
def test_capi_round_trip(tiles):
    assert os.path.exists(EXE), 'tools/capi_example is built by kompressor_amd/_build.py'
    r = subprocess.run([EXE, str(tiles)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert 'capi ok' in r.stdout
