"""CPU-only checks of the product package: host logic and the C-ABI library (no GPU compute)."""

import ast
import os
import re

import numpy as np
import pytest

import oracle
from conftest import ROOT


def test_library_exports_every_header_symbol():
    import kompressor_amd._lib as L
    header = open(os.path.join(ROOT, 'include', 'kompressor_hip.h')).read()
    declared = set(re.findall(r'^\s*(?:const char\*|int64_t|int)\s+(kmp_\w+)\s*\(', header, re.M))
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(L.lib, name), name
    assert set(L.EXPORTED) >= declared
    assert 'gfx950' in L.version()


def test_debug_library_exports_the_same_c_abi():
    """The KMP_DEBUG=1 variant (device bounds checks compiled in) is built beside the release
    library and exports the identical C-ABI, so the parity suite can run against either."""
    import subprocess
    import sys
    import kompressor_amd._lib as L
    path = os.path.join(ROOT, 'kompressor_amd', 'libkompressor_hip_debug.so')
    if not os.path.exists(path):
        pytest.skip('debug library not built (__graft_entry__.build() builds it)')
    # loaded in a child process: the library is chosen when kompressor_amd._lib is imported
    code = ('import os, sys; os.environ["KMP_DEBUG"] = "1"; sys.path.insert(0, %r); '
            'import kompressor_amd._lib as L; print(L.LIB_PATH); print(L.version()); '
            'print([n for n in L.EXPORTED if not hasattr(L.lib, n)])' % ROOT)
    out = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    assert lines[0].endswith('libkompressor_hip_debug.so')
    assert 'debug' in lines[1] and 'debug' not in L.version()
    assert lines[2] == '[]'


def test_package_imports_and_version():
    import kompressor_amd as kom
    assert isinstance(kom.VERSION, str)  # tests/test_import_module.py:36-40
    for ns in (kom.volume, kom.image):
        for name in ('encode', 'decode', 'encode_chunks', 'decode_chunks', 'targets_from_highres',
                     'lowres_from_highres', 'maps_from_predictions', 'maps_from_highres',
                     'highres_from_lowres_and_maps', 'features_from_lowres', 'pad_neighborhood',
                     'encode_values_raw', 'decode_values_raw', 'encode_values_uint8', 'decode_values_uint8',
                     'encode_values_uint16', 'decode_values_uint16', 'encode_categorical', 'decode_categorical',
                     'mean_squared_error', 'mean_abs_error', 'mean_charbonnier_error', 'mean_total_variation'):
            assert callable(getattr(ns, name)), name
        for name in ('validate_highres', 'validate_lowres', 'validate_chunk', 'validate_padding', 'yield_chunks',
                     'pad_highres', 'pad_lowres', 'pad_map', 'pad_maps', 'trim', 'trim_maps'):
            assert callable(getattr(ns.utils, name)), name


def test_product_never_imports_oracle():
    pkg = os.path.join(ROOT, 'kompressor_amd')
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith('.py'):
                tree = ast.parse(open(os.path.join(dirpath, f)).read())
                for node in ast.walk(tree):
                    if isinstance(node, ast.Import):
                        assert not any(a.name.split('.')[0] == 'oracle' for a in node.names), f
                    if isinstance(node, ast.ImportFrom) and node.module:
                        assert node.module.split('.')[0] != 'oracle', f


def test_no_gpu_means_loud_failure():
    import torch
    import kompressor_amd as kom
    if torch.cuda.is_available():
        pytest.skip('a GPU is visible')
    with pytest.raises(RuntimeError, match='GPU'):
        kom.volume.lowres_from_highres(np.zeros((1, 3, 3, 3, 1), np.uint16))


@pytest.mark.parametrize('max_value', [1, 2, 5, 16, 17, 33, 257])
@pytest.mark.parametrize('chunk', [4, 5, 6, 11, 32])
def test_yield_chunks_matches_oracle(max_value, chunk):
    import kompressor_amd as kom
    assert list(kom.utils.yield_chunks(max_value, chunk)) == list(oracle.common.yield_chunks(max_value, chunk))


def test_validators_volume():
    # tests/volume/test_utils.py:347-444 re-expressed against kompressor_amd
    import kompressor_amd as kom
    V = kom.volume.utils
    z = lambda s: np.zeros(s, np.uint16)  # noqa: E731
    with pytest.raises(AssertionError):
        V.validate_highres(z((2, 3, 3, 3)))
    with pytest.raises(AssertionError):
        V.validate_highres(z((0, 3, 3, 3, 1)))
    for s in [(0, 0, 0), (1, 1, 1), (2, 2, 2), (2, 2, 3), (2, 3, 2), (3, 2, 2), (4, 4, 4), (6, 6, 6)]:
        with pytest.raises(AssertionError):
            V.validate_highres(z((2, *s, 3)))
    for s in [(3, 3, 3), (3, 3, 5), (3, 5, 3), (5, 3, 3)]:
        assert V.validate_highres(z((2, *s, 3))) == s
    for s in [(0, 0, 0), (1, 1, 1), (1, 1, 2), (1, 2, 1), (2, 1, 1)]:
        with pytest.raises(AssertionError):
            V.validate_lowres(z((2, *s, 3)))
    for s in [(2, 2, 2), (2, 2, 3), (2, 3, 2), (3, 2, 2)]:
        assert V.validate_lowres(z((2, *s, 3))) == s
    for p in [None, -2, -1, 1.0]:
        with pytest.raises(Exception):
            V.validate_padding(p)
    for p in [0, 1]:
        V.validate_padding(p)
    for c in [(4,), (4, 4), (4, 4, 4, 4), None, (None, 4, 4), (4, None, 4), (4, 4, None), 3, (3, 4, 4),
              (4, 3, 4), (4, 4, 3)]:
        with pytest.raises(Exception):
            V.validate_chunk(c)
    for c in [4, 5, (4, 4, 5), (4, 5, 4), (5, 4, 4)]:
        assert len(V.validate_chunk(c)) == 3


def test_validators_image():
    import kompressor_amd as kom
    I = kom.image.utils  # noqa: E741
    z = lambda s: np.zeros(s, np.uint8)  # noqa: E731
    with pytest.raises(AssertionError):
        I.validate_highres(z((2, 3, 3)))
    for s in [(0, 0), (1, 1), (2, 2), (2, 3), (3, 2), (4, 4)]:
        with pytest.raises(AssertionError):
            I.validate_highres(z((2, *s, 3)))
    assert I.validate_highres(z((2, 3, 5, 3))) == (3, 5)
    for s in [(1, 1), (1, 2), (2, 1)]:
        with pytest.raises(AssertionError):
            I.validate_lowres(z((2, *s, 3)))
    assert I.validate_lowres(z((2, 2, 3, 3))) == (2, 3)
    for c in [(4,), (4, 4, 4), None, (None, 4), 3, (3, 4)]:
        with pytest.raises(Exception):
            I.validate_chunk(c)
    assert I.validate_chunk(5) == (5, 5)


def test_encode_validates_before_touching_the_device():
    import kompressor_amd as kom
    pred = kom.MeanPredictor(0, 3)
    with pytest.raises(AssertionError):
        kom.volume.encode(pred, kom.volume.encode_values_uint16, np.zeros((2, 1, 3, 3, 1), np.uint16))
    with pytest.raises(AssertionError):
        kom.volume.encode(pred, kom.volume.encode_values_uint16, np.zeros((2, 3, 3, 3, 1), np.uint16), padding=-1)
    with pytest.raises(AssertionError):
        kom.image.encode(kom.MeanPredictor(0, 2), kom.image.encode_values_uint8, np.zeros((2, 3, 3), np.uint8))


def test_encoded_shapes_match_oracle():
    import kompressor_amd as kom
    for shape in [(2, 17, 17, 17, 1), (2, 16, 16, 16, 1), (1, 9, 10, 12, 3), (512, 64, 64, 64, 1)]:
        lo, maps, dims = kom._nd.encoded_shapes(shape, 3)
        o_hi, o_dims = oracle.volume.pad_highres(np.zeros((1, *shape[1:]), np.uint8))
        o_lo = oracle.volume.trim(oracle.volume.lowres_from_highres(o_hi), o_dims)
        o_maps = oracle.volume.trim_maps(oracle.volume.maps_from_highres(o_hi), o_dims)
        assert dims == o_dims and lo[1:] == o_lo.shape[1:]
        assert [m[1:] for m in maps] == [m.shape[1:] for m in o_maps]


def test_fused_chunk_regions_merge_and_cover():
    from kompressor_amd._nd import fused_chunk_regions, yield_chunks
    from itertools import product
    E = (32, 32, 32)
    L = (33, 33, 33)
    chunks = list(product(*[yield_chunks(l, 32) for l in L]))
    regions, covered = fused_chunk_regions(chunks, E, 3)
    assert covered
    # the two slabs (overlapping planes launched once) tile the frame: merged into ONE launch
    assert regions == [[(0, 32), (0, 32), (0, 32)]]
    # odd extents, small chunks, 2D
    for E2, L2, c in [((8, 9), (9, 9), 6), ((17, 16), (17, 17), 11), ((5, 5), (5, 5), 4)]:
        ch = list(product(*[yield_chunks(l, c) for l in L2]))
        regs, cov = fused_chunk_regions(ch, E2, 2)
        assert cov
        lead = np.zeros(E2[0], int)
        for r in regs:
            lead[r[0][0]:r[0][1]] += 1
        assert (lead == 1).all()
    # a filtered chunk list leaves outputs unreached -> not covered
    regs, cov = fused_chunk_regions(chunks[:-1], E, 3)
    assert not cov


def test_pyramid_validates_levels():
    import kompressor_amd as kom
    for bad in (0, -1, 1.5, True):
        with pytest.raises(AssertionError):
            kom.volume.encode_pyramid(kom.MeanPredictor(0, 3), kom.volume.encode_values_uint16,
                                      np.zeros((1, 9, 9, 9, 1), np.uint16), bad)
    with pytest.raises(AssertionError):
        kom.volume.encode_pyramid([kom.MeanPredictor(0, 3)], kom.volume.encode_values_uint16,
                                  np.zeros((1, 9, 9, 9, 1), np.uint16), 2)


def test_container_rejects_foreign_and_truncated_files(tmp_path):
    """kompressor_amd.container reads and checks the file header and the payload CRC on the host
    before anything touches the GPU."""
    import kompressor_amd as kom
    (tmp_path / 'foreign.kmp').write_bytes(b'GIF89a' + bytes(64))
    (tmp_path / 'short.kmp').write_bytes(b'KMP')
    import json
    import struct
    meta = json.dumps({'bundle_bytes': 64, 'crc32': 0}).encode()
    meta += b' ' * (-len(meta) % 8)
    (tmp_path / 'trunc.kmp').write_bytes(struct.pack('<4sHHQ', b'KMPF', 1, 0, len(meta)) + meta + bytes(10))
    (tmp_path / 'crc.kmp').write_bytes(struct.pack('<4sHHQ', b'KMPF', 1, 0, len(meta)) + meta + bytes(range(64)))
    for name in ('foreign.kmp', 'short.kmp', 'trunc.kmp', 'crc.kmp'):
        with pytest.raises(ValueError):
            kom.container.decompress(str(tmp_path / name))


def test_dispatch_options_are_a_table_not_the_environment():
    """Kernel dispatch options live in a process-wide table the library seeds
    from the environment once, at load; set / get / clear work without a GPU and unknown names are
    refused (no getenv per launch)."""
    from kompressor_amd import _lib as L
    assert L.get_option('KMP_DISABLE_FAST') is None
    with L.option('KMP_DISABLE_FAST', 1):
        assert L.get_option('KMP_DISABLE_FAST') == 1
        with L.option('KMP_DISABLE_FAST', None):
            assert L.get_option('KMP_DISABLE_FAST') is None
        assert L.get_option('KMP_DISABLE_FAST') == 1
    assert L.get_option('KMP_DISABLE_FAST') is None
    os.environ['KMP_W3_XCD'] = '0'  # read at load only: changing it now has no effect
    try:
        assert L.get_option('KMP_W3_XCD') is None
    finally:
        del os.environ['KMP_W3_XCD']
    for bad in ('KMP_MP_PPB', 'KMP_W3P_ROLL', 'KMP_W2R_RUN', 'NOT_AN_OPTION'):
        with pytest.raises(L.KompressorHipError):
            L.set_option(bad, 1)
    src = ''.join(open(os.path.join(ROOT, 'kompressor_amd', 'csrc', f)).read()
                  for f in os.listdir(os.path.join(ROOT, 'kompressor_amd', 'csrc')) if f != 'kmp_options.hip')
    assert 'getenv' not in src


def test_linear_auto_arith_rule():
    """LinearPredictor(arith='auto'), the default, resolves by configuration only: the matrix cores
    (bf16x2) for volumes with padding 1 and uint16 samples, the f32 chain elsewhere."""
    import torch
    from kompressor_amd.predictors import resolve_arith
    assert resolve_arith('auto', 1, 3, torch.uint16) == 'bf16x2'
    assert resolve_arith('auto', 1, 3, torch.uint8) == 'bf16x2'
    for p, nd, dt in ((0, 3, torch.uint16), (2, 3, torch.uint16), (0, 3, torch.uint8), (1, 2, torch.uint16),
                      (1, 2, torch.uint8),
                      (1, 3, torch.int32), (1, 3, torch.uint32)):
        assert resolve_arith('auto', p, nd, dt) == 'f32'
    for a in ('f32', 'bf16x2'):
        assert resolve_arith(a, 1, 3, torch.uint16) == a


def test_release_pinned_exported():
    """The package exports the pinned-memory release ("Host memory of numpy
    results"), and the pinned-result threshold is the documented 512 MiB."""
    import kompressor_amd as kom
    from kompressor_amd import _device
    assert kom.release_pinned is _device.release_pinned
    assert _device.PINNED_OUT_MAX == 512 << 20


def test_arith_revision_check():
    """LinearPredictor files carry the arithmetic's revision (predictors.ARITH_REV); a file coded
    under another revision -- or a pre-version-3 bf16x2 file, whose accumulation order is
    ambiguous -- is refused with ValueError, never decoded into wrong samples."""
    from kompressor_amd.container import _check_arith_rev
    from kompressor_amd.predictors import ARITH_REV
    lin = lambda **kw: {'predictor': dict({'kind': 'linear'}, **kw)}  # noqa: E731
    _check_arith_rev({'predictor': {'kind': 'mean'}})
    _check_arith_rev({'predictor': None})
    _check_arith_rev(lin(arith='f32'))                      # version-2 f32 file: the chain is revision 1
    _check_arith_rev(lin())                                 # round-3 file: no arith at all = f32
    for a, r in ARITH_REV.items():
        _check_arith_rev(lin(arith=a, arith_rev=r))
        with pytest.raises(ValueError, match='revision'):
            _check_arith_rev(lin(arith=a, arith_rev=r + 1))
    with pytest.raises(ValueError, match='unrecorded'):
        _check_arith_rev(lin(arith='bf16x2'))               # version-2 bf16x2: round 4 or round 5 order
    with pytest.raises(ValueError):
        _check_arith_rev(lin(arith='bf16x2', arith_rev=1))  # the round-4 accumulation order
    with pytest.raises(ValueError, match='unknown'):
        _check_arith_rev(lin(arith='tf32', arith_rev=1))
