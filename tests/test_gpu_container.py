"""Compressed files (kompressor_amd.container): compress -> file -> decompress is
lossless for every sample type the codec takes (uint8 images, uint16 volumes, int32, float32 bit
patterns), with the predictor recorded in the file; the Rice payload is smaller than the
bit-plane one on structured data; corrupt or foreign files raise ValueError.  The reference has no
file format (volume/encode_decode.py:56), so the byte layout is the build's own ("parity
unpinned"; the payload bytes are pinned to oracle/rice.py by tests/test_packing.py)."""

import numpy as np
import pytest
import torch

from conftest import ROOT  # noqa: F401


def structured(shape, dtype, noise, seed=0):
    """A smooth field (a few Gaussian blobs + a slow wave) plus Gaussian noise of std ``noise`` --
    the kind of data a predictive codec is for (random data is incompressible)."""
    rng = np.random.default_rng(seed)
    grids = np.meshgrid(*[np.arange(s, dtype=np.float32) for s in shape[1:-1]], indexing='ij')
    field = np.zeros(shape[1:-1], np.float32)
    for _ in range(4):
        c = [rng.uniform(0, s) for s in shape[1:-1]]
        w = rng.uniform(8, 24)
        field += rng.uniform(0.3, 1.0) * np.exp(-sum((g - ci) ** 2 for g, ci in zip(grids, c)) / (2 * w * w))
    field += 0.2 * np.sin(grids[-1] / 7.0) * np.cos(grids[0] / 11.0)
    hi = 200 if dtype == np.uint8 else 4000  # a 12-bit-like dynamic range (CT / EM volumes)
    out = np.empty(shape, np.float32)
    for b in range(shape[0]):
        out[b, ..., 0] = 20 + hi * (field - field.min()) / (np.ptp(field) + 1e-6) + rng.normal(0, noise, shape[1:-1])
    if dtype == np.float32:
        return out
    info = np.iinfo(dtype)
    return np.clip(np.round(out), info.min, info.max).astype(dtype)


CASES = [
    ('mean0_u16', 3, (4, 64, 64, 64, 1), np.uint16, 2.0),
    ('mean1_u16_odd', 3, (2, 33, 40, 31, 1), np.uint16, 2.0),
    ('mean0_u8_img', 2, (16, 256, 256, 1), np.uint8, 1.0),
    ('mean0_f32', 3, (2, 64, 64, 64, 1), np.float32, 0.5),
    ('linear0_u16', 3, (2, 32, 32, 32, 1), np.uint16, 2.0),
    ('linearmx0_u16', 3, (2, 32, 64, 64, 1), np.uint16, 2.0),  # arith='bf16x2' (the matrix cores)
    ('mean2_u16', 3, (2, 40, 36, 64, 1), np.uint16, 2.0),      # the z-rolling p = 2 kernel
    ('mean2_u8_img', 2, (4, 100, 256, 1), np.uint8, 1.0),      # the y-rolling image kernel
]


def _predictor(kom, name, ndim):
    p = int(name[4]) if name.startswith('mean') else 0
    if name.startswith('linear'):
        n, k = 8, 19
        w = (np.full((n, k), 1.0 / n) + np.random.default_rng(3).standard_normal((n, k)) * 0.01).astype(np.float32)
        return kom.LinearPredictor(w, np.zeros(k, np.float32), p, ndim,
                                   arith='bf16x2' if name.startswith('linearmx') else 'f32')
    return kom.MeanPredictor(p, ndim)


@pytest.mark.gpu
@pytest.mark.parametrize('method', ['rice', 'planes'])
@pytest.mark.parametrize('name,ndim,shape,dtype,noise', CASES)
def test_compress_decompress_lossless(kom, tmp_path, name, ndim, shape, dtype, noise, method):
    x = structured(shape, dtype, noise)
    pred = _predictor(kom, name, ndim)
    path = str(tmp_path / f'{name}.kmp')
    info = kom.container.compress(path, x, pred, method=method)
    assert info['bytes'] < info['raw_bytes'], info      # structured data shrinks
    back = kom.container.decompress(path)
    assert back.dtype == x.dtype and back.shape == x.shape
    assert np.array_equal(back.view(np.uint8), x.view(np.uint8))
    assert info['levels'] >= 2
    # every stored level equals the reference's single-level encode applied to the previous
    # level's lowres (the predictor came from the file)
    lo, (maps, _), meta = kom.container.load(path)
    assert meta['predictor']['kind'] == ('linear' if name.startswith('linear') else 'mean')
    assert len(meta['levels']) == info['levels'] and len(maps) == info['levels'] * (7 if ndim == 3 else 3)
    h = torch.from_numpy(x).cuda()
    if dtype == np.float32:
        h = h.view(torch.uint32)
    ns = kom.volume if ndim == 3 else kom.image
    enc = {torch.uint16: ns.encode_values_uint16, torch.uint8: ns.encode_values_uint8,
           torch.uint32: kom.volume.encode_values_uint32}[h.dtype]
    nm = 7 if ndim == 3 else 3
    for lvl, ml in enumerate(meta['levels']):
        h, (rmaps, rdims) = ns.encode(pred, enc, h, padding=pred.padding)
        assert tuple(ml['dims']) == tuple(rdims)
        assert all(torch.equal(a, b) for a, b in zip(maps[nm * lvl:nm * (lvl + 1)], rmaps)), lvl
    assert torch.equal(lo, h)


@pytest.mark.gpu
def test_rice_smaller_than_planes_on_structured_volumes(kom, tmp_path):
    """The entropy coder's point: on structured volumes (smooth field + noise of std 1, 4, 16) the
    Rice container is clearly smaller than the bit-plane container, and both beat raw storage."""
    for noise in (1.0, 4.0, 16.0):
        x = structured((4, 64, 64, 64, 1), np.uint16, noise, seed=int(noise))
        pred = kom.MeanPredictor(0, 3)
        r = kom.container.compress(str(tmp_path / 'r.kmp'), x, pred, method='rice')
        p = kom.container.compress(str(tmp_path / 'p.kmp'), x, pred, method='planes')
        assert r['bytes'] < 0.93 * p['bytes'], (noise, r, p)
        assert np.array_equal(kom.container.decompress(str(tmp_path / 'r.kmp')), x)


@pytest.mark.gpu
def test_pyramid_levels_shrink_the_file(kom, tmp_path):
    """Only the coarsest lowres is stored unpredicted: each extra level replaces raw lowres samples
    (1/8 of the voxels at level 1) by small residuals, so the file shrinks with the level count."""
    x = structured((8, 64, 64, 64, 1), np.uint16, 2.0, seed=4)
    pred = kom.MeanPredictor(0, 3)
    sizes = []
    for levels in (1, 2, 4):
        info = kom.container.compress(str(tmp_path / f'l{levels}.kmp'), x, pred, levels=levels)
        assert np.array_equal(kom.container.decompress(str(tmp_path / f'l{levels}.kmp')), x)
        sizes.append(info['bytes'])
    assert sizes[0] > sizes[1] > sizes[2], sizes
    assert sizes[2] < 0.95 * sizes[0], sizes


@pytest.mark.gpu
def test_external_predictor_must_be_passed(kom, tmp_path):
    inner = kom.MeanPredictor(0, 3)

    def my_predictor(lowres):  # an opaque predictions_fn (a trained network would sit here)
        return inner(lowres)

    x = structured((2, 32, 32, 32, 1), np.uint16, 2.0)
    lo, enc = kom.volume.encode(my_predictor, kom.volume.encode_values_uint16, x)
    path = str(tmp_path / 'ext.kmp')
    kom.container.save(path, lo, enc, predictor=my_predictor)
    with pytest.raises(AssertionError, match='external'):
        kom.container.decompress(path)
    assert np.array_equal(kom.container.decompress(path, predictor=inner), x)


@pytest.mark.gpu
@pytest.mark.parametrize('kind,p', [('mean', 1), ('mean', 2), ('linear', 1), ('linear', 0)])
def test_save_records_the_predictors_padding(kom, tmp_path, kind, p):
    """save() of an encode() result made with a padded built-in predictor records the predictor's
    own padding (the default ``padding=None``), so decompress() decodes it without being told;
    a conflicting explicit padding is refused."""
    x = structured((2, 32, 32, 32, 1), np.uint16, 2.0, seed=p)
    if kind == 'mean':
        pred = kom.MeanPredictor(p, 3)
    else:
        n, k = (2 * p + 2) ** 3, 19
        w = (np.full((n, k), 1.0 / n) + np.random.default_rng(p).standard_normal((n, k)) * 0.01).astype(np.float32)
        pred = kom.LinearPredictor(w, np.zeros(k, np.float32), p, 3)
    lo, enc = kom.volume.encode(pred, kom.volume.encode_values_uint16, x, padding=p)
    path = str(tmp_path / f'{kind}{p}.kmp')
    kom.container.save(path, lo, enc, predictor=pred)
    assert kom.container.load(path)[2]['padding'] == p
    assert np.array_equal(kom.container.decompress(path), x)
    if p:
        with pytest.raises(AssertionError, match='padding'):
            kom.container.save(path, lo, enc, predictor=pred, padding=0)


@pytest.mark.gpu
def test_corrupt_files_raise(kom, tmp_path):
    x = structured((2, 32, 32, 32, 1), np.uint16, 2.0)
    path = tmp_path / 'c.kmp'
    kom.container.compress(str(path), x, kom.MeanPredictor(0, 3))
    raw = bytearray(path.read_bytes())
    flipped = bytearray(raw)
    flipped[-9] ^= 0x40                      # one payload bit: the CRC catches it
    (tmp_path / 'flip.kmp').write_bytes(bytes(flipped))
    (tmp_path / 'trunc.kmp').write_bytes(bytes(raw[:-100]))
    (tmp_path / 'foreign.kmp').write_bytes(b'GIF89a' + bytes(64))
    for name in ('flip.kmp', 'trunc.kmp', 'foreign.kmp'):
        with pytest.raises(ValueError):
            kom.container.decompress(str(tmp_path / name))


@pytest.mark.gpu
def test_device_crc_matches_zlib(kom):
    """kmp_crc32 (the file CRC, computed on the device) equals zlib.crc32 for lengths around its
    16-byte chunks, 1 KiB wave steps and 32 KiB wave regions, with the length given directly or read
    by the kernel from device memory (capped at the buffer)."""
    import zlib
    from kompressor_amd import container
    rng = np.random.default_rng(9)
    data = rng.integers(0, 256, size=(3 << 20) + 77, dtype=np.uint8)
    dev_data = torch.from_numpy(data).cuda()
    for n in [0, 1, 15, 16, 17, 1023, 1024, 1025, 32767, 32768, 32769, 100000, (1 << 20) + 3, data.size]:
        got = int(container._device_crc(dev_data, n).cpu().view(torch.uint32).item())
        assert got == zlib.crc32(data[:n].tobytes()), n
    lens = torch.tensor([5000, 10 ** 9], dtype=torch.int64, device='cuda')
    got = int(container._device_crc(dev_data, 70000, lens[0:1].data_ptr()).cpu().view(torch.uint32).item())
    assert got == zlib.crc32(data[:5000].tobytes())
    got = int(container._device_crc(dev_data, 70000, lens[1:2].data_ptr()).cpu().view(torch.uint32).item())
    assert got == zlib.crc32(data[:70000].tobytes())  # a length past the buffer is capped


@pytest.mark.gpu
def test_file_crc_is_zlib_and_split_is_recorded(kom, tmp_path):
    """The CRC a file stores is zlib's CRC-32 of its bundle bytes (files stay readable by any zlib),
    and compress / decompress record their host / device time split."""
    import json
    import struct
    import zlib
    x = structured((2, 32, 32, 32, 1), np.uint16, 2.0)
    path = str(tmp_path / 'z.kmp')
    kom.container.compress(path, x, kom.MeanPredictor(0, 3))
    assert set(kom.container.last_timing) >= {'device', 'd2h_write', 'total'}
    raw = open(path, 'rb').read()
    mlen = struct.unpack('<4sHHQ', raw[:16])[3]
    meta = json.loads(raw[16:16 + mlen])
    body = raw[16 + mlen:]
    assert len(body) == meta['bundle_bytes'] and zlib.crc32(body) == meta['crc32']
    assert np.array_equal(kom.container.decompress(path), x)
    assert set(kom.container.last_timing) >= {'read_upload', 'crc', 'device', 'd2h', 'total'}


@pytest.mark.gpu
def test_oversized_bundle_length_is_rejected_before_allocation(kom, tmp_path):
    """A header whose recorded payload length exceeds the file raises the clean ValueError before any
    host or device buffer is sized from it."""
    import json
    import struct
    x = structured((2, 32, 32, 32, 1), np.uint16, 2.0)
    path = tmp_path / 'c.kmp'
    kom.container.compress(str(path), x, kom.MeanPredictor(0, 3))
    raw = path.read_bytes()
    magic, ver, z, mlen = struct.unpack('<4sHHQ', raw[:16])
    meta = json.loads(raw[16:16 + mlen])
    for bad in (10 ** 15, meta['bundle_bytes'] + 1, -1):
        js = json.dumps(dict(meta, bundle_bytes=bad)).encode()
        js += b' ' * (-len(js) % 8)
        p = tmp_path / 'big.kmp'
        p.write_bytes(struct.pack('<4sHHQ', magic, ver, z, len(js)) + js + raw[16 + mlen:])
        with pytest.raises(ValueError):
            kom.container.decompress(str(p))


@pytest.mark.gpu
def test_arith_mismatch_is_rejected(kom, tmp_path):
    """Decoding a bf16x2-coded file with an f32 LinearPredictor of the same weights (or the reverse)
    raises instead of returning wrong samples (the two arithmetics are not bit-equal)."""
    rng = np.random.default_rng(3)
    w = (rng.standard_normal((8, 19)) / 8).astype(np.float32)
    b = np.zeros(19, np.float32)
    x = structured((2, 32, 32, 32, 1), np.uint16, 2.0)
    for enc, dec in (('bf16x2', 'f32'), ('f32', 'bf16x2')):
        path = str(tmp_path / f'{enc}.kmp')
        kom.container.compress(path, x, kom.LinearPredictor(w, b, 0, 3, arith=enc))
        assert np.array_equal(kom.container.decompress(path), x)
        with pytest.raises(AssertionError):
            kom.container.decompress(path, predictor=kom.LinearPredictor(w, b, 0, 3, arith=dec))


@pytest.mark.gpu
@pytest.mark.parametrize('chunk', [1 << 20, 16 << 20])
def test_chunked_host_transfers(kom, tmp_path, monkeypatch, chunk):
    """The pinned chunk rings (``_device.d2h_stream`` / ``h2d_stream``): to_host of tensors spanning
    several chunks with a ragged tail (the ring path: results above ``PINNED_OUT_MAX``; and the
    pinned-result path below it), and a file whose payload spans several chunks, are exact."""
    from kompressor_amd import _device as dev
    monkeypatch.setattr(dev, 'RING_CHUNK', chunk)
    g = torch.Generator(device='cuda').manual_seed(5)
    for pin_max in (0, dev.PINNED_OUT_MAX):
        monkeypatch.setattr(dev, 'PINNED_OUT_MAX', pin_max)
        for nbytes in (5 << 20, 3 * chunk + 12345, 7 * chunk + 2):
            t = torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device='cuda', generator=g)
            assert np.array_equal(dev.to_host(t), t.cpu().numpy())
        t16 = torch.randint(0, 65536, (3, 77, 129, 131), dtype=torch.int32, device='cuda', generator=g).to(torch.uint16)
        h16 = dev.to_host(t16)
        assert h16.dtype == np.uint16 and h16.shape == tuple(t16.shape) and np.array_equal(h16, t16.cpu().numpy())
    x = np.random.default_rng(1).integers(0, 65536, size=(3, 96, 96, 96, 1), dtype=np.uint16)  # ~5 MiB, incompressible
    path = str(tmp_path / 'r.kmp')
    kom.container.compress(path, x, kom.MeanPredictor(0, 3))
    assert np.array_equal(kom.container.decompress(path), x)


@pytest.mark.gpu
def test_pinned_results_are_released(kom):
    """A to_host result is a pinned array from torch's caching host allocator; once freed,
    ``release_pinned`` hands the cached pinned blocks back (the process does not keep them)."""
    from kompressor_amd import _device as dev
    t = torch.full((48 << 20,), 7, dtype=torch.uint8, device='cuda')
    h = dev.to_host(t)
    assert h.shape == (48 << 20,) and int(h[::4096].sum()) == 7 * ((48 << 20) // 4096)
    del h
    dev.release_pinned()
    st = torch.cuda.host_memory_stats()
    assert st.get('reserved_bytes.current', st.get('segment.current', 0)) < (48 << 20)
    assert np.array_equal(dev.to_host(t[:5 << 20]), np.full(5 << 20, 7, np.uint8))


def _rewrite_meta(src, dst, version=None, **pred_changes):
    """Copy a file with its metadata's predictor entry changed (keys set to None are removed)."""
    import json
    import struct
    raw = open(src, 'rb').read()
    magic, ver, z, mlen = struct.unpack('<4sHHQ', raw[:16])
    meta = json.loads(raw[16:16 + mlen].decode())
    for k, v in pred_changes.items():
        if v is None:
            meta['predictor'].pop(k, None)
        else:
            meta['predictor'][k] = v
    js = json.dumps(meta).encode()
    js += b' ' * (-len(js) % 8)
    open(dst, 'wb').write(struct.pack('<4sHHQ', magic, ver if version is None else version, z, len(js)) + js
                          + raw[16 + mlen:])


@pytest.mark.gpu
def test_arith_revision_recorded_and_enforced(kom, tmp_path):
    """Files record the LinearPredictor arithmetic's revision; a bf16x2 file of another revision (or
    a version-2 file, whose bf16x2 order is ambiguous) raises ValueError instead of decoding into wrong
    samples, while a version-2 f32 file still decodes."""
    from kompressor_amd.predictors import ARITH_REV
    rng = np.random.default_rng(4)
    w = (1 / 64 + rng.standard_normal((64, 19)) * 0.005).astype(np.float32)
    b = np.zeros(19, np.float32)
    x = structured((2, 32, 32, 32, 1), np.uint16, 2.0)
    for arith in ('bf16x2', 'f32'):
        path = str(tmp_path / f'{arith}.kmp')
        kom.container.compress(path, x, kom.LinearPredictor(w, b, 1, 3, arith=arith))
        meta = kom.container.load(path)[2]
        assert meta['predictor']['arith'] == arith and meta['predictor']['arith_rev'] == ARITH_REV[arith]
        assert np.array_equal(kom.container.decompress(path), x)
        old = str(tmp_path / f'{arith}_v2.kmp')
        _rewrite_meta(path, old, version=2, arith_rev=None)
        if arith == 'f32':
            assert np.array_equal(kom.container.decompress(old), x)
        else:
            with pytest.raises(ValueError, match='unrecorded'):
                kom.container.decompress(old)
        other = str(tmp_path / f'{arith}_rev.kmp')
        _rewrite_meta(path, other, arith_rev=ARITH_REV[arith] + 1)
        with pytest.raises(ValueError, match='revision'):
            kom.container.decompress(other)
        with pytest.raises(ValueError, match='revision'):
            kom.container.decompress(other, predictor=kom.LinearPredictor(w, b, 1, 3, arith=arith))


@pytest.mark.gpu
def test_default_predictor_takes_the_files_arith(kom, tmp_path):
    """A default-constructed LinearPredictor (arith='auto') passed to decompress evaluates with the
    arithmetic the file records -- a u16 p = 1 file written with arith='f32' (the pre-round-5
    default) decodes with it, although 'auto' would resolve to bf16x2 there."""
    rng = np.random.default_rng(5)
    w = (1 / 64 + rng.standard_normal((64, 19)) * 0.005).astype(np.float32)
    b = np.zeros(19, np.float32)
    x = structured((1, 32, 32, 32, 1), np.uint16, 2.0)
    path = str(tmp_path / 'f32.kmp')
    kom.container.compress(path, x, kom.LinearPredictor(w, b, 1, 3, arith='f32'))
    auto = kom.LinearPredictor(w, b, 1, 3)
    assert auto.arith_for(torch.uint16) == 'bf16x2'
    assert np.array_equal(kom.container.decompress(path, predictor=auto), x)
    with pytest.raises(AssertionError):  # an explicit mismatch still raises
        kom.container.decompress(path, predictor=kom.LinearPredictor(w, b, 1, 3, arith='bf16x2'))


@pytest.mark.gpu
def test_pinned_results_are_capped(kom, monkeypatch):
    """to_host pins results only while the live pinned bytes stay within PINNED_LIVE_MAX; past it
    results are pageable (ring path), and freeing a pinned result returns its bytes to the budget."""
    from kompressor_amd import _device as dev
    import gc
    gc.collect()
    base = dev.pinned_result_bytes()
    monkeypatch.setattr(dev, 'PINNED_LIVE_MAX', base + (12 << 20))
    t = torch.arange(8 << 20, dtype=torch.int32, device='cuda').to(torch.uint8)  # 8 MiB
    a = dev.to_host(t)
    assert dev.pinned_result_bytes() == base + (8 << 20)
    b = dev.to_host(t)       # would exceed the cap: pageable, not counted
    assert dev.pinned_result_bytes() == base + (8 << 20)
    assert np.array_equal(a, b) and np.array_equal(a, t.cpu().numpy())
    del a
    gc.collect()
    assert dev.pinned_result_bytes() == base
    c = dev.to_host(t)       # the budget is back
    assert dev.pinned_result_bytes() == base + (8 << 20) and np.array_equal(c, b)
    del b, c
    gc.collect()
    assert dev.pinned_result_bytes() == base
