"""Container payloads: the numpy specifications (oracle/packing.py: bit-planes,
oracle/rice.py: block-adaptive Rice) on the CPU, and the HIP kernels (kmp_pack.hip, kmp_rice.hip)
byte-for-byte against them on the GPU.  The reference has no container stage, so these pin the
build's own formats ("parity unpinned" by the reference)."""

import numpy as np
import pytest

from oracle import packing as OPK
from oracle import rice as ORC


def _residuals(n, dtype, rng, spread=4):
    """Small signed residuals as the coders store them (wrapped modulo 2^W for unsigned dtypes)."""
    r = rng.integers(-spread, spread + 1, size=n)
    if dtype == np.int32:
        return r.astype(np.int32)
    return (r % (int(np.iinfo(dtype).max) + 1)).astype(dtype)


def test_spec_known_answer():
    # residuals 0, -1, 1, -2 (uint16 wrap) zigzag to 0, 1, 2, 3: one block of width 2;
    # bit-plane 0 = samples 1, 3 -> 0b1010, bit-plane 1 = samples 2, 3 -> 0b1100
    x = np.array([0, 65535, 1, 65534], np.uint16)
    w, payload = OPK.pack(x)
    assert w.tolist() == [2] and payload.tolist() == [0b1010, 0b1100]
    assert np.array_equal(OPK.unpack(w, payload, 4, np.uint16), x)
    w, payload = OPK.pack(np.zeros(130, np.uint8))  # all-zero blocks take no payload
    assert w.tolist() == [0, 0, 0] and payload.size == 0


@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.int32, np.uint32])
@pytest.mark.parametrize('n', [1, 63, 64, 65, 1000])
def test_spec_round_trip(dtype, n):
    rng = np.random.default_rng(n)
    info = np.iinfo(dtype)
    x = rng.integers(info.min, int(info.max) + 1, size=n, dtype=np.int64).astype(dtype)
    x[: n // 2] = _residuals(n // 2, dtype, rng)
    w, payload = OPK.pack(x)
    assert len(w) == -(-n // 64) and payload.size == int(w.astype(np.int64).sum())
    assert w.max() <= np.dtype(dtype).itemsize * 8
    assert np.array_equal(OPK.unpack(w, payload, n, dtype), x)


def test_rice_spec_known_answer():
    # residuals 0, -1, 1, -2 zigzag to 0, 1, 2, 3 (+ 60 zero-padded samples): S_0 = 6, S_1 = 2,
    # words(0) = 0 + ceil(70 / 32) = 3, words(1) = 2 + ceil(66 / 32) = 5 -> k = 0, 3 unary words:
    # sample 0 '1', sample 1 '01', sample 2 '001', sample 3 '0001', then 60 x '1'
    x = np.array([0, 65535, 1, 65534], np.uint16)
    params, bw, payload = ORC.pack(x)
    assert params.tolist() == [1] and bw.tolist() == [3]
    bits = '1' + '01' + '001' + '0001' + '1' * 60
    want = [sum(1 << t for t in range(32) if 32 * i + t < len(bits) and bits[32 * i + t] == '1') for i in range(3)]
    assert payload.tolist() == want
    assert np.array_equal(ORC.unpack(params, bw, payload, 4, np.uint16), x)
    params, bw, payload = ORC.pack(np.zeros(130, np.uint8))  # all-zero blocks take no payload
    assert params.tolist() == [0, 0, 0] and bw.tolist() == [0, 0, 0] and payload.size == 0


@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.int32, np.uint32])
@pytest.mark.parametrize('n', [1, 63, 64, 65, 1000])
def test_rice_spec_round_trip(dtype, n):
    rng = np.random.default_rng(n + 7)
    info = np.iinfo(dtype)
    x = rng.integers(info.min, int(info.max) + 1, size=n, dtype=np.int64).astype(dtype)
    x[: n // 2] = _residuals(n // 2, dtype, rng, spread=40)
    params, bw, payload = ORC.pack(x)
    W = np.dtype(dtype).itemsize * 8
    assert len(params) == -(-n // 64) and payload.size == int(bw.astype(np.int64).sum())
    assert params.max() <= W and bw.max() <= 2 * W + 2
    assert np.array_equal(ORC.unpack(params, bw, payload, n, dtype), x)


def test_rice_beats_planes_on_laplacian_residuals():
    """The reason for the Rice format: on Laplacian residuals (what a good predictor leaves) it is
    within ~0.7 bit/sample of the empirical entropy and clearly below the bit-plane format."""
    rng = np.random.default_rng(0)
    for scale in (1, 4, 16, 100):
        r = np.round(rng.laplace(0, scale, size=1 << 16)).astype(np.int64)
        x = (r % 65536).astype(np.uint16)
        params, bw, payload = ORC.pack(x)
        w, planes = OPK.pack(x)
        rice_bits = (payload.size * 32 + 16 * len(params)) / x.size
        plane_bits = (planes.size * 64 + 8 * len(w)) / x.size
        _, c = np.unique(r, return_counts=True)
        pr = c / c.sum()
        H = float(-(pr * np.log2(pr)).sum())
        assert rice_bits < H + 0.75 and rice_bits < plane_bits - 0.5, (scale, H, rice_bits, plane_bits)


# --------------------------------------------------------------------------------------------- GPU

@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.int32, np.uint32, np.float32])
@pytest.mark.parametrize('shape', [(1,), (64,), (65,), (513,), (3, 17, 19), (2, 4096 * 64 + 5), (3 * 1024 * 64 + 8 * 64 + 17,)])
@pytest.mark.parametrize('spread', [3, 40, 3000])
def test_rice_matches_spec(kom, dtype, shape, spread):
    rng = np.random.default_rng(sum(shape) + spread)
    if dtype == np.float32:
        x = rng.standard_normal(shape).astype(np.float32)
        bits = x.view(np.uint32)
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.min, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)
        flat = x.reshape(-1)
        flat[: flat.size * 3 // 4] = _residuals(flat.size * 3 // 4, dtype, rng, spread=spread)
        flat[: min(flat.size, 200)] = 0  # all-zero blocks too
        bits = x
    blob = kom.packing.pack(x)  # the default method is 'rice': a one-array v2 bundle
    assert isinstance(blob, np.ndarray) and blob.dtype == np.uint8 and bytes(blob[:4]) == b'KMPB'
    want = ORC.pack_bundle([x])
    assert blob.size == want.size
    bad = np.flatnonzero(blob != want)
    assert bad.size == 0, f'{bad.size} bytes differ from the spec, first at {bad[:5].tolist()}'
    back = kom.packing.unpack(blob)
    assert back.dtype == x.dtype and back.shape == x.shape
    assert np.array_equal(back.view(np.uint8), x.view(np.uint8))
    assert np.array_equal(ORC.unpack_bundle(blob)[0][0].view(np.uint8), x.view(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.uint32])
def test_rice_long_unary_runs(kom, dtype):
    """Blocks whose unary part is lopsided: the 8 samples of one lane (8 consecutive samples) are
    large and the rest of the block small, so that lane's 8 codes span more than 64 stream bits and
    the unpack kernel leaves its 64-bit window path for the word-by-word walk; every lane position,
    several magnitudes, and single spikes.  Byte-exact to the spec, lossless."""
    rng = np.random.default_rng(11)
    W = np.dtype(dtype).itemsize * 8
    top = (1 << min(W, 16)) - 1
    blocks = []
    for lane in range(8):
        for mag in (40, 255, 3000, top):
            b = rng.integers(0, 3, size=64)
            b[8 * lane:8 * lane + 8] = rng.integers(mag // 2, mag + 1, size=8)
            blocks.append(b)
            s1 = np.zeros(64, np.int64)
            s1[8 * lane + int(rng.integers(0, 8))] = mag  # one spike, the rest zero
            blocks.append(s1)
    x = (np.concatenate(blocks) * np.where(rng.random(64 * len(blocks)) < 0.5, 1, -1)).astype(np.int64)
    x = (x % (1 << W)).astype(dtype)  # signed residuals in the coder's modular form
    blob = kom.packing.pack(x)
    assert np.array_equal(blob, ORC.pack_bundle([x]))
    assert np.array_equal(kom.packing.unpack(blob), x)


@pytest.mark.gpu
def test_rice_bundle_matches_spec(kom):
    """A bundle of many arrays in one call: mixed sample widths (one launch per run of a dtype),
    an empty array, more than 32 arrays of one dtype (two launches continuing one tile chain), and
    arrays whose tiles end ragged -- byte-exact to oracle/rice.py pack_bundle, lossless both ways."""
    rng = np.random.default_rng(21)
    arrays = [_residuals(70000, np.uint16, rng, spread=30).reshape(70, 1000),
              _residuals(3000, np.int32, rng, spread=500),
              _residuals(5, np.int32, rng),
              np.zeros((0, 4), np.uint16),
              rng.standard_normal((9, 9)).astype(np.float32)]
    arrays += [_residuals(int(rng.integers(1, 9000)), np.uint8, rng, spread=6) for _ in range(40)]
    arrays.append(_residuals(16384 * 3, np.uint16, rng, spread=2))  # exactly 3 tiles
    dims = (1, 0, 1)
    lo, maps = arrays[0], tuple(arrays[1:])
    blob = kom.packing.pack_encoded(lo, (maps, dims))
    want = ORC.pack_bundle(arrays, dims)
    assert blob.size == want.size
    bad = np.flatnonzero(blob != want)
    assert bad.size == 0, f'{bad.size} bytes differ from the spec, first at {bad[:5].tolist()}'
    lo2, (maps2, dims2) = kom.packing.unpack_encoded(blob)
    assert tuple(dims2) == dims
    for a, b in zip(arrays, (lo2, *maps2)):
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.gpu
def test_rice_bundle_rejects_corruption(kom):
    """Flipped side information, tile offsets, records or a truncated bundle raise ValueError (the
    decode kernel bounds every read by the tile / payload extents and counts inconsistent tiles)."""
    rng = np.random.default_rng(3)
    arrays = [_residuals(50000, np.uint16, rng, spread=40), _residuals(9000, np.uint16, rng, spread=3)]
    blob = kom.packing.pack_encoded(arrays[0], ((arrays[1],), (1, 1)))
    side0 = int(blob[80 + 96:80 + 104].view(np.int64)[0])
    toff0 = int(blob[80 + 104:80 + 112].view(np.int64)[0])
    for where, val in ((side0 + 5, 30), (side0 + 5, 0), (side0 + (-(-50000 // 64) + 7) // 8 * 8 + 9, 200),
                       (toff0 + 8, 0x7f), (toff0 + 9, 0x10), (80 + 72, 1), (80 + 112, 3), (56, 0)):
        bad = blob.copy()
        bad[where] = val if bad[where] != val else val ^ 1
        with pytest.raises(ValueError):
            kom.packing.unpack_encoded(bad)
    with pytest.raises(ValueError):
        kom.packing.unpack_encoded(blob[:-16])
    a, (m, _) = kom.packing.unpack_encoded(blob)  # the intact bundle still decodes
    assert np.array_equal(a, arrays[0]) and np.array_equal(m[0], arrays[1])


@pytest.mark.gpu
def test_rice_torch_round_trip_large(kom):
    """A full C3-sized coded map (512 x 32^3 uint16, device-resident): lossless through the Rice
    kernels, and the numpy spec agrees on a slice of blocks."""
    import torch
    rng = np.random.default_rng(5)
    r = np.round(rng.laplace(0, 6, size=(512, 32, 32, 32, 1))).astype(np.int64)
    x = torch.from_numpy((r % 65536).astype(np.uint16)).cuda()
    blob = kom.packing.pack(x)
    assert blob.is_cuda
    back = kom.packing.unpack(blob)
    assert torch.equal(back, x)
    assert blob.numel() < 0.45 * x.numel() * 2



@pytest.mark.gpu
@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.int32, np.uint32, np.float32])
@pytest.mark.parametrize('shape', [(1,), (64,), (65,), (513,), (3, 17, 19), (2, 4096 * 64 + 5), (3 * 1024 * 64 + 8 * 64 + 17,)])
def test_pack_matches_spec(kom, dtype, shape):
    rng = np.random.default_rng(sum(shape))
    if dtype == np.float32:
        x = rng.standard_normal(shape).astype(np.float32)
        bits = x.view(np.uint32)
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.min, int(info.max) + 1, size=shape, dtype=np.int64).astype(dtype)
        flat = x.reshape(-1)
        flat[: flat.size // 2] = _residuals(flat.size // 2, dtype, rng, spread=9)
        bits = x
    blob = kom.packing.pack(x, 'planes')
    assert isinstance(blob, np.ndarray) and blob.dtype == np.uint8
    w, payload = OPK.pack(bits)
    head = 40 + 8 * x.ndim
    nb = len(w)
    assert np.array_equal(blob[head:head + nb], w)
    poff = head + (nb + 7) // 8 * 8
    assert np.array_equal(blob[poff:].view(np.uint64), payload)
    back = kom.packing.unpack(blob)
    assert back.dtype == x.dtype and back.shape == x.shape
    assert np.array_equal(back.view(np.uint8), x.view(np.uint8))


@pytest.mark.gpu
def test_pack_encoded_round_trip_and_ratio(kom):
    """encode -> pack_encoded -> unpack_encoded -> decode is lossless, and a smooth volume's coded
    maps shrink (the container's purpose; random data cannot)."""
    import torch
    z, y, x = np.meshgrid(*[np.arange(64)] * 3, indexing='ij')
    smooth = (1000 + 300 * np.sin(x / 9.0) * np.cos(y / 7.0) + 200 * np.sin(z / 11.0)).astype(np.uint16)
    vol = np.stack([smooth + np.uint16(k) for k in range(8)])[..., None]
    pred = kom.MeanPredictor(0, 3)
    for data in (vol, torch.from_numpy(vol).cuda()):
        lo, enc = kom.volume.encode(pred, kom.volume.encode_values_uint16, data)
        blob = kom.packing.pack_encoded(lo, enc)
        lo2, (maps2, dims2) = kom.packing.unpack_encoded(blob)
        assert tuple(dims2) == tuple(enc[1])
        rec = kom.volume.decode(pred, kom.volume.decode_values_uint16, lo2, (maps2, dims2))
        rec = rec.cpu().numpy() if isinstance(rec, torch.Tensor) else rec
        assert np.array_equal(rec, vol)
        nbytes = blob.numel() if isinstance(blob, torch.Tensor) else blob.size
        assert nbytes < 0.5 * vol.nbytes, nbytes / vol.nbytes


@pytest.mark.gpu
@pytest.mark.parametrize('method', ['rice', 'planes'])
@pytest.mark.parametrize('shape', [(0,), (3, 0, 5)])
def test_pack_empty(kom, shape, method):
    x = np.zeros(shape, np.uint16)
    blob = kom.packing.pack(x, method)
    # header (+ shape), no side information, no payload
    assert blob.size == (80 + 128 if method == 'rice' else 40 + 8 * x.ndim)
    if method == 'rice':
        assert np.array_equal(blob, ORC.pack_bundle([x]))
    back = kom.packing.unpack(blob)
    assert back.shape == x.shape and back.dtype == x.dtype


@pytest.mark.gpu
@pytest.mark.parametrize('method', ['rice', 'planes'])
def test_unpack_rejects_bad_blobs(kom, method):
    x = np.arange(1000, dtype=np.uint16)
    blob = kom.packing.pack(x, method)
    with pytest.raises(ValueError):
        kom.packing.unpack(blob[:-8])          # truncated payload
    bad = blob.copy()
    bad[:4] = np.frombuffer(b'XXXX', np.uint8)
    with pytest.raises(ValueError):
        kom.packing.unpack(bad)                # not a container
    with pytest.raises(ValueError):
        kom.packing.unpack(blob[:10])          # shorter than a header


def _poke(blob, off, fmt, value):
    import struct
    bad = blob.copy()
    bad[off:off + struct.calcsize(fmt)] = np.frombuffer(struct.pack(fmt, value), np.uint8)
    return bad


@pytest.mark.gpu
@pytest.mark.parametrize('method', ['rice', 'planes'])
def test_unpack_rejects_inconsistent_headers(kom, method):
    """every header field is checked against the others before a kernel runs --
    a sample count that disagrees with the shape, a wrong block count, an unknown dtype, a block
    width past the sample size, a payload word count that the widths do not add up to."""
    x = (np.arange(1000) % 7).astype(np.uint16)
    blob = kom.packing.pack(x, method)
    if method == 'planes':
        head = 40 + 8 * x.ndim
        cases = [
            _poke(blob, 16, '<q', 1 << 20),   # n past prod(shape): the kernel would write past `out`
            _poke(blob, 40, '<q', 1 << 20),   # shape past n
            _poke(blob, 24, '<q', 3),         # nblocks too small for n
            _poke(blob, 6, '<H', 99),         # unknown dtype code (ValueError, not KeyError)
            _poke(blob, 32, '<q', 1),         # words smaller than the widths add up to
            _poke(blob, head, '<B', 200),     # a block width past 16 bits
            _poke(blob, head, '<B', 16),      # a legal width whose sum no longer matches words
        ]
    else:  # v2 bundle: header 80 bytes, the array record at 80, params at 208, bw at 224
        cases = [
            _poke(blob, 152, '<q', 1 << 20),  # n past prod(shape)
            _poke(blob, 88, '<q', 1 << 20),   # shape past n
            _poke(blob, 160, '<q', 3),        # nblocks too small for n
            _poke(blob, 168, '<q', 9),        # a tile count that does not match n
            _poke(blob, 80, '<I', 99),        # unknown dtype code
            _poke(blob, 176, '<q', 4096),     # side information moved off the layout
            _poke(blob, 56, '<Q', 1),         # payload words that do not match the bundle size
            _poke(blob, 200, '<Q', 3),        # the array's payload end before its start's blocks
            _poke(blob, 208, '<B', 200),      # a Rice k past 16 bits
            _poke(blob, 208, '<B', 16),       # k = 15 with too few payload words for its planes
            _poke(blob, 224, '<B', 0),        # a coded block claiming no payload
            _poke(blob, 224, '<B', 90),       # more words than a 16-bit block can take
        ]
    for bad in cases:
        with pytest.raises(ValueError):
            kom.packing.unpack(bad)
    assert np.array_equal(kom.packing.unpack(blob), x)


def test_rice_bundle_spec_round_trip():
    """oracle/rice.py's v2 bundle: mixed widths, an empty array, float32 bit patterns, dims."""
    rng = np.random.default_rng(9)
    arrays = [_residuals(3000, np.uint16, rng, spread=20).reshape(3, 1000), _residuals(70, np.int32, rng),
              np.zeros(0, np.uint8), rng.standard_normal((2, 33)).astype(np.float32),
              _residuals(2048 * 2, np.uint8, rng)]
    blob = ORC.pack_bundle(arrays, (1, 0))
    assert bytes(blob[:4]) == b'KMPB' and blob.size % 8 == 0
    back, dims = ORC.unpack_bundle(blob)
    assert dims == (1, 0)
    for a, b in zip(arrays, back):
        assert a.dtype == b.dtype and a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.gpu
def test_rice_layout_caches_follow_the_shapes_and_bytes(kom):
    """packing.py caches bundle layouts by the arrays' dtypes / shapes (pack) and by the header
    bytes (unpack): interleaved packs of differently shaped results give the spec's bytes each
    time; a cached header with a flipped record or a truncated blob still raises."""
    from oracle import rice as ORC
    rng = np.random.default_rng(77)
    a = [rng.integers(-40, 40, size=s).astype(np.int16).view(np.uint16) for s in [(3, 17, 19), (5000,), (64,)]]
    b = [rng.integers(0, 256, size=s).astype(np.uint8) for s in [(2, 70000), (1,)]]
    import torch
    ta = [torch.from_numpy(x).cuda() for x in a]
    tb = [torch.from_numpy(x).cuda() for x in b]
    wa, wb = ORC.pack_bundle(a, (1, 0, 1)), ORC.pack_bundle(b, (1,))
    for _ in range(2):  # the second round hits the caches
        ga = kom.packing.pack_encoded(ta[0], (tuple(ta[1:]), (1, 0, 1))).cpu().numpy()
        gb = kom.packing.pack_encoded(tb[0], (tuple(tb[1:]), (1,))).cpu().numpy()
        assert np.array_equal(ga, wa) and np.array_equal(gb, wb)
        for blob, want in ((ga, a), (gb, b)):
            lo, (maps, _) = kom.packing.unpack_encoded(blob)
            assert all(np.array_equal(x, y) for x, y in zip((lo, *maps), want))
    with pytest.raises(ValueError):
        kom.packing.unpack_encoded(_poke(ga, 80 + 72, '<q', 999))   # record sample count of a cached layout
    with pytest.raises(ValueError):
        kom.packing.unpack_encoded(ga[:-8])                          # truncated blob, cached header


@pytest.mark.gpu
def test_rice_blob_holds_only_its_bytes(kom):
    """A device blob is an exact-size tensor, not a view into the encode's worst-case buffer (which
    is ~1.06x the raw samples for u16): holding many compressed results keeps only their bytes."""
    import torch
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.integers(-3, 4, size=(200_000,)).astype(np.int16).view(np.uint16)).cuda()
    blob = kom.packing.pack(x)
    assert blob.untyped_storage().nbytes() == blob.numel()
    lo = x[:1000].contiguous()
    blob2 = kom.packing.pack_encoded(lo, ((x,), (0,)))
    assert blob2.untyped_storage().nbytes() == blob2.numel()
    assert torch.equal(kom.packing.unpack(blob), x)


@pytest.mark.gpu
def test_rice_pack_unpack_from_threads(kom):
    """pack / unpack from several threads at once on same-shaped inputs (the layout caches are
    shared; the launch records and the pinned header buffer are per call / per thread): every
    thread gets its own blob and its own arrays back."""
    import threading
    import torch
    rng = np.random.default_rng(11)
    xs = [torch.from_numpy(rng.integers(-50, 50, size=(8, 4096)).astype(np.int16).view(np.uint16)).cuda()
          for _ in range(8)]
    want = [ORC.pack_bundle([x.cpu().numpy()], ()) for x in xs]
    errors = []

    def work(i):
        try:
            torch.cuda.set_device(0)
            for _ in range(20):
                blob = kom.packing.pack(xs[i])
                if not np.array_equal(blob.cpu().numpy(), want[i]):
                    errors.append(f'thread {i}: pack bytes')
                if not torch.equal(kom.packing.unpack(blob), xs[i]):
                    errors.append(f'thread {i}: unpack')
        except Exception as e:  # noqa: BLE001
            errors.append(f'thread {i}: {e!r}')

    th = [threading.Thread(target=work, args=(i,)) for i in range(len(xs))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:5]


@pytest.mark.gpu
def test_unpack_names_the_bundle_kind(kom):
    """unpack() of a several-array 'planes' bundle (format v1) names the function to use instead of
    reading it as a rice (v2) header; a rice header with another version is rejected."""
    import torch
    x = torch.from_numpy(np.arange(300, dtype=np.uint16)).cuda()
    b1 = kom.packing.pack_encoded(x, ((x, x), (1, 1)), method='planes')
    with pytest.raises(ValueError, match='unpack_encoded'):
        kom.packing.unpack(b1)
    lo, (maps, dims) = kom.packing.unpack_encoded(b1)
    assert torch.equal(lo, x) and tuple(dims) == (1, 1)
    b2 = kom.packing.pack(x).cpu().numpy().copy()
    b2[4:6] = np.frombuffer(np.uint16(7).tobytes(), np.uint8)
    with pytest.raises(ValueError):
        kom.packing.unpack(b2)
