"""Container for coded arrays: entropy-coded payloads of one array or of
a whole ``encode`` result.

The reference stops at residual arrays: ``encode`` returns lowres plus maps of the same total size
as the input (volume/encode_decode.py:56), so nothing gets smaller.  A good predictor leaves small
residuals (modulo 2^W) with a roughly Laplacian distribution; two payload formats store them in
about as many bits as they need, both lossless for every bit pattern:

* ``'rice'`` (default, ``kmp_rice.hip``, spec ``oracle/rice.py``): block-adaptive Golomb-Rice --
  per 64-sample block the parameter k minimising the block's size; k low bit-planes plus the
  unary quotients.  About 0.5 bit/sample above the order-0 entropy of the residuals: 16 bits of
  side information per 64-sample block plus the unary part padded to a 32-bit word
  (tests/test_ratio.py).
* ``'planes'`` (``kmp_pack.hip``, spec ``oracle/packing.py``): zigzag samples in blocks of 64 as
  ``width`` 64-bit bit-planes, width = the block's largest value's bit length.  Faster to unpack,
  ~0.8 bit/sample larger.

The formats are the build's own -- no reference counterpart, parity pinned to their numpy
specifications ("parity unpinned" by the reference).

    blob = pack(x[, method])                          # one array -> uint8 blob
    x2 = unpack(blob)                                 # bit-identical, same dtype and shape
    blob = pack_encoded(lowres, (maps, dims)[, method])  # a whole encode() result
    lowres, (maps, dims) = unpack_encoded(blob)

Blobs are device uint8 tensors for torch inputs and numpy uint8 arrays for numpy inputs.

'rice' blobs are BUNDLES (format v2, spec ``oracle/rice.py`` pack_bundle): one header, the
arrays' records, their side information and tile-offset tables, then ONE payload region holding
every array's blocks in order.  ``pack`` of one array is a one-array bundle.  Encoding is one
single-pass launch per run of same-dtype arrays (kmp_rice_bundle_encode: the samples are read once;
per-block parameters, a decoupled look-back scan of the tiles' word counts and the payload in the
same pass) and ONE synchronisation for the bundle's size; decoding is one launch per run
(kmp_rice_bundle_decode: tile offsets from the table, no scan) and one synchronisation for the
side-information check.

'planes' blobs keep format v1: array layout (little-endian, 8-byte aligned) ``magic u16 version
u16 dtype u32 ndim u32 0 i64 n i64 nblocks i64 words`` (40 bytes), ``i64 shape[ndim]``, then
``u8 widths[nblocks]`` padded to 8 bytes, ``u64 payload[words]``; bundle v1: ``'KMPB' u16 version=1
u16 count u32 nsp``, ``i32 dims[nsp]`` padded to 8, ``i64 lengths[count]``, then the array blobs
(each padded to 8 bytes), lowres first.
"""

import struct
import threading

import torch

from . import _device as dev
from . import _lib
from ._lib import check, lib

ARRAY_MAGIC = b'KMPA'
BUNDLE_MAGIC = b'KMPB'
VERSION = 1         # planes arrays and bundles
RICE_VERSION = 2    # rice bundles
METHODS = ('rice', 'planes')
_HEAD = struct.Struct('<4sHHIIqqq')  # magic, version, dtype, ndim, reserved, n, nblocks, words (40 bytes)
_HEAD_MAX = _HEAD.size + 8 * 8       # header + the largest shape (ndim <= 8)
_SAMPLE_BITS = {1: 8, 2: 16, 4: 32}


_TLS = threading.local()  # per thread: a pinned staging buffer for header reads (reused: every read synchronises)


def _head_bytes(b, n):
    """The first ``n`` bytes of the device blob ``b`` on the host: one copy into a reused pinned
    buffer (one per thread) and one stream synchronisation (a pageable ``.cpu()`` copy costs a
    fresh allocation)."""
    n = min(int(n), b.numel())
    buf = getattr(_TLS, 'head', None)
    if buf is None or buf.numel() < n:
        buf = _TLS.head = torch.empty((max(n, 4096),), dtype=torch.uint8, pin_memory=True)
    buf[:n].copy_(b[:n], non_blocking=True)
    torch.cuda.current_stream().synchronize()
    return buf[:n].numpy().tobytes()



def _pad8(n):
    return (n + 7) // 8 * 8


# ---------------------------------------------------------------------------------------------
# pack, in two phases so the payloads land in their final place: (1) per array the plan kernels
# (block widths / Rice parameters + the offset scan) write the side information into a small
# buffer and the payload length into the workspace; ONE host synchronisation reads every length;
# (2) the output is allocated at its exact size and every array's header, side information and
# payload are written straight into it (no concatenation copy of the payloads)
# ---------------------------------------------------------------------------------------------

class _Plan:
    """Phase 1 of packing one array; ``write`` is phase 2 once the payload length is known."""

    def __init__(self, t):
        self.t = t
        self.code, self.n = dev.dtype_code(t), t.numel()
        self.nb = nb = int(lib.kmp_pack_blocks(self.n))
        self.ws = dev.empty((int(lib.kmp_pack_workspace_bytes(self.n)),), torch.uint8)
        self.hlen = _HEAD.size + 8 * t.dim()
        self.side = torch.zeros((_pad8(nb),), dtype=torch.uint8, device='cuda')  # widths, padded to 8 bytes
        check(lib.kmp_pack_plan(self.code, t.data_ptr(), self.n, self.side.data_ptr(), self.ws.data_ptr(),
                                dev.stream()), 'pack')
        self.magic, self.unit = ARRAY_MAGIC, 8
        self.poff = self.hlen + self.side.numel()

    def words_view(self):
        off = int(lib.kmp_pack_total_offset(self.n))
        return self.ws[off:off + 8].view(torch.int64)

    def size(self, words):
        return _pad8(self.poff + self.unit * words)

    def write(self, dst, words):
        """Header, side information and payload into the device byte view ``dst`` (``size`` bytes)."""
        t, used = self.t, self.poff + self.unit * words
        head = _HEAD.pack(self.magic, VERSION, self.code, t.dim(), 0, self.n, self.nb, words)
        head += struct.pack(f'<{t.dim()}q', *t.shape)
        base = dst.data_ptr()
        check(lib.kmp_pack_header(base, head, len(head), used, dst.numel(), None, 0, -1, dev.stream()), 'pack')
        dst[self.hlen:self.poff].copy_(self.side)
        check(lib.kmp_pack(self.code, t.data_ptr(), self.n, self.side.data_ptr(), self.ws.data_ptr(),
                           base + self.poff, dev.stream()), 'pack')


def _plan_all(arrays):
    """Phase 1 for every array, then the ONE synchronisation: (plans, payload words)."""
    plans = [_Plan(dev.to_device(a)[0].contiguous()) for a in arrays]
    words = torch.cat([p.words_view() for p in plans]).tolist() if plans else []
    return plans, words


def _write_bytes(dst, data):
    """Host bytes into the device byte view ``dst`` through the header kernel (no host copy sync)."""
    for i in range(0, len(data), 128):
        chunk = data[i:i + 128]
        check(lib.kmp_pack_header(dst.data_ptr() + i, chunk, len(chunk), 0, 0, None, 0, -1, dev.stream()), 'pack')


# ---------------------------------------------------------------------------------------------
# unpack: the headers of all arrays of a call in one device-to-host copy; every header field
# checked against the others on the host; the side information checked on the device and read
# back with ONE synchronisation for all arrays; then the unpack kernels
# ---------------------------------------------------------------------------------------------

def _parse_head(hb, avail):
    """Header fields of an array blob from its first bytes ``hb`` (``avail`` bytes in the blob).
    Every field is checked against the others before anything is launched, so a corrupt or
    hostile blob raises ValueError instead of steering a kernel outside its buffers."""
    if len(hb) < _HEAD.size:
        raise ValueError('truncated array blob')
    magic, version, code, ndim, _, n, nb, words = _HEAD.unpack(hb[:_HEAD.size])
    if magic != ARRAY_MAGIC or version != VERSION or ndim > 8:
        raise ValueError(f'not a kompressor_amd array blob (magic {magic!r}, version {version})')
    if code not in dev.CODE_TO_TORCH:
        raise ValueError(f'array blob has an unknown dtype code {code}')
    if len(hb) < _HEAD.size + 8 * ndim:
        raise ValueError('truncated array blob')
    shape = struct.unpack(f'<{ndim}q', hb[_HEAD.size:_HEAD.size + 8 * ndim])
    if any(s < 0 for s in shape) or n != dev.prod(shape):
        raise ValueError(f'array blob sample count {n} does not match its shape {shape}')
    if nb != int(lib.kmp_pack_blocks(n)):
        raise ValueError(f'array blob has {nb} blocks, {n} samples need {int(lib.kmp_pack_blocks(n))}')
    bits = _SAMPLE_BITS[torch.empty(0, dtype=dev.CODE_TO_TORCH[code]).element_size()]
    if words < 0 or words > nb * bits:
        raise ValueError(f'array blob payload of {words} words exceeds {nb} blocks of {bits} words')
    woff = _HEAD.size + 8 * ndim
    poff, total = woff + _pad8(nb), woff + _pad8(nb) + 8 * words
    if avail < total:
        raise ValueError(f'truncated array blob ({avail} < {total} bytes)')
    return dict(magic=magic, code=code, shape=shape, n=n, nb=nb, woff=woff, poff=poff, words=words, bits=bits)


def _prepare(b, h):
    """Output buffer + the block-offset scan for one parsed blob; returns the device tensor of
    [scanned payload words, bad side-information blocks] to check before unpacking."""
    h['out'] = dev.empty(h['shape'], dev.CODE_TO_TORCH[h['code']])
    if h['n'] == 0:
        return None
    n, nb, woff = h['n'], h['nb'], h['woff']
    ws = h['ws'] = dev.empty((int(lib.kmp_pack_workspace_bytes(n)),), torch.uint8)
    widths = h['widths'] = b[woff:woff + nb]
    check(lib.kmp_unpack_plan(widths.data_ptr(), n, ws.data_ptr(), dev.stream()), 'unpack')
    check(lib.kmp_unpack_check(0, h['code'], widths.data_ptr(), None, n, ws.data_ptr(), dev.stream()), 'unpack')
    # [payload words the stored block sizes add up to, blocks with impossible side information]
    # (kmp_unpack_check: widths past W)
    off = int(lib.kmp_pack_total_offset(n))
    return ws[off:off + 16].view(torch.int64)


def _run_unpack(b, h):
    if h['n'] == 0:
        return h['out']
    n, code, ws, out = h['n'], h['code'], h['ws'], h['out']
    check(lib.kmp_unpack(code, b.data_ptr() + h['poff'], n, h['widths'].data_ptr(), ws.data_ptr(),
                         out.data_ptr(), dev.stream()), 'unpack')
    return out


def _unpack_many(b, spans):
    """The arrays stored at byte ``spans`` [(offset, length)] of the device blob ``b``."""
    if not spans:
        return []
    heads = torch.cat([b[o:o + min(ln, _HEAD_MAX)] for o, ln in spans]).cpu().numpy().tobytes()
    parsed, pos = [], 0
    for o, ln in spans:
        k = min(ln, _HEAD_MAX)
        parsed.append(_parse_head(heads[pos:pos + k], ln))
        pos += k
    views = [b[o:o + ln] for o, ln in spans]
    checks = [(i, _prepare(v, h)) for i, (v, h) in enumerate(zip(views, parsed))]
    live = [(i, c) for i, c in checks if c is not None]
    if live:
        vals = torch.stack([c for _, c in live]).tolist()  # the one synchronisation
        for (i, _), (total, nbad) in zip(live, vals):
            if nbad or total != parsed[i]['words']:
                raise ValueError(f'array blob side information is inconsistent ({nbad} bad blocks, {total} '
                                 f'payload words, header says {parsed[i]["words"]})')
    return [_run_unpack(v, h) for v, h in zip(views, parsed)]


# ---------------------------------------------------------------------------------------------
# rice bundles (format v2): layout on the host, one single-pass launch per run of same-dtype
# arrays, one synchronisation for the size; decode likewise
# ---------------------------------------------------------------------------------------------

_RHEAD = struct.Struct('<4sHHII8i4Q')       # 80 bytes: magic, version, count, nsp, 0, dims[8], payload_off,
_RREC = struct.Struct('<II8q5q2Q')          # payload words, bytes, 0 / 128-byte array record
_TILE_BLOCKS = 256
_MAX_ARRAYS = 1 << 12


def _bundle_layout(ns):
    """``(header bytes, [(side_off, toff_off)], payload_off)`` of a v2 bundle of arrays of ``ns``
    samples (oracle/rice.py bundle_layout)."""
    head = _RHEAD.size + _RREC.size * len(ns)
    off, sides, tofs = head, [], []
    for n in ns:
        sides.append(off)
        off += 2 * _pad8(int(lib.kmp_pack_blocks(n)))
    for n in ns:
        tofs.append(off)
        off += 8 * int(lib.kmp_rice_tiles(n))
    return head, list(zip(sides, tofs)), _pad8(off)


def _runs(ts):
    """Maximal runs of same-dtype arrays, at most 32 per launch: [(first index, count)]."""
    runs, i = [], 0
    while i < len(ts):
        k = i + 1
        while k < len(ts) and k - i < 32 and ts[k].dtype == ts[i].dtype:
            k += 1
        runs.append((i, k - i))
        i = k
    return runs


def _rice_arrays_n(ns, offs, first, count, ptrs):
    """The launch records of arrays ``first .. first + count - 1`` (a fresh ctypes array per call)."""
    arr = (_lib.RiceArray * count)()
    for q in range(count):
        i = first + q
        arr[q].samples = ptrs[i]
        arr[q].n = ns[i]
        arr[q].side_off, arr[q].toff_off = offs[i]
        arr[q].rec_off = _RHEAD.size + _RREC.size * i + 112
    return arr


def _rice_pack_bundle(arrays, dims, exact=True):
    """The bundle as a device byte tensor.  The encode writes into a worst-case sized buffer (the
    size is known only after the launch); ``exact`` returns a copy of the ``total`` bytes so the
    blob does not hold the worst-case allocation alive (callers that copy the blob to the host
    right away pass False and take the view)."""
    out, poff, launched, keep = _rice_encode_launch(arrays, dims)
    if launched:  # the kernel zeroes the side arrays' and the payload's padding
        words, total = struct.unpack('<2q', _head_bytes(out[56:72], 16))  # the one synchronisation
    else:
        total = poff
    del keep
    return out[:total].clone() if exact else out[:total]


# Layouts of recent bundle shapes (header bytes, offsets, tile counts, launch records), keyed by
# the arrays' dtypes and shapes: a repeated pack of same-shaped results (a volume's chunks, a
# series) skips the host-side layout work.  The header is copied from a device copy.
_ENC_PLANS = {}
_DEC_PLANS = {}
_PLAN_CACHE_MAX = 64


def _remember(cache, key, plan):
    if len(cache) >= _PLAN_CACHE_MAX:
        cache.clear()
    cache[key] = plan
    return plan


def _rice_enc_plan(ts, dims):
    key = (tuple((t.dtype, tuple(t.shape)) for t in ts), tuple(int(d) for d in dims))
    plan = _ENC_PLANS.get(key)
    if plan is not None:
        return plan
    if not ts or len(ts) > _MAX_ARRAYS or len(dims) > 8:
        raise ValueError(f'a bundle holds 1 .. {_MAX_ARRAYS} arrays and <= 8 dims')
    for t in ts:
        dev.dtype_code(t)
        if t.dim() > 8:
            raise ValueError('arrays of at most 8 dimensions')
    ns = [t.numel() for t in ts]
    head, offs, poff = _bundle_layout(ns)
    tiles = [int(lib.kmp_rice_tiles(n)) for n in ns]
    worst = sum(int(lib.kmp_pack_blocks(n)) * (2 * 8 * t.element_size() + 2) * 4 for n, t in zip(ns, ts))
    hdr = bytearray(_RHEAD.pack(BUNDLE_MAGIC, RICE_VERSION, len(ts), len(dims), 0,
                                *(list(int(d) for d in dims) + [0] * (8 - len(dims))), poff, 0, poff, 0))
    for t, (side, toff), nt in zip(ts, offs, tiles):
        hdr += _RREC.pack(dev.dtype_code(t), t.dim(), *(list(t.shape) + [0] * (8 - t.dim())), t.numel(),
                          int(lib.kmp_pack_blocks(t.numel())), nt, side, toff, 0, 0)
    T = sum(tiles)
    runs = []
    tile_begin = 0
    for first, count in _runs(ts):
        runs.append((first, count, tile_begin, dev.dtype_code(ts[first])))
        tile_begin += sum(tiles[first:first + count])
    return _remember(_ENC_PLANS, key, {
        'ns': ns, 'offs': offs,
        'head': head, 'poff': poff, 'worst': worst, 'T': T, 'runs': runs,
        'hdr': torch.frombuffer(hdr, dtype=torch.uint8).to('cuda'),
        'ws_bytes': int(lib.kmp_rice_bundle_workspace_bytes(T)) if T else 0})


def _rice_encode_launch(arrays, dims):
    """Everything of a rice pack up to the synchronisation: ``(worst-case sized output, payload
    offset, whether a kernel ran, objects the queued work still reads)``."""
    ts = [dev.to_device(a)[0] for a in arrays]
    plan = _rice_enc_plan(ts, dims)
    poff, head = plan['poff'], plan['head']
    out = dev.empty((poff + plan['worst'] + 8,), torch.uint8)
    out[:head].copy_(plan['hdr'], non_blocking=True)
    if not plan['T'] and poff > head:
        out[head:poff].zero_()
    if plan['T']:
        ws = dev.empty((plan['ws_bytes'],), torch.uint8)
        for first, count, tile_begin, code in plan['runs']:
            # the launch records are built per call (a cached ctypes record shared between threads
            # could be rewritten by another thread while a launch reads it)
            arr = _rice_arrays_n(plan['ns'], plan['offs'], first, count, [t.data_ptr() for t in ts])
            check(lib.kmp_rice_bundle_encode(code, arr, count, tile_begin, plan['T'], out.data_ptr(), poff,
                                             ws.data_ptr(), dev.stream()), 'rice bundle')
    return out, poff, plan['T'] > 0, ts


def _rice_unpack_bundle(b, hb):
    """``(arrays, dims)`` of the v2 bundle ``b`` (device uint8) whose first bytes are ``hb``."""
    outs, dims, bad = _rice_decode_launch(b, hb)
    if bad is not None:
        nbad = int(bad.item())  # the one synchronisation
        if nbad:
            raise ValueError(f'rice bundle side information is inconsistent in {nbad} tiles (corrupt bundle)')
    return outs, dims


def _rice_decode_launch(b, hb):
    """Header checks and the decode launches, no synchronisation: ``(arrays, dims, bad-tile
    counter or None)``."""
    if len(hb) < _RHEAD.size:
        raise ValueError('truncated bundle')
    f = _RHEAD.unpack(hb[:_RHEAD.size])
    count = f[2]
    head = _RHEAD.size + _RREC.size * count if 1 <= count <= _MAX_ARRAYS else _RHEAD.size
    if len(hb) < head:
        hb = b[:head].cpu().numpy().tobytes()
    key = bytes(hb[:head])  # the plan depends on these bytes only (the blob size is checked per call)
    plan = _DEC_PLANS.get(key)
    if plan is None:
        plan = _remember(_DEC_PLANS, key, _rice_dec_plan(b, hb))
    if plan['total'] > b.numel():
        raise ValueError(f'truncated bundle ({b.numel()} < {plan["total"]} bytes)')
    outs = [dev.empty(shape, dev.CODE_TO_TORCH[code]) for shape, code in zip(plan['shapes'], plan['codes'])]
    if plan['T']:
        bad = torch.zeros((1,), dtype=torch.int64, device='cuda')
        for first, count, tile_begin, code in plan['runs']:
            arr = _rice_arrays_n(plan['ns'], plan['offs'], first, count, [t.data_ptr() for t in outs])
            check(lib.kmp_rice_bundle_decode(code, arr, count, tile_begin, b.data_ptr(), plan['poff'], plan['words'],
                                             bad.data_ptr(), dev.stream()), 'rice bundle')
    else:
        bad = None
    return outs, plan['dims'], bad


def _rice_dec_plan(b, hb):
    """The checked layout of a v2 bundle header (everything a decode needs but the payload)."""
    if len(hb) < _RHEAD.size:
        raise ValueError('truncated bundle')
    f = _RHEAD.unpack(hb[:_RHEAD.size])
    magic, version, count, nsp, flags = f[:5]
    if magic != BUNDLE_MAGIC or version != RICE_VERSION:
        raise ValueError(f'not a rice bundle (magic {magic!r}, version {version}; expected {RICE_VERSION})')
    dims = f[5:13]
    poff, words, total, _ = f[13:17]
    if count < 1 or count > _MAX_ARRAYS or nsp > 8 or flags:
        raise ValueError(f'bad rice bundle header (count {count}, nsp {nsp})')
    head = _RHEAD.size + _RREC.size * count
    if len(hb) < head:
        hb = b[:head].cpu().numpy().tobytes()
        if len(hb) < head:
            raise ValueError('truncated bundle')
    recs = [_RREC.unpack(hb[_RHEAD.size + _RREC.size * i:_RHEAD.size + _RREC.size * (i + 1)]) for i in range(count)]
    shapes, codes, ns = [], [], []
    for r in recs:
        code, ndim = r[0], r[1]
        if code not in dev.CODE_TO_TORCH or ndim > 8:
            raise ValueError(f'bad array record (dtype code {code}, ndim {ndim})')
        shape = tuple(r[2:2 + ndim])
        n, nb, nt = r[10], r[11], r[12]
        if any(x < 0 for x in shape) or n != dev.prod(shape) or nb != int(lib.kmp_pack_blocks(n)) or \
                nt != int(lib.kmp_rice_tiles(n)):
            raise ValueError(f'array record sample / block / tile counts do not match its shape {shape}')
        shapes.append(shape)
        codes.append(code)
        ns.append(n)
    ehead, offs, epoff = _bundle_layout(ns)
    if poff != epoff or [(r[13], r[14]) for r in recs] != offs:
        raise ValueError('bundle layout does not match its records')
    if total != poff + _pad8(4 * words):
        raise ValueError(f'bundle size field {total} does not match its payload')
    prev_end = 0
    for r, n, code in zip(recs, ns, codes):
        first, end = r[15], r[16]
        bits = 8 * torch.empty(0, dtype=dev.CODE_TO_TORCH[code]).element_size()
        if n and (first != prev_end or end < first or end > words or end - first > r[11] * (2 * bits + 2)):
            raise ValueError('array payload ranges are inconsistent')
        if n:
            prev_end = end
    if prev_end != words:
        raise ValueError('bundle payload words do not match its arrays')
    tiles = [int(lib.kmp_rice_tiles(n)) for n in ns]
    runs = []
    tile_begin = 0
    for first, count in _runs([torch.empty(0, dtype=dev.CODE_TO_TORCH[c]) for c in codes]):
        runs.append((first, count, tile_begin, codes[first]))
        tile_begin += sum(tiles[first:first + count])
    return {'ns': ns, 'offs': offs, 'shapes': shapes, 'codes': codes, 'dims': tuple(int(d) for d in dims[:nsp]), 'poff': poff,
            'words': words, 'total': total, 'T': sum(tiles), 'runs': runs}


# ---------------------------------------------------------------------------------------------
# public API
# ---------------------------------------------------------------------------------------------

def _check_method(method):
    if method not in METHODS:
        raise ValueError(f'unknown packing method {method!r} (expected one of {METHODS})')


def pack(x, method='rice'):
    """Pack one array (uint8 / uint16 / int32 / uint32 / float32 samples) into a blob ('rice': a
    one-array bundle)."""
    _check_method(method)
    t, kind = dev.to_device(x)
    if method == 'rice':
        return dev.from_device(_rice_pack_bundle([t], ()), kind)
    (plan,), (words,) = _plan_all([t])
    out = dev.empty((plan.size(words),), torch.uint8)
    plan.write(out, words)
    return dev.from_device(out, kind)


def unpack(blob):
    """Inverse of :func:`pack`: the array, bit for bit."""
    b, kind = dev.to_device(blob)
    hb = _head_bytes(b, 4096)
    if hb[:4] == BUNDLE_MAGIC:
        version = struct.unpack('<H', hb[4:6])[0] if len(hb) >= 6 else None
        if version == VERSION:
            raise ValueError('a planes bundle of several arrays (pack_encoded(method="planes")): use unpack_encoded')
        if version != RICE_VERSION:
            raise ValueError(f'unknown bundle version {version}')
        arrays, _ = _rice_unpack_bundle(b, hb)
        if len(arrays) != 1:
            raise ValueError(f'a bundle of {len(arrays)} arrays: use unpack_encoded')
        return dev.from_device(arrays[0], kind)
    return dev.from_device(_unpack_many(b, [(0, b.numel())])[0], kind)


def pack_encoded(lowres, encoded, method='rice'):
    """One blob for an ``encode`` result ``(lowres, (maps, dims))`` (any number of maps; ``dims``
    may be empty).  'rice': one v2 bundle -- a single-pass launch per run of same-dtype arrays and
    ONE synchronisation; 'planes': every array's plan kernels, ONE synchronisation, then every
    array written in place (v1)."""
    _check_method(method)
    maps, dims = encoded
    kind = 'torch' if isinstance(lowres, torch.Tensor) else 'numpy'
    if method == 'rice':
        return dev.from_device(_rice_pack_bundle((lowres, *maps), dims), kind)
    plans, words = _plan_all((lowres, *maps))
    sizes = [p.size(w) for p, w in zip(plans, words)]
    nsp = len(dims)
    head = struct.pack('<4sHHI', BUNDLE_MAGIC, VERSION, len(plans), nsp)
    head += struct.pack(f'<{nsp}i', *[int(d) for d in dims])
    head += b'\0' * (_pad8(len(head)) - len(head))
    head += struct.pack(f'<{len(plans)}q', *sizes)  # every blob is a multiple of 8 bytes
    out = dev.empty((len(head) + sum(sizes),), torch.uint8)
    _write_bytes(out, head)
    off = len(head)
    for p, w, sz in zip(plans, words, sizes):
        p.write(out[off:off + sz], w)
        off += sz
    return dev.from_device(out, kind)


def unpack_encoded(blob):
    """Inverse of :func:`pack_encoded`: ``(lowres, (maps, dims))``."""
    b, kind = dev.to_device(blob)
    hb = _head_bytes(b, 4096)
    if len(hb) < 12:
        raise ValueError('truncated bundle')
    magic, version, count, nsp = struct.unpack('<4sHHI', hb[:12])
    if magic == BUNDLE_MAGIC and version == RICE_VERSION:
        arrays, dims = _rice_unpack_bundle(b, hb)
        arrays = [dev.from_device(a, kind) for a in arrays]
        return arrays[0], (tuple(arrays[1:]), dims)
    if magic != BUNDLE_MAGIC or version != VERSION or nsp > 8:
        raise ValueError(f'not a kompressor_amd bundle (magic {magic!r}, version {version})')
    off = _pad8(12 + 4 * nsp)
    if len(hb) < off + 8 * count:
        hb = b[:off + 8 * count].cpu().numpy().tobytes()
        if len(hb) < off + 8 * count:
            raise ValueError('truncated bundle')
    dims = struct.unpack(f'<{nsp}i', hb[12:12 + 4 * nsp])
    lengths = struct.unpack(f'<{count}q', hb[off:off + 8 * count])
    off += 8 * count
    spans = []
    for ln in lengths:
        if ln < 0 or off + ln > b.numel():
            raise ValueError('truncated bundle')
        spans.append((off, ln))
        off += _pad8(ln)
    arrays = [dev.from_device(a, kind) for a in _unpack_many(b, spans)]
    if not arrays:
        raise ValueError('empty bundle')
    return arrays[0], (tuple(arrays[1:]), tuple(int(d) for d in dims))
