"""Container for coded arrays: entropy-coded payloads of one array or of
a whole ``encode`` result.

The reference stops at residual arrays: ``encode`` returns lowres plus maps of the same total size
as the input (volume/encode_decode.py:56), so nothing gets smaller.  A good predictor leaves small
residuals (modulo 2^W) with a roughly Laplacian distribution; two payload formats store them in
about as many bits as they need, both lossless for every bit pattern:

* ``'rice'`` (default, ``kmp_rice.hip``, spec ``oracle/rice.py``): block-adaptive Golomb-Rice --
  per 64-sample block the parameter k minimising the block's size; k low bit-planes plus the
  unary quotients.  Within ~0.6 bit/sample of the empirical entropy of Laplacian residuals.
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
Array layout (little-endian, 8-byte aligned): ``magic u16 version u16 dtype u32 ndim u32 0 i64 n
i64 nblocks i64 words`` (40 bytes), ``i64 shape[ndim]``, then
  'KMPA' (planes): ``u8 widths[nblocks]`` padded to 8 bytes, ``u64 payload[words]``;
  'KMPR' (rice):   ``u8 params[nblocks]`` padded to 8, ``u8 bw[nblocks]`` padded to 8,
                   ``u32 payload[words]`` padded to 8.
Bundle: ``'KMPB' u16 version u16 count u32 nsp``, ``i32 dims[nsp]`` padded to 8, ``i64
lengths[count]``, then the array blobs (each padded to 8 bytes), lowres first.
"""

import struct

import torch

from . import _device as dev
from ._lib import check, lib

ARRAY_MAGIC = b'KMPA'
RICE_MAGIC = b'KMPR'
BUNDLE_MAGIC = b'KMPB'
VERSION = 1
METHODS = ('rice', 'planes')
_HEAD = struct.Struct('<4sHHIIqqq')  # magic, version, dtype, ndim, reserved, n, nblocks, words (40 bytes)
_HEAD_MAX = _HEAD.size + 8 * 8       # header + the largest shape (ndim <= 8)
_SAMPLE_BITS = {1: 8, 2: 16, 4: 32}


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

    def __init__(self, t, method):
        if method not in METHODS:
            raise ValueError(f'unknown packing method {method!r} (expected one of {METHODS})')
        self.t, self.method = t, method
        self.code, self.n = dev.dtype_code(t), t.numel()
        self.nb = nb = int(lib.kmp_pack_blocks(self.n))
        self.ws = dev.empty((int(lib.kmp_pack_workspace_bytes(self.n)),), torch.uint8)
        self.hlen = _HEAD.size + 8 * t.dim()
        if method == 'rice':  # params | bw, each padded to 8 bytes
            self.side = torch.zeros((2 * _pad8(nb),), dtype=torch.uint8, device='cuda')
            check(lib.kmp_rice_plan(self.code, t.data_ptr(), self.n, self.side.data_ptr(),
                                    self.side.data_ptr() + _pad8(nb), self.ws.data_ptr(), dev.stream()), 'rice')
            self.magic, self.unit = RICE_MAGIC, 4
        else:  # widths, padded to 8 bytes
            self.side = torch.zeros((_pad8(nb),), dtype=torch.uint8, device='cuda')
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
        if self.method == 'rice':
            check(lib.kmp_rice_pack(self.code, t.data_ptr(), self.n, self.side.data_ptr(), self.ws.data_ptr(),
                                    base + self.poff, dev.stream()), 'rice')
        else:
            check(lib.kmp_pack(self.code, t.data_ptr(), self.n, self.side.data_ptr(), self.ws.data_ptr(),
                               base + self.poff, dev.stream()), 'pack')


def _plan_all(arrays, method):
    """Phase 1 for every array, then the ONE synchronisation: (plans, payload words)."""
    plans = [_Plan(dev.to_device(a)[0].contiguous(), method) for a in arrays]
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
    if magic not in (ARRAY_MAGIC, RICE_MAGIC) or version != VERSION or ndim > 8:
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
    per_block = bits if magic == ARRAY_MAGIC else 2 * bits + 2
    if words < 0 or words > nb * per_block:
        raise ValueError(f'array blob payload of {words} words exceeds {nb} blocks of {per_block} words')
    woff = _HEAD.size + 8 * ndim
    if magic == ARRAY_MAGIC:
        poff, total = woff + _pad8(nb), woff + _pad8(nb) + 8 * words
    else:
        poff = woff + 2 * _pad8(nb)
        total = poff + 4 * words
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
    if h['magic'] == ARRAY_MAGIC:
        widths = h['widths'] = b[woff:woff + nb]
        check(lib.kmp_unpack_plan(widths.data_ptr(), n, ws.data_ptr(), dev.stream()), 'unpack')
        check(lib.kmp_unpack_check(0, h['code'], widths.data_ptr(), None, n, ws.data_ptr(), dev.stream()), 'unpack')
    else:
        params = h['params'] = b[woff:woff + nb]
        bw = h['bw'] = b[woff + _pad8(nb):woff + _pad8(nb) + nb]
        check(lib.kmp_unpack_plan(bw.data_ptr(), n, ws.data_ptr(), dev.stream()), 'rice unpack')
        check(lib.kmp_unpack_check(1, h['code'], params.data_ptr(), bw.data_ptr(), n, ws.data_ptr(), dev.stream()),
              'rice unpack')
    # [payload words the stored block sizes add up to, blocks with impossible side information]
    # (kmp_unpack_check: widths past W; Rice k >= W, a zero block with payload, a coded block
    # smaller than its planes + 2 unary words or larger than 2W + 2 words)
    off = int(lib.kmp_pack_total_offset(n))
    return ws[off:off + 16].view(torch.int64)


def _run_unpack(b, h):
    if h['n'] == 0:
        return h['out']
    n, code, ws, out = h['n'], h['code'], h['ws'], h['out']
    if h['magic'] == ARRAY_MAGIC:
        check(lib.kmp_unpack(code, b.data_ptr() + h['poff'], n, h['widths'].data_ptr(), ws.data_ptr(),
                             out.data_ptr(), dev.stream()), 'unpack')
    else:
        check(lib.kmp_rice_unpack(code, b.data_ptr() + h['poff'], n, h['params'].data_ptr(), h['bw'].data_ptr(),
                                  ws.data_ptr(), out.data_ptr(), dev.stream()), 'rice unpack')
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
# public API
# ---------------------------------------------------------------------------------------------

def pack(x, method='rice'):
    """Pack one array (uint8 / uint16 / int32 / uint32 / float32 samples) into a blob."""
    t, kind = dev.to_device(x)
    (plan,), (words,) = _plan_all([t], method)
    out = dev.empty((plan.size(words),), torch.uint8)
    plan.write(out, words)
    return dev.from_device(out, kind)


def unpack(blob):
    """Inverse of :func:`pack`: the array, bit for bit."""
    b, kind = dev.to_device(blob)
    return dev.from_device(_unpack_many(b, [(0, b.numel())])[0], kind)


def pack_encoded(lowres, encoded, method='rice'):
    """One blob for an ``encode`` result ``(lowres, (maps, dims))`` (any number of maps; ``dims``
    may be empty): every array's plan kernels, ONE synchronisation, then every array written in
    place."""
    maps, dims = encoded
    kind = 'torch' if isinstance(lowres, torch.Tensor) else 'numpy'
    plans, words = _plan_all((lowres, *maps), method)
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
    hb = b[:min(b.numel(), 4096)].cpu().numpy().tobytes()
    if len(hb) < 12:
        raise ValueError('truncated bundle')
    magic, version, count, nsp = struct.unpack('<4sHHI', hb[:12])
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
