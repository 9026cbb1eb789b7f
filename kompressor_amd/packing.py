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


def _pad8(n):
    return (n + 7) // 8 * 8


def _device_bytes(b):
    """A device uint8 tensor holding ``b`` (<= 128 bytes), written by a kernel, no host copy."""
    out = dev.empty((len(b),), torch.uint8)
    check(lib.kmp_pack_header(out.data_ptr(), b, len(b), 0, 0, None, 0, -1, dev.stream()), 'pack')
    return out


def _pack_device(t):
    """Plan (block widths + scan) and pack straight into a worst-case-sized blob, then ONE host
    synchronisation to learn the payload length; the blob returned is a view of that buffer."""
    t = t.contiguous()
    code = dev.dtype_code(t)
    n = t.numel()
    nb = int(lib.kmp_pack_blocks(n))
    ws = dev.empty((int(lib.kmp_pack_workspace_bytes(n)),), torch.uint8)
    head = _HEAD.pack(ARRAY_MAGIC, VERSION, code, t.dim(), 0, n, nb, 0) + struct.pack(f'<{t.dim()}q', *t.shape)
    woff = len(head)
    poff = woff + _pad8(nb)
    cap = poff + nb * t.element_size() * 64  # every block at full width
    out = dev.empty((cap,), torch.uint8)
    wptr = out.data_ptr() + woff
    check(lib.kmp_pack_plan(code, t.data_ptr(), n, wptr, ws.data_ptr(), dev.stream()), 'pack')
    check(lib.kmp_pack(code, t.data_ptr(), n, wptr, ws.data_ptr(), out.data_ptr() + poff, dev.stream()), 'pack')
    # header + widths padding + the scan's word count (offset 32), from kernel arguments
    check(lib.kmp_pack_header(out.data_ptr(), head, len(head), woff + nb, poff, ws.data_ptr(), n, 32, dev.stream()),
          'pack')
    words = int(out[32:40].view(torch.int64).item())  # the one host synchronisation
    return out[:poff + 8 * words]


_SAMPLE_BITS = {1: 8, 2: 16, 4: 32}


def _pack_rice_device(t):
    """Rice plan (params + bw + scan) and pack straight into a worst-case-sized blob; header and
    padding written by kernels; ONE host synchronisation for the payload length."""
    t = t.contiguous()
    code = dev.dtype_code(t)
    n = t.numel()
    nb = int(lib.kmp_pack_blocks(n))
    bits = _SAMPLE_BITS[t.element_size()]
    ws = dev.empty((int(lib.kmp_pack_workspace_bytes(n)),), torch.uint8)
    head = _HEAD.pack(RICE_MAGIC, VERSION, code, t.dim(), 0, n, nb, 0) + struct.pack(f'<{t.dim()}q', *t.shape)
    aoff = len(head)
    boff = aoff + _pad8(nb)
    poff = boff + _pad8(nb)
    cap = poff + _pad8(4 * nb * (2 * bits + 2))  # every block at its largest
    out = dev.empty((cap,), torch.uint8)
    base = out.data_ptr()
    check(lib.kmp_rice_plan(code, t.data_ptr(), n, base + aoff, base + boff, ws.data_ptr(), dev.stream()), 'rice')
    check(lib.kmp_rice_pack(code, t.data_ptr(), n, base + aoff, ws.data_ptr(), base + poff, dev.stream()), 'rice')
    check(lib.kmp_pack_header(base, b'', 0, aoff + nb, boff, None, 0, -1, dev.stream()), 'rice')
    check(lib.kmp_pack_header(base, head, len(head), boff + nb, poff, ws.data_ptr(), n, 32, dev.stream()), 'rice')
    words = int(out[32:40].view(torch.int64).item())  # the one host synchronisation
    end = poff + _pad8(4 * words)
    if end > poff + 4 * words:  # zero the payload's tail padding
        check(lib.kmp_pack_header(base, b'', 0, poff + 4 * words, end, None, 0, -1, dev.stream()), 'rice')
    return out[:end]


def _parse_array(b):
    """(dtype code, shape, n, nb, widths offset, payload offset, total bytes, words) of an array
    blob: one device-to-host read of the header.  Every header field is checked against the others
    before anything is launched, so a corrupt or hostile blob raises ValueError instead of steering
    a kernel outside its buffers."""
    hb = bytes(b[:min(b.numel(), _HEAD.size + 8 * 8)].cpu().numpy())
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
        poff = woff + _pad8(nb)
        return magic, code, shape, n, nb, woff, poff, poff + 8 * words, words
    poff = woff + 2 * _pad8(nb)
    return magic, code, shape, n, nb, woff, poff, poff + 4 * words, words


def _unpack_device(b):
    magic, code, shape, n, nb, woff, poff, total, words = _parse_array(b)
    if b.numel() < total:
        raise ValueError(f'truncated array blob ({b.numel()} < {total} bytes)')
    out = dev.empty(shape, dev.CODE_TO_TORCH[code])
    if n == 0:
        return out
    if magic == RICE_MAGIC:
        return _unpack_rice(b, code, n, nb, woff, poff, words, out)
    widths = b[woff:woff + nb]
    bits = _SAMPLE_BITS[out.element_size()]
    ws = dev.empty((int(lib.kmp_pack_workspace_bytes(n)),), torch.uint8)
    check(lib.kmp_unpack_plan(widths.data_ptr(), n, ws.data_ptr(), dev.stream()), 'unpack')
    # the widths must fit the sample type and add up to the header's payload length (the unpack
    # kernel derives every block's payload offset from them): one synchronisation for both
    off = int(lib.kmp_pack_total_offset(n))
    scanned = ws[off:off + 8].view(torch.int64)
    wmax, total_words = torch.cat([widths.max().to(torch.int64).reshape(1), scanned]).tolist()
    if wmax > bits or total_words != words:
        raise ValueError(f'array blob block widths are inconsistent (max {wmax} of {bits} bits, '
                         f'{total_words} payload words, header says {words})')
    check(lib.kmp_unpack(code, b.data_ptr() + poff, n, widths.data_ptr(), ws.data_ptr(), out.data_ptr(),
                         dev.stream()), 'unpack')
    return out


def _unpack_rice(b, code, n, nb, aoff, poff, words, out):
    params, bw = b[aoff:aoff + nb], b[aoff + _pad8(nb):aoff + _pad8(nb) + nb]
    bits = _SAMPLE_BITS[out.element_size()]
    ws = dev.empty((int(lib.kmp_pack_workspace_bytes(n)),), torch.uint8)
    check(lib.kmp_unpack_plan(bw.data_ptr(), n, ws.data_ptr(), dev.stream()), 'rice unpack')
    # every block's side information must be one the encoder can produce (k < W; an all-zero
    # block has no payload; a coded block holds its 2k plane words and >= 2 unary words, at most
    # 2W + 2 in all) and the sizes must add up to the header's payload length: one synchronisation
    off = int(lib.kmp_pack_total_offset(n))
    k = params.to(torch.int32) - 1
    bwi = bw.to(torch.int32)
    coded = params > 0
    bad = (k >= bits) | (coded & ((bwi < 2 * k + 2) | (bwi > 2 * bits + 2))) | (~coded & (bwi != 0))
    nbad, total_words = torch.cat([bad.sum().to(torch.int64).reshape(1), ws[off:off + 8].view(torch.int64)]).tolist()
    if nbad or total_words != words:
        raise ValueError(f'rice blob side information is inconsistent ({nbad} bad blocks, {total_words} payload '
                         f'words, header says {words})')
    check(lib.kmp_rice_unpack(code, b.data_ptr() + poff, n, params.data_ptr(), bw.data_ptr(), ws.data_ptr(),
                              out.data_ptr(), dev.stream()), 'rice unpack')
    return out


def _pack_any(t, method):
    if method == 'rice':
        return _pack_rice_device(t)
    if method == 'planes':
        return _pack_device(t)
    raise ValueError(f'unknown packing method {method!r} (expected one of {METHODS})')


def pack(x, method='rice'):
    """Pack one array (uint8 / uint16 / int32 / uint32 / float32 samples) into a blob."""
    t, kind = dev.to_device(x)
    return dev.from_device(_pack_any(t, method), kind)


def unpack(blob):
    """Inverse of :func:`pack`: the array, bit for bit."""
    b, kind = dev.to_device(blob)
    return dev.from_device(_unpack_device(b), kind)


def pack_encoded(lowres, encoded, method='rice'):
    """One blob for an ``encode`` result ``(lowres, (maps, dims))``."""
    maps, dims = encoded
    kind = 'torch' if isinstance(lowres, torch.Tensor) else 'numpy'
    blobs = [_pack_any(dev.to_device(a)[0], method) for a in (lowres, *maps)]
    nsp = len(dims)
    head = struct.pack('<4sHHI', BUNDLE_MAGIC, VERSION, len(blobs), nsp)
    head += struct.pack(f'<{nsp}i', *[int(d) for d in dims])
    head += b'\0' * (_pad8(len(head)) - len(head))
    head += struct.pack(f'<{len(blobs)}q', *[int(bl.numel()) for bl in blobs])
    parts = [_device_bytes(head)]
    for bl in blobs:
        parts.append(bl)
        if bl.numel() % 8:
            parts.append(_device_bytes(bytes(8 - bl.numel() % 8)))
    return dev.from_device(torch.cat(parts), kind)


def unpack_encoded(blob):
    """Inverse of :func:`pack_encoded`: ``(lowres, (maps, dims))``."""
    b, kind = dev.to_device(blob)
    magic, version, count, nsp = struct.unpack('<4sHHI', bytes(b[:12].cpu().numpy()))
    if magic != BUNDLE_MAGIC or version != VERSION:
        raise ValueError(f'not a kompressor_amd bundle (magic {magic!r}, version {version})')
    dims = struct.unpack(f'<{nsp}i', bytes(b[12:12 + 4 * nsp].cpu().numpy()))
    off = _pad8(12 + 4 * nsp)
    lengths = struct.unpack(f'<{count}q', bytes(b[off:off + 8 * count].cpu().numpy()))
    off += 8 * count
    arrays = []
    for ln in lengths:
        arrays.append(dev.from_device(_unpack_device(b[off:off + ln]), kind))
        off += _pad8(ln)
    return arrays[0], (tuple(arrays[1:]), tuple(int(d) for d in dims))
