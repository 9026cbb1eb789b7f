"""Bit-plane container for coded arrays -- ``kmp_pack.hip``.

The reference stops at residual arrays: ``encode`` returns lowres plus maps of the same total size
as the input (volume/encode_decode.py:56), so nothing gets smaller.  A good predictor leaves small
residuals (modulo 2^W), and this container stores them in about as many bits as they need:
zigzag-mapped samples in blocks of 64, each block as ``width`` 64-bit bit-planes (one wavefront
ballot per plane on the GPU).  The format is the build's own -- no reference counterpart, parity
pinned to its numpy specification ``oracle/packing.py`` -- and lossless for every bit pattern.

    blob = pack(x)                    # one array -> uint8 blob
    x2 = unpack(blob)                 # bit-identical, same dtype and shape
    blob = pack_encoded(lowres, (maps, dims))         # a whole encode() result
    lowres, (maps, dims) = unpack_encoded(blob)

Blobs are device uint8 tensors for torch inputs and numpy uint8 arrays for numpy inputs.
Array layout (little-endian, 8-byte aligned): ``'KMPA' u16 version u16 dtype u32 ndim u32 0 i64 n
i64 nblocks i64 words`` (40 bytes), ``i64 shape[ndim]``, ``u8 widths[nblocks]`` padded to 8
bytes, ``u64 payload[words]``.  Bundle: ``'KMPB' u16 version u16 count u32 nsp``, ``i32 dims[nsp]`` padded to
8, ``i64 lengths[count]``, then the array blobs (each padded to 8 bytes), lowres first.
"""

import struct

import torch

from . import _device as dev
from ._lib import check, lib

ARRAY_MAGIC = b'KMPA'
BUNDLE_MAGIC = b'KMPB'
VERSION = 1
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


def _parse_array(b):
    """(dtype code, shape, n, nb, widths offset, payload offset, total bytes, words) of an array
    blob: one device-to-host read of the header.  Every header field is checked against the others
    before anything is launched, so a corrupt or hostile blob raises ValueError instead of steering
    a kernel outside its buffers."""
    hb = bytes(b[:min(b.numel(), _HEAD.size + 8 * 8)].cpu().numpy())
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
        raise ValueError(f'array blob payload of {words} words exceeds {nb} blocks of {bits} planes')
    woff = _HEAD.size + 8 * ndim
    poff = woff + _pad8(nb)
    return code, shape, n, nb, woff, poff, poff + 8 * words, words


def _unpack_device(b):
    code, shape, n, nb, woff, poff, total, words = _parse_array(b)
    if b.numel() < total:
        raise ValueError(f'truncated array blob ({b.numel()} < {total} bytes)')
    out = dev.empty(shape, dev.CODE_TO_TORCH[code])
    if n == 0:
        return out
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


def pack(x):
    """Pack one array (uint8 / uint16 / int32 / uint32 / float32 samples) into a blob."""
    t, kind = dev.to_device(x)
    return dev.from_device(_pack_device(t), kind)


def unpack(blob):
    """Inverse of :func:`pack`: the array, bit for bit."""
    b, kind = dev.to_device(blob)
    return dev.from_device(_unpack_device(b), kind)


def pack_encoded(lowres, encoded):
    """One blob for an ``encode`` result ``(lowres, (maps, dims))``."""
    maps, dims = encoded
    kind = 'torch' if isinstance(lowres, torch.Tensor) else 'numpy'
    blobs = [_pack_device(dev.to_device(a)[0]) for a in (lowres, *maps)]
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
