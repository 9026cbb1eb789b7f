"""Self-describing compressed files ("on-disk format + entropy coding").

The reference has no file format -- ``encode`` returns ``(lowres, (maps, dims))`` in memory
(volume/encode_decode.py:56) -- so this is the build's own container: one file holds the
entropy-coded ``encode`` result (``packing.pack_encoded``: block-adaptive Rice by default) plus
everything needed to decode it without outside knowledge -- the pyramid levels (``compress``
applies the reference's single-level ``encode`` recursively to the lowres, so only the coarsest
lowres is stored raw), the spatial rank, the predictor
(kind, padding, and a LinearPredictor's weights), the coder, the even-size ``dims``, the original
sample dtype (float32 volumes travel bit-cast to uint32) and a CRC-32 of the payload.

    info = compress(path, highres, predictor)     # pyramid encode on the GPU + Rice + one write
    highres = decompress(path)                    # read + unpack + decode on the GPU
    save(path, lowres, encoded, predictor=...)    # an encode() result you already have
    lowres, encoded, meta = load(path)

File layout (little-endian): ``b'KMPF' u16 version u16 0 u64 meta_len``, the metadata as UTF-8
JSON padded to 8 bytes, then the ``pack_encoded`` bundle (``meta['bundle_bytes']`` bytes).

The host side of the file path (round 4): the bundle's CRC-32 (zlib's, the value the file stores)
is computed on the device (``kmp_crc32``) -- over the bundle the encode just wrote, its length read
by the kernel from the bundle header, so one synchronisation returns length and CRC together; on
read, over the bundle as uploaded, checked with the decode's side-information counter.  The bundle
crosses the link through a reused pinned staging buffer (57 GB/s instead of ~8 GB/s pageable) and
files are read straight into it; numpy results come back through the same pinned path
(``_device.to_host``).  ``last_timing`` holds the wall-time split of the last call.
"""

import json
import os
import struct
import time

import numpy as np
import torch

from . import _device as dev
from . import _nd, packing
from ._lib import check, lib
from .predictors import ARITH_REV, LinearPredictor, MeanPredictor

# wall-time split (seconds) of the last compress / decompress / save / load of this process
last_timing = {}

MAGIC = b'KMPF'
VERSION = 3  # 2: rice payloads are v2 bundles (packing.py); 3: a LinearPredictor's arith_rev recorded
_HEAD = struct.Struct('<4sHHQ')
_NP_NAME = {torch.uint8: 'uint8', torch.uint16: 'uint16', torch.int32: 'int32', torch.uint32: 'uint32',
            torch.float32: 'float32'}


def _predictor_meta(predictor, padding, ndim, dtype):
    """(``dtype``: the coded samples' torch dtype -- a LinearPredictor's arithmetic is recorded
    resolved for it, so a reader needs no rule for ``'auto'``)"""
    if isinstance(predictor, MeanPredictor):
        return {'kind': 'mean', 'padding': predictor.padding, 'ndim': predictor.ndim}
    if isinstance(predictor, LinearPredictor):
        return {'kind': 'linear', 'padding': predictor.padding, 'ndim': predictor.ndim,
                'arith': predictor.arith_for(dtype), 'arith_rev': ARITH_REV[predictor.arith_for(dtype)],
                'weights': predictor.weights.tolist(), 'bias': predictor.bias.tolist()}
    # an opaque predictions_fn: recorded by name; decoding needs the caller to pass it again
    return {'kind': 'external', 'padding': padding, 'ndim': ndim,
            'name': getattr(predictor, '__qualname__', type(predictor).__name__)}


def predictor_from_meta(meta):
    """The built-in predictor a file was coded with (None for an external predictions_fn)."""
    p = meta['predictor']
    if p['kind'] == 'mean':
        return MeanPredictor(p['padding'], p['ndim'])
    if p['kind'] == 'linear':
        _check_arith_rev(meta)
        return LinearPredictor(np.asarray(p['weights'], np.float32), np.asarray(p['bias'], np.float32),
                               p['padding'], p['ndim'], p.get('arith', 'f32'))
    return None


def _check_arith_rev(meta, path='file'):
    """A LinearPredictor file decodes only under the arithmetic revision it was coded with
    (predictors.ARITH_REV): a different revision rounds some predictions differently and would
    return wrong samples.  Files before container version 3 carry no revision; their f32 chain is
    revision 1, their bf16x2 data is ambiguous (round 4 and round 5 builds wrote it with different
    accumulation orders) and is refused."""
    p = meta.get('predictor') or {}
    if p.get('kind') != 'linear':
        return
    arith = p.get('arith', 'f32')
    rev = p.get('arith_rev', 1 if arith == 'f32' else None)
    if arith not in ARITH_REV:
        raise ValueError(f"{path}: unknown LinearPredictor arithmetic {arith!r}")
    if rev != ARITH_REV[arith]:
        raise ValueError(f"{path}: coded with arith={arith!r} revision {rev if rev is not None else 'unrecorded'}; "
                         f"this build evaluates revision {ARITH_REV[arith]}, whose rounding differs -- decode it "
                         f"with the build that wrote it")


def _device_crc(blob, n_max, n_dev=None):
    """zlib CRC-32 of the device bytes ``blob[:n]`` (n = ``n_max``, or the device int64 at ``n_dev``
    capped to ``n_max``) as a 1-element device uint32 tensor; no synchronisation."""
    out = torch.empty((1,), dtype=torch.int32, device='cuda')
    check(lib.kmp_crc32(blob.data_ptr(), int(n_max), n_dev, out.data_ptr(), dev.stream()), 'crc32')
    return out


def _bundle(x, arrays, dims, method):
    """Entropy-code an encode result on the device: ``(device bytes, bundle length, crc32)`` with ONE
    synchronisation (length and CRC read back together)."""
    if method == 'rice':
        out, poff, launched, keep = packing._rice_encode_launch((x, *arrays), dims)
        if not launched:  # no samples: the header and side arrays only
            total = poff
            crc = _device_crc(out, total)
            head = dev.pinned_staging(64, 'head')
            head[:4].copy_(crc.view(torch.uint8), non_blocking=True)
        else:
            crc = _device_crc(out, out.numel(), out[64:72].data_ptr())  # the size field of the header
            head = dev.pinned_staging(64, 'head')
            head[:16].copy_(out[56:72], non_blocking=True)
            head[16:20].copy_(crc.view(torch.uint8), non_blocking=True)
        torch.cuda.current_stream().synchronize()
        hb = head[:20].numpy().tobytes()
        del keep
        if launched:
            _, total = struct.unpack('<2q', hb[:16])
            return out, int(total), struct.unpack('<I', hb[16:20])[0]
        return out, int(total), struct.unpack('<I', hb[:4])[0]
    blob = packing.pack_encoded(x, (arrays, dims), method)
    crc = _device_crc(blob, blob.numel())
    return blob, blob.numel(), int(crc.cpu().view(torch.uint32).item())


def _write(path, meta, blob, total, crc, t0):
    """Header, metadata and the first ``total`` device bytes of ``blob`` to ``path``: the bundle
    crosses the link in pinned chunks (``_device.d2h_stream``), each written to the file while the
    next ones are in flight."""
    t1 = time.perf_counter()
    meta = dict(meta, bundle_bytes=int(total), crc32=int(crc) & 0xffffffff)
    js = json.dumps(meta, separators=(',', ':')).encode()
    js += b' ' * (-len(js) % 8)
    tmp = f'{path}.tmp{os.getpid()}'
    with open(tmp, 'wb') as f:
        try:  # the file's blocks allocated up front: the write then only copies (8.0 vs 10.0 ms for
            os.posix_fallocate(f.fileno(), 0, _HEAD.size + len(js) + total)  # 112 MB, write_probe_r5w2.log)
        except OSError:
            pass  # a filesystem without fallocate: the writes allocate
        f.write(_HEAD.pack(MAGIC, VERSION, 0, len(js)))
        f.write(js)
        if total:
            dev.d2h_stream(blob[:total], lambda lo, piece: f.write(memoryview(piece)))
    os.replace(tmp, path)  # a reader never sees a half-written file
    t2 = time.perf_counter()
    last_timing.clear()
    last_timing.update(device=t1 - t0, d2h_write=t2 - t1, total=t2 - t0)
    return _HEAD.size + len(js) + total


def _builtin_padding(predictor, padding):
    """The padding a file records: a built-in predictor carries its own (a conflicting explicit
    ``padding`` is an error); an external predictions_fn needs it passed (default 0)."""
    if isinstance(predictor, (MeanPredictor, LinearPredictor)):
        if padding is not None and int(padding) != predictor.padding:
            raise AssertionError(f'padding={padding} conflicts with the predictor\'s padding {predictor.padding}')
        return predictor.padding
    return 0 if padding is None else int(padding)


def save(path, lowres, encoded, predictor=None, padding=None, ndim=None, method='rice', sample_dtype=None):
    """Write an ``encode`` result ``(lowres, (maps, dims))`` to ``path``; returns the file size.
    ``predictor`` is recorded so :func:`decompress` can decode without being told.  ``padding``
    defaults to a built-in predictor's own padding (0 for an external predictions_fn)."""
    maps, dims = encoded
    ndim = ndim or len(dims)
    padding = _builtin_padding(predictor, padding)
    t0 = time.perf_counter()
    packing._check_method(method)
    lo_t = dev.to_device(lowres)[0]
    maps_t = [dev.to_device(m)[0] for m in maps]
    meta = {'format': 'kompressor_amd', 'ndim': ndim, 'padding': padding, 'dims': [int(d) for d in dims],
            'method': method, 'lowres_shape': list(lo_t.shape), 'lowres_dtype': _NP_NAME[lo_t.dtype],
            'map_dtype': _NP_NAME[maps_t[0].dtype],
            'sample_dtype': sample_dtype or _NP_NAME[lo_t.dtype],
            'predictor': _predictor_meta(predictor, padding, ndim, lo_t.dtype) if predictor is not None else None}
    blob, total, crc = _bundle(lo_t, maps_t, dims, method)
    return _write(path, meta, blob, total, crc, t0)


def _read(path):
    """``(meta, device bundle, device crc, timing)``: the file's bundle read straight into the pinned
    staging buffer, uploaded, and its CRC-32 launched on the device (checked by the caller together
    with the decode's own synchronisation -- ``_check_crc``)."""
    t0 = time.perf_counter()
    with open(path, 'rb') as f:
        head = f.read(_HEAD.size)
        if len(head) < _HEAD.size:
            raise ValueError(f'{path}: not a kompressor_amd file (too short)')
        magic, version, _, mlen = _HEAD.unpack(head)
        if magic != MAGIC or version not in (1, 2, VERSION) or mlen > (1 << 26):
            raise ValueError(f'{path}: not a kompressor_amd file (magic {magic!r}, version {version})')
        try:
            meta = json.loads(f.read(mlen).decode())
            n = int(meta['bundle_bytes'])
        except (ValueError, KeyError, TypeError) as e:
            raise ValueError(f'{path}: corrupt metadata ({e})') from None
        if version == 1 and meta.get('method') != 'planes':
            # version-1 'rice' payloads were the per-array KMPR format, replaced by the v2 bundle;
            # version-1 'planes' payloads are unchanged and still read
            raise ValueError(f'{path}: a version-1 rice file (the retired per-array KMPR format): re-compress it')
        # the payload length is checked against the file before anything is allocated for it
        avail = os.fstat(f.fileno()).st_size - (_HEAD.size + mlen)
        if not 0 <= n <= avail:
            raise ValueError(f'{path}: truncated or corrupt ({n} payload bytes recorded, {max(avail, 0)} present)')
        # the payload: parallel page-cache reads into pinned chunks, each uploaded while the next is read
        blob = torch.empty((max(n, 1),), dtype=torch.uint8, device='cuda')[:n]
        fd, base = f.fileno(), _HEAD.size + mlen
        got = dev.h2d_stream(blob, lambda lo, piece: dev.pread_into(fd, piece, base + lo)) if n else 0
    if got != n:
        raise ValueError(f'{path}: truncated ({got} of {n} payload bytes)')
    t1 = time.perf_counter()
    crc = _device_crc(blob, n) if n else torch.zeros((1,), dtype=torch.int32, device='cuda')
    return meta, blob, crc, {'read_upload': t1 - t0, 't_upload': t1}


def _check_crc(path, meta, crc):
    """The device CRC against the file's (one small read-back; the caller's own synchronisation
    usually has already drained the stream)."""
    got = int(crc.cpu().view(torch.uint32).item()) if meta['bundle_bytes'] else 0
    if got != (int(meta['crc32']) & 0xffffffff):
        raise ValueError(f'{path}: payload CRC mismatch (corrupt file)')


def load(path, device=True):
    """``(lowres, (maps, dims), meta)`` from a file written by :func:`save` / :func:`compress`;
    device tensors by default, numpy arrays with ``device=False``."""
    meta, blob, crc, _ = _read(path)
    _check_crc(path, meta, crc)  # before any header parsing of a possibly corrupt bundle
    lowres, (maps, dims) = packing.unpack_encoded(blob)
    if not device:
        lowres, maps = dev.to_host(lowres), tuple(dev.to_host(m) for m in maps)
    return lowres, (maps, dims), meta


def _auto_levels(shape, ndim, max_levels=4):
    """Pyramid levels while every spatial extent stays >= 3 (its lowres >= 2, volume/utils.py:295-303)."""
    sp, levels = list(shape[1:1 + ndim]), 0
    while levels < max_levels and all(s >= 3 for s in sp):
        sp = [(s + (s + 1) % 2 + 1) // 2 - (s + 1) % 2 for s in sp]  # the trimmed lowres extent
        levels += 1
    return max(levels, 1)


def compress(path, highres, predictor, levels='auto', method='rice'):
    """Encode ``highres`` with a built-in ``predictor`` (:class:`MeanPredictor` /
    :class:`LinearPredictor`) and the lossless coder of its dtype (uint8 / uint16 modular, int32
    raw, float32 bit-cast to uint32 modulo 2^32) as a ``levels``-deep pyramid -- each level is the
    reference's single-level ``encode`` (volume/encode_decode.py:30-56) applied to the previous
    level's lowres, so only the coarsest lowres is stored raw -- entropy-code every array and write
    ``path``.  Returns ``{'bytes', 'raw_bytes', 'ratio', 'bits_per_sample', 'levels'}``."""
    t0 = time.perf_counter()
    packing._check_method(method)
    ndim, padding = predictor.ndim, predictor.padding
    h, _ = dev.to_device(highres)
    sample = _NP_NAME[h.dtype]
    if h.dtype == torch.float32:
        h = h.view(torch.uint32)
    coder = _nd.NATURAL_CODER.get(h.dtype)
    if coder is None:
        raise TypeError(f'no lossless coder for {h.dtype}')
    levels = _auto_levels(h.shape, ndim) if levels == 'auto' else int(levels)
    _nd._require(levels >= 1, 'levels must be >= 1')
    x, arrays, meta_levels = h, [], []
    for _ in range(levels):
        sp = _nd._sp(x.shape, ndim)
        _nd.validate_highres_shape((x.shape[0], *[s + (s + 1) % 2 for s in sp], *x.shape[1 + ndim:]), ndim)
        lowres, maps, dims = _nd._alloc_encoded(x, coder, ndim)
        _nd.fused_encode_into(x, predictor, coder, lowres, maps, ndim)
        arrays.extend(maps)
        meta_levels.append({'highres_shape': list(x.shape), 'dims': [int(d) for d in dims]})
        x = lowres
    meta = {'format': 'kompressor_amd', 'ndim': ndim, 'padding': padding, 'method': method,
            'sample_dtype': sample, 'levels': meta_levels, 'lowres_shape': list(x.shape),
            'predictor': _predictor_meta(predictor, padding, ndim, x.dtype)}
    # one bundle: the coarsest lowres, then every level's maps finest first (no bundle dims: the
    # per-level dims live in the metadata)
    blob, total, crc = _bundle(x, arrays, (), method)
    nbytes = _write(path, meta, blob, total, crc, t0)
    raw = h.numel() * h.element_size()
    return {'bytes': nbytes, 'raw_bytes': raw, 'ratio': raw / nbytes, 'bits_per_sample': 8.0 * nbytes / h.numel(),
            'levels': levels}


def decompress(path, predictor=None, as_numpy=True):
    """Decode a file written by :func:`compress` (or :func:`save`) back to the original array, bit
    for bit, coarsest level first.  A file coded with an external predictions_fn needs it passed."""
    t0 = time.perf_counter()
    meta, blob, crc, tm = _read(path)
    _check_crc(path, meta, crc)
    t1 = time.perf_counter()
    lowres, (arrays, bundle_dims) = packing.unpack_encoded(blob)
    pred = predictor or predictor_from_meta(meta)
    if pred is None:
        raise AssertionError(f'{path} was coded with an external predictions_fn '
                             f'({meta["predictor"]["name"] if meta["predictor"] else "unknown"}): pass it')
    ndim, padding = meta['ndim'], meta['padding']
    if isinstance(pred, (MeanPredictor, LinearPredictor)) and pred.padding != padding:
        raise AssertionError(f'{path} was coded with padding {padding}; the predictor passed has {pred.padding}')
    if isinstance(pred, LinearPredictor) and meta['predictor'] and meta['predictor'].get('kind') == 'linear':
        # the two arithmetics are not bit-equal: decoding with the other one returns wrong samples
        _check_arith_rev(meta, path)
        arith = meta['predictor'].get('arith', 'f32')
        if pred.arith == 'auto':  # a default-constructed predictor takes the file's arithmetic
            pred = LinearPredictor(pred.weights, pred.bias, pred.padding, pred.ndim, arith=arith)
        if pred.arith_for(lowres.dtype) != arith:
            raise AssertionError(f"{path} was coded with arith='{arith}'; the predictor passed evaluates with "
                                 f"arith='{pred.arith_for(lowres.dtype)}'")
    nmaps = _nd.NMAPS[ndim]
    levels = meta.get('levels') or [{'dims': list(bundle_dims)}]  # save(): one level, dims in the bundle
    if len(arrays) != nmaps * len(levels):
        raise ValueError(f'{path}: {len(arrays)} coded maps for {len(levels)} levels of {nmaps}')
    coder = _nd.NATURAL_CODER[lowres.dtype]
    dec_fn = _coder_fn(coder, ndim)
    x = lowres
    for lvl in reversed(range(len(levels))):
        maps = list(arrays[nmaps * lvl:nmaps * (lvl + 1)])
        dims = tuple(levels[lvl]['dims'])
        if _nd.fused_plan(pred, dec_fn, padding, x.dtype, ndim, 1) is not None:
            out = torch.empty((x.shape[0], *[2 * e - 1 + d for e, d in zip(_nd._sp(x.shape, ndim), dims)],
                               *x.shape[1 + ndim:]), dtype=x.dtype, device='cuda')
            _nd.fused_decode_into(x, maps, dims, pred, coder, out, ndim)
        else:
            out = _nd.decode(pred, dec_fn, x, (maps, dims), padding, ndim)
        x = out
    if meta.get('sample_dtype') == 'float32':
        x = x.view(torch.float32)
    torch.cuda.current_stream().synchronize()
    t2 = time.perf_counter()
    out = dev.to_host(x) if as_numpy else x
    t3 = time.perf_counter()
    last_timing.clear()
    last_timing.update(read_upload=tm['read_upload'], crc=t1 - tm['t_upload'], device=t2 - t1, d2h=t3 - t2,
                       total=t3 - t0)
    return out


def _coder_fn(coder, ndim):
    from . import utils
    name = {0: 'decode_values_raw', 1: 'decode_values_uint8', 2: 'decode_values_uint16', 3: 'decode_values_uint32'}
    return getattr(utils, name[coder])
