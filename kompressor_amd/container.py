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
Reads and writes move the bundle with one host<->device copy; numpy arrays in, numpy out.
"""

import json
import os
import struct
import zlib

import numpy as np
import torch

from . import _device as dev
from . import _nd, packing
from .predictors import LinearPredictor, MeanPredictor

MAGIC = b'KMPF'
VERSION = 2  # 2: rice payloads are v2 bundles (packing.py)
_HEAD = struct.Struct('<4sHHQ')
_NP_NAME = {torch.uint8: 'uint8', torch.uint16: 'uint16', torch.int32: 'int32', torch.uint32: 'uint32',
            torch.float32: 'float32'}


def _predictor_meta(predictor, padding, ndim):
    if isinstance(predictor, MeanPredictor):
        return {'kind': 'mean', 'padding': predictor.padding, 'ndim': predictor.ndim}
    if isinstance(predictor, LinearPredictor):
        return {'kind': 'linear', 'padding': predictor.padding, 'ndim': predictor.ndim,
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
        return LinearPredictor(np.asarray(p['weights'], np.float32), np.asarray(p['bias'], np.float32),
                               p['padding'], p['ndim'])
    return None


def _write(path, meta, blob):
    host = blob.detach().cpu().numpy() if isinstance(blob, torch.Tensor) else np.asarray(blob, np.uint8)
    meta = dict(meta, bundle_bytes=int(host.size), crc32=zlib.crc32(memoryview(host)) & 0xffffffff)
    js = json.dumps(meta, separators=(',', ':')).encode()
    js += b' ' * (-len(js) % 8)
    tmp = f'{path}.tmp{os.getpid()}'
    with open(tmp, 'wb') as f:
        f.write(_HEAD.pack(MAGIC, VERSION, 0, len(js)))
        f.write(js)
        f.write(memoryview(host))
    os.replace(tmp, path)  # a reader never sees a half-written file
    return _HEAD.size + len(js) + host.size


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
    lo_t = dev.to_device(lowres)[0]
    meta = {'format': 'kompressor_amd', 'ndim': ndim, 'padding': padding, 'dims': [int(d) for d in dims],
            'method': method, 'lowres_shape': list(lo_t.shape), 'lowres_dtype': _NP_NAME[lo_t.dtype],
            'map_dtype': _NP_NAME[dev.to_device(maps[0])[0].dtype],
            'sample_dtype': sample_dtype or _NP_NAME[lo_t.dtype],
            'predictor': _predictor_meta(predictor, padding, ndim) if predictor is not None else None}
    return _write(path, meta, packing.pack_encoded(lo_t, (maps, dims), method))


def _read(path):
    with open(path, 'rb') as f:
        head = f.read(_HEAD.size)
        if len(head) < _HEAD.size:
            raise ValueError(f'{path}: not a kompressor_amd file (too short)')
        magic, version, _, mlen = _HEAD.unpack(head)
        if magic != MAGIC or version not in (1, VERSION) or mlen > (1 << 26):
            raise ValueError(f'{path}: not a kompressor_amd file (magic {magic!r}, version {version})')
        meta = json.loads(f.read(mlen).decode())
        if version == 1 and meta.get('method') != 'planes':
            # version-1 'rice' payloads were the per-array KMPR format, replaced by the v2 bundle;
            # version-1 'planes' payloads are unchanged and still read
            raise ValueError(f'{path}: a version-1 rice file (the retired per-array KMPR format): re-compress it')
        body = np.fromfile(f, dtype=np.uint8, count=int(meta['bundle_bytes']))
    if body.size != meta['bundle_bytes']:
        raise ValueError(f'{path}: truncated ({body.size} of {meta["bundle_bytes"]} payload bytes)')
    if zlib.crc32(memoryview(body)) & 0xffffffff != meta['crc32']:
        raise ValueError(f'{path}: payload CRC mismatch (corrupt file)')
    return meta, body


def load(path, device=True):
    """``(lowres, (maps, dims), meta)`` from a file written by :func:`save` / :func:`compress`;
    device tensors by default, numpy arrays with ``device=False``."""
    meta, body = _read(path)
    blob = torch.from_numpy(body).cuda() if device else body
    lowres, (maps, dims) = packing.unpack_encoded(blob)
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
            'predictor': _predictor_meta(predictor, padding, ndim)}
    # one bundle: the coarsest lowres, then every level's maps finest first (no bundle dims: the
    # per-level dims live in the metadata)
    nbytes = _write(path, meta, packing.pack_encoded(x, (arrays, ()), method))
    raw = h.numel() * h.element_size()
    return {'bytes': nbytes, 'raw_bytes': raw, 'ratio': raw / nbytes, 'bits_per_sample': 8.0 * nbytes / h.numel(),
            'levels': levels}


def decompress(path, predictor=None, as_numpy=True):
    """Decode a file written by :func:`compress` (or :func:`save`) back to the original array, bit
    for bit, coarsest level first.  A file coded with an external predictions_fn needs it passed."""
    meta, body = _read(path)
    lowres, (arrays, bundle_dims) = packing.unpack_encoded(torch.from_numpy(body).cuda())
    pred = predictor or predictor_from_meta(meta)
    if pred is None:
        raise AssertionError(f'{path} was coded with an external predictions_fn '
                             f'({meta["predictor"]["name"] if meta["predictor"] else "unknown"}): pass it')
    ndim, padding = meta['ndim'], meta['padding']
    if isinstance(pred, (MeanPredictor, LinearPredictor)) and pred.padding != padding:
        raise AssertionError(f'{path} was coded with padding {padding}; the predictor passed has {pred.padding}')
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
    return x.cpu().numpy() if as_numpy else x


def _coder_fn(coder, ndim):
    from . import utils
    name = {0: 'decode_values_raw', 1: 'decode_values_uint8', 2: 'decode_values_uint16', 3: 'decode_values_uint32'}
    return getattr(utils, name[coder])
