"""Shared N-d engine behind ``kompressor_amd.image`` (N = 2) and ``kompressor_amd.volume`` (N = 3).

Every function here mirrors one of the reference's (cited at the thin per-module wrappers in
``image/`` and ``volume/``) and runs its arithmetic in ``libkompressor_hip.so``.  ``d_*`` helpers
take and return contiguous device tensors; the public wrappers accept numpy arrays or torch
tensors and return the same kind they were given.
"""

import ctypes
import os
from itertools import product

import numpy as np
import torch

from . import _device as dev
from . import _lib, _trace
from ._lib import check, lib

PARITY = {
    3: ((1, 1, 0), (1, 0, 1), (0, 1, 1), (1, 1, 1), (1, 0, 0), (0, 1, 0), (0, 0, 1)),  # volume/utils.py:161-169
    2: ((1, 0), (0, 1), (1, 1)),                                                       # image/utils.py:92-94
}
NMAPS = {3: 7, 2: 3}
NPRED = {3: 19, 2: 5}
CODER_DTYPE = {_lib.CODER_RAW: torch.int32, _lib.CODER_U8: torch.uint8, _lib.CODER_U16: torch.uint16,
               _lib.CODER_U32: torch.uint32}
NATURAL_CODER = {torch.uint8: _lib.CODER_U8, torch.uint16: _lib.CODER_U16, torch.int32: _lib.CODER_RAW,
                 torch.uint32: _lib.CODER_U32}


def _sp(shape, nsp):
    return tuple(int(s) for s in shape[1:1 + nsp])


def _ch(shape, nsp):
    return tuple(int(s) for s in shape[1 + nsp:])


def _C(shape, nsp):
    return dev.prod(_ch(shape, nsp))


def _dev(x):
    return dev.to_device(x)[0]


def _zeros(shape, dtype):
    # zero-filled device buffer without relying on fill kernels for unsigned 16/32-bit types
    alias = {torch.uint16: torch.int16, torch.uint32: torch.int32}.get(dtype)
    if alias is None:
        return torch.zeros(tuple(shape), dtype=dtype, device='cuda')
    return torch.zeros(tuple(shape), dtype=alias, device='cuda').view(dtype)


# =============================================================================================
# Validators (pure host logic; raise AssertionError explicitly so ``python -O`` keeps them)
# =============================================================================================

def _require(cond, msg):
    if not cond:
        raise AssertionError(msg)


def validate_padding(padding):
    """utils.py:158-161."""
    _require(isinstance(padding, int) and not isinstance(padding, bool), 'padding must be an int')
    _require(padding >= 0, 'padding must be >= 0')


def validate_highres_shape(shape, nsp):
    """volume/utils.py:284-292 / image/utils.py:201-208 on a shape."""
    _require(len(shape) >= nsp + 2, f'highres needs ndim >= {nsp + 2} (batch, spatial, channels)')
    _require(dev.prod(shape) > 0, 'highres is empty')
    sp = _sp(shape, nsp)
    for s in sp:
        _require(s > 2 and s % 2 != 0, f'highres spatial dims must be odd and > 2 (after even padding), got {sp}')
    return sp


def validate_lowres_shape(shape, nsp):
    """volume/utils.py:295-303 / image/utils.py:211-218 on a shape."""
    _require(len(shape) >= nsp + 2, f'lowres needs ndim >= {nsp + 2}')
    _require(dev.prod(shape) > 0, 'lowres is empty')
    sp = _sp(shape, nsp)
    for s in sp:
        _require(s >= 2, f'lowres spatial dims must be >= 2, got {sp}')
    return sp


def validate_chunk(chunk, nsp):
    """volume/utils.py:306-318 / image/utils.py:221-232."""
    if isinstance(chunk, int) and not isinstance(chunk, bool):
        _require(chunk > 3, 'chunk must be > 3')
        return (chunk,) * nsp
    if isinstance(chunk, tuple):
        if len(chunk) != nsp:
            raise ValueError(f'chunk tuple must have {nsp} entries')
        for c in chunk:
            if not isinstance(c, int) or isinstance(c, bool):
                raise TypeError('chunk entries must be ints')
            _require(c > 3, 'chunk must be > 3 in every dimension')
        return tuple(chunk)
    raise AssertionError(f'chunk must be int or tuple of {nsp} ints')


def yield_chunks(max_value, chunk):
    """utils.py:114-155 -- constant-size lowres windows with a one-sided halo (p0 + p1 == 2)."""
    _require(max_value > 0, 'max_value must be > 0')
    _require(chunk > 3, 'chunk must be > 3')
    if chunk >= max_value:
        yield (0, max_value), (0, 0)
        return
    step, span = chunk - 3, chunk - 2
    for start in range(0, max_value, step):
        i1 = min(max_value, start + span)
        last = i1 == max_value
        i0 = max(0, i1 - span) if last else start
        first = i0 == 0
        p0 = 0 if first else (2 if last else 1)
        p1 = 0 if last else (2 if first else 1)
        _require(not (first and last) and p0 + p1 == 2, 'yield_chunks invariant')
        yield (i0, i1), (p0, p1)
        if last:
            return


# =============================================================================================
# Primitives on device tensors
# =============================================================================================

def _empty_ok(*tensors):
    return all(t.numel() > 0 for t in tensors)


def d_lowres_from_highres(h, nsp):
    sp = _sp(h.shape, nsp)
    out = dev.empty((h.shape[0], *[(s + 1) // 2 for s in sp], *_ch(h.shape, nsp)), h.dtype)
    if _empty_ok(h, out):
        check(lib.kmp_lowres_from_highres(nsp, dev.dtype_code(h), h.data_ptr(), h.shape[0], _lib.i64x3(sp),
                                          _C(h.shape, nsp), out.data_ptr(), dev.stream()), 'lowres_from_highres')
    return out


def d_maps_from_highres(h, nsp):
    sp = _sp(h.shape, nsp)
    ch = _ch(h.shape, nsp)
    outs = [dev.empty((h.shape[0], *[(s // 2 if p else (s + 1) // 2) for s, p in zip(sp, par)], *ch), h.dtype)
            for par in PARITY[nsp]]
    if _empty_ok(h, *outs):
        check(lib.kmp_maps_from_highres(nsp, dev.dtype_code(h), h.data_ptr(), h.shape[0], _lib.i64x3(sp),
                                        _C(h.shape, nsp), _lib.ptrs(outs), dev.stream()), 'maps_from_highres')
    return tuple(outs)


def d_targets_from_highres(h, nsp):
    sp = _sp(h.shape, nsp)
    out = dev.empty((h.shape[0], *[(s - 1) // 2 for s in sp], NPRED[nsp], *_ch(h.shape, nsp)), h.dtype)
    if _empty_ok(h, out):
        check(lib.kmp_targets_from_highres(nsp, dev.dtype_code(h), h.data_ptr(), h.shape[0], _lib.i64x3(sp),
                                           _C(h.shape, nsp), out.data_ptr(), dev.stream()), 'targets_from_highres')
    return out


def d_copy_box(src, in_off, ext, dst, out_off, nsp):
    """dst[:, out_off:out_off+ext] = cast(src[:, in_off:in_off+ext]) (HIP box copy)."""
    if dev.prod(ext) == 0 or src.shape[0] == 0:
        return dst
    C = _C(src.shape, nsp)
    _require(C == _C(dst.shape, nsp) and src.shape[0] == dst.shape[0], 'box copy: batch/channel mismatch')
    check(lib.kmp_copy_box(nsp, dev.dtype_code(src), src.data_ptr(), _lib.i64x3(_sp(src.shape, nsp)),
                           _lib.i64x3(in_off), dev.dtype_code(dst), dst.data_ptr(), _lib.i64x3(_sp(dst.shape, nsp)),
                           _lib.i64x3(out_off), src.shape[0], C, _lib.i64x3(ext), dev.stream()), 'copy_box')
    return dst


def d_crop(src, start, ext, nsp):
    out = dev.empty((src.shape[0], *ext, *_ch(src.shape, nsp)), src.dtype)
    return d_copy_box(src, start, ext, out, (0,) * nsp, nsp)


def d_cast(src, dtype, nsp):
    if src.dtype == dtype:
        return src
    out = dev.empty(src.shape, dtype)
    return d_copy_box(src, (0,) * nsp, _sp(src.shape, nsp), out, (0,) * nsp, nsp)


def d_highres_from_lowres_and_maps(lowres, maps, nsp):
    L = _sp(lowres.shape, nsp)
    ch = _ch(lowres.shape, nsp)
    maps = list(maps)
    _require(len(maps) == NMAPS[nsp], f'expected {NMAPS[nsp]} maps')
    for i, (m, par) in enumerate(zip(maps, PARITY[nsp])):
        want = (lowres.shape[0], *[(l - 1 if p else l) for l, p in zip(L, par)], *ch)
        _require(tuple(m.shape) == want, f'map {i} has shape {tuple(m.shape)}, expected {want}')
        maps[i] = d_cast(m, lowres.dtype, nsp)
    out = dev.empty((lowres.shape[0], *[2 * l - 1 for l in L], *ch), lowres.dtype)
    if _empty_ok(lowres, out):
        check(lib.kmp_highres_from_lowres_and_maps(nsp, dev.dtype_code(lowres), lowres.data_ptr(), _lib.ptrs(maps),
                                                   lowres.shape[0], _lib.i64x3(L), _C(lowres.shape, nsp),
                                                   out.data_ptr(), dev.stream()), 'highres_from_lowres_and_maps')
    return out


def d_features_from_lowres(lowres, padding, nsp):
    S = _sp(lowres.shape, nsp)
    k = 2 * padding + 2
    cells = [s - 2 * padding - 1 for s in S]
    _require(all(c >= 0 for c in cells), 'lowres window smaller than the neighbourhood')
    out = dev.empty((lowres.shape[0], *cells, k ** nsp, *_ch(lowres.shape, nsp)), lowres.dtype)
    if _empty_ok(lowres, out):
        check(lib.kmp_features_from_lowres(nsp, dev.dtype_code(lowres), lowres.data_ptr(), lowres.shape[0],
                                           _lib.i64x3(S), _C(lowres.shape, nsp), padding, out.data_ptr(),
                                           dev.stream()), 'features_from_lowres')
    return out


def d_maps_from_predictions(preds, nsp):
    cells = _sp(preds.shape, nsp)
    _require(preds.ndim >= nsp + 2 and preds.shape[1 + nsp] == NPRED[nsp],
             f'predictions must be [B, cells..., {NPRED[nsp]}, ...]')
    ch = tuple(int(s) for s in preds.shape[2 + nsp:])
    C = dev.prod(ch)
    outs = [dev.empty((preds.shape[0], *[(c if p else c + 1) for c, p in zip(cells, par)], *ch), preds.dtype)
            for par in PARITY[nsp]]
    if _empty_ok(preds, *outs):
        check(lib.kmp_maps_from_predictions(nsp, dev.dtype_code(preds), preds.data_ptr(), preds.shape[0],
                                            _lib.i64x3(cells), C, _lib.ptrs(outs), dev.stream()),
              'maps_from_predictions')
    return tuple(outs)


def d_mean_predict_maps(window, padding, nsp, out_dtype=None):
    """The mean predictor's 7 (3) maps of a padded lowres window, in the sample dtype or (out_dtype
    torch.float32) as float32 maps written by the kernel itself -- the shape of a network's output.
    Windows the float32 kernels do not take (2D, C > 1) convert the sample-dtype maps on the device."""
    S = _sp(window.shape, nsp)
    cells = [s - 2 * padding - 1 for s in S]
    _require(all(c >= 1 for c in cells), 'window has no cells')
    ch = _ch(window.shape, nsp)
    od = window.dtype if out_dtype is None else out_dtype
    _require(od in (window.dtype, torch.float32), 'maps dtype must be the sample dtype or float32')
    outs = [dev.empty((window.shape[0], *[(c if p else c + 1) for c, p in zip(cells, par)], *ch), od)
            for par in PARITY[nsp]]
    if _empty_ok(window, *outs):
        st = lib.kmp_mean_predict_maps_typed(nsp, dev.dtype_code(window), dev.dtype_code(outs[0]), window.data_ptr(),
                                             window.shape[0], _lib.i64x3(S), _C(window.shape, nsp), padding,
                                             _lib.ptrs(outs), dev.stream())
        if st == _lib.KMP_ERR_UNSUPPORTED and od != window.dtype:
            return tuple(m.to(od) for m in d_mean_predict_maps(window, padding, nsp))
        check(st, 'mean_predict_maps')
    return tuple(outs)


def d_pad(x, lo, hi, mode, nsp):
    """jnp.pad of the spatial axes, mode 'symmetric' (0) / 'reflect' (1); negative pads crop."""
    if all(v == 0 for v in lo) and all(v == 0 for v in hi):
        return x
    sp = _sp(x.shape, nsp)
    out_sp = [s + a + b for s, a, b in zip(sp, lo, hi)]
    out = dev.empty((x.shape[0], *out_sp, *_ch(x.shape, nsp)), x.dtype)
    if _empty_ok(x, out):
        check(lib.kmp_pad(nsp, dev.dtype_code(x), x.data_ptr(), x.shape[0], _lib.i64x3(sp), _C(x.shape, nsp),
                          _lib.i64x3(lo), _lib.i64x3(hi), mode, out.data_ptr(), dev.stream()), 'pad')
    return out


def d_pad_neighborhood(lowres, padding, nsp):
    return d_pad(lowres, (padding,) * nsp, (padding,) * nsp, 0, nsp)


def highres_dims(shape, nsp):
    return tuple((s + 1) % 2 for s in _sp(shape, nsp))


def d_pad_highres(h, nsp):
    dims = highres_dims(h.shape, nsp)
    return d_pad(h, (0,) * nsp, dims, 1, nsp), dims


def d_pad_lowres(lowres, dims, nsp):
    return d_pad(lowres, (0,) * nsp, tuple(dims), 0, nsp)


def map_dims(dims, nsp):
    # a map is padded / trimmed on the axes where it lies on the node lattice (volume/utils.py:258-276)
    return [tuple(d if p == 0 else 0 for d, p in zip(dims, par)) for par in PARITY[nsp]]


def d_pad_maps(maps, dims, nsp):
    return tuple(d_pad(m, (0,) * nsp, md, 0, nsp) for m, md in zip(maps, map_dims(dims, nsp)))


def d_trim(x, dims, nsp):
    return d_pad(x, (0,) * nsp, tuple(-int(d) for d in dims), 0, nsp)


def d_trim_maps(maps, dims, nsp):
    return tuple(d_trim(m, md, nsp) for m, md in zip(maps, map_dims(dims, nsp)))


# ---------------------------------------------------------------------------------------------
# Coders
# ---------------------------------------------------------------------------------------------

def d_code(direction, coder, pred, x):
    pred, x = _dev(pred), _dev(x)
    _require(tuple(pred.shape) == tuple(x.shape),
             f'coder operands must have equal shapes, got {tuple(pred.shape)} and {tuple(x.shape)}')
    out = dev.empty(x.shape, CODER_DTYPE[coder])
    if x.numel():
        check(lib.kmp_code(direction, coder, dev.dtype_code(pred), pred.data_ptr(), dev.dtype_code(x), x.data_ptr(),
                           x.numel(), out.data_ptr(), dev.stream()), 'code')
    return out


def d_categorical(direction, logits, x):
    logits, x = _dev(logits), _dev(x)
    _require(logits.dtype == torch.float32, 'categorical logits must be float32')
    _require(tuple(logits.shape[:-1]) == tuple(x.shape), 'logits must be [..., L] over the values [...]')
    out = dev.empty(x.shape, x.dtype)
    if x.numel():
        check(lib.kmp_categorical(direction, logits.data_ptr(), x.numel(), logits.shape[-1], dev.dtype_code(x),
                                  x.data_ptr(), out.data_ptr(), dev.stream()), 'categorical')
    return out


# =============================================================================================
# Fused one-pass codec (built-in predictor + built-in coder)
# =============================================================================================

def fused_enabled():
    return os.environ.get('KOMPRESSOR_AMD_FUSED', '1') != '0'


def fused_plan(predictions_fn, code_fn, padding, dtype, nsp, direction):
    """(predictor, coder) when the call can run as one fused kernel, else None."""
    if not fused_enabled():
        return None
    kmp_pred = getattr(predictions_fn, '_kmp_predictor', None)
    kmp_code = getattr(code_fn, '_kmp_coder', None)
    if kmp_pred is None or kmp_code is None:
        return None
    if kmp_code[1] != direction or predictions_fn.padding != padding or predictions_fn.ndim != nsp:
        return None
    if NATURAL_CODER.get(dtype) != kmp_code[0]:
        return None
    return predictions_fn, kmp_code[0]


def callback_coder(code_fn, dtype, direction):
    """The built-in coder id when ``code_fn`` is the natural coder of ``dtype`` (the callback path
    then runs the steps around an opaque predictions_fn as two fused launches), else None."""
    if not fused_enabled():
        return None
    kc = getattr(code_fn, '_kmp_coder', None)
    if kc is None or kc[1] != direction or NATURAL_CODER.get(dtype) != kc[0]:
        return None
    return kc[0]


def d_window_from_highres(h, padding, nsp):
    """pad_neighborhood(lowres_from_highres(pad_highres(h)), padding), one gather."""
    sp = _sp(h.shape, nsp)
    L = [(s + d + 1) // 2 for s, d in zip(sp, highres_dims(h.shape, nsp))]
    out = dev.empty((h.shape[0], *[l + 2 * padding for l in L], *_ch(h.shape, nsp)), h.dtype)
    if _empty_ok(h, out):
        check(lib.kmp_window_from_highres(nsp, dev.dtype_code(h), h.data_ptr(), h.shape[0], _lib.i64x3(sp),
                                          _C(h.shape, nsp), padding, out.data_ptr(), dev.stream()), 'window')
    return out


def d_window_from_lowres(lo, dims, padding, nsp):
    """pad_neighborhood(pad_lowres(lo, dims), padding), one gather."""
    E = _sp(lo.shape, nsp)
    out = dev.empty((lo.shape[0], *[e + d + 2 * padding for e, d in zip(E, dims)], *_ch(lo.shape, nsp)), lo.dtype)
    if _empty_ok(lo, out):
        check(lib.kmp_window_from_lowres(nsp, dev.dtype_code(lo), lo.data_ptr(), lo.shape[0], _lib.i64x3(E),
                                         _C(lo.shape, nsp), _lib.i32xn(dims), padding, out.data_ptr(), dev.stream()),
              'window')
    return out


def _preds_fit(preds, dtype, B, L, ch, nsp):
    """The prediction maps' dtype code when predictions_fn's maps can feed the fused coder kernels
    directly -- contiguous device tensors in the untrimmed map shapes, all of the sample dtype or all
    float32 (a network's output, which the coder reads as ``jnp.int32(pred)``, utils.py:28-55) --
    else None."""
    pdt = preds[0].dtype if isinstance(preds[0], torch.Tensor) else None
    if pdt not in (dtype, torch.float32):
        return None
    for m, par in zip(preds, PARITY[nsp]):
        want = (B, *[(l - 1 if p else l) for l, p in zip(L, par)], *ch)
        if not (isinstance(m, torch.Tensor) and m.is_cuda and m.dtype == pdt and m.is_contiguous()
                and tuple(m.shape) == want):
            return None
    return dev.dtype_code(preds[0])


def _workspace(nbytes):
    return dev.empty((max(int(nbytes), 1),), torch.uint8)


def _region(nsp, region):
    if region is None:
        return None
    r = _lib.Region()
    off = 3 - nsp
    for a in range(3):
        if a < off:
            r.begin[a], r.end[a] = 0, 1
        else:
            r.begin[a], r.end[a] = region[a - off]
    return r


def encoded_shapes(shape, nsp):
    """Shapes of (lowres, maps) produced by encode for a highres ``shape``."""
    sp = _sp(shape, nsp)
    ch = _ch(shape, nsp)
    dims = highres_dims(shape, nsp)
    L = [(s + d + 1) // 2 for s, d in zip(sp, dims)]
    E = [l - d for l, d in zip(L, dims)]
    lo = (shape[0], *E, *ch)
    maps = [(shape[0], *[(l - 1 if p else e) for l, e, p in zip(L, E, par)], *ch) for par in PARITY[nsp]]
    return lo, maps, dims


def _ptr(t):
    """Device address of ``t``: its data pointer for a device tensor; for a pinned host tensor the
    device mapping of the page-locked buffer (zero-copy: the kernel reads / writes host memory
    over the host link directly, ``kmp_host_device_pointer``).  The mapping is looked up on every
    call (about a microsecond): a cache keyed by host address would hand out a stale mapping once
    a freed pinned buffer's address is reused."""
    if t.is_cuda:
        return t.data_ptr()
    if not t.is_pinned():
        raise TypeError('fused kernels take device tensors or pinned host tensors')
    base = t.untyped_storage().data_ptr()
    out = ctypes.c_void_p()
    check(lib.kmp_host_device_pointer(ctypes.c_void_p(base), ctypes.byref(out)), 'host_device_pointer')
    return out.value + (t.data_ptr() - base)


def _ptrs(tensors):
    arr = (ctypes.c_void_p * 7)()
    for i, t in enumerate(tensors):
        arr[i] = _ptr(t)
    return arr


def workspace_bytes(h, predictor, nsp):
    """Device workspace the fused calls may need for highres ``h`` (0 on the one-pass path)."""
    B, sp, C = h.shape[0], _sp(h.shape, nsp), _C(h.shape, nsp)
    pstruct = predictor._kmp_predictor(h.dtype)
    fn = lib.kmp_volume_workspace_bytes if nsp == 3 else lib.kmp_image_workspace_bytes
    return int(fn(dev.dtype_code(h), B, *sp, C, ctypes.byref(pstruct)))


def fused_encode_into(h, predictor, coder, lowres, maps, nsp, region=None, workspace=None):
    B, sp, C = h.shape[0], _sp(h.shape, nsp), _C(h.shape, nsp)
    pstruct = predictor._kmp_predictor(h.dtype)
    if nsp == 3:
        need = lib.kmp_volume_workspace_bytes(dev.dtype_code(h), B, *sp, C, ctypes.byref(pstruct))
    else:
        need = lib.kmp_image_workspace_bytes(dev.dtype_code(h), B, *sp, C, ctypes.byref(pstruct))
    ws = workspace if workspace is not None and workspace.numel() >= need else _workspace(need)
    dims = (ctypes.c_int32 * 3)()
    reg = _region(nsp, region)
    args = (dev.dtype_code(h), _ptr(h), B, *sp, C, ctypes.byref(pstruct), coder, _ptr(lowres),
            _ptrs(maps), dims, ctypes.byref(reg) if reg is not None else None, ws.data_ptr(), ws.numel(),
            dev.stream())
    fn = lib.kmp_volume_encode if nsp == 3 else lib.kmp_image_encode
    check(fn(*args), 'fused encode')
    return tuple(int(dims[a]) for a in range(nsp))


def fused_decode_into(lowres, maps, dims, predictor, coder, out, nsp, region=None, workspace=None):
    B, E, C = lowres.shape[0], _sp(lowres.shape, nsp), _C(lowres.shape, nsp)
    pstruct = predictor._kmp_predictor(lowres.dtype)
    hs = [2 * e - 1 + d for e, d in zip(E, dims)]
    if nsp == 3:
        need = lib.kmp_volume_workspace_bytes(dev.dtype_code(lowres), B, *hs, C, ctypes.byref(pstruct))
    else:
        need = lib.kmp_image_workspace_bytes(dev.dtype_code(lowres), B, *hs, C, ctypes.byref(pstruct))
    ws = workspace if workspace is not None and workspace.numel() >= need else _workspace(need)
    reg = _region(nsp, region)
    dims_c = _lib.i32xn(dims)
    args = (dev.dtype_code(lowres), _ptr(lowres), _ptrs(maps), B, *E, C, dims_c, ctypes.byref(pstruct),
            coder, _ptr(out), ctypes.byref(reg) if reg is not None else None, ws.data_ptr(), ws.numel(),
            dev.stream())
    fn = lib.kmp_volume_decode if nsp == 3 else lib.kmp_image_decode
    check(fn(*args), 'fused decode')
    return out


def _alloc_encoded(h, coder, nsp):
    lo_shape, map_shapes, dims = encoded_shapes(h.shape, nsp)
    lowres = dev.empty(lo_shape, h.dtype)
    maps = [dev.empty(s, CODER_DTYPE[coder]) for s in map_shapes]
    return lowres, maps, dims


def _check_encoded_maps(lowres, maps, dims, nsp):
    E = _sp(lowres.shape, nsp)
    ch = _ch(lowres.shape, nsp)
    _require(len(maps) == NMAPS[nsp], f'expected {NMAPS[nsp]} encoded maps')
    _require(len(dims) == nsp and all(int(d) in (0, 1) for d in dims), 'dims must be 0/1 per spatial axis')
    for i, (m, par) in enumerate(zip(maps, PARITY[nsp])):
        want = (lowres.shape[0], *[(e + int(d) - 1 if p else e) for e, d, p in zip(E, dims, par)], *ch)
        _require(tuple(m.shape) == want, f'encoded map {i} has shape {tuple(m.shape)}, expected {want}')


# =============================================================================================
# encode / decode -- volume/encode_decode.py:30-85, image/encode_decode.py:30-85
# =============================================================================================

def _callback_maps(maps, nsp):
    maps = list(maps)
    _require(len(maps) == NMAPS[nsp], f'predictions_fn must return {NMAPS[nsp]} maps')
    return [_dev(m) for m in maps]


@_trace.traced('kmp.encode')
def encode(predictions_fn, encode_fn, highres, padding, nsp):
    validate_padding(padding)
    dims = highres_dims(highres.shape, nsp)
    padded_shape = (highres.shape[0], *[s + d for s, d in zip(_sp(highres.shape, nsp), dims)],
                    *_ch(highres.shape, nsp))
    validate_highres_shape(padded_shape, nsp)
    h, kind = dev.to_device(highres)
    plan = fused_plan(predictions_fn, encode_fn, padding, h.dtype, nsp, _lib.ENCODE)
    if plan is not None:
        predictor, coder = plan
        lowres, maps, dims = _alloc_encoded(h, coder, nsp)
        fused_encode_into(h, predictor, coder, lowres, maps, nsp)
        encoded = tuple(maps)
    else:
        coder = callback_coder(encode_fn, h.dtype, _lib.ENCODE)
        L = [(s + d + 1) // 2 for s, d in zip(_sp(h.shape, nsp), dims)]
        if coder is not None:
            # the callback path with a built-in coder: window gather, predictions_fn, one coder launch
            validate_lowres_shape((h.shape[0], *L, *_ch(h.shape, nsp)), nsp)
            with _trace.stage('kmp.predictions_fn'):
                pred_maps = _callback_maps(predictions_fn(d_window_from_highres(h, padding, nsp)), nsp)
            pdt = _preds_fit(pred_maps, h.dtype, h.shape[0], L, _ch(h.shape, nsp), nsp)
            if pdt is not None:
                lowres, encoded, dims = _alloc_encoded(h, coder, nsp)
                check(lib.kmp_encode_with_predictions_typed(nsp, dev.dtype_code(h), coder, pdt, h.data_ptr(),
                                                            h.shape[0], _lib.i64x3(_sp(h.shape, nsp)),
                                                            _C(h.shape, nsp), _lib.ptrs(pred_maps), lowres.data_ptr(),
                                                            _lib.ptrs(encoded), dev.stream()),
                      'encode_with_predictions')
                return (dev.from_device(lowres, kind),
                        (tuple(dev.from_device(m, kind) for m in encoded), tuple(dims)))
        else:
            pred_maps = None
        hp, dims = d_pad_highres(h, nsp)
        lowres = d_lowres_from_highres(hp, nsp)
        validate_lowres_shape(lowres.shape, nsp)
        gt_maps = d_maps_from_highres(hp, nsp)
        if pred_maps is None:
            pred_maps = _callback_maps(predictions_fn(d_pad_neighborhood(lowres, padding, nsp)), nsp)
        encoded = [_dev(encode_fn(p, g)) for p, g in zip(pred_maps, gt_maps)]
        encoded = d_trim_maps(encoded, dims, nsp)
        lowres = d_trim(lowres, dims, nsp)
    return dev.from_device(lowres, kind), (tuple(dev.from_device(m, kind) for m in encoded), tuple(dims))


@_trace.traced('kmp.decode')
def decode(predictions_fn, decode_fn, lowres, encoded, padding, nsp):
    encoded_maps, dims = encoded
    dims = tuple(int(d) for d in dims)
    validate_padding(padding)
    validate_lowres_shape(lowres.shape, nsp)
    lo, kind = dev.to_device(lowres)
    maps = [_dev(m) for m in encoded_maps]
    plan = fused_plan(predictions_fn, decode_fn, padding, lo.dtype, nsp, _lib.DECODE)
    if plan is not None and all(m.dtype == CODER_DTYPE[plan[1]] for m in maps):
        predictor, coder = plan
        _check_encoded_maps(lo, maps, dims, nsp)
        out = dev.empty((lo.shape[0], *[2 * e - 1 + d for e, d in zip(_sp(lo.shape, nsp), dims)],
                         *_ch(lo.shape, nsp)), lo.dtype)
        fused_decode_into(lo, maps, dims, predictor, coder, out, nsp)
        return dev.from_device(out, kind)
    coder = callback_coder(decode_fn, lo.dtype, _lib.DECODE)
    pred_maps = None
    if coder is not None and all(m.dtype == CODER_DTYPE[coder] and m.is_contiguous() for m in maps):
        # the callback path with a built-in coder: window gather, predictions_fn, one coder launch
        _check_encoded_maps(lo, maps, dims, nsp)
        L = [e + d for e, d in zip(_sp(lo.shape, nsp), dims)]
        with _trace.stage('kmp.predictions_fn'):
            pred_maps = _callback_maps(predictions_fn(d_window_from_lowres(lo, dims, padding, nsp)), nsp)
        pdt = _preds_fit(pred_maps, lo.dtype, lo.shape[0], L, _ch(lo.shape, nsp), nsp)
        if pdt is not None:
            lo = lo.contiguous()
            out = dev.empty((lo.shape[0], *[2 * l - 1 - d for l, d in zip(L, dims)], *_ch(lo.shape, nsp)), lo.dtype)
            check(lib.kmp_decode_with_predictions_typed(nsp, dev.dtype_code(lo), coder, pdt, lo.data_ptr(),
                                                        _lib.ptrs(maps), lo.shape[0], _lib.i64x3(_sp(lo.shape, nsp)),
                                                        _C(lo.shape, nsp), _lib.i32xn(dims), _lib.ptrs(pred_maps),
                                                        out.data_ptr(), dev.stream()), 'decode_with_predictions')
            return dev.from_device(out, kind)
    lo_p = d_pad_lowres(lo, dims, nsp)
    maps_p = d_pad_maps(maps, dims, nsp)
    if pred_maps is None:
        pred_maps = _callback_maps(predictions_fn(d_pad_neighborhood(lo_p, padding, nsp)), nsp)
    decoded = [_dev(decode_fn(p, e)) for p, e in zip(pred_maps, maps_p)]
    hi = d_highres_from_lowres_and_maps(lo_p, decoded, nsp)
    return dev.from_device(d_trim(hi, dims, nsp), kind)


# =============================================================================================
# Multi-level pyramid: the reference's single level applied recursively
# =============================================================================================

def _per_level(fn, levels, what):
    if isinstance(fn, (list, tuple)):
        _require(len(fn) == levels, f'{what}: one per level ({levels}) expected, got {len(fn)}')
        return list(fn)
    return [fn] * levels


@_trace.traced('kmp.encode_pyramid')
def encode_pyramid(predictions_fn, encode_fn, highres, levels, padding, nsp):
    """``levels`` applications of ``encode`` (volume/encode_decode.py:30-56), each on the previous
    level's lowres.  ``predictions_fn`` / ``encode_fn`` may be one callable or one per level
    (finest first).  Returns ``(lowres, [(maps, dims), ...])`` finest level first."""
    _require(isinstance(levels, int) and not isinstance(levels, bool) and levels >= 1, 'levels must be an int >= 1')
    preds, encs = _per_level(predictions_fn, levels, 'predictions_fn'), _per_level(encode_fn, levels, 'encode_fn')
    x, out = highres, []
    for lvl in range(levels):
        x, enc = encode(preds[lvl], encs[lvl], x, padding, nsp)
        out.append(enc)
    return x, out


@_trace.traced('kmp.decode_pyramid')
def decode_pyramid(predictions_fn, decode_fn, lowres, encoded, padding, nsp):
    """Inverse of :func:`encode_pyramid`: decode the coarsest level first."""
    encoded = list(encoded)
    levels = len(encoded)
    _require(levels >= 1, 'encoded must hold at least one level')
    preds, decs = _per_level(predictions_fn, levels, 'predictions_fn'), _per_level(decode_fn, levels, 'decode_fn')
    x = lowres
    for lvl in reversed(range(levels)):
        x = decode(preds[lvl], decs[lvl], x, encoded[lvl], padding, nsp)
    return x


# =============================================================================================
# Chunked drivers -- volume/encode_decode_chunk.py:33-117, image/encode_decode_chunk.py:33-115
# =============================================================================================

def _chunk_list(L, chunk, nsp, progress_fn):
    cks = validate_chunk(chunk, nsp)
    chunks = product(*[yield_chunks(l, c) for l, c in zip(L, cks)])
    if progress_fn is not None:
        return progress_fn(list(chunks))
    return chunks


def fused_chunk_regions(chunk_list, E, nsp):
    """Output-frame regions for the fused chunked drivers.

    The reference codes one chunk window at a time (encode_decode_chunk.py:98-115) and its tests
    pin that the result equals the whole-array call (tests/volume/test_encode_decode.py:509-539).
    The fused kernels never materialise windows, so the chunks of one slab along the leading
    spatial axis (consecutive in the reference's z-major order) are merged into ONE launch
    whenever together they cover that slab's whole cross-section -- the normal case; a chunk that
    is not part of such a covered slab keeps its own launch.  ``covered`` is False when the chunks
    leave part of the output unreached (a progress_fn that filters chunks): the callers then run
    the reference's step sequence instead, whose unreached map entries stay zero (``zeros_like``,
    :91).  Returns ``(regions, covered)``."""
    boxes = [[(i0, min(i1, e)) for ((i0, i1), _), e in zip(ranges, E)] for ranges in chunk_list]
    key = (tuple(tuple(b) for b in boxes), tuple(int(e) for e in E))
    hit = _REGION_CACHE.get(key)
    if hit is not None:  # the plan depends only on the boxes and the frame: ~35 us of numpy per call
        return [list(r) for r in hit[0]], hit[1]
    regions, covered = _chunk_regions(boxes, E)
    if len(_REGION_CACHE) > 256:
        _REGION_CACHE.clear()
    _REGION_CACHE[key] = (tuple(tuple(r) for r in regions), covered)
    return regions, covered


_REGION_CACHE = {}


def _covers(regions, E):
    """True when the union of the boxes ``regions`` covers the frame ``[0, E)``.  Checked on the
    grid the boxes' own edges cut the frame into (a few cells per window per axis), not on a dense
    per-element mask -- a 2048^3 volume's lowres frame would be a 1 GB mask."""
    cuts = [sorted({0, int(e)} | {min(max(int(v), 0), int(e)) for r in regions for v in r[a]})
            for a, e in enumerate(E)]
    grid = np.zeros(tuple(max(len(c) - 1, 0) for c in cuts), dtype=bool)
    for r in regions:
        grid[tuple(slice(int(np.searchsorted(c, min(max(a, 0), e))), int(np.searchsorted(c, min(max(b, 0), e))))
                   for (a, b), c, e in zip(r, cuts, E))] = True
    return bool(grid.all())


def _chunk_regions(boxes, E):
    regions = []
    done = np.zeros(E[0], dtype=bool)  # leading-axis planes written by a full-slab launch
    k = 0
    while k < len(boxes):
        lead = boxes[k][0]
        j = k
        while j < len(boxes) and boxes[j][0] == lead:
            j += 1
        if _covers([b[1:] for b in boxes[k:j]], E[1:]):
            # overlapping windows (yield_chunks steps by chunk - 3) rewrite planes an earlier slab
            # already wrote with identical values: launch only the planes not yet written
            a = lead[0]
            while a < lead[1]:
                if done[a]:
                    a += 1
                    continue
                b = a
                while b < lead[1] and not done[b]:
                    b += 1
                regions.append([(a, b)] + [(0, e) for e in E[1:]])
                done[a:b] = True
                a = b
        else:
            regions.extend(boxes[k:j])
        k = j
    return _merge_slabs(regions, E), _covers(regions, E)


def _merge_slabs(regions, E):
    """Adjacent full-cross-section slabs merged into one region: the fused kernels give any region
    the whole-array call's values (chunk invariance, tests/volume/test_encode_decode.py:509-539), so
    slabs that tile [a, b) along the leading axis are ONE launch -- at chunk = 32 on 64^3 tiles the
    windows' two slabs become the single whole-frame launch."""
    full = [r for r in regions if all(tuple(r[a]) == (0, e) for a, e in enumerate(E) if a > 0)]
    rest = [r for r in regions if not all(tuple(r[a]) == (0, e) for a, e in enumerate(E) if a > 0)]
    merged = []
    for r in sorted(full, key=lambda r: r[0][0]):
        if merged and merged[-1][0][1] == r[0][0]:
            merged[-1] = [(merged[-1][0][0], r[0][1])] + list(merged[-1][1:])
        else:
            merged.append(list(r))
    return merged + rest


def d_process_chunks(predictions_fn, code_fn, lowres, reference_maps, chunk_list, padding, nsp):
    """encode_decode_chunk.py:77-117 over an already enumerated (and progress_fn-filtered) chunk list."""
    padded = d_pad_neighborhood(lowres, padding, nsp)
    coded = [_zeros(r.shape, r.dtype) for r in reference_maps]
    for ranges in chunk_list:
        starts = [i0 - p0 for (i0, _), (p0, _) in ranges]
        ext = [(i1 + p1 + 2 * padding) - (i0 - p0) for (i0, i1), (p0, p1) in ranges]
        window = d_crop(padded, starts, ext, nsp)
        preds = _callback_maps(predictions_fn(window), nsp)
        for idx, (pm, ref) in enumerate(zip(preds, reference_maps)):
            sub = [pm.shape[1 + a] - (ranges[a][1][0] + ranges[a][1][1]) for a in range(nsp)]
            sub_pred = d_crop(pm, [r[1][0] for r in ranges], sub, nsp)
            sub_ref = d_crop(ref, [r[0][0] for r in ranges], sub, nsp)
            value = _dev(code_fn(sub_pred, sub_ref))
            d_copy_box(value, (0,) * nsp, sub, coded[idx], [r[0][0] for r in ranges], nsp)
    return coded


def _chunks_for(L, chunk, padding, progress_fn, nsp):
    # process_chunks' checks (encode_decode_chunk.py:77-96), then the one progress_fn call
    validate_padding(padding)
    validate_chunk(chunk, nsp)
    _require(all(l >= 2 for l in L), f'lowres spatial dims must be >= 2, got {tuple(L)}')
    return list(_chunk_list(L, chunk, nsp, progress_fn))


@_trace.traced('kmp.encode_chunks')
def encode_chunks(predictions_fn, encode_fn, highres, chunk, padding, progress_fn, nsp):
    dims = highres_dims(highres.shape, nsp)
    padded_shape = (highres.shape[0], *[s + d for s, d in zip(_sp(highres.shape, nsp), dims)],
                    *_ch(highres.shape, nsp))
    validate_highres_shape(padded_shape, nsp)
    validate_padding(padding)
    h, kind = dev.to_device(highres)
    L = [(s + 1) // 2 for s in _sp(padded_shape, nsp)]
    chunk_list = _chunks_for(L, chunk, padding, progress_fn, nsp)
    plan = fused_plan(predictions_fn, encode_fn, padding, h.dtype, nsp, _lib.ENCODE)
    if plan is not None:
        predictor, coder = plan
        lowres, maps, dims = _alloc_encoded(h, coder, nsp)
        regions, covered = fused_chunk_regions(chunk_list, _sp(lowres.shape, nsp), nsp)
        if covered:
            for region in regions:
                fused_encode_into(h, predictor, coder, lowres, maps, nsp, region=region)
            return dev.from_device(lowres, kind), (tuple(dev.from_device(m, kind) for m in maps), tuple(dims))
    hp, dims = d_pad_highres(h, nsp)
    lowres = d_lowres_from_highres(hp, nsp)
    gt_maps = d_maps_from_highres(hp, nsp)
    coded = d_process_chunks(predictions_fn, encode_fn, lowres, gt_maps, chunk_list, padding, nsp)
    encoded = d_trim_maps(coded, dims, nsp)
    lowres = d_trim(lowres, dims, nsp)
    return dev.from_device(lowres, kind), (tuple(dev.from_device(m, kind) for m in encoded), tuple(dims))


@_trace.traced('kmp.decode_chunks')
def decode_chunks(predictions_fn, decode_fn, lowres, encoded, chunk, padding, progress_fn, nsp):
    encoded_maps, dims = encoded
    dims = tuple(int(d) for d in dims)
    validate_padding(padding)
    validate_lowres_shape(lowres.shape, nsp)
    lo, kind = dev.to_device(lowres)
    maps = [_dev(m) for m in encoded_maps]
    E = _sp(lo.shape, nsp)
    L = [e + d for e, d in zip(E, dims)]
    chunk_list = _chunks_for(L, chunk, padding, progress_fn, nsp)
    plan = fused_plan(predictions_fn, decode_fn, padding, lo.dtype, nsp, _lib.DECODE)
    if plan is not None and all(m.dtype == CODER_DTYPE[plan[1]] for m in maps):
        predictor, coder = plan
        _check_encoded_maps(lo, maps, dims, nsp)
        regions, covered = fused_chunk_regions(chunk_list, E, nsp)
        if covered:
            out = dev.empty((lo.shape[0], *[2 * e - 1 + d for e, d in zip(E, dims)], *_ch(lo.shape, nsp)),
                            lo.dtype)
            for region in regions:
                fused_decode_into(lo, maps, dims, predictor, coder, out, nsp, region=region)
            return dev.from_device(out, kind)
    lo_p = d_pad_lowres(lo, dims, nsp)
    maps_p = d_pad_maps(maps, dims, nsp)
    decoded = d_process_chunks(predictions_fn, decode_fn, lo_p, maps_p, chunk_list, padding, nsp)
    hi = d_highres_from_lowres_and_maps(lo_p, decoded, nsp)
    return dev.from_device(d_trim(hi, dims, nsp), kind)


# =============================================================================================
# Public wrappers for the primitives (numpy or torch in, same kind out)
# =============================================================================================

def _fresh(out, src):
    """``out``, or a copy of it when it shares memory with the caller's ``src`` (a zero-width pad or
    trim returns its input on the device path): the reference is purely functional -- every
    output is a new array (SURVEY.md §8b "Ownership") -- so a torch caller must never get its own
    tensor back and see later writes to one through the other."""
    if isinstance(src, torch.Tensor) and src.is_cuda and out.numel() and src.numel() and \
            out.untyped_storage().data_ptr() == src.untyped_storage().data_ptr():
        return out.clone()
    return out


def wrap1(fn):
    def inner(x, *args):
        t, kind = dev.to_device(x)
        out = fn(t, *args)
        if isinstance(out, tuple):
            return tuple(dev.from_device(_fresh(o, x), kind) for o in out)
        return dev.from_device(_fresh(out, x), kind)
    return inner


def highres_from_lowres_and_maps(lowres, maps, nsp):
    lo, kind = dev.to_device(lowres)
    return dev.from_device(d_highres_from_lowres_and_maps(lo, [_dev(m) for m in maps], nsp), kind)


def pad_maps(maps, dims, nsp):
    maps = list(maps)
    kinds = [dev.to_device(m) for m in maps]
    outs = d_pad_maps([t for t, _ in kinds], dims, nsp)
    return tuple(dev.from_device(_fresh(o, m), k) for o, m, (_, k) in zip(outs, maps, kinds))


def trim_maps(maps, dims, nsp):
    maps = list(maps)
    kinds = [dev.to_device(m) for m in maps]
    outs = d_trim_maps([t for t, _ in kinds], dims, nsp)
    return tuple(dev.from_device(_fresh(o, m), k) for o, m, (_, k) in zip(outs, maps, kinds))


def to_numpy(x):
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)
