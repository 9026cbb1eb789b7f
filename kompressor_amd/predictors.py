"""Built-in predictors: callable ``predictions_fn`` objects that the fused kernels recognise.

The reference leaves the predictor to the caller (``predictions_fn`` slot,
volume/encode_decode.py:48) and its tests use a "mean of the neighbourhood" double
(tests/volume/test_encode_decode.py:43-55, tests/image/test_encode_decode.py:43-55).  These
classes are that predictor (``MeanPredictor``) and a dense per-cell linear predictor
(``LinearPredictor``, the "learned predictor apply" of the north star).  Called as plain
``predictions_fn(padded_lowres)`` they return the 7 (3) prediction maps exactly as the
reference's callback would; passed to ``encode`` / ``decode`` together with a built-in coder
they run as one fused HIP kernel per direction.
"""

import ctypes

import numpy as np
import torch

from . import _device as dev
from . import _lib
from ._nd import d_mean_predict_maps, d_maps_from_predictions, NPRED, _sp, _ch, _C
from ._lib import check, lib


class MeanPredictor:
    """``maps_from_predictions(repeat(astype(mean(features_from_lowres(x, p)), dtype)))``.

    ``maps_dtype=None`` returns the maps in the sample dtype (the reference test predictor);
    ``maps_dtype=float32`` returns the same values as float32 maps, written by the kernel -- the
    shape of a trained network's output, which the coders read as int32 (utils.py:38-55)."""

    def __init__(self, padding=0, ndim=3, maps_dtype=None):
        if ndim not in (2, 3):
            raise ValueError('ndim must be 2 (image) or 3 (volume)')
        if not isinstance(padding, int) or padding < 0:
            raise ValueError('padding must be an int >= 0')
        if maps_dtype is not None and maps_dtype is not torch.float32 and (
                isinstance(maps_dtype, torch.dtype) or np.dtype(maps_dtype) != np.float32):
            raise ValueError('maps_dtype must be None (the sample dtype) or float32')
        self.padding, self.ndim = padding, ndim
        self.maps_dtype = None if maps_dtype is None else torch.float32

    def _kmp_predictor(self, dtype=None):
        return _lib.Predictor(_lib.PRED_MEAN, self.padding, None, None)

    def __call__(self, lowres):
        t, kind = dev.to_device(lowres)
        return tuple(dev.from_device(m, kind) for m in d_mean_predict_maps(t, self.padding, self.ndim,
                                                                          self.maps_dtype))

    def __repr__(self):
        md = '' if self.maps_dtype is None else ', maps_dtype=float32'
        return f'MeanPredictor(padding={self.padding}, ndim={self.ndim}{md})'


ARITHS = ('auto', 'f32', 'bf16x2')

# Revision of each arithmetic's rounding behaviour.  A revision changes whenever the bits an
# arithmetic produces change (e.g. the order in which the matrix-core form accumulates its
# products), so data coded under one revision is never decoded under another: files record it
# (container.py) and a reader refuses a mismatch instead of returning wrong samples.
#   f32 1     the k-ordered fma chain from the bias (unchanged since round 1)
#   bf16x2 1  round 4: one MFMA per 8 consecutive features
#   bf16x2 2  round 5: one MFMA per node row of a plane pair (kmp_bf16x2.h step_feature)
ARITH_REV = {'f32': 1, 'bf16x2': 2}


def resolve_arith(arith, padding, ndim, dtype):
    """The arithmetic a LinearPredictor evaluates with for samples of ``dtype``: ``'auto'`` is the
    matrix-core form (``'bf16x2'``) for volumes with padding 1 and 8- or 16-bit samples -- the
    learned-predictor configuration SURVEY.md §8d prices, where the fused ``linear3pm`` kernel codes a
    C3 direction in about half the f32 chain's time (profiles/round5/rows_linear_auto_r5a1.log; uint8
    since round 6) -- and the f32 chain everywhere else (padding 0, where the f32 kernel is the faster
    one; images; 32-bit samples, which bf16x2 cannot split exactly).  A function of the predictor and
    the sample dtype only, so encode, decode, chunked and whole-volume calls, and a file's reader all
    resolve it the same way."""
    if arith != 'auto':
        return arith
    return 'bf16x2' if ndim == 3 and padding == 1 and dtype in (torch.uint16, torch.uint8) else 'f32'


class LinearPredictor:
    """``pred[cell, k] = sum_n features[cell, n] * W[n, k] + b[k]``, cast to the sample dtype, then
    ``maps_from_predictions``.  ``W`` is ``[(2p+2)^ndim, 19 or 5]``.

    ``arith`` picks the arithmetic, and every path (fused codec kernels, the callable, the generic
    codec) evaluates a predictor with the same one, so encode and decode agree bit for bit:

    * ``'f32'``: the k-ordered float32 fma chain from the bias -- bit-identical to the oracle's
      restatement (``oracle.predictors.linear_fma_chain``);
    * ``'bf16x2'``: the matrix cores (kmp_bf16x2.h) -- features split into two exact bf16 bytes,
      weights into two bf16 terms, one ``v_mfma_f32_16x16x32_bf16`` per 8 features; within the north
      star's 1e-5 (relative to sum|f w| + |b|) of the float64 value rather than equal to the f32
      chain.  uint8 / uint16 samples;
    * ``'auto'`` (default): ``'bf16x2'`` where the matrix cores are the fast path (volumes, padding 1,
      uint8 / uint16 samples), ``'f32'`` elsewhere (:func:`resolve_arith`).  Breaking change (round 5,
      uint8 in round 6): the default was ``'f32'``; in-memory encodings made with the old default must
      be decoded with ``arith='f32'`` (files record their arithmetic, and ``container.decompress``
      takes it from the file for a default-constructed predictor)."""

    def __init__(self, weights, bias, padding=0, ndim=3, arith='auto'):
        if ndim not in (2, 3):
            raise ValueError('ndim must be 2 (image) or 3 (volume)')
        if arith not in ARITHS:
            raise ValueError(f'arith must be one of {ARITHS}')
        self.arith = arith
        n, k = (2 * padding + 2) ** ndim, NPRED[ndim]
        w = torch.as_tensor(np.asarray(weights, dtype=np.float32) if not isinstance(weights, torch.Tensor)
                            else weights, dtype=torch.float32)
        b = torch.as_tensor(np.asarray(bias, dtype=np.float32) if not isinstance(bias, torch.Tensor)
                            else bias, dtype=torch.float32)
        if tuple(w.shape) != (n, k) or tuple(b.shape) != (k,):
            raise ValueError(f'weights must be [{n}, {k}] and bias [{k}] for padding={padding}, ndim={ndim}')
        self.padding, self.ndim = padding, ndim
        self._w_host, self._b_host = w.contiguous(), b.contiguous()
        self._w = self._b = None

    @property
    def weights(self):
        return self._w_host

    @property
    def bias(self):
        return self._b_host

    def _device_params(self):
        if self._w is None:
            dev.require_gpu()
            self._w = self._w_host.to('cuda')
            self._b = self._b_host.to('cuda')
        return self._w, self._b

    def arith_for(self, dtype):
        """The arithmetic for samples of ``dtype`` (``arith`` with ``'auto'`` resolved)."""
        return resolve_arith(self.arith, self.padding, self.ndim, dtype)

    def _kmp_predictor(self, dtype):
        w, b = self._device_params()
        kind = _lib.PRED_LINEAR if self.arith_for(dtype) == 'f32' else _lib.PRED_LINEAR_MFMA
        return _lib.Predictor(kind, self.padding, w.data_ptr(), b.data_ptr())

    def predict_cells(self, lowres, with_f32=False):
        """Per-cell predictions ``[B, cells..., K, C...]`` in the sample dtype (and the f32 pre-cast
        values if ``with_f32``) for a padded lowres window."""
        t, kind = dev.to_device(lowres)
        w, b = self._device_params()
        nsp = self.ndim
        S = _sp(t.shape, nsp)
        cells = [s - 2 * self.padding - 1 for s in S]
        shape = (t.shape[0], *cells, NPRED[nsp], *_ch(t.shape, nsp))
        out = dev.empty(shape, t.dtype)
        f32 = dev.empty(shape, torch.float32) if with_f32 else None
        fn = lib.kmp_linear_predict if self.arith_for(t.dtype) == 'f32' else lib.kmp_linear_predict_mfma
        check(fn(nsp, dev.dtype_code(t), t.data_ptr(), t.shape[0], _lib.i64x3(S),
                                     _C(t.shape, nsp), self.padding, w.data_ptr(), b.data_ptr(), out.data_ptr(),
                                     f32.data_ptr() if f32 is not None else None, dev.stream()), 'linear_predict')
        if with_f32:
            return dev.from_device(out, kind), dev.from_device(f32, kind)
        return dev.from_device(out, kind)

    def __call__(self, lowres):
        t, kind = dev.to_device(lowres)
        cells = self.predict_cells(t)
        return tuple(dev.from_device(m, kind) for m in d_maps_from_predictions(cells, self.ndim))

    def __repr__(self):
        ar = '' if self.arith == 'auto' else f", arith='{self.arith}'"
        return f'LinearPredictor(padding={self.padding}, ndim={self.ndim}{ar})'
