"""Codec plans replayed from HIP graphs: the fused encode / decode of a fixed tile batch captured
once and replayed with one graph launch per direction.

The fused path costs ~40 us of Python, ctypes and allocator work per call (``tools/host_overhead.py``)
next to ~0.1-0.2 ms of kernel time for a C3 batch, so small batches coded in a loop are
host-bound.  The C-ABI allocates and synchronises nothing (``include/kompressor_hip.h``), so its
launches capture into a graph on the current stream; a plan owns static device buffers (the
highres batch, lowres, the maps, the reconstruction and the workspace) and replays the captured
launches.  Fill ``plan.highres`` (or pass a tensor to :meth:`encode`, copied in), replay, read
``plan.lowres`` / ``plan.maps``; :meth:`decode` reconstructs into ``plan.out`` from the static
lowres / maps.  Same kernels and arithmetic as ``volume.encode`` / ``decode`` with a built-in
predictor (reference semantics: volume/encode_decode.py:30-85).

    plan = CodecPlan(kom.MeanPredictor(0, 3), (64, 64, 64, 64, 1), torch.uint16)
    plan.highres.copy_(tiles)          # or plan.encode(tiles)
    plan.encode()                      # one graph launch
    lowres, maps = plan.lowres, plan.maps
    plan.decode()                      # plan.out == tiles

An opaque ``predictions_fn`` (a trained network, the reference's real use: volume/encode_decode.py:48)
is planned the same way when it is capture-safe -- torch ops on the device, no host synchronisation
(``.item()``, ``.cpu()``), no CPU tensors: the callback path (window gather, the callable, one coder
launch) is captured as it runs eagerly, and ``padding`` must be given:

    plan = CodecPlan(net, (64, 64, 64, 64, 1), torch.uint16, padding=1)
"""

import torch

from . import _device as dev
from . import _lib
from . import _nd


def _natural_coder_fns(coder):
    from . import utils
    return {_lib.CODER_U8: (utils.encode_values_uint8, utils.decode_values_uint8),
            _lib.CODER_U16: (utils.encode_values_uint16, utils.decode_values_uint16),
            _lib.CODER_RAW: (utils.encode_values_raw, utils.decode_values_raw),
            _lib.CODER_U32: (utils.encode_values_uint32, utils.decode_values_uint32)}[coder]


class CodecPlan:
    """Captured encode and decode of ``shape`` / ``dtype`` batches with the natural coder of the
    dtype (uint8 / uint16 modular, int32 raw, uint32 modular) and a built-in predictor (one fused
    kernel per direction) or a capture-safe ``predictions_fn`` (the callback path; ``padding``
    required, ``ndim`` defaults to ``len(shape) - 2``)."""

    def __init__(self, predictor, shape, dtype, warmup=1, padding=None, ndim=None):
        dev.require_gpu()
        self.predictor = predictor
        builtin = getattr(predictor, '_kmp_predictor', None) is not None
        self.nsp = predictor.ndim if builtin else (ndim if ndim is not None else len(shape) - 2)
        self.coder = _nd.NATURAL_CODER.get(dtype)
        if self.coder is None:
            raise TypeError(f'no lossless coder for {dtype}')
        if builtin:
            padding = predictor.padding if padding is None else padding
            if padding != predictor.padding:
                raise ValueError(f'padding {padding} differs from the predictor\'s {predictor.padding}')
        elif padding is None:
            raise ValueError('a predictions_fn plan needs padding=')
        _nd.validate_padding(padding)
        self.padding = padding
        sp = _nd._sp(shape, self.nsp)
        dims = _nd.highres_dims(shape, self.nsp)
        _nd.validate_highres_shape((shape[0], *[s + d for s, d in zip(sp, dims)], *_nd._ch(shape, self.nsp)),
                                   self.nsp)
        self.highres = dev.empty(shape, dtype)
        self.highres.zero_()
        self.fused = builtin and _nd.fused_enabled()
        if self.fused:
            self.lowres, self.maps, self.dims = _nd._alloc_encoded(self.highres, self.coder, self.nsp)
            self.out = torch.empty_like(self.highres)
            self.workspace = torch.empty(max(1, _nd.workspace_bytes(self.highres, predictor, self.nsp)),
                                         dtype=torch.uint8, device='cuda')
            enc = lambda: _nd.fused_encode_into(self.highres, predictor, self.coder, self.lowres,  # noqa: E731
                                                self.maps, self.nsp, workspace=self.workspace)
            dec = lambda: _nd.fused_decode_into(self.lowres, self.maps, self.dims, predictor,  # noqa: E731
                                                self.coder, self.out, self.nsp, workspace=self.workspace)
        else:
            # the eager callback path, captured: its outputs come from the graph's memory pool and
            # stay the plan's static buffers (each replay rewrites them in place)
            enc_fn, dec_fn = _natural_coder_fns(self.coder)
            enc = lambda: self._set_encoded(_nd.encode(predictor, enc_fn, self.highres,  # noqa: E731
                                                       padding, self.nsp))
            dec = lambda: setattr(self, 'out', _nd.decode(predictor, dec_fn, self.lowres,  # noqa: E731
                                                          (tuple(self.maps), self.dims), padding, self.nsp))
        # warm up outside the capture (first-launch initialisation), on a side stream as torch
        # requires for capture, then capture each direction
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                enc()
                dec()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self._g_enc, self._g_dec = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(self._g_enc):
            enc()
        with torch.cuda.graph(self._g_dec):
            dec()
        torch.cuda.synchronize()

    def _set_encoded(self, result):
        self.lowres, (maps, dims) = result
        self.maps, self.dims = list(maps), tuple(dims)

    def encode(self, highres=None, copy=False):
        """Replay the encode (after copying ``highres`` into the static input, if given);
        returns ``(lowres, (maps, dims))``.  Unlike the eager ``encode``, these are the plan's
        static buffers: the next replay overwrites them in place, so a caller that keeps a result
        across two calls must clone it -- or pass ``copy=True`` to get fresh tensors."""
        if highres is not None:
            self.highres.copy_(dev.to_device(highres)[0])
        self._g_enc.replay()
        if copy:
            return self.lowres.clone(), (tuple(m.clone() for m in self.maps), tuple(self.dims))
        return self.lowres, (tuple(self.maps), tuple(self.dims))

    def decode(self, copy=False):
        """Replay the decode of the static lowres / maps into ``plan.out`` and return it -- a static
        buffer the next replay overwrites (``copy=True`` returns a fresh tensor)."""
        self._g_dec.replay()
        return self.out.clone() if copy else self.out
