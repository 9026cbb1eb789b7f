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
"""

import torch

from . import _device as dev
from . import _nd


class CodecPlan:
    """Captured encode and decode of ``shape`` / ``dtype`` batches with a built-in predictor and
    the natural coder of the dtype (uint8 / uint16 modular, int32 raw, uint32 modular)."""

    def __init__(self, predictor, shape, dtype, warmup=1):
        dev.require_gpu()
        self.predictor = predictor
        self.nsp = predictor.ndim
        self.coder = _nd.NATURAL_CODER.get(dtype)
        if self.coder is None:
            raise TypeError(f'no lossless coder for {dtype}')
        sp = _nd._sp(shape, self.nsp)
        dims = _nd.highres_dims(shape, self.nsp)
        _nd.validate_highres_shape((shape[0], *[s + d for s, d in zip(sp, dims)], *_nd._ch(shape, self.nsp)),
                                   self.nsp)
        self.highres = dev.empty(shape, dtype)
        self.highres.zero_()
        self.lowres, self.maps, self.dims = _nd._alloc_encoded(self.highres, self.coder, self.nsp)
        self.out = torch.empty_like(self.highres)
        self.workspace = torch.empty(max(1, _nd.workspace_bytes(self.highres, predictor, self.nsp)),
                                     dtype=torch.uint8, device='cuda')
        enc = lambda: _nd.fused_encode_into(self.highres, predictor, self.coder, self.lowres, self.maps,  # noqa: E731
                                            self.nsp, workspace=self.workspace)
        dec = lambda: _nd.fused_decode_into(self.lowres, self.maps, self.dims, predictor, self.coder,  # noqa: E731
                                            self.out, self.nsp, workspace=self.workspace)
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

    def encode(self, highres=None):
        """Replay the encode (after copying ``highres`` into the static input, if given);
        returns ``(lowres, (maps, dims))`` -- the plan's static buffers."""
        if highres is not None:
            self.highres.copy_(dev.to_device(highres)[0])
        self._g_enc.replay()
        return self.lowres, (tuple(self.maps), tuple(self.dims))

    def decode(self):
        """Replay the decode of the static lowres / maps into ``plan.out``."""
        self._g_dec.replay()
        return self.out
