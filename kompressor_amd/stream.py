"""Host-resident tile batches streamed through the GPU codec with copy / compute overlap.

The reference's path starts and ends in host memory (``encode`` takes a host array and returns
host arrays, ``volume/encode_decode.py:30-56``); the north star asks for that end-to-end rate
next to the device-resident one, and BASELINE config C5 streams a 2048^3 float32 volume as
128^3 chunks through pinned host memory.  :class:`TileStream` keeps ``slots`` device buffer
sets, each with its own HIP stream, and runs chunk ``i`` on slot ``i % slots``:

    H2D(chunk i) -> fused encode/decode kernel -> D2H(outputs of chunk i)

all on that slot's stream, so a slot is reused only after its previous chunk's D2H has been
issued ahead of it (stream order), while the other slots' copies and kernels overlap it (the
host->device and device->host DMA engines and the CUs run concurrently).  Host buffers must be
pinned (``torch.empty(..., pin_memory=True)``) for the copies to be asynchronous DMA.

For 8/16-bit samples the default is **zero-copy** instead: pinned host memory is mapped into the
GPU's address space (``kmp_host_device_pointer``), so ONE fused launch reads the host input and
writes the host outputs over the link itself -- reads and writes interleave, using both link
directions at once, with no staging buffers and no per-map DMA descriptors (8 outputs per chunk
made the copy pipeline descriptor-bound: 16.4 GB/s vs 20.1 GB/s end to end at C3 on MI355X,
``profiles/round1/h2d_probe.log``).  32-bit samples (float32 bit-cast to uint32, int32) have a
one-pass kernel too (``kmp_codec_wave3d32.hip``) and stream zero-copy as well; ``zero_copy=False``
(or ``KMP_STREAM_COPY=1``) selects the copy pipeline.

float32 data (config C5) is coded losslessly by bit-casting to uint32 and using the mod-2^32
coder (``encode_values_uint32``), a build extension: the reference has no lossless float coder
(``encode_values_raw`` truncates through ``int32``, ``utils.py:28-30``).
"""

import os

import torch

from . import _device as dev
from . import _nd


def pinned(shape, dtype):
    """A pinned (page-locked) host tensor, the only kind the DMA engines copy asynchronously."""
    return torch.empty(tuple(int(s) for s in shape), dtype=dtype, pin_memory=True)


def _as_codec_dtype(t):
    return t.view(torch.uint32) if t.dtype == torch.float32 else t


class TileStream:
    """Stream host tile batches ``[n, *tile, C...]`` through the fused codec on the current GPU.

    ``predictor`` is a built-in predictor (:class:`kompressor_amd.MeanPredictor` /
    :class:`~kompressor_amd.LinearPredictor`); the coder is the one whose modulus matches the
    sample dtype (uint8 / uint16 / uint32 for bit-cast float32; int32 -> raw).  ``chunk`` tiles
    move per copy.
    """

    def __init__(self, predictor, tile_shape, dtype, chunk, slots=3, ndim=3, zero_copy=None):
        dev.require_gpu()
        self.ndim = ndim
        if zero_copy is None:
            zero_copy = os.environ.get('KMP_STREAM_COPY', '0') == '0'
        self.zero_copy = bool(zero_copy)
        self.predictor = predictor
        self.chunk = int(chunk)
        self.slots = int(slots)
        self.dtype = dtype
        self.tile_shape = tuple(int(s) for s in tile_shape)
        cdt = torch.uint32 if dtype == torch.float32 else dtype
        if cdt not in _nd.NATURAL_CODER:
            raise TypeError(f'no lossless coder for {dtype}')
        self.coder = _nd.NATURAL_CODER[cdt]
        probe = torch.empty((self.chunk, *self.tile_shape), dtype=cdt, device='meta')
        lo_shape, map_shapes, self.dims = _nd.encoded_shapes(probe.shape, ndim)
        self.lowres_shape = lo_shape[1:]
        self.map_shapes = [s[1:] for s in map_shapes]
        self.map_dtype = _nd.CODER_DTYPE[self.coder]
        ws_bytes = _nd.workspace_bytes(probe, predictor, ndim)
        self._streams = [torch.cuda.Stream() for _ in range(self.slots)]
        self._hi = [dev.empty((self.chunk, *self.tile_shape), cdt) for _ in range(self.slots)]
        self._lo = [dev.empty((self.chunk, *self.lowres_shape), cdt) for _ in range(self.slots)]
        self._maps = [[dev.empty((self.chunk, *s), self.map_dtype) for s in self.map_shapes] for _ in range(self.slots)]
        self._ws = [dev.empty((max(1, ws_bytes),), torch.uint8) for _ in range(self.slots)]

    # -- host buffers -------------------------------------------------------------------------
    def alloc_encoded(self, n):
        """Pinned host outputs of :meth:`encode` for ``n`` tiles: ``(lowres, maps)``."""
        cdt = torch.uint32 if self.dtype == torch.float32 else self.dtype
        return pinned((n, *self.lowres_shape), cdt), [pinned((n, *s), self.map_dtype) for s in self.map_shapes]

    def _check_buffers(self, tiles, host_lowres, host_maps, n, what):
        """Every host buffer against the shapes :meth:`alloc_encoded` gives for ``n`` tiles --
        raised before any launch: on the zero-copy path the kernel reads / writes these buffers
        directly, so a short or mis-shaped one would be overrun in pinned host memory."""
        cdt = torch.uint32 if self.dtype == torch.float32 else self.dtype
        want = [((n, *self.tile_shape), cdt, tiles), ((n, *self.lowres_shape), cdt, host_lowres)]
        host_maps = list(host_maps)
        if len(host_maps) != len(self.map_shapes):
            raise AssertionError(f'{what}: expected {len(self.map_shapes)} maps, got {len(host_maps)}')
        want += [((n, *s), self.map_dtype, m) for s, m in zip(self.map_shapes, host_maps)]
        for shape, dtype, t in want:
            if not isinstance(t, torch.Tensor) or tuple(t.shape) != shape or t.dtype != dtype or not t.is_contiguous():
                got = (tuple(t.shape), t.dtype, t.is_contiguous()) if isinstance(t, torch.Tensor) else type(t)
                raise AssertionError(f'{what}: buffer {got} does not match the stream\'s '
                                     f'{shape} {dtype} (contiguous)')
        return host_maps

    def _chunks(self, n):
        for i, b in enumerate(range(0, n, self.chunk)):
            yield i % self.slots, b, min(n, b + self.chunk)

    # -- the two directions -------------------------------------------------------------------
    def encode(self, host_tiles, host_lowres, host_maps):
        """Encode pinned ``host_tiles`` into the pinned ``host_lowres`` / ``host_maps`` (from
        :meth:`alloc_encoded`).  Returns once every copy is queued; :meth:`synchronize` waits."""
        src = _as_codec_dtype(host_tiles)
        n = int(src.shape[0])
        host_maps = self._check_buffers(src, host_lowres, host_maps, n, 'TileStream.encode')
        cur = torch.cuda.current_stream()
        for s in self._streams:
            s.wait_stream(cur)
        if self.zero_copy and src.is_pinned() and host_lowres.is_pinned() and all(m.is_pinned() for m in host_maps):
            with torch.cuda.stream(self._streams[0]):
                _nd.fused_encode_into(src, self.predictor, self.coder, host_lowres, list(host_maps), self.ndim,
                                      workspace=self._ws[0] if n <= self.chunk else None)
            return host_lowres, host_maps
        for slot, b, e in self._chunks(n):
            k = e - b
            with torch.cuda.stream(self._streams[slot]):
                hi, lo = self._hi[slot][:k], self._lo[slot][:k]
                maps = [m[:k] for m in self._maps[slot]]
                hi.copy_(src[b:e], non_blocking=True)
                _nd.fused_encode_into(hi, self.predictor, self.coder, lo, maps, self.ndim, workspace=self._ws[slot])
                host_lowres[b:e].copy_(lo, non_blocking=True)
                for hm, m in zip(host_maps, maps):
                    hm[b:e].copy_(m, non_blocking=True)
        return host_lowres, host_maps

    def decode(self, host_lowres, host_maps, host_out):
        """Decode pinned encoded tiles into the pinned ``host_out`` ``[n, *tile, C...]``."""
        dst = _as_codec_dtype(host_out)
        n = int(host_lowres.shape[0])
        host_maps = self._check_buffers(dst, host_lowres, host_maps, n, 'TileStream.decode')
        cur = torch.cuda.current_stream()
        for s in self._streams:
            s.wait_stream(cur)
        if self.zero_copy and dst.is_pinned() and host_lowres.is_pinned() and all(m.is_pinned() for m in host_maps):
            with torch.cuda.stream(self._streams[0]):
                _nd.fused_decode_into(host_lowres, list(host_maps), self.dims, self.predictor, self.coder, dst,
                                      self.ndim, workspace=self._ws[0] if n <= self.chunk else None)
            return host_out
        for slot, b, e in self._chunks(n):
            k = e - b
            with torch.cuda.stream(self._streams[slot]):
                hi, lo = self._hi[slot][:k], self._lo[slot][:k]
                maps = [m[:k] for m in self._maps[slot]]
                lo.copy_(host_lowres[b:e], non_blocking=True)
                for m, hm in zip(maps, host_maps):
                    m.copy_(hm[b:e], non_blocking=True)
                _nd.fused_decode_into(lo, maps, self.dims, self.predictor, self.coder, hi, self.ndim,
                                      workspace=self._ws[slot])
                dst[b:e].copy_(hi, non_blocking=True)
        return host_out

    def synchronize(self):
        for s in self._streams:
            s.synchronize()
