"""Device plumbing: numpy / torch <-> contiguous device tensors, dtype codes, the current stream.

PyTorch-ROCm is used only for device memory, host<->device copies and the stream handle; all
arithmetic on the hot path runs in ``libkompressor_hip.so``.
"""

import os
import threading
import weakref
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

from . import _lib

TORCH_TO_CODE = {torch.uint8: _lib.U8, torch.uint16: _lib.U16, torch.int32: _lib.I32,
                 torch.float32: _lib.F32, torch.uint32: _lib.U32}
CODE_TO_TORCH = {v: k for k, v in TORCH_TO_CODE.items()}
NP_TO_TORCH = {np.dtype(np.uint8): torch.uint8, np.dtype(np.uint16): torch.uint16,
               np.dtype(np.int32): torch.int32, np.dtype(np.float32): torch.float32,
               np.dtype(np.uint32): torch.uint32}

_device_checked = False


def require_gpu():
    """Fail loudly unless a gfx950 device is visible (there is no CPU fallback)."""
    global _device_checked
    if _device_checked:
        return
    if not torch.cuda.is_available():
        raise RuntimeError('kompressor_amd computes on an MI355X (gfx950) GPU through libkompressor_hip.so; '
                           'no GPU is visible to this process')
    if not _lib.lib.kmp_device_ok():
        arch = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
        raise RuntimeError(f'kompressor_amd: libkompressor_hip.so (gfx950 only) cannot run on the visible GPU '
                           f'({arch}): {_lib.lib.kmp_last_error().decode(errors="replace")}')
    _device_checked = True


# The current stream's raw handle without building a torch.cuda.Stream object (a few microseconds
# per call through torch.cuda.current_stream(), paid once or more per API call)
# (0.19 vs 2.67 us, tools/stream_check.py; profiles/round2/r2s14_host_overhead.log)
_RAW_STREAM = getattr(torch._C, '_cuda_getCurrentRawStream', None)
_GET_DEVICE = getattr(torch._C, '_cuda_getDevice', None)


def stream():
    if _RAW_STREAM is not None and _GET_DEVICE is not None:
        return _RAW_STREAM(_GET_DEVICE())
    return torch.cuda.current_stream().cuda_stream


def is_torch(x):
    return isinstance(x, torch.Tensor)


def to_device(x):
    """Return ``(tensor, kind)``: a contiguous device tensor and 'torch' / 'numpy' for the result."""
    require_gpu()
    if isinstance(x, torch.Tensor):
        t = x if x.is_cuda else x.to('cuda')
        return (t if t.is_contiguous() else t.contiguous()), 'torch'
    a = np.ascontiguousarray(np.asarray(x))
    if a.dtype not in NP_TO_TORCH:
        raise TypeError(f'kompressor_amd: unsupported dtype {a.dtype}')
    return torch.from_numpy(a).to('cuda'), 'numpy'


def from_device(t, kind):
    if kind == 'numpy':
        return to_host(t)
    return t


# ---------------------------------------------------------------------------------------------
# Host copies.  A pageable ``.cpu()`` of a large tensor runs at ~8 GB/s on the MI355X box (the
# driver stages it); a copy into pinned memory runs at the link rate (~57 GB/s) and a parallel
# memcpy from there into the numpy result at ~100 GB/s (profiles/round4/file_probe_r4s2.log).
# Large transfers stream through a small ring of pinned chunks (``PinnedRing``): the link moves
# chunk i+1 while the host copies chunk i, and the pinned memory a thread keeps is bounded
# (``RING_CHUNK * RING_SLOTS`` per ring, whatever the transfer size).
# ---------------------------------------------------------------------------------------------

_TLS = threading.local()
_POOL = None
_POOL_LOCK = threading.Lock()
_COPY_THREADS = 8
_SMALL = 4 << 20  # below this a plain .cpu() costs less than the hand-off
RING_CHUNK = 16 << 20
RING_SLOTS = 4
_STAGING_CAP = 64 << 20  # pinned_staging buffers above this are not kept
# page-locked result bytes alive at once (to_host): past it results go through the ring into pageable
# memory, so a caller holding many results (a data loader) cannot pin an unbounded share of the host
PINNED_LIVE_MAX = int(os.environ.get('KMP_PINNED_RESULTS_MAX', 2 << 30))
_pinned_live = [0]
_pinned_lock = threading.Lock()
PINNED_OUT_MAX = 512 << 20  # to_host results up to this size are pinned arrays (kept in torch's host cache once freed, up to the peak in use; release_pinned() returns them)


def pinned_staging(nbytes, slot='stage'):
    """A pinned host byte buffer of at least ``nbytes``: reused per thread and ``slot`` up to
    ``_STAGING_CAP`` bytes; a larger request gets a buffer of its own, freed with its last reference
    (so no thread keeps more than the cap pinned for the life of the process)."""
    nbytes = int(nbytes)
    if nbytes > _STAGING_CAP:
        return torch.empty((nbytes,), dtype=torch.uint8, pin_memory=True)
    buf = getattr(_TLS, slot, None)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty((max(nbytes, 1 << 20),), dtype=torch.uint8, pin_memory=True)
        setattr(_TLS, slot, buf)
    return buf


def release_pinned():
    """Free this thread's cached pinned buffers (staging slots and chunk rings) and return the
    pinned blocks of freed ``to_host`` results from torch's caching host allocator to the system."""
    for k in list(vars(_TLS)):
        delattr(_TLS, k)
    empty = getattr(torch._C, '_host_emptyCache', None)  # torch's caching host allocator (private API)
    if empty is not None:
        empty()


class PinnedRing:
    """``RING_SLOTS`` pinned chunks of ``RING_CHUNK`` bytes with one event each, reused per thread
    (``ring()``).  ``slot(i)`` is chunk i's buffer; ``done(i)`` records chunk i's transfer on
    ``stream``; ``wait(i)`` blocks until it landed."""

    def __init__(self):
        self.chunk = RING_CHUNK
        self.bufs = [torch.empty((RING_CHUNK,), dtype=torch.uint8, pin_memory=True) for _ in range(RING_SLOTS)]
        self.events = [torch.cuda.Event() for _ in range(RING_SLOTS)]

    def slot(self, i):
        return self.bufs[i % RING_SLOTS]

    def done(self, i, stream):
        self.events[i % RING_SLOTS].record(stream)

    def wait(self, i):
        self.events[i % RING_SLOTS].synchronize()


def ring(name='d2h', device=None):
    """This thread's ring for ``name`` on ``device`` (a CUDA event belongs to the device it is first
    recorded on, so each device has its own ring)."""
    idx = torch.cuda.current_device() if device is None else (device.index if isinstance(device, torch.device)
                                                              else int(device))
    if idx is None:
        idx = torch.cuda.current_device()
    key = f'ring_{name}_{idx}'
    r = getattr(_TLS, key, None)
    if r is None or r.chunk != RING_CHUNK:
        with torch.cuda.device(idx):
            r = PinnedRing()
        setattr(_TLS, key, r)
    return r


def d2h_stream(src, sink, stream=None):
    """Stream the device byte tensor ``src`` to the host in ``RING_CHUNK`` pieces:
    ``sink(offset, pinned uint8 numpy view)`` is called for each piece in order, while the next
    pieces are in flight on ``stream`` (default: the current stream of ``src``'s device)."""
    n = src.numel()
    s = stream or torch.cuda.current_stream(src.device)
    r = ring('d2h', src.device)
    nch = -(-n // RING_CHUNK)

    def issue(i):
        lo = i * RING_CHUNK
        hi = min(n, lo + RING_CHUNK)
        with torch.cuda.stream(s):
            r.slot(i)[:hi - lo].copy_(src[lo:hi], non_blocking=True)
        r.done(i, s)

    for i in range(min(RING_SLOTS - 1, nch)):
        issue(i)
    for i in range(nch):
        if i + RING_SLOTS - 1 < nch:
            issue(i + RING_SLOTS - 1)  # its slot's previous chunk (i - 1) was consumed last step
        r.wait(i)
        lo = i * RING_CHUNK
        sink(lo, r.slot(i)[:min(n, lo + RING_CHUNK) - lo].numpy())


def h2d_stream(dst, source, stream=None):
    """Fill the device byte tensor ``dst`` from the host in ``RING_CHUNK`` pieces:
    ``source(offset, pinned uint8 numpy view)`` fills each piece and returns the bytes it wrote;
    the piece's upload is queued on ``stream`` while the next piece is filled.  Returns the bytes
    filled (short when ``source`` came up short)."""
    n = dst.numel()
    s = stream or torch.cuda.current_stream(dst.device)
    r = ring('h2d', dst.device)
    for i in range(-(-n // RING_CHUNK)):
        r.wait(i)  # the slot's previous upload (this call's chunk i - RING_SLOTS, or an earlier call's) landed
        lo = i * RING_CHUNK
        hi = min(n, lo + RING_CHUNK)
        buf = r.slot(i)[:hi - lo]
        got = source(lo, buf.numpy())
        if got:
            with torch.cuda.stream(s):
                dst[lo:lo + got].copy_(buf[:got], non_blocking=True)
            r.done(i, s)
        if got != hi - lo:
            return lo + got
    return n


def pread_into(fd, view, offset):
    """``os.preadv`` of ``view.size`` bytes at ``offset`` into the numpy uint8 ``view``, split over
    the copy threads for large views (page-cache reads of one file run in parallel); returns the
    bytes read."""
    n = view.size
    k = copy_pool()._max_workers if n >= (8 << 20) else 1
    step = -(-n // k)

    def part(i):
        lo, hi = i * step, min(n, (i + 1) * step)
        got = 0
        while lo + got < hi:
            r = os.preadv(fd, [memoryview(view[lo + got:hi])], offset + lo + got)
            if r <= 0:
                break
            got += r
        return got, hi - lo

    parts = list(copy_pool().map(part, range(k))) if k > 1 else [part(0)]
    total = 0
    for got, want in parts:
        total += got
        if got != want:
            break
    return total


def copy_pool():
    global _POOL
    if _POOL is None:
        with _POOL_LOCK:
            if _POOL is None:
                n = max(1, min(_COPY_THREADS, len(os.sched_getaffinity(0))))
                _POOL = ThreadPoolExecutor(n, thread_name_prefix='kmp-copy')
    return _POOL


def parallel_copy(dst, src):
    """``dst[:] = src`` for two equal-size flat uint8 numpy arrays, split over the copy threads
    (numpy releases the GIL for the copy)."""
    n = dst.size
    pool = copy_pool()
    k = pool._max_workers if n >= (8 << 20) else 1
    if k == 1:
        np.copyto(dst, src)
        return
    step = -(-n // k)
    list(pool.map(lambda i: np.copyto(dst[i * step:(i + 1) * step], src[i * step:(i + 1) * step]), range(k)))


def _pin_result(nbytes):
    with _pinned_lock:
        if _pinned_live[0] + nbytes > PINNED_LIVE_MAX:
            return False
        _pinned_live[0] += nbytes
        return True


def _unpin_result(nbytes):
    with _pinned_lock:
        _pinned_live[0] -= nbytes


def pinned_result_bytes():
    """Page-locked bytes held by live ``to_host`` results."""
    return _pinned_live[0]


def to_host(t):
    """A device tensor as a new numpy array, ordered after the work queued on the current stream of
    ``t``'s device.  Up to ``PINNED_OUT_MAX`` bytes the array lives in pinned host memory from
    torch's caching host allocator (one D2H at the link rate, ~57 GB/s, straight into the result;
    the block returns to torch's cache when the array is freed) while the live pinned results stay
    within ``PINNED_LIVE_MAX``; larger tensors, and results past that cap, stream through the
    pinned chunk ring, each chunk copied out (in parallel) into ordinary pageable memory while the
    next ones cross the link."""
    nbytes = t.numel() * t.element_size()
    if nbytes < _SMALL:
        return t.cpu().numpy()
    t = t.contiguous()
    if nbytes <= PINNED_OUT_MAX and _pin_result(nbytes):
        host = torch.empty(tuple(t.shape), dtype=t.dtype, pin_memory=True)
        with torch.cuda.device(t.device):
            s = torch.cuda.current_stream(t.device)
            with torch.cuda.stream(s):
                host.copy_(t, non_blocking=True)
            s.synchronize()
        arr = host.numpy()
        # the array (and any view of it, whose base it is) holds the pinned storage; the Python
        # tensor object may go away first, so the budget follows the array
        weakref.finalize(arr, _unpin_result, nbytes)
        return arr
    out = np.empty(tuple(t.shape), dtype=torch.empty(0, dtype=t.dtype).numpy().dtype)
    dst = out.reshape(-1).view(np.uint8)
    with torch.cuda.device(t.device):
        d2h_stream(t.view(-1).view(torch.uint8), lambda lo, piece: parallel_copy(dst[lo:lo + piece.size], piece))
    return out


def dtype_code(t):
    try:
        return TORCH_TO_CODE[t.dtype]
    except KeyError:
        raise TypeError(f'kompressor_amd: unsupported dtype {t.dtype} '
                        f'(supported: uint8, uint16, int32, uint32, float32)') from None


_CUDA = torch.device('cuda')


def empty(shape, dtype):
    return torch.empty(tuple(int(s) for s in shape), dtype=dtype, device=_CUDA)


def prod(shape):
    p = 1
    for s in shape:
        p *= int(s)
    return p
