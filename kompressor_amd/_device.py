"""Device plumbing: numpy / torch <-> contiguous device tensors, dtype codes, the current stream.

PyTorch-ROCm is used only for device memory, host<->device copies and the stream handle; all
arithmetic on the hot path runs in ``libkompressor_hip.so``.
"""

import os
import threading
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
# ---------------------------------------------------------------------------------------------

_TLS = threading.local()
_POOL = None
_POOL_LOCK = threading.Lock()
_COPY_THREADS = 8
_SMALL = 4 << 20  # below this a plain .cpu() costs less than the hand-off


def pinned_staging(nbytes, slot='stage'):
    """A reused pinned host byte buffer of at least ``nbytes`` (one per thread and ``slot``)."""
    buf = getattr(_TLS, slot, None)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty((max(int(nbytes), 1 << 20),), dtype=torch.uint8, pin_memory=True)
        setattr(_TLS, slot, buf)
    return buf


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


def to_host(t):
    """A device tensor as a new numpy array: pinned D2H at the link rate, then a parallel copy out of
    the staging buffer (the result is ordinary pageable memory the caller owns)."""
    nbytes = t.numel() * t.element_size()
    if nbytes < _SMALL:
        return t.cpu().numpy()
    t = t.contiguous()
    stage = pinned_staging(nbytes)
    stage[:nbytes].copy_(t.view(-1).view(torch.uint8), non_blocking=True)
    torch.cuda.current_stream().synchronize()
    out = np.empty(tuple(t.shape), dtype=torch.empty(0, dtype=t.dtype).numpy().dtype)
    parallel_copy(out.reshape(-1).view(np.uint8), stage[:nbytes].numpy())
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
