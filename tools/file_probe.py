"""Where the time of the file path goes (container.compress / decompress of a C3-sized volume from
and to numpy), and the host-side primitives it is built from, on this box.

    python tools/file_probe.py [--dir DIR]

One JSON line per measurement (milliseconds, GB/s of the bytes each step moves)."""
import argparse
import json
import os
import sys
import tempfile
import time
import zlib
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def wall(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts))


def emit(what, t, nbytes, **kw):
    print(json.dumps({'what': what, 'ms': round(t * 1e3, 3), 'GBps': round(nbytes / t / 1e9, 2), **kw}), flush=True)


def structured_volume(noise=4.0):
    zz, yy, xx = torch.meshgrid(*[torch.arange(512, device='cuda', dtype=torch.float32)] * 3, indexing='ij')
    f = torch.sin(xx / 41.0) * torch.cos(yy / 29.0) + torch.sin(zz / 53.0 + xx / 97.0)
    f = 4000 + 9000 * (f - f.min()) / (f.max() - f.min())
    g = torch.Generator(device='cuda').manual_seed(0)
    v = (f + noise * torch.randn(f.shape, device='cuda', generator=g)).round().clamp(0, 65535).to(torch.int32)
    v = v.to(torch.uint16).view(8, 64, 8, 64, 8, 64).permute(0, 2, 4, 1, 3, 5).reshape(512, 64, 64, 64, 1)
    return v.contiguous()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--dir', default=None)
    args = ap.parse_args()
    import kompressor_amd as kom
    torch.cuda.set_device(0)
    d = tempfile.mkdtemp(dir=args.dir)
    vol_d = structured_volume()
    vol = vol_d.cpu().numpy()
    raw = vol.nbytes
    pred = kom.MeanPredictor(0, 3)
    path = os.path.join(d, 'c3.kmp')

    info = kom.container.compress(path, vol, pred, levels=1)
    back = kom.container.decompress(path)
    assert np.array_equal(back, vol)
    fsize = os.path.getsize(path)
    print(json.dumps({'what': 'file', 'raw_bytes': raw, 'file_bytes': fsize, 'ratio': round(raw / fsize, 3),
                      'dir': d}), flush=True)
    tc = wall(lambda: kom.container.compress(path, vol, pred, levels=1))
    emit('compress numpy -> file (levels=1)', tc, raw, split=getattr(kom.container, 'last_timing', None))
    td = wall(lambda: kom.container.decompress(path))
    emit('decompress file -> numpy', td, raw, split=getattr(kom.container, 'last_timing', None))

    # the primitives
    blob = np.fromfile(path, dtype=np.uint8)
    nb = blob.size
    emit('zlib.crc32 of the file bytes', wall(lambda: zlib.crc32(memoryview(blob))), nb)
    emit('np.fromfile (page cache)', wall(lambda: np.fromfile(path, dtype=np.uint8)), nb)
    out = os.path.join(d, 'w.bin')

    def write_np():
        with open(out, 'wb') as f:
            f.write(memoryview(blob))
    emit('file write from pageable numpy', wall(write_np), nb)
    pin = torch.empty(max(nb, raw), dtype=torch.uint8, pin_memory=True)
    pin_np = pin.numpy()
    pin_np[:nb] = blob

    def write_pin():
        with open(out, 'wb') as f:
            f.write(memoryview(pin_np[:nb]))
    emit('file write from pinned', wall(write_pin), nb)

    def read_pin():
        with open(path, 'rb') as f:
            f.readinto(memoryview(pin_np[:nb]))
    emit('file readinto pinned', wall(read_pin), nb)

    pool = ThreadPoolExecutor(8)

    def pwrite_par(k):
        fd = os.open(out, os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
        try:
            os.ftruncate(fd, nb)
            step = (nb + k - 1) // k
            list(pool.map(lambda i: os.pwrite(fd, memoryview(pin_np[i * step:min(nb, (i + 1) * step)]), i * step),
                          range(k)))
        finally:
            os.close(fd)
    for k in (2, 4, 8):
        emit(f'file pwrite from pinned, {k} threads', wall(lambda: pwrite_par(k)), nb)

    import mmap

    def mmap_write_par(k):
        # the file sized first, then filled through a shared mapping by k threads (page faults of
        # one file's mapping run in parallel; write() serialises on the inode)
        fd = os.open(out, os.O_RDWR | os.O_CREAT | os.O_TRUNC)
        try:
            os.ftruncate(fd, nb)
            mm = mmap.mmap(fd, nb, mmap.MAP_SHARED, mmap.PROT_WRITE | mmap.PROT_READ)
            dst = np.frombuffer(mm, dtype=np.uint8)
            step = (nb + k - 1) // k
            list(pool.map(lambda i: np.copyto(dst[i * step:min(nb, (i + 1) * step)], pin_np[i * step:min(nb, (i + 1) * step)]),
                          range(k)))
            del dst
            mm.close()
        finally:
            os.close(fd)
    for k in (1, 4, 8):
        emit(f'file write via mmap from pinned, {k} threads', wall(lambda: mmap_write_par(k)), nb)

    def pread_par(k):
        fd = os.open(path, os.O_RDONLY)
        try:
            step = (nb + k - 1) // k
            list(pool.map(lambda i: os.preadv(fd, [memoryview(pin_np[i * step:min(nb, (i + 1) * step)])], i * step),
                          range(k)))
        finally:
            os.close(fd)
    for k in (2, 4, 8):
        emit(f'file preadv into pinned, {k} threads', wall(lambda: pread_par(k)), nb)

    flat = vol.reshape(-1).view(np.uint8)
    emit('memcpy numpy -> pinned, 1 thread', wall(lambda: np.copyto(pin_np[:raw], flat)), raw)

    def par_copy(k):
        step = (raw + k - 1) // k
        list(pool.map(lambda i: np.copyto(pin_np[i * step:min(raw, (i + 1) * step)], flat[i * step:min(raw, (i + 1) * step)]),
                      range(k)))
    for k in (4, 8):
        emit(f'memcpy numpy -> pinned, {k} threads', wall(lambda: par_copy(k)), raw)
    dev = torch.empty(raw, dtype=torch.uint8, device='cuda')
    emit('H2D pageable (torch.from_numpy().cuda())', wall(lambda: torch.from_numpy(vol).cuda()), raw)
    emit('H2D pinned', wall(lambda: dev.copy_(pin[:raw], non_blocking=True)), raw)
    emit('D2H pinned', wall(lambda: pin[:raw].copy_(dev, non_blocking=True)), raw)
    emit('D2H pageable (.cpu().numpy())', wall(lambda: vol_d.cpu().numpy()), raw)
    try:
        cudart = torch.cuda.cudart()
        host = np.empty_like(vol)
        t = time.perf_counter()
        rc = cudart.cudaHostRegister(host.ctypes.data, host.nbytes, 0)
        treg = time.perf_counter() - t
        t = time.perf_counter()
        cudart.cudaHostUnregister(host.ctypes.data)
        tun = time.perf_counter() - t
        emit('hipHostRegister of a 256 MiB numpy array', treg, raw, rc=int(rc), unregister_ms=round(tun * 1e3, 3))
    except Exception as e:  # noqa: BLE001
        print(json.dumps({'what': 'hipHostRegister', 'error': repr(e)}), flush=True)


if __name__ == '__main__':
    main()
