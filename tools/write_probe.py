"""Page-cache write probe for the container's file write (112 MB, the C3 levels=1 file): plain
write, write into a preallocated (posix_fallocate) file, ftruncate first, and the cost of the
preallocation itself.  python tools/write_probe.py [MB]"""
import os
import sys
import tempfile
import time

import numpy as np

MB = int(sys.argv[1]) if len(sys.argv) > 1 else 112
buf = np.random.default_rng(0).integers(0, 256, size=MB << 20, dtype=np.uint8)
d = tempfile.mkdtemp()
print('dir', d, os.statvfs(d).f_bsize, flush=True)


def run(name, fn, reps=5):
    ts = []
    for i in range(reps):
        p = os.path.join(d, f'{name}{i}.bin')
        t = time.perf_counter()
        fn(p)
        ts.append(time.perf_counter() - t)
        os.remove(p)
    ts.sort()
    print(f'{name:28s} median {ts[len(ts) // 2] * 1e3:7.2f} ms  min {ts[0] * 1e3:7.2f} ms', flush=True)


def plain(p):
    with open(p, 'wb') as f:
        f.write(memoryview(buf))


def chunked(p):
    with open(p, 'wb') as f:
        for i in range(0, buf.size, 16 << 20):
            f.write(memoryview(buf[i:i + (16 << 20)]))


def falloc_write(p):
    fd = os.open(p, os.O_WRONLY | os.O_CREAT, 0o644)
    os.posix_fallocate(fd, 0, buf.size)
    os.write(fd, memoryview(buf))
    os.close(fd)


def falloc_only(p):
    fd = os.open(p, os.O_WRONLY | os.O_CREAT, 0o644)
    os.posix_fallocate(fd, 0, buf.size)
    os.close(fd)


def trunc_write(p):
    with open(p, 'wb') as f:
        f.truncate(buf.size)
        f.write(memoryview(buf))


def prealloc_then_write(p):  # preallocation outside the timed region (as if overlapped with device work)
    pass


for name, fn in (('plain write', plain), ('16 MiB chunks', chunked), ('fallocate + write', falloc_write),
                 ('fallocate only', falloc_only), ('ftruncate + write', trunc_write)):
    run(name, fn)
ts = []
for i in range(5):
    p = os.path.join(d, f'pre{i}.bin')
    fd = os.open(p, os.O_WRONLY | os.O_CREAT, 0o644)
    os.posix_fallocate(fd, 0, buf.size)
    t = time.perf_counter()
    os.pwrite(fd, memoryview(buf), 0)
    ts.append(time.perf_counter() - t)
    os.close(fd)
    os.remove(p)
ts.sort()
print(f'{"write into fallocated file":28s} median {ts[2] * 1e3:7.2f} ms  min {ts[0] * 1e3:7.2f} ms', flush=True)

# the container's path: a device buffer to the file through the pinned chunk ring (d2h_stream), vs a
# whole pinned copy then one write
if len(sys.argv) > 2 and sys.argv[2] == 'gpu':
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from kompressor_amd import _device as dev
    g = torch.from_numpy(buf).cuda()
    torch.cuda.synchronize()

    def ring(p):
        with open(p, 'wb') as f:
            os.posix_fallocate(f.fileno(), 0, buf.size)
            dev.d2h_stream(g, lambda lo, piece: f.write(memoryview(piece)))

    def whole(p):
        h = torch.empty(buf.size, dtype=torch.uint8, pin_memory=True)
        h.copy_(g, non_blocking=True)
        torch.cuda.current_stream().synchronize()
        with open(p, 'wb') as f:
            os.posix_fallocate(f.fileno(), 0, buf.size)
            f.write(memoryview(h.numpy()))

    for chunk in (16 << 20, 4 << 20, 64 << 20):
        dev.RING_CHUNK = chunk
        run(f'ring {chunk >> 20} MiB + write', ring)
    dev.RING_CHUNK = 16 << 20
    run('whole pinned + write', whole)
