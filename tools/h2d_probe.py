"""Host link ceilings on this box and the TileStream end-to-end rate vs chunk size / streams.
    python tools/h2d_probe.py"""
import os, sys, time, json
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

n = 256 << 20
h1 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
d1 = torch.empty(n, dtype=torch.uint8, device='cuda')
d2 = torch.empty(n, dtype=torch.uint8, device='cuda')
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def t(fn, reps=5):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def both():
    with torch.cuda.stream(s1):
        d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2):
        h2.copy_(d2, non_blocking=True)

th = t(lambda: d1.copy_(h1, non_blocking=True))
td = t(lambda: h2.copy_(d2, non_blocking=True))
tb = t(both)
print(json.dumps({'h2d_GBps': round(n / th / 1e9, 1), 'd2h_GBps': round(n / td / 1e9, 1),
                  'concurrent_each_GBps': round(n / tb / 1e9, 1)}), flush=True)

import kompressor_amd as kom
host = np.random.default_rng(0).integers(0, 65536, size=(512, 64, 64, 64, 1), dtype=np.int64).astype(np.uint16)
src = kom.stream.pinned(host.shape, torch.uint16)
src.copy_(torch.from_numpy(host))
out = kom.stream.pinned(host.shape, torch.uint16)
pred = kom.MeanPredictor(0, 3)
for chunk in (16, 32, 64, 128):
    for slots in (2, 3, 4):
        ts = kom.stream.TileStream(pred, host.shape[1:], torch.uint16, chunk, slots, 3)
        lo, maps = ts.alloc_encoded(512)
        def rnd():
            ts.encode(src, lo, maps); ts.synchronize()
            ts.decode(lo, maps, out); ts.synchronize()
        tt = t(rnd, 3)
        print(json.dumps({'chunk': chunk, 'slots': slots, 'e2e_GBps': round(src.numel() * 2 / tt / 1e9, 2)}), flush=True)
        del ts
assert torch.equal(out, src)

# zero-copy: the fused kernels read the pinned input and write the pinned outputs directly
from kompressor_amd import _nd
coder = _nd.NATURAL_CODER[torch.uint16]
lo_h, maps_h = kom.stream.TileStream(pred, host.shape[1:], torch.uint16, 32, 1, 3).alloc_encoded(512)
out2 = kom.stream.pinned(host.shape, torch.uint16)
dims = (1, 1, 1)
def zc():
    _nd.fused_encode_into(src, pred, coder, lo_h, maps_h, 3)
    torch.cuda.synchronize()
    _nd.fused_decode_into(lo_h, maps_h, dims, pred, coder, out2, 3)
    torch.cuda.synchronize()
tt = t(zc, 3)
assert torch.equal(out2, src)
print(json.dumps({'zero_copy_e2e_GBps': round(src.numel() * 2 / tt / 1e9, 2)}), flush=True)
