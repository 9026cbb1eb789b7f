"""Practical HBM ceiling for a read-N/write-N stream on this box: torch's device copy of the
same byte counts as one fused encode (256 MiB in, 256 MiB out), back to back and alternating."""
import torch, numpy as np
n = 256 * 1024 * 1024
a = torch.empty(n, dtype=torch.uint8, device='cuda').random_(0, 255)
b = torch.empty_like(a); c = torch.empty_like(a); d = torch.empty_like(a)
for _ in range(3):
    b.copy_(a); d.copy_(c)
torch.cuda.synchronize()
def t(fn, reps=20):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3
s1 = t(lambda: b.copy_(a))
s2 = t(lambda: (b.copy_(a), a.copy_(b)), 10) / 2
print(f'copy 256MiB->256MiB back-to-back: {s1*1e6:.1f} us, {2*n/s1/1e9:.0f} GB/s')
print(f'copy ping-pong (a->b, b->a):       {s2*1e6:.1f} us, {2*n/s2/1e9:.0f} GB/s')
