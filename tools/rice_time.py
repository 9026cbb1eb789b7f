"""Rice bundle encode / decode launches only (for rocprofv3 --kernel-trace --stats A/B of kernel
variants; the decode's output is checked once at the end).   python tools/rice_time.py [sigma] [reps]"""
import os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kompressor_amd import packing as kpk
sigma = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
gen = torch.Generator(device='cuda').manual_seed(0)
arrays = [(sigma * torch.randn((512, 32, 32, 32, 1), device='cuda', generator=gen)).round().to(torch.int32)
          .to(torch.int16).view(torch.uint16) for _ in range(8)]
for _ in range(reps):
    kpk._rice_encode_launch(arrays, (1, 1, 1))
blob = kpk.pack_encoded(arrays[0], (tuple(arrays[1:]), (1, 1, 1)))
hb = blob[:4096].cpu().numpy().tobytes()
for _ in range(reps):
    outs, _, bad = kpk._rice_decode_launch(blob, hb)
torch.cuda.synchronize()
ok = int(bad.item()) == 0 and all(torch.equal(a, b) for a, b in zip(outs, arrays))
print('ok' if ok else 'MISMATCH')
