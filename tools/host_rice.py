"""Host-side cost of pack_encoded / unpack_encoded on a C3 encode result: wall time per call vs
the device time of its kernels, and a cProfile of 50 calls (where the host time goes).
    python tools/host_rice.py"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom  # noqa: E402
from kompressor_amd import packing as kpk  # noqa: E402

torch.cuda.set_device(0)
gen = torch.Generator(device='cuda').manual_seed(0)
vol = (30000 + 4 * torch.randn((512, 64, 64, 64, 1), device='cuda', generator=gen)).round().to(torch.int32).to(torch.uint16)
lo, enc = kom.volume.encode(kom.MeanPredictor(0, 3), kom.volume.encode_values_uint16, vol)
blob = kpk.pack_encoded(lo, enc)
for name, fn in (('pack_encoded', lambda: kpk.pack_encoded(lo, enc)), ('unpack_encoded', lambda: kpk.unpack_encoded(blob))):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    print(f'{name}: {(time.perf_counter() - t0) / 50 * 1e3:.3f} ms per call', flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats('tottime').print_stats(14)
