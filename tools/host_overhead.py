#!/usr/bin/env python3
"""Host-side cost of one API call: cProfile over N back-to-back calls of the callback-path encode
and decode (128 C3 tiles, opaque predictions_fn), the fused encode, and graph-replayed
CodecPlans (kompressor_amd.graphs) of the fused and the callback path, with one synchronisation at the end, so the Python / ctypes /
allocator time per call is visible next to the kernels' time.

    python tools/host_overhead.py [N]
"""
import cProfile
import pstats
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __file__.rsplit('/tools/', 1)[0])
import kompressor_amd as kom  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 200
V = kom.volume
vol = torch.from_numpy(np.random.default_rng(0).integers(0, 65536, (128, 64, 64, 64, 1), dtype=np.uint16)).cuda()
pred = kom.MeanPredictor(0, 3)
cb = lambda lowres: pred(lowres)  # noqa: E731
lo, enc = V.encode(cb, V.encode_values_uint16, vol)
torch.cuda.synchronize()
plan = kom.graphs.CodecPlan(pred, tuple(vol.shape), vol.dtype)
plan.highres.copy_(vol)
cplan = kom.graphs.CodecPlan(cb, tuple(vol.shape), vol.dtype, padding=0)  # the callback path, captured
cplan.highres.copy_(vol)
for name, fn in (('encode', lambda: V.encode(cb, V.encode_values_uint16, vol)),
                 ('decode', lambda: V.decode(cb, V.decode_values_uint16, lo, enc)),
                 ('fused_encode', lambda: V.encode(pred, V.encode_values_uint16, vol)),
                 ('chunks_encode', lambda: V.encode_chunks(pred, V.encode_values_uint16, vol, chunk=32)),
                 ('graph_encode', lambda: plan.encode()),
                 ('graph_decode', lambda: plan.decode()),
                 ('graph_callback_encode', lambda: cplan.encode()),
                 ('graph_callback_decode', lambda: cplan.decode())):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(N):
        fn()
    host = time.perf_counter() - t
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    print(f'{name}: host {1e6 * host / N:.1f} us/call, wall {1e6 * wall / N:.1f} us/call', flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(N):
        fn()
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats('tottime').print_stats(14)
