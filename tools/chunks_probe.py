"""Per-launch view of the fused chunked drivers at C3 (encode_chunks / decode_chunks, chunk 32):
run under rocprofv3 --kernel-trace to see each region launch.
    python tools/chunks_probe.py [reps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
V = kom.volume
vol = torch.from_numpy(np.random.default_rng(0).integers(0, 65536, (512, 64, 64, 64, 1)).astype(np.uint16)).cuda()
pred = kom.MeanPredictor(0, 3)
lo, (maps, dims) = V.encode(pred, V.encode_values_uint16, vol)
for _ in range(reps):
    V.encode_chunks(pred, V.encode_values_uint16, vol, chunk=32)
    V.decode_chunks(pred, V.decode_values_uint16, lo, (maps, dims), chunk=32)
torch.cuda.synchronize()
from kompressor_amd import _nd  # noqa: E402
L = [(s + 1 + 1) // 2 for s in (64, 64, 64)]
print('regions', _nd.fused_chunk_regions(_nd._chunks_for(L, 32, 0, None, 3), [32, 32, 32], 3))
