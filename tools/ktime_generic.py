"""Launch one generic-path configuration N times per direction (for rocprofv3 --kernel-trace --stats).
    python tools/ktime_generic.py NAME [reps]   (NAME: a key of CFG)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom  # noqa: E402
from kompressor_amd import _nd  # noqa: E402

name = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
w64 = (1.0 / 64 + np.random.default_rng(1).standard_normal((64, 19)) * 0.005).astype(np.float32)
w216 = (1.0 / 216 + np.random.default_rng(1).standard_normal((216, 19)) * 0.001).astype(np.float32)
w16 = (1.0 / 16 + np.random.default_rng(1).standard_normal((16, 5)) * 0.02).astype(np.float32)
CFG = {'odd': ((512, 63, 63, 63, 1), np.uint16, kom.MeanPredictor(0, 3), 3),
       'odd1': ((512, 63, 63, 63, 1), np.uint16, kom.MeanPredictor(1, 3), 3),
       'c2': ((256, 64, 64, 64, 2), np.uint16, kom.MeanPredictor(0, 3), 3),
       'img_c3': ((1024, 256, 256, 3), np.uint8, kom.MeanPredictor(0, 2), 2),
       'img_odd': ((1024, 255, 255, 1), np.uint8, kom.MeanPredictor(0, 2), 2),
       'img_lin1': ((1024, 256, 256, 1), np.uint8, kom.LinearPredictor(w16, np.zeros(5, np.float32), 1, 2), 2),
       'big': ((1, 512, 512, 1024, 1), np.uint16, kom.MeanPredictor(0, 3), 3),
       'lin1_odd': ((256, 63, 63, 63, 1), np.uint16, kom.LinearPredictor(w64, np.zeros(19, np.float32), 1, 3), 3),
       'lin2': ((128, 64, 64, 64, 1), np.uint16, kom.LinearPredictor(w216, np.zeros(19, np.float32), 2, 3), 3),
       'lin1_odd_f32': ((256, 63, 63, 63, 1), np.uint16,
                        kom.LinearPredictor(w64, np.zeros(19, np.float32), 1, 3, arith='f32'), 3)}
shape, dt, pred, ndim = CFG[name]
hi = torch.from_numpy(np.random.default_rng(0).integers(0, np.iinfo(dt).max + 1, size=shape,
                                                         dtype=np.int64).astype(dt)).cuda()
coder = _nd.NATURAL_CODER[hi.dtype]
lo, maps, dims = _nd._alloc_encoded(hi, coder, ndim)
rec = torch.empty_like(hi)
ws = torch.empty(max(1, _nd.workspace_bytes(hi, pred, ndim)), dtype=torch.uint8, device='cuda')
for _ in range(reps):
    _nd.fused_encode_into(hi, pred, coder, lo, maps, ndim, workspace=ws)
    _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, ndim, workspace=ws)
torch.cuda.synchronize()
assert torch.equal(rec, hi)
print('ok', name)
