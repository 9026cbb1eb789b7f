import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
import kompressor_amd as kom
from kompressor_amd import _nd
x = torch.from_numpy(np.random.default_rng(0).integers(0, 65536, size=(512, 64, 64, 64, 1)).astype(np.uint16)).cuda()
rng = np.random.default_rng(1)
w = (1.0 / 64 + rng.standard_normal((64, 19)) * (0.3 / 64)).astype(np.float32)
pred = kom.LinearPredictor(w, np.zeros(19, np.float32), 1, 3, arith='f32')
coder = _nd.NATURAL_CODER[x.dtype]
lo, maps, dims = _nd._alloc_encoded(x, coder, 3)
rec = torch.empty_like(x)
ws = torch.empty(max(1, _nd.workspace_bytes(x, pred, 3)), dtype=torch.uint8, device='cuda')
for _ in range(3):
    _nd.fused_encode_into(x, pred, coder, lo, maps, 3, workspace=ws)
    _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, 3, workspace=ws)
torch.cuda.synchronize()
assert torch.equal(rec, x)
print('ok')
