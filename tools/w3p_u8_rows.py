import os, sys, json
import numpy as np, torch
sys.path.insert(0, '/root/repo' if os.path.exists('/root/repo') else '.')
import kompressor_amd as kom
from kompressor_amd import _nd
hi = torch.from_numpy(np.random.default_rng(0).integers(0, 256, size=(512, 64, 64, 64, 1), dtype=np.int64).astype(np.uint8)).cuda()
coder = _nd.NATURAL_CODER[hi.dtype]
def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps): fn()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3
for p in (1, 2):
    pred = kom.MeanPredictor(p, 3)
    lo, maps, dims = _nd._alloc_encoded(hi, coder, 3)
    rec = torch.empty_like(hi)
    ws = torch.empty(max(1, _nd.workspace_bytes(hi, pred, 3)), dtype=torch.uint8, device='cuda')
    for pl in (0, 1, 2):
        with kom._lib.option('KMP_W3P_PL', pl):
            enc = lambda: _nd.fused_encode_into(hi, pred, coder, lo, maps, 3, workspace=ws)
            dec = lambda: _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, 3, workspace=ws)
            enc(); dec(); torch.cuda.synchronize(); assert torch.equal(rec, hi)
            print(json.dumps({'p': p, 'pl_opt': pl, 'kernel': kom._lib.lib.kmp_last_launch().decode(),
                              'enc_us': round(t(enc), 1), 'dec_us': round(t(dec), 1)}), flush=True)
