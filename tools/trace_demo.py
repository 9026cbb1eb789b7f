"""KMP_TRACE=1 rocprofv3 --marker-trace --kernel-trace --stats -- python3 tools/trace_demo.py
One fused and one callback round trip of 64 C3 tiles: the roctx ranges (kmp.encode, kmp.decode,
kmp.predictions_fn, kmp.encode_chunks) bracket the kernels each stage launched."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom  # noqa: E402

V = kom.volume
x = torch.randint(0, 65536, (64, 64, 64, 64, 1), dtype=torch.int32, device='cuda').to(torch.uint16)
pred = kom.MeanPredictor(0, 3)
for _ in range(3):
    lo, enc = V.encode(pred, V.encode_values_uint16, x)
    assert torch.equal(V.decode(pred, V.decode_values_uint16, lo, enc), x)
    cb = lambda w: pred(w)  # noqa: E731  an opaque predictions_fn
    lo, enc = V.encode(cb, V.encode_values_uint16, x)
    assert torch.equal(V.decode(cb, V.decode_values_uint16, lo, enc), x)
    lo2, enc2 = V.encode_chunks(pred, V.encode_values_uint16, x, chunk=32)
    assert torch.equal(lo2, lo)
torch.cuda.synchronize()
print('trace demo ok, tracing', kom._trace.ENABLED)
