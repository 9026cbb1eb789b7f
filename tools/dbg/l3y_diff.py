"""Per-map mismatch positions of the fused LinearPredictor p = 0 encode vs the oracle (debug aid)."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import kompressor_amd as kom
import oracle
from oracle import predictors as OP

shape = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else '2,64,64,64,1').split(','))
rng = np.random.default_rng(3)
hi = rng.integers(0, 65536, size=shape, dtype=np.int64).astype(np.uint16)
n, k = 8, 19
r2 = np.random.default_rng(4)
w = (1.0 / n + r2.standard_normal((n, k)) * (0.3 / n)).astype(np.float32)
b = (r2.standard_normal(k) * float(os.environ.get('BIAS', '50'))).astype(np.float32)
pred = kom.LinearPredictor(w, b, 0, 3)
want_lo, (want_maps, _) = oracle.volume.encode(OP.linear_predictions_fn(0, w, b, 3), oracle.volume.encode_values_uint16, hi)
lo, (maps, dims) = kom.volume.encode(pred, kom.volume.encode_values_uint16, hi)
print('kernel', kom._lib.lib.kmp_last_launch().decode(), 'lowres equal', np.array_equal(lo, want_lo))
names = ['LR', 'UD', 'FB', 'C', 'Z', 'Y', 'X']
for i, (a, c) in enumerate(zip(maps, want_maps)):
    bad = np.argwhere(a != c)
    print(names[i], a.shape, 'mismatches', len(bad), bad[:6].tolist(),
          [(int(a[tuple(p)]), int(c[tuple(p)])) for p in bad[:3]])
rec = kom.volume.decode(pred, kom.volume.decode_values_uint16, lo, (maps, dims))
print('roundtrip', np.array_equal(rec, hi))
