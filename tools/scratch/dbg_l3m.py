import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import kompressor_amd as kom
sys.path.insert(0, 'tests')
from test_gpu_linear import _weights, _data
for shape in [(8, 64, 64, 64, 1), (2, 12, 33, 32, 1), (1, 10, 40, 32, 1), (1, 9, 14, 128, 1)]:
    hi = _data(shape, np.uint16, 7)
    w, b = _weights(3, 1, 8, np.uint16)
    pred = kom.LinearPredictor(w, b, 1, 3)
    V = kom.volume
    os.environ['KMP_L3P_MFMA'] = '0'
    lo0, (m0, d0) = V.encode(pred, V.encode_values_uint16, hi, padding=1)
    os.environ['KMP_L3P_MFMA'] = '1'
    lo1, (m1, d1) = V.encode(pred, V.encode_values_uint16, hi, padding=1)
    print(shape, 'enc', kom._lib.lib.kmp_last_launch().decode(), all(np.array_equal(a, c) for a, c in zip(m0, m1)))
    r1 = V.decode(pred, V.decode_values_uint16, lo1, (m1, d1), padding=1)
    print('  dec', kom._lib.lib.kmp_last_launch().decode(), np.array_equal(r1, hi))
    bad = np.argwhere(r1 != hi)
    if bad.size:
        print('  nbad', len(bad), 'first', bad[:6].tolist())
        par = (bad[:, 1] % 2) * 4 + (bad[:, 2] % 2) * 2 + (bad[:, 3] % 2)
        print('  parity hist', np.bincount(par, minlength=8).tolist(), 'z', np.unique(bad[:, 1] // 2)[:20].tolist(), 'y', np.unique(bad[:, 2] // 2)[:40].tolist(), 'x', np.unique(bad[:,3]//2).tolist()[:40])
