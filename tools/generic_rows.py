"""Per-direction times of configurations outside the fused kernels' fast paths (the generic and
callback kernels), to find pathologically slow ones.  Event-timed, back to back, median of 3 x reps.
    python tools/generic_rows.py [reps]"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom  # noqa: E402
from kompressor_amd import _nd  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5


def w_b(n, k, seed=1):
    rng = np.random.default_rng(seed)
    return (1.0 / n + rng.standard_normal((n, k)) * (0.3 / n)).astype(np.float32), np.zeros(k, np.float32)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) / reps * 1e3)
    return float(np.median(out))


def row(name, shape, dtype, pred, ndim):
    rng = np.random.default_rng(0)
    hi = torch.from_numpy(rng.integers(0, np.iinfo(dtype).max + 1, size=shape, dtype=np.int64).astype(dtype)).cuda()
    coder = _nd.NATURAL_CODER[hi.dtype]
    lo, maps, dims = _nd._alloc_encoded(hi, coder, ndim)
    rec = torch.empty_like(hi)
    ws = torch.empty(max(1, _nd.workspace_bytes(hi, pred, ndim)), dtype=torch.uint8, device='cuda')
    enc = lambda: _nd.fused_encode_into(hi, pred, coder, lo, maps, ndim, workspace=ws)  # noqa: E731
    dec = lambda: _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, ndim, workspace=ws)  # noqa: E731
    enc()
    ke = kom._lib.lib.kmp_last_launch().decode()
    dec()
    kd = kom._lib.lib.kmp_last_launch().decode()
    torch.cuda.synchronize()
    assert torch.equal(rec, hi), name
    te, td = timed(enc), timed(dec)
    raw = hi.numel() * hi.element_size()
    print(json.dumps({'row': name, 'shape': list(shape), 'dtype': np.dtype(dtype).name, 'pred': repr(pred),
                      'kernels': [ke, kd], 'us': [round(te, 1), round(td, 1)],
                      'GBps': round(2 * raw / (te + td) / 1e3, 1)}), flush=True)


V3, I2 = (512, 64, 64, 64, 1), (1024, 256, 256, 1)
row('vol_mean_p0_c2', (256, 64, 64, 64, 2), np.uint16, kom.MeanPredictor(0, 3), 3)
row('vol_mean_p1_u8', V3, np.uint8, kom.MeanPredictor(1, 3), 3)
row('vol_mean_p2_u8', V3, np.uint8, kom.MeanPredictor(2, 3), 3)
row('vol_mean_p3_u16', (128, 64, 64, 64, 1), np.uint16, kom.MeanPredictor(3, 3), 3)
row('vol_mean_p0_odd', (512, 63, 63, 63, 1), np.uint16, kom.MeanPredictor(0, 3), 3)
row('vol_lin_p2_u16', (128, 64, 64, 64, 1), np.uint16, kom.LinearPredictor(*w_b(216, 19), 2, 3), 3)
row('vol_lin_p0_u8', V3, np.uint8, kom.LinearPredictor(*w_b(8, 19), 0, 3), 3)
row('img_mean_p1_u16', (512, 256, 256, 1), np.uint16, kom.MeanPredictor(1, 2), 2)
row('img_lin_p0_u8', I2, np.uint8, kom.LinearPredictor(*w_b(4, 5), 0, 2), 2)
row('img_lin_p1_u8', I2, np.uint8, kom.LinearPredictor(*w_b(16, 5), 1, 2), 2)
row('img_lin_p1_u16', (512, 256, 256, 1), np.uint16, kom.LinearPredictor(*w_b(16, 5), 1, 2), 2)
row('img_mean_p0_c3', (1024, 256, 256, 3), np.uint8, kom.MeanPredictor(0, 2), 2)
row('vol_mean_p0_i32', (128, 64, 64, 64, 1), np.int32, kom.MeanPredictor(0, 3), 3)

if len(sys.argv) > 2 and sys.argv[2] == 'more':
    row('img_mean_p0_odd', (1024, 255, 255, 1), np.uint8, kom.MeanPredictor(0, 2), 2)
    row('img_mean_p1_odd', (1024, 255, 255, 1), np.uint8, kom.MeanPredictor(1, 2), 2)
    row('vol_mean_p1_odd', (512, 63, 63, 63, 1), np.uint16, kom.MeanPredictor(1, 3), 3)
    row('vol_mean_p0_w100', (64, 128, 128, 100, 1), np.uint16, kom.MeanPredictor(0, 3), 3)
    row('vol_mean_p0_big', (1, 512, 512, 1024, 1), np.uint16, kom.MeanPredictor(0, 3), 3)
    row('vol_lin_p1_odd', (256, 63, 63, 63, 1), np.uint16, kom.LinearPredictor(*w_b(64, 19), 1, 3), 3)
    # the callback path (an opaque predictions_fn) on an odd shape
    V = kom.volume
    hi = torch.from_numpy(np.random.default_rng(0).integers(0, 65536, size=(256, 63, 63, 63, 1), dtype=np.int64)
                          .astype(np.uint16)).cuda()
    inner = kom.MeanPredictor(0, 3)
    cb = lambda x: inner(x)  # noqa: E731
    lo, enc = V.encode(cb, V.encode_values_uint16, hi)
    te = timed(lambda: V.encode(cb, V.encode_values_uint16, hi))
    td = timed(lambda: V.decode(cb, V.decode_values_uint16, lo, enc))
    raw = hi.numel() * 2
    print(json.dumps({'row': 'vol_callback_p0_odd', 'us': [round(te, 1), round(td, 1)],
                      'GBps': round(2 * raw / (te + td) / 1e3, 1)}), flush=True)
    # categorical with class counts the vector kernel does not take
    for L in (10, 255):
        torch.manual_seed(0)
        logits = torch.rand((1 << 18, L), device='cuda')
        gt = torch.randint(0, L, (1 << 18,), device='cuda', dtype=torch.uint8)
        enc_c = V.encode_categorical(logits, gt)
        te = timed(lambda: V.encode_categorical(logits, gt))
        td = timed(lambda: V.decode_categorical(logits, enc_c))
        assert torch.equal(V.decode_categorical(logits, enc_c), gt)
        nb = logits.numel() * 4
        print(json.dumps({'row': f'categorical_L{L}', 'us': [round(te, 1), round(td, 1)],
                          'GBps_read': [round(nb / te / 1e3, 1), round(nb / td / 1e3, 1)]}), flush=True)
