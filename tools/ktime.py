"""Launch the fused volume/image codec N times per direction (for rocprofv3 --kernel-trace --stats).
    python tools/ktime.py [volume|image] [padding] [reps] [mean|linear|linearmx]
    python tools/ktime.py rice SIGMA [reps]   (the Rice bundle kernels on a C3 encode result)"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom
from kompressor_amd import _nd

wl = sys.argv[1] if len(sys.argv) > 1 else 'volume'
p = int(sys.argv[2]) if len(sys.argv) > 2 else 0
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
if wl == 'categorical':  # rank coder, 1M elements x 256 logits (tools/bench_rows.py's row)
    torch.manual_seed(0)
    logits = torch.rand((1 << 20, 256), device='cuda')
    gt = torch.randint(0, 256, (1 << 20,), device='cuda', dtype=torch.uint8)
    small = torch.randint(0, 4, (1 << 20,), device='cuda', dtype=torch.uint8)
    for _ in range(reps):
        enc = kom.volume.encode_categorical(logits, gt)
        dec = kom.volume.decode_categorical(logits, enc)
        if os.environ.get('KMP_CAT_SMALL', '1') != '0':  # 0: the uniform-rank decode only (counters)
            kom.volume.decode_categorical(logits, small)
    torch.cuda.synchronize()
    assert torch.equal(dec, gt)
    print('ok', os.environ.get('KMP_TAG', ''))
    sys.exit(0)
if wl == 'rice':  # Rice bundle encode + decode of 8 C3-sized u16 maps of N(0, sigma^2) residuals (sigma = argv[2])
    from kompressor_amd import packing as kpk
    gen = torch.Generator(device='cuda').manual_seed(0)
    arrays = [(max(p, 1) * torch.randn((512, 32, 32, 32, 1), device='cuda', generator=gen)).round().to(torch.int32)
              .to(torch.int16).view(torch.uint16) for _ in range(8)]
    blob = kpk.pack_encoded(arrays[0], (tuple(arrays[1:]), (1, 1, 1)))
    hb = blob[:4096].cpu().numpy().tobytes()
    for _ in range(reps):
        kpk._rice_encode_launch(arrays, (1, 1, 1))
        outs, _, bad = kpk._rice_decode_launch(blob, hb)
    torch.cuda.synchronize()
    if os.environ.get('KMP_NOCHECK', '0') == '0':
        assert int(bad.item()) == 0 and all(torch.equal(a, b) for a, b in zip(outs, arrays))
    print('ok', os.environ.get('KMP_TAG', ''), 'bundle bytes', blob.numel())
    sys.exit(0)
ndim = 3 if wl == 'volume' else 2
shape, dt = ((512, 64, 64, 64, 1), np.uint16) if ndim == 3 else ((1024, 256, 256, 1), np.uint8)
if os.environ.get('KMP_KT_U8') == '1' and ndim == 3:  # uint8 volumes at C3 geometry
    dt = np.uint8
host = np.random.default_rng(0).integers(0, np.iinfo(dt).max + 1, size=shape, dtype=np.int64).astype(dt)
hi = torch.from_numpy(host).cuda()
if len(sys.argv) > 4 and sys.argv[4] in ('linear', 'linearmx'):
    n, k = (2 * p + 2) ** ndim, 19 if ndim == 3 else 5
    w = (1.0 / n + np.random.default_rng(1).standard_normal((n, k)) * (0.3 / n)).astype(np.float32)
    pred = kom.LinearPredictor(w, np.zeros(k, np.float32), p, ndim,
                               arith='bf16x2' if sys.argv[4] == 'linearmx' else 'f32')
else:
    pred = kom.MeanPredictor(p, ndim)
if len(sys.argv) > 4 and sys.argv[4] == 'callback':  # the callback path: opaque predictions_fn
    ns = kom.volume if ndim == 3 else kom.image
    enc_fn, dec_fn = ((ns.encode_values_uint16, ns.decode_values_uint16) if ndim == 3
                      else (ns.encode_values_uint8, ns.decode_values_uint8))
    cb = lambda lowres: pred(lowres)  # noqa: E731
    lo, enc = ns.encode(cb, enc_fn, hi, padding=p)
    for _ in range(reps):
        lo, enc = ns.encode(cb, enc_fn, hi, padding=p)
        rec = ns.decode(cb, dec_fn, lo, enc, padding=p)
    torch.cuda.synchronize()
    assert torch.equal(rec, hi)
    print('ok', os.environ.get('KMP_TAG', ''))
    sys.exit(0)
coder = _nd.NATURAL_CODER[hi.dtype]
lo, maps, dims = _nd._alloc_encoded(hi, coder, ndim)
rec = torch.empty_like(hi)
for _ in range(reps):
    _nd.fused_encode_into(hi, pred, coder, lo, maps, ndim)
    _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, ndim)
torch.cuda.synchronize()
if os.environ.get('KMP_NOCHECK', '0') == '0':  # 1: experiment builds that skip work (timing only)
    assert torch.equal(rec, hi)
print('ok', os.environ.get('KMP_TAG', ''))
