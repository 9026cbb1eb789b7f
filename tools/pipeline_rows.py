#!/usr/bin/env python3
"""Store policy of the one-pass encode, measured on the pipelines that follow it (VERDICT r2
item 3): the encode's lowres / map stores either allocate in the MALL (default policy, knob = 1)
or stream past it (non-temporal, 0).  Volume: C3, 512 x 64^3 uint16 (KMP_W3_ST_ENC for p = 0,
KMP_W3P_ST_ENC for p = 1, 2); image: C2, 1024 x 256^2 uint8 (KMP_W2_ST_ENC / KMP_W2P_ST_ENC).

    python tools/pipeline_rows.py [--reps N] [--workload volume|image] [--padding P]

Rows (one JSON line each, per policy; device time from HIP events over ``reps`` iterations):
  bench      encode -> decode alternating (bench.py's timed loop)
  enc_stream encode back to back with itself (a producer that only encodes)
  compress   encode -> Rice bundle encode of its 8 outputs (the file path: container.compress)
  decompress Rice bundle decode -> decode (container.decompress)
The Rice launches are kompressor_amd.packing's own (no host synchronisation inside the loop).
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=20)
    ap.add_argument('--workload', default='volume')
    ap.add_argument('--padding', type=int, default=0)
    args = ap.parse_args()
    vol3 = args.workload == 'volume'
    knob = ('KMP_W3_ST_ENC' if args.padding == 0 else 'KMP_W3P_ST_ENC') if vol3 else \
           ('KMP_W2_ST_ENC' if args.padding == 0 else 'KMP_W2P_ST_ENC')
    import kompressor_amd as kom
    from kompressor_amd import _nd, packing as kpk
    torch.cuda.set_device(0)
    # a structured volume / image set (the Rice stage's cost depends on the residuals): smooth field + noise
    gen = torch.Generator(device='cuda').manual_seed(0)
    if vol3:
        zz, yy, xx = torch.meshgrid(*[torch.arange(512, device='cuda', dtype=torch.float32)] * 3, indexing='ij')
        f = torch.sin(xx / 41.0) * torch.cos(yy / 29.0) + torch.sin(zz / 53.0 + xx / 97.0)
        f = 4000 + 9000 * (f - f.min()) / (f.max() - f.min())
        del zz, yy, xx
        vol = (f + 4 * torch.randn(f.shape, device='cuda', generator=gen)).round().clamp(0, 65535).to(torch.int32)
        hi = vol.to(torch.uint16).view(8, 64, 8, 64, 8, 64).permute(0, 2, 4, 1, 3, 5).reshape(512, 64, 64, 64, 1).contiguous()
        del f, vol
    else:
        yy, xx = torch.meshgrid(*[torch.arange(256, device='cuda', dtype=torch.float32)] * 2, indexing='ij')
        ph = torch.rand((1024, 1, 1), device='cuda', generator=gen) * 6.28
        f = 128 + 80 * torch.sin(xx / 23.0 + ph) * torch.cos(yy / 31.0 - ph)
        hi = (f + 2 * torch.randn(f.shape, device='cuda', generator=gen)).round().clamp(0, 255).to(torch.uint8)
        hi = hi.reshape(1024, 256, 256, 1).contiguous()
        del f
    ndim = 3 if vol3 else 2
    pred = kom.MeanPredictor(args.padding, ndim)
    coder = _nd.NATURAL_CODER[hi.dtype]
    lo, maps, dims = _nd._alloc_encoded(hi, coder, ndim)
    rec = torch.empty_like(hi)
    ws = torch.empty(max(1, _nd.workspace_bytes(hi, pred, ndim)), dtype=torch.uint8, device='cuda')
    enc = lambda: _nd.fused_encode_into(hi, pred, coder, lo, maps, ndim, workspace=ws)  # noqa: E731
    dec = lambda: _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, ndim, workspace=ws)  # noqa: E731
    enc()
    blob = kpk.pack_encoded(lo, (maps, dims))
    hb = blob[:4096].cpu().numpy().tobytes()
    raw = hi.numel() * hi.element_size()

    def timed(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(50_000_000)  # keep the GPU busy while the host enqueues (no host-bound intervals)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / args.reps / 1e3

    pipes = {
        'bench': lambda: (enc(), dec()),
        'enc_stream': enc,
        'compress': lambda: (enc(), kpk._rice_encode_launch((lo, *maps), dims)),
        'decompress': lambda: (kpk._rice_decode_launch(blob, hb), dec()),
    }
    for rep in range(2):
        for name, fn in pipes.items():
            for pol in ('1', '0'):
                os.environ[knob] = pol
                t = timed(fn)
                print(json.dumps({'row': f'pipeline:{args.workload}_p{args.padding}:{name}', knob: int(pol), 'us_per_iter': round(t * 1e6, 1),
                                  'raw_GBps': round(raw / t / 1e9, 1), 'rep': rep}), flush=True)
    os.environ.pop(knob, None)
    enc()
    dec()
    torch.cuda.synchronize()
    assert torch.equal(rec, hi)


if __name__ == '__main__':
    main()
