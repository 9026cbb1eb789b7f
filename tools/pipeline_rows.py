#!/usr/bin/env python3
"""Store policy of the one-pass encode, measured on the pipelines that follow it (VERDICT r2
item 3): the encode's lowres / map stores either allocate in the MALL (default policy,
KMP_W3_ST_ENC=1) or stream past it (non-temporal, 0).  C3: 512 x 64^3 uint16, MeanPredictor(0).

    python tools/pipeline_rows.py [--reps N]

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
    args = ap.parse_args()
    import kompressor_amd as kom
    from kompressor_amd import _nd, packing as kpk
    torch.cuda.set_device(0)
    # a structured volume (the Rice stage's cost depends on the residuals): smooth field + N(0, 4^2)
    zz, yy, xx = torch.meshgrid(*[torch.arange(512, device='cuda', dtype=torch.float32)] * 3, indexing='ij')
    f = torch.sin(xx / 41.0) * torch.cos(yy / 29.0) + torch.sin(zz / 53.0 + xx / 97.0)
    f = 4000 + 9000 * (f - f.min()) / (f.max() - f.min())
    del zz, yy, xx
    gen = torch.Generator(device='cuda').manual_seed(0)
    vol = (f + 4 * torch.randn(f.shape, device='cuda', generator=gen)).round().clamp(0, 65535).to(torch.int32)
    hi = vol.to(torch.uint16).view(8, 64, 8, 64, 8, 64).permute(0, 2, 4, 1, 3, 5).reshape(512, 64, 64, 64, 1).contiguous()
    del f, vol
    pred = kom.MeanPredictor(0, 3)
    coder = _nd.NATURAL_CODER[hi.dtype]
    lo, maps, dims = _nd._alloc_encoded(hi, coder, 3)
    rec = torch.empty_like(hi)
    ws = torch.empty(max(1, _nd.workspace_bytes(hi, pred, 3)), dtype=torch.uint8, device='cuda')
    enc = lambda: _nd.fused_encode_into(hi, pred, coder, lo, maps, 3, workspace=ws)  # noqa: E731
    dec = lambda: _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, 3, workspace=ws)  # noqa: E731
    enc()
    blob = kpk.pack_encoded(lo, (maps, dims))
    hb = blob[:4096].cpu().numpy().tobytes()
    raw = hi.numel() * 2

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
                os.environ['KMP_W3_ST_ENC'] = pol
                t = timed(fn)
                print(json.dumps({'row': f'pipeline:{name}', 'KMP_W3_ST_ENC': int(pol), 'us_per_iter': round(t * 1e6, 1),
                                  'raw_GBps': round(raw / t / 1e9, 1), 'rep': rep}), flush=True)
    os.environ.pop('KMP_W3_ST_ENC', None)
    enc()
    dec()
    torch.cuda.synchronize()
    assert torch.equal(rec, hi)


if __name__ == '__main__':
    main()
