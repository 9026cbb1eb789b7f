"""Interleaved A/B timing of fast-kernel launch geometries (env knobs read per call)."""
import os, sys, time, json
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom
from kompressor_amd import _nd

def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else 'volume'
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    ndim = 3 if wl == 'volume' else 2
    shape, dt = ((512, 64, 64, 64, 1), np.uint16) if ndim == 3 else ((1024, 256, 256, 1), np.uint8)
    rng = np.random.default_rng(0)
    host = rng.integers(0, np.iinfo(dt).max + 1, size=shape, dtype=np.int64).astype(dt)
    hi = torch.from_numpy(host).cuda()
    pred = kom.MeanPredictor(p, ndim)
    coder = _nd.NATURAL_CODER[hi.dtype]
    lo, maps, dims = _nd._alloc_encoded(hi, coder, ndim)
    rec = torch.empty_like(hi)
    ws = torch.empty(1, dtype=torch.uint8, device='cuda')
    if len(sys.argv) > 3:
        configs = json.loads(sys.argv[3])
    else:
        configs = [dict(KMP_WG_TARGET=str(w), KMP_MIN_SLAB=str(s), KMP_NT=str(nt)) for w in (1024, 2048, 4096, 8192) for s in (2, 4) for nt in (0, 1)]
    res = {i: ([], []) for i in range(len(configs))}
    for rnd in range(8):
        for i, cfg in enumerate(configs):
            os.environ.update(cfg)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            _nd.fused_encode_into(hi, pred, coder, lo, maps, ndim, workspace=ws)
            _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, ndim, workspace=ws)
            ev[0].record()
            for _ in range(5):
                _nd.fused_encode_into(hi, pred, coder, lo, maps, ndim, workspace=ws)
            ev[1].record()
            for _ in range(5):
                _nd.fused_decode_into(lo, maps, dims, pred, coder, rec, ndim, workspace=ws)
            ev[2].record()
            torch.cuda.synchronize()
            res[i][0].append(ev[0].elapsed_time(ev[1]) / 5)
            res[i][1].append(ev[1].elapsed_time(ev[2]) / 5)
    assert torch.equal(rec, hi)
    nbytes = 2 * hi.numel() * hi.element_size()
    for i, cfg in enumerate(configs):
        e, d = np.median(res[i][0]), np.median(res[i][1])
        print(json.dumps(cfg), f'enc {e*1e3:.1f} us ({nbytes/e/1e6:.0f} GB/s)  dec {d*1e3:.1f} us ({nbytes/d/1e6:.0f} GB/s)')

if __name__ == '__main__':
    main()
