"""The trained-network callback path at C3 (512 x 64^3 uint16), for a per-kernel rocprofv3 split
(VERDICT r2 item 5): encode + decode with an opaque predictions_fn returning uint16 maps (the mean
predictor's primitive) and returning float32 maps (a network's output: the stand-in writes them itself).
    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/callback_split.py [reps] [u16|f32|both]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import kompressor_amd as kom  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
which = sys.argv[2] if len(sys.argv) > 2 else 'both'
V = kom.volume
vol = torch.from_numpy(np.random.default_rng(0).integers(0, 65536, size=(512, 64, 64, 64, 1)).astype(np.uint16)).cuda()
pred = kom.MeanPredictor(0, 3)
pred32 = kom.MeanPredictor(0, 3, maps_dtype=torch.float32)
fns = {'u16': lambda lowres: pred(lowres), 'f32': lambda lowres: pred32(lowres)}
for name, fn in fns.items():
    if which not in (name, 'both'):
        continue
    lo, enc = V.encode(fn, V.encode_values_uint16, vol)
    for _ in range(reps):
        lo, enc = V.encode(fn, V.encode_values_uint16, vol)
        rec = V.decode(fn, V.decode_values_uint16, lo, enc)
    torch.cuda.synchronize()
    assert torch.equal(rec, vol)
    print('ok', name)
