"""Device CRC-32 of a C3-bundle-sized buffer, N times (for rocprofv3 --kernel-trace --stats).
    python tools/crc_time.py [MiB] [reps]"""
import os
import sys
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kompressor_amd import container  # noqa: E402

mib = int(sys.argv[1]) if len(sys.argv) > 1 else 107
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
host = np.random.default_rng(0).integers(0, 256, size=mib << 20, dtype=np.uint8)
dev = torch.from_numpy(host).cuda()
for _ in range(reps):
    crc = container._device_crc(dev, dev.numel())
torch.cuda.synchronize()
assert int(crc.cpu().view(torch.uint32).item()) == zlib.crc32(host.tobytes())
print('ok', mib, 'MiB')
