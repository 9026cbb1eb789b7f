"""The raw current-stream handle kompressor_amd._device.stream() passes to the C-ABI equals
torch.cuda.current_stream().cuda_stream (default stream and inside a torch.cuda.stream context),
and what each costs per call; plus torch.empty's cost.   python tools/stream_check.py"""
import time, torch, sys
sys.path.insert(0, '.')
from kompressor_amd import _device as dev
torch.cuda.init()
s = torch.cuda.Stream()
a = dev.stream(); b = torch.cuda.current_stream().cuda_stream
assert a == b, (a, b)
with torch.cuda.stream(s):
    assert dev.stream() == s.cuda_stream == torch.cuda.current_stream().cuda_stream
n = 20000
t = time.perf_counter()
for _ in range(n): torch.cuda.current_stream().cuda_stream
t1 = time.perf_counter()
for _ in range(n): dev.stream()
t2 = time.perf_counter()
for _ in range(n): torch.empty((128, 32, 32, 32, 1), dtype=torch.uint16, device='cuda')
t3 = time.perf_counter()
for _ in range(n): dev.empty((128, 32, 32, 32, 1), torch.uint16)
t4 = time.perf_counter()
print(f'current_stream {1e6*(t1-t)/n:.2f} us, raw {1e6*(t2-t1)/n:.2f} us, empty(str) {1e6*(t3-t2)/n:.2f} us, dev.empty {1e6*(t4-t3)/n:.2f} us')
