// probe_bw.hip -- HBM ceilings for the codec's access shapes on this box (standalone).
//   hipcc -O3 --offload-arch=gfx950 tools/probe_bw.hip -o tools/probe_bw && ./tools/probe_bw
// 1. copy: 256 MiB -> 256 MiB, 16 B per lane, grid-stride
// 2. split8: read 256 MiB at 16 B/lane, write 8 output streams of 32 MiB at 8 B/lane per lane
//    (the fused encode's store shape), one 2x2x2 block class per stream
// 3. merge8: the inverse (decode's shape)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__global__ void copy16(const u32x4* __restrict__ a, u32x4* __restrict__ b, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), b + i);
}

// element i of the input (16 B = 8 u16) -> 8 outputs of 2 B?  Keep it byte-shaped: lane reads 16 B,
// writes 8 B to stream (i & 7) ... simplest equal-volume shape: each lane reads 16 B and writes two
// 8-B halves to streams s and s+4 at the same index, s = (i / chunk) & 3.
__global__ void split8(const u32x4* __restrict__ a, u32x2* __restrict__ out, int64_t n, int64_t per) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    u32x4 v = __builtin_nontemporal_load(a + i);
    int64_t row = i / 256, col = i % 256;   // 256 lanes = one "plane"
    int s = row & 3;
    int64_t o = (row >> 2) * 256 + col;
    u32x2 lo = {v.x, v.y}, hi = {v.z, v.w};
    __builtin_nontemporal_store(lo, out + (int64_t)s * per + o);
    __builtin_nontemporal_store(hi, out + (int64_t)(s + 4) * per + o);
  }
}

__global__ void merge8(const u32x2* __restrict__ in, u32x4* __restrict__ b, int64_t n, int64_t per) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t row = i / 256, col = i % 256;
    int s = row & 3;
    int64_t o = (row >> 2) * 256 + col;
    u32x2 lo = __builtin_nontemporal_load(in + (int64_t)s * per + o);
    u32x2 hi = __builtin_nontemporal_load(in + (int64_t)(s + 4) * per + o);
    u32x4 v = {lo.x, lo.y, hi.x, hi.y};
    __builtin_nontemporal_store(v, b + i);
  }
}

int main() {
  const size_t bytes = 256ull << 20;
  const int64_t n16 = bytes / 16;
  void *a, *b;
  hipMalloc(&a, bytes);
  hipMalloc(&b, bytes);
  hipMemset(a, 1, bytes);
  hipMemset(b, 2, bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto fn) {
    for (int w = 0; w < 3; ++w) fn();
    hipEventRecord(e0);
    const int reps = 20;
    for (int r = 0; r < reps; ++r) fn();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double us = ms * 1e3 / reps;
    printf("%-28s %8.1f us  %7.0f GB/s (read+write %zu MiB)\n", name, us, 2.0 * bytes / (us * 1e3), 2 * (bytes >> 20));
  };
  for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
    char nm[64];
    snprintf(nm, sizeof nm, "copy16 grid=%d", blocks);
    run(nm, [&] { copy16<<<blocks, 256>>>((const u32x4*)a, (u32x4*)b, n16); });
  }
  const int64_t per = n16 / 4;  // u32x2 elements per output stream
  for (int blocks : {2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "split8 grid=%d", blocks);
    run(nm, [&] { split8<<<blocks, 256>>>((const u32x4*)a, (u32x2*)b, n16, per); });
    snprintf(nm, sizeof nm, "merge8 grid=%d", blocks);
    run(nm, [&] { merge8<<<blocks, 256>>>((const u32x2*)b, (u32x4*)a, n16, per); });
  }
  return 0;
}
