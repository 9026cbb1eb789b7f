// probe_unaligned.hip -- cost of 16-byte accesses at 2-byte alignment (rows of 33 uint16, the
// untrimmed prediction maps and windows of the callback path) vs aligned rows (standalone).
//   hipcc -O3 --offload-arch=gfx950 tools/probe_unaligned.hip -o tools/probe_unaligned && ./tools/probe_unaligned
// Copies R rows of 32 uint16 (64 B): 4 lanes per row, 16 B per lane.  Source / destination row
// pitch is 32 (aligned) or 33 elements (2-byte aligned rows); "shift" reads the unaligned rows as
// two aligned 16-byte loads + a funnel shift.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int SP, int DP>
__global__ void __launch_bounds__(256) rows_copy(const uint16_t* __restrict__ a, uint16_t* __restrict__ b, int32_t R) {
  const int32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= 4 * R) return;
  const int32_t r = t >> 2, j = t & 3;
  const u32x4u v = *(const u32x4u*)(a + (int64_t)r * SP + 8 * j);
  *(u32x4u*)(b + (int64_t)r * DP + 8 * j) = v;
}

// odd rows start 2 bytes past a 4-byte boundary: read the covering aligned 16-byte chunks
__global__ void __launch_bounds__(256) rows_copy_shift(const uint16_t* __restrict__ a, uint16_t* __restrict__ b,
                                                        int32_t R) {
  const int32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= 4 * R) return;
  const int32_t r = t >> 2, j = t & 3;
  const int64_t e = (int64_t)r * 33 + 8 * j;  // first element
  const int64_t e0 = e & ~7ll;                // aligned chunk start
  const int sh = (int)(e - e0);               // 0..7 elements
  const u32x4 lo = *(const u32x4*)(a + e0), hi = *(const u32x4*)(a + e0 + 8);
  uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w}, o[4];
  const int dw = sh >> 1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t x0 = 0, x1 = 0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      if (q == dw) { x0 = w[k + q]; x1 = w[k + q + 1 < 8 ? k + q + 1 : 7]; }
    }
    o[k] = (sh & 1) ? __builtin_amdgcn_alignbit(x1, x0, 16) : x0;
  }
  *(u32x4*)(b + (int64_t)r * 32 + 8 * j) = (u32x4){o[0], o[1], o[2], o[3]};
}

template <typename K>
static float timeit(K k, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) k();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / reps;
}

int main() {
  const int32_t R = 4 * 1024 * 1024;  // 4 Mi rows = 256 MiB of payload each way
  uint16_t *a, *b;
  hipMalloc(&a, (size_t)R * 34 * 2);
  hipMalloc(&b, (size_t)R * 34 * 2);
  hipMemset(a, 1, (size_t)R * 34 * 2);
  const unsigned grid = (unsigned)((4 * (int64_t)R + 255) / 256);
  const double bytes = 2.0 * R * 64;
  auto rep = [&](const char* name, float us) { printf("%-28s %8.1f us  %7.1f GB/s\n", name, us, bytes / us / 1e3); };
  rep("aligned -> aligned", timeit([&] { rows_copy<32, 32><<<grid, 256>>>(a, b, R); }, 20));
  rep("pitch33 read -> aligned", timeit([&] { rows_copy<33, 32><<<grid, 256>>>(a, b, R); }, 20));
  rep("aligned -> pitch33 write", timeit([&] { rows_copy<32, 33><<<grid, 256>>>(a, b, R); }, 20));
  rep("pitch33 -> pitch33", timeit([&] { rows_copy<33, 33><<<grid, 256>>>(a, b, R); }, 20));
  rep("pitch33 shift-read -> aligned", timeit([&] { rows_copy_shift<<<grid, 256>>>(a, b, R); }, 20));
  rep("aligned -> aligned", timeit([&] { rows_copy<32, 32><<<grid, 256>>>(a, b, R); }, 20));
  hipFree(a);
  hipFree(b);
  return 0;
}
