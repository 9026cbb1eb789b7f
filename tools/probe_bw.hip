// probe_bw.hip -- HBM ceilings for the codec's access shapes on this box (standalone).
//   hipcc -O3 --offload-arch=gfx950 tools/probe_bw.hip -o tools/probe_bw && ./tools/probe_bw
// 1. copy: 256 MiB -> 256 MiB, 16 B per lane, grid-stride
// 2. split8: read 256 MiB at 16 B/lane, write 8 output streams of 32 MiB at 8 B/lane per lane
//    (the fused encode's store shape), one 2x2x2 block class per stream
// 3. merge8: the inverse (decode's shape)
// ./tools/probe_bw c2: only the C2-sized probes -- 64 MiB -> 64 MiB copies alternating X -> M and
//    M -> R like bench.py's encode / decode pairs (the 192 MiB working set fits the 256 MiB MALL)
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

// split16: each lane reads 32 B (two 16-B loads) and writes two 16-B halves to streams s and
// s+4: the store shape of a codec lane owning 8 outputs (16 B of each map) instead of 4
__global__ void split16(const u32x4* __restrict__ a, u32x4* __restrict__ out, int64_t n2, int64_t per) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / 256, col = i % 256;
    const u32x4 v0 = __builtin_nontemporal_load(a + (row * 512 + col));
    const u32x4 v1 = __builtin_nontemporal_load(a + (row * 512 + 256 + col));
    const int s = row & 3;
    const int64_t o = (row >> 2) * 256 + col;
    __builtin_nontemporal_store(v0, out + (int64_t)s * per + o);
    __builtin_nontemporal_store(v1, out + (int64_t)(s + 4) * per + o);
  }
}

// merge16: the inverse of split16 (a decode lane reading 16 B of each map row)
__global__ void merge16(const u32x4* __restrict__ in, u32x4* __restrict__ b, int64_t n2, int64_t per) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / 256, col = i % 256;
    const int s = row & 3;
    const int64_t o = (row >> 2) * 256 + col;
    const u32x4 v0 = __builtin_nontemporal_load(in + (int64_t)s * per + o);
    const u32x4 v1 = __builtin_nontemporal_load(in + (int64_t)(s + 4) * per + o);
    __builtin_nontemporal_store(v0, b + (row * 512 + col));
    __builtin_nontemporal_store(v1, b + (row * 512 + 256 + col));
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

// block-owned regions: block k streams its own ``region`` bytes in 16 KiB steps (the codec's
// z-slab walk), optionally with XCD-contiguous block order
__global__ void region_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, int64_t region16, int steps,
                            int xcd_per) {
  const int blk = xcd_per > 0 ? (int)(blockIdx.x % 8) * xcd_per + (int)(blockIdx.x / 8) : (int)blockIdx.x;
  const int64_t base = (int64_t)blk * region16;
  const int64_t per_step = region16 / steps;
  for (int s = 0; s < steps; ++s)
    for (int64_t i = threadIdx.x; i < per_step; i += blockDim.x) {
      const int64_t o = base + s * per_step + i;
      __builtin_nontemporal_store(__builtin_nontemporal_load(a + o), b + o);
    }
}

// row-strided reads: a wave covers 2 KiB = 16 lines of 128 B; instruction 1 reads the even
// lines (8 x 128 B at 256 B stride, the codec's "row 2Y" loads), instruction 2 the odd lines.
// STRIDED = 0 reads the same 2 KiB as two contiguous 1 KiB halves.  Writes 2 x 1 KiB contiguous.
template <int STRIDED>
__global__ void rows_copy(const u32x4* __restrict__ a, u32x4* __restrict__ b, int64_t nchunks) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t c = wave; c < nchunks; c += nw) {
    const int64_t base = c * 128;  // 2 KiB in 16-B units
    int64_t i0, i1;
    if (STRIDED) {
      i0 = base + (lane >> 3) * 16 + (lane & 7);
      i1 = i0 + 8;
    } else {
      i0 = base + lane;
      i1 = base + 64 + lane;
    }
    u32x4 v0 = __builtin_nontemporal_load(a + i0);
    u32x4 v1 = __builtin_nontemporal_load(a + i1);
    __builtin_nontemporal_store(v0, b + base + lane);
    __builtin_nontemporal_store(v1, b + base + 64 + lane);
  }
}

// codec-shaped copy: the exact access pattern of the volume encode at C3 (512 tiles of 64^3 u16,
// 256-thread workgroup = one z-slab of one tile, wave w owns rows 8w..8w+7, lane = (row, 8 x 16 B)):
// per output plane, read rows 2Y, 2Y+1 of planes 2c, 2c+1 (4 x 16 B per lane), write 8 x 8 B per
// lane into 8 separate [512, 32, 32, 32] arrays.  No arithmetic.
__global__ void __launch_bounds__(256) codec_shape(const uint16_t* __restrict__ hi, uint16_t* __restrict__ out,
                                                   int nslab) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int tx = lane & 7, Y = w * 8 + (lane >> 3), X = tx * 4;
  const int b = blockIdx.x / nslab, sl = blockIdx.x % nslab;
  const int slab = 32 / nslab;
  const uint16_t* t = hi + (int64_t)b * 262144;
  for (int c = sl * slab; c < (sl + 1) * slab; ++c) {
    const uint16_t* p = t + 2 * c * 4096 + 2 * Y * 64 + 2 * X;
    u32x4 e0 = __builtin_nontemporal_load((const u32x4*)p);
    u32x4 e1 = __builtin_nontemporal_load((const u32x4*)(p + 64));
    u32x4 o0 = __builtin_nontemporal_load((const u32x4*)(p + 4096));
    u32x4 o1 = __builtin_nontemporal_load((const u32x4*)(p + 4096 + 64));
    const int64_t o = (int64_t)b * 32768 + c * 1024 + Y * 32 + X;
    u32x2 v[8] = {{e0.x, e0.y}, {e0.z, e0.w}, {e1.x, e1.y}, {e1.z, e1.w}, {o0.x, o0.y}, {o0.z, o0.w}, {o1.x, o1.y}, {o1.z, o1.w}};
#pragma unroll
    for (int k = 0; k < 8; ++k) __builtin_nontemporal_store(v[k], (u32x2*)(out + (int64_t)k * 16777216 + o));
  }
}

int main(int argc, char** argv) {
  if (argc > 1 && argv[1][0] == 'c') {  // C2- (64 MiB) or C3-sized (256 MiB: "c3") ceilings
    const bool c3 = argv[1][1] == '3';
    const size_t sb = (c3 ? 256ull : 64ull) << 20;
    void *x, *m, *r;
    hipMalloc(&x, sb);
    hipMalloc(&m, sb);
    hipMalloc(&r, sb);
    hipMemset(x, 1, sb);
    hipMemset(m, 2, sb);
    hipMemset(r, 3, sb);
    hipEvent_t t0, t1;
    hipEventCreate(&t0);
    hipEventCreate(&t1);
    for (int blocks : {1024, 2048, 4096, 8192, 16384}) {
      for (int alt : {0, 1}) {
        auto pair = [&] {
          copy16<<<blocks, 256>>>((const u32x4*)x, (u32x4*)m, sb / 16);
          copy16<<<blocks, 256>>>((const u32x4*)(alt ? m : x), (u32x4*)(alt ? r : m), sb / 16);
        };
        for (int w = 0; w < 3; ++w) pair();
        hipEventRecord(t0);
        const int reps = 50;
        for (int i = 0; i < reps; ++i) pair();
        hipEventRecord(t1);
        hipEventSynchronize(t1);
        float ms;
        hipEventElapsedTime(&ms, t0, t1);
        const double us = ms * 1e3 / (2 * reps);
        printf("%s copy16 %s grid=%-6d %7.1f us per copy  %7.0f GB/s (read+write %zu MiB)\n", c3 ? "c3" : "c2",
               alt ? "X->M, M->R" : "X->M twice", blocks, us, 2.0 * sb / (us * 1e3), 2 * (sb >> 20));
      }
    }
    if (c3) {  // the codec's store / load shapes, alternating like bench.py: split8 X->M, merge8 M->R
      const int64_t n16 = sb / 16, per = n16 / 4;
      for (int shape = 0; shape < 2; ++shape)
      for (int blocks : {4096, 8192, 16384}) {
        auto enc = [&] {
          if (shape) split16<<<blocks, 256>>>((const u32x4*)x, (u32x4*)m, n16 / 2, n16 / 8);
          else split8<<<blocks, 256>>>((const u32x4*)x, (u32x2*)m, n16, per);
        };
        auto dec = [&] {
          if (shape) merge16<<<blocks, 256>>>((const u32x4*)m, (u32x4*)r, n16 / 2, n16 / 8);
          else merge8<<<blocks, 256>>>((const u32x2*)m, (u32x4*)r, n16, per);
        };
        auto pair = [&] {
          enc();
          dec();
        };
        for (int w = 0; w < 3; ++w) pair();
        hipEvent_t ev[41];
        for (auto& e : ev) hipEventCreate(&e);
        hipEventRecord(ev[0]);
        for (int i = 0; i < 20; ++i) {  // an event between every two launches: per-direction times
          enc();
          hipEventRecord(ev[2 * i + 1]);
          dec();
          hipEventRecord(ev[2 * i + 2]);
        }
        hipEventSynchronize(ev[40]);
        double se = 0, sd = 0;
        for (int i = 0; i < 20; ++i) {
          float a, b;
          hipEventElapsedTime(&a, ev[2 * i], ev[2 * i + 1]);
          hipEventElapsedTime(&b, ev[2 * i + 1], ev[2 * i + 2]);
          se += a;
          sd += b;
        }
        se *= 1e3 / 20;
        sd *= 1e3 / 20;
        printf("c3 %s grid=%-6d %7.1f / %7.1f us  %7.0f / %7.0f GB/s (read+write %zu MiB)\n",
               shape ? "split16 X->M / merge16 M->R" : "split8 X->M / merge8 M->R", blocks,
               se, sd, 2.0 * sb / (se * 1e3), 2.0 * sb / (sd * 1e3), 2 * (sb >> 20));
      }
    }
    return 0;
  }
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
  for (int nslab : {1, 4, 8, 32}) {
    char nm[64];
    snprintf(nm, sizeof nm, "codec_shape nslab=%d", nslab);
    run(nm, [&] { codec_shape<<<512 * nslab, 256>>>((const uint16_t*)a, (uint16_t*)b, nslab); });
  }
  for (int blocks : {4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "rows contiguous grid=%d", blocks);
    run(nm, [&] { rows_copy<0><<<blocks, 256>>>((const u32x4*)a, (u32x4*)b, n16 / 128); });
    snprintf(nm, sizeof nm, "rows strided grid=%d", blocks);
    run(nm, [&] { rows_copy<1><<<blocks, 256>>>((const u32x4*)a, (u32x4*)b, n16 / 128); });
  }
  for (int steps : {1, 4}) {
    for (int xcd : {0, 1}) {
      for (int64_t region : {16384, 65536}) {
        const int64_t r16 = region / 16 * steps / (region == 16384 ? steps : 1);
        const int blocks = (int)(n16 / r16);
        char nm[96];
        snprintf(nm, sizeof nm, "region %lldK steps=%d xcd=%d", (long long)(r16 * 16 / 1024), steps, xcd);
        run(nm, [&] { region_copy<<<blocks, 256>>>((const u32x4*)a, (u32x4*)b, r16, steps, xcd ? blocks / 8 : 0); });
      }
    }
  }
  const int64_t per = n16 / 4;  // u32x2 elements per output stream
  for (int blocks : {2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "split8 grid=%d", blocks);
    run(nm, [&] { split8<<<blocks, 256>>>((const u32x4*)a, (u32x2*)b, n16, per); });
    snprintf(nm, sizeof nm, "merge8 grid=%d", blocks);
    run(nm, [&] { merge8<<<blocks, 256>>>((const u32x2*)b, (u32x4*)a, n16, per); });
  }
  for (int blocks : {2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "split16 grid=%d", blocks);
    run(nm, [&] { split16<<<blocks, 256>>>((const u32x4*)a, (u32x4*)b, n16 / 2, n16 / 8); });
  }
  return 0;
}
