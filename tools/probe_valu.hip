// probe_valu.hip -- f32 FMA issue rate on gfx950: packed (v_pk_fma_f32) vs plain (v_fma_f32),
// weight operand in a scalar register, 16 independent accumulator chains per lane.
//   hipcc -O3 --offload-arch=gfx950 tools/probe_valu.hip -o tools/probe_valu && tools/probe_valu
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ void __launch_bounds__(256) fma_kernel(float* out, float w0, float w1, int iters) {
  float x = (float)threadIdx.x * 1e-3f;
  f32x2 acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = (f32x2){x + i, x - i};
  const f32x2 f = {x, x + 1.0f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float w = (i & 1) ? w1 : w0;
      if constexpr (PK) {
        acc[i] = __builtin_elementwise_fma(f, (f32x2){w, w}, acc[i]);
      } else {
        acc[i].x = __builtin_fmaf(f.x, w, acc[i].x);
        acc[i].y = __builtin_fmaf(f.y, w, acc[i].y);
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  const int blocks = 256 * 16, threads = 256, iters = 4096;
  hipMalloc(&out, sizeof(float) * blocks * threads);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int pk = 0; pk < 2; ++pk) {
    for (int rep = 0; rep < 3; ++rep) {
      hipEventRecord(e0);
      if (pk) fma_kernel<true><<<blocks, threads>>>(out, 1.0001f, 0.9999f, iters);
      else fma_kernel<false><<<blocks, threads>>>(out, 1.0001f, 0.9999f, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double flop = 2.0 * 32 * (double)iters * blocks * threads;
      printf("%s rep %d: %.3f ms, %.1f TFLOP/s\n", pk ? "v_pk_fma_f32" : "v_fma_f32   ", rep, ms, flop / ms / 1e9);
    }
  }
  hipFree(out);
  return 0;
}
