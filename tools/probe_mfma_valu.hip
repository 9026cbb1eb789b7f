// Does v_mfma_f32_16x16x4_f32 overlap packed-f32 VALU work on the same SIMD?
//   hipcc --offload-arch=gfx950 -O3 tools/probe_mfma_valu.hip -o tools/probe_mfma_valu && tools/probe_mfma_valu
// Kernels (1024 workgroups x 256 threads, every wave independent):
//   mfma  : each wave runs NM rounds of 8 independent 16x16x4 f32 MFMAs
//   valu  : each wave runs NV rounds of 8 independent v_pk_fma_f32
//   split : even waves do the mfma work, odd waves the valu work (co-resident on each SIMD)
//   mixed : every wave does both streams interleaved in its own instruction stream
//   split1: 1-wave workgroups, even workgroups mfma, odd valu (the SIMDs get both kinds)
//   bf16 control: the same split / mixed with v_mfma_f32_16x16x16_bf16 (16 cycles) in place of the
//   f32 MFMA -- a matrix op the guide measures overlapping VALU (MI355X_MICROARCH.md)
// If the matrix pipe and the VALU share nothing, split ~ max(mfma, valu); if they share the
// f32 datapath, split ~ mfma + valu.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int NM = 512, NV = 1024;

__device__ __forceinline__ void do_mfma(float a, float b, f32x4 (&acc)[8]) {
#pragma unroll 1
  for (int i = 0; i < NM; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[k], 0, 0, 0);
  }
}
__device__ __forceinline__ void do_valu(f32x2 x, f32x2 w, f32x2 (&v)[8]) {
#pragma unroll 1
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = __builtin_elementwise_fma(x, w, v[k]);
  }
}

typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void do_bf16(bf16x4 a, bf16x4 b, f32x4 (&acc)[8]) {
#pragma unroll 1
  for (int i = 0; i < NM; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a, b, acc[k], 0, 0, 0);
  }
}

template <int MODE>
__global__ void __launch_bounds__(256) probe(float* out, float a, float b) {
  f32x4 acc[8];
  f32x2 v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    acc[k] = (f32x4){a, b, a, b};
    v[k] = (f32x2){a + k, b - k};
  }
  const int wave = MODE >= 4 ? blockIdx.x : threadIdx.x >> 6;
  const bf16x4 ab = {(__bf16)a, (__bf16)b, (__bf16)a, (__bf16)b};
  const f32x2 x = {a, b}, w = {b, a};
  if (MODE == 0 || ((MODE == 2 || MODE == 4) && (wave & 1) == 0)) do_mfma(a, b, acc);
  if (MODE == 1 || ((MODE == 2 || MODE == 4 || MODE == 6) && (wave & 1) == 1)) do_valu(x, w, v);
  if (MODE == 5 || (MODE == 6 && (wave & 1) == 0)) do_bf16(ab, ab, acc);
  if (MODE == 7) {
#pragma unroll 1
    for (int i = 0; i < NM; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc[k] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ab, ab, acc[k], 0, 0, 0);
        v[k] = __builtin_elementwise_fma(x, w, v[k]);
        v[k] = __builtin_elementwise_fma(x, w, v[k]);
      }
    }
  }
  if (MODE == 3) {
#pragma unroll 1
    for (int i = 0; i < NM; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        acc[k] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[k], 0, 0, 0);
        v[k] = __builtin_elementwise_fma(x, w, v[k]);
        v[k] = __builtin_elementwise_fma(x, w, v[k]);
      }
    }
  }
  float s = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) s += acc[k].x + acc[k].y + acc[k].z + acc[k].w + v[k].x + v[k].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  float* out;
  hipMalloc(&out, 1024 * 256 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[8] = {"mfma f32          ", "valu pk_fma       ", "split f32/valu    ", "mixed f32+valu    ",
                          "split1 f32/valu   ", "mfma bf16         ", "split1 bf16/valu  ", "mixed bf16+valu   "};
  for (int rep = 0; rep < 2; ++rep) {
    for (int m = 0; m < 8; ++m) {
      auto launch = [&]() {
        switch (m) {
          case 0: probe<0><<<1024, 256>>>(out, 1.0f, 0.5f); break;
          case 1: probe<1><<<1024, 256>>>(out, 1.0f, 0.5f); break;
          case 2: probe<2><<<1024, 256>>>(out, 1.0f, 0.5f); break;
          case 3: probe<3><<<1024, 256>>>(out, 1.0f, 0.5f); break;
          case 4: probe<4><<<4096, 64>>>(out, 1.0f, 0.5f); break;
          case 5: probe<5><<<1024, 256>>>(out, 1.0f, 0.5f); break;
          case 6: probe<6><<<4096, 64>>>(out, 1.0f, 0.5f); break;
          default: probe<7><<<1024, 256>>>(out, 1.0f, 0.5f); break;
        }
      };
      launch();
      hipEventRecord(e0);
      for (int i = 0; i < 5; ++i) launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      printf("%s %7.1f us   (4 waves per SIMD; an MFMA wave issues %d MFMAs, a VALU wave %d v_pk_fma_f32)\n",
             names[m], ms * 1e3 / 5, NM * 8, NV * 8);
    }
  }
  return 0;
}
