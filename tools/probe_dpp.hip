// DPP semantics probe (gfx950): the Rice kernels' 8-lane group helpers, full and partial exec
#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ uint32_t group8_incl(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
  return v - (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x157, 0xf, 0xc, false);
}
__device__ __forceinline__ uint32_t group8_incl_sel(uint32_t v, int j8) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);
  const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x157, 0xf, 0xf, false);
  return j8 ? v - t : v;
}
__device__ __forceinline__ uint32_t group8_last(uint32_t x) {
  const int b = __builtin_amdgcn_update_dpp(0, (int)x, 0x15F, 0xf, 0xf, false);
  return (uint32_t)__builtin_amdgcn_update_dpp(b, (int)x, 0x157, 0xf, 0x3, false);
}
__device__ __forceinline__ uint32_t group8_first(uint32_t x) {
  const int b = __builtin_amdgcn_update_dpp(0, (int)x, 0x158, 0xf, 0xf, false);
  return (uint32_t)__builtin_amdgcn_update_dpp(b, (int)x, 0x150, 0xf, 0x3, false);
}
__global__ void k(const uint32_t* in, uint32_t* o) {
  const int l = threadIdx.x;
  uint32_t v = in[l];
  asm volatile("" : "+v"(v));
  const uint32_t inc = group8_incl(v);
  o[0 * 64 + l] = inc;
  o[1 * 64 + l] = group8_last(inc);
  o[2 * 64 + l] = group8_first(v);
  const uint32_t inc2 = group8_incl_sel(v, l & 8);
  o[3 * 64 + l] = inc2;
  o[4 * 64 + l] = group8_last(inc2);
}
int main() {
  uint32_t h_in[64], h[5 * 64];
  for (int l = 0; l < 64; ++l) h_in[l] = (uint32_t)(l * 7 + 3) % 50;
  uint32_t *d_in, *d; hipMalloc((void**)&d_in, sizeof(h_in)); hipMalloc((void**)&d, sizeof(h));
  hipMemcpy(d_in, h_in, sizeof(h_in), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d_in, d);
  hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    uint32_t inc = 0, tot = 0;
    for (int m = l & ~7; m <= l; ++m) inc += h_in[m];
    for (int m = l & ~7; m < (l & ~7) + 8; ++m) tot += h_in[m];
    const uint32_t first = h_in[l & ~7];
    if (h[l] != inc || h[64 + l] != tot || h[128 + l] != first || h[192 + l] != inc || h[256 + l] != tot) {
      ++bad;
      printf("lane %d: incl %u/%u last %u/%u first %u/%u incl_sel %u last_sel %u\n", l, h[l], inc, h[64 + l], tot,
             h[128 + l], first, h[192 + l], h[256 + l]);
    }
  }
  printf("bad lanes: %d\n", bad);
  return 0;
}
