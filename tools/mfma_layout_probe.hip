// mfma_layout_probe.hip -- operand / result lane layout of v_mfma_f32_4x4x1f32 (16 blocks) on gfx950.
//   hipcc -O2 --offload-arch=gfx950 tools/mfma_layout_probe.hip -o tools/mfma_layout_probe
// Pass 1: A one-hot on lane la, B = lane + 1: every nonzero D entry names the B lane paired with la.
// Pass 2: B one-hot on lane lb, A = lane + 1: names the A lane paired with lb.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out, int pass, int hot) {
  const int l = threadIdx.x;
  const float a = pass == 0 ? (l == hot ? 1.0f : 0.0f) : (float)(l + 1);
  const float b = pass == 0 ? (float)(l + 1) : (l == hot ? 1.0f : 0.0f);
  f32x4 c = {0, 0, 0, 0};
  f32x4 d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) out[l * 4 + r] = d[r];
}
int main() {
  float* o;
  (void)hipMalloc(&o, 256 * 4);
  for (int pass = 0; pass < 2; ++pass)
    for (int hot : {0, 1, 2, 3, 4, 5, 17}) {
      k<<<1, 64>>>(o, pass, hot);
      float h[256];
      (void)hipMemcpy(h, o, sizeof h, hipMemcpyDeviceToHost);
      printf("%s one-hot lane %2d:", pass ? "B" : "A", hot);
      for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r)
          if (h[l * 4 + r] != 0.0f) printf("  D[lane %d][r%d] <- %s lane %d", l, r, pass ? "A" : "B", (int)h[l * 4 + r] - 1);
      printf("\n");
    }
  return 0;
}
