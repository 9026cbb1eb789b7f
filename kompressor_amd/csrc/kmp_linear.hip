// kmp_linear.hip -- LinearPredictor apply on f32 MFMA (v_mfma_f32_32x32x2_f32).
//
// pred[cell, k] = fma-chain over n = 0..N-1 of features[cell, n] * W[n, k], started from b[k]:
//     acc = b[k];  acc = fmaf(f[n], W[n, k], acc)  for n = 0, 1, ...
// then ``astype(T)`` (XLA truncating, saturating cast).  N = (2p+2)^d features in the
// reference's order (z-major, y, x: features_from_lowres, volume/utils.py:199-210), K = 19 (3D)
// or 5 (2D) outputs in the predictions order maps_from_predictions expects (volume/utils.py:83).
//
// On gfx950 an f32-input MFMA is bit-for-bit that k-ordered fmaf chain (cdna_hip_programming.md
// §3 'FP32-input MFMA'), so one wave computes a 32-cell x 32-output tile (19 / 5 used) as N/2
// 32x32x2 MFMAs with the accumulator seeded by the bias; the oracle reproduces the chain exactly.
// Lane l feeds A[cell l&31][feature 2s + (l>>5)] and B[feature 2s + (l>>5)][output l&31]; the
// result row (cell) of accumulator register r is (r&3) + 8(r>>2) + 4(l>>5), column l&31.
#include "kmp_bf16x2.h"
#include "kmp_codec.h"

namespace kmp {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct LinSrc {
  int64_t S[3];   // source spatial extents
  int32_t mult;   // 2: highres (lowres node j = sample 2*sym(j)), 1: lowres, 0: padded window
  int64_t L[3], E[3];
  int64_t cbeg[3], cext[3];  // box of cells to compute
  int64_t Lc[3];             // cells of the full grid (output indexing)
};

template <typename T>
__device__ __forceinline__ float lin_feature(const T* __restrict__ src, const LinSrc& s, int nsp, int p, int64_t b,
                                            int64_t c, int64_t C, int64_t cz, int64_t cy, int64_t cx, int n) {
  const int k = 2 * p + 2;
  int dz = 0, dy, dx;
  if (nsp == 3) {
    dz = n / (k * k);
    dy = (n / k) % k;
  } else {
    dy = n / k;
  }
  dx = n % k;
  int64_t z, y, x;
  if (s.mult == 0) {  // already padded window: the neighbourhood is [c, c + 2p + 1]
    z = nsp == 3 ? cz + dz : 0;
    y = cy + dy;
    x = cx + dx;
  } else {
    const int pz = nsp == 3 ? p : 0;
    z = s.mult * sym_index(sym_index(cz - pz + dz, s.L[0]), s.E[0]);
    y = s.mult * sym_index(sym_index(cy - p + dy, s.L[1]), s.E[1]);
    x = s.mult * sym_index(sym_index(cx - p + dx, s.L[2]), s.E[2]);
  }
  return (float)src[(((b * s.S[0] + z) * s.S[1] + y) * s.S[2] + x) * C + c];
}

// One wave per 32-row tile; rows = (b, cell in box, c) flattened.  Writes preds[row-major
// [B, Lc..., K, C]] in T and optionally the f32 values.
template <typename T>
__global__ void __launch_bounds__(256) linear_mfma_kernel(const T* __restrict__ src, LinSrc s, int nsp, int p,
                                                          int64_t B, int64_t C, const float* __restrict__ W,
                                                          const float* __restrict__ bias, int N, int K,
                                                          T* __restrict__ out, float* __restrict__ out_f32,
                                                          int64_t rows) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int j = lane & 31;  // output column this lane feeds (B operand) and holds (D)
  const int h = lane >> 5;  // k within the 2-wide step
  for (int64_t tile = wave; tile * 32 < rows; tile += nwaves) {
    // decode this lane's A row (cell)
    const int64_t row = tile * 32 + (lane & 31);
    const bool row_ok = row < rows;
    int64_t b, z, y, x, c;
    unflat5(row_ok ? row : 0, s.cext[0], s.cext[1], s.cext[2], C, b, z, y, x, c);
    z += s.cbeg[0];
    y += s.cbeg[1];
    x += s.cbeg[2];
    f32x16 acc;
    const float bj = j < K ? bias[j] : 0.0f;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = bj;  // every row of column j starts at b[j]
    for (int st = 0; st < N / 2; ++st) {
      const int n = 2 * st + h;
      const float a = row_ok ? lin_feature(src, s, nsp, p, b, c, C, z, y, x, n) : 0.0f;
      const float w = j < K ? W[n * K + j] : 0.0f;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w, acc, 0, 0, 0);
    }
    if (j >= K) continue;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int64_t orow = tile * 32 + (q & 3) + 8 * (q >> 2) + 4 * h;
      if (orow >= rows) continue;
      int64_t ob, oz, oy, ox, oc;
      unflat5(orow, s.cext[0], s.cext[1], s.cext[2], C, ob, oz, oy, ox, oc);
      oz += s.cbeg[0];
      oy += s.cbeg[1];
      ox += s.cbeg[2];
      const int64_t cell = ((ob * s.Lc[0] + oz) * s.Lc[1] + oy) * s.Lc[2] + ox;
      const int64_t o = (cell * K + j) * C + oc;
      out[o] = cast_f32<T>(acc[q]);
      if (out_f32) out_f32[o] = acc[q];
    }
  }
}

// KMP_PRED_LINEAR_MFMA (kmp_bf16x2.h): one wave per 16-row tile (rows = (b, cell, c) as above),
// the K outputs in column tiles of 16, per accumulation step (8 features, kmp_bf16x2.h
// step_feature) one v_mfma_f32_16x16x32_bf16 per column tile.  u8 / u16 samples only (the byte split is exact for them).
template <typename T>
__global__ void __launch_bounds__(256) linear_bf16x2_kernel(const T* __restrict__ src, LinSrc s, int nsp, int p,
                                                            int64_t B, int64_t C, const float* __restrict__ W,
                                                            const float* __restrict__ bias, int N, int K,
                                                            T* __restrict__ out, float* __restrict__ out_f32,
                                                            int64_t rows) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int m = lane & 15, g = lane >> 4;
  const int nq = (N + 7) / 8, nct = (K + 15) / 16;
  for (int64_t tile = wave; tile * 16 < rows; tile += nwaves) {
    const int64_t row = tile * 16 + m;  // this lane's A row (cell)
    const bool row_ok = row < rows;
    int64_t b, z, y, x, c;
    unflat5(row_ok ? row : 0, s.cext[0], s.cext[1], s.cext[2], C, b, z, y, x, c);
    z += s.cbeg[0];
    y += s.cbeg[1];
    x += s.cbeg[2];
    for (int ct = 0; ct < nct; ++ct) {
      const int k = 16 * ct + m;  // this lane's B / D column
      const bool col_ok = k < K;
      const float bk = col_ok ? bias[k] : 0.0f;
      bx::f32x4 acc = {bk, bk, bk, bk};
      for (int t = 0; t < nq; ++t) {  // accumulation steps (kmp_bf16x2.h step_feature)
        bx::u32x4 a;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = bx::step_feature(nsp, p, nq, t, g & 1, i);
          const uint32_t v = (row_ok && n < N) ? (uint32_t)lin_feature(src, s, nsp, p, b, c, C, z, y, x, n) : 0u;
          a[i] = bx::feature_dword(v);
        }
        acc = bx::mfma(a, bx::b_fragment(W + (col_ok ? k : 0), K, N, nsp, p, t, g, col_ok), acc);
      }
      if (!col_ok) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t orow = tile * 16 + 4 * g + r;
        if (orow >= rows) continue;
        int64_t ob, oz, oy, ox, oc;
        unflat5(orow, s.cext[0], s.cext[1], s.cext[2], C, ob, oz, oy, ox, oc);
        oz += s.cbeg[0];
        oy += s.cbeg[1];
        ox += s.cbeg[2];
        const int64_t cell = ((ob * s.Lc[0] + oz) * s.Lc[1] + oy) * s.Lc[2] + ox;
        const int64_t o = (cell * K + k) * C + oc;
        out[o] = cast_f32<T>(acc[r]);
        if (out_f32) out_f32[o] = acc[r];
      }
    }
  }
}

template <typename T>
static int launch_linear(const T* src, const LinSrc& s, int nsp, int p, int64_t B, int64_t C, const float* W,
                         const float* bias, T* out, float* out_f32, hipStream_t stream, int kind = KMP_PRED_LINEAR) {
  const int k = 2 * p + 2;
  const int N = nsp == 3 ? k * k * k : k * k;
  const int K = nsp == 3 ? 19 : 5;
  const int64_t rows = B * s.cext[0] * s.cext[1] * s.cext[2] * C;
  if (rows == 0) return KMP_OK;
  if (kind == KMP_PRED_LINEAR_MFMA) {
    if constexpr (std::is_same<T, uint8_t>::value || std::is_same<T, uint16_t>::value) {
      int64_t blocks = ceil_div(ceil_div(rows, 16), 4);
      if (blocks > 65536) blocks = 65536;
      linear_bf16x2_kernel<T><<<(unsigned)blocks, 256, 0, stream>>>(src, s, nsp, p, B, C, W, bias, N, K, out, out_f32,
                                                                    rows);
      return check_launch("linear_bf16x2");
    }
    return fail(KMP_ERR_UNSUPPORTED, "the matrix-core LinearPredictor (bf16x2) takes uint8 / uint16 samples");
  }
  int64_t waves = ceil_div(rows, 32);
  int64_t blocks = ceil_div(waves, 4);
  if (blocks > 65536) blocks = 65536;
  linear_mfma_kernel<T><<<(unsigned)blocks, 256, 0, stream>>>(src, s, nsp, p, B, C, W, bias, N, K, out, out_f32, rows);
  return check_launch("linear_mfma");
}

template <typename T>
int linear_cells(const T* src, const int64_t* S, int mult, const Geo& g, int nsp, int64_t B, int64_t C,
                 const kmp_predictor* pred, const int64_t* cbegin, const int64_t* cext, T* cells, hipStream_t stream) {
  LinSrc s{};
  for (int a = 0; a < 3; ++a) {
    s.S[a] = S[a];
    s.L[a] = g.L[a];
    s.E[a] = g.E[a];
    s.cbeg[a] = cbegin[a];
    s.cext[a] = cext[a];
    s.Lc[a] = g.Lc[a];
  }
  s.mult = mult;
  return launch_linear<T>(src, s, nsp, pred->padding, B, C, pred->weights, pred->bias, cells, nullptr, stream,
                          pred->kind);
}

#define KMP_INSTL(T)                                                                                             \
  template int linear_cells<T>(const T*, const int64_t*, int, const Geo&, int, int64_t, int64_t,               \
                               const kmp_predictor*, const int64_t*, const int64_t*, T*, hipStream_t);
KMP_INSTL(uint8_t)
KMP_INSTL(uint16_t)
KMP_INSTL(int32_t)
KMP_INSTL(uint32_t)

}  // namespace kmp

using namespace kmp;

static int linear_predict(int kind, int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B,
                          const int64_t shape[3], int64_t C, int32_t padding, const float* weights, const float* bias,
                          void* preds_out, float* preds_f32, kmp_stream_t stream);

extern "C" int kmp_linear_predict(int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B,
                                  const int64_t shape[3], int64_t C, int32_t padding, const float* weights,
                                  const float* bias, void* preds_out, float* preds_f32, kmp_stream_t stream) {
  return linear_predict(KMP_PRED_LINEAR, nsp, dtype, padded_lowres, B, shape, C, padding, weights, bias, preds_out,
                        preds_f32, stream);
}

extern "C" int kmp_linear_predict_mfma(int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B,
                                       const int64_t shape[3], int64_t C, int32_t padding, const float* weights,
                                       const float* bias, void* preds_out, float* preds_f32, kmp_stream_t stream) {
  return linear_predict(KMP_PRED_LINEAR_MFMA, nsp, dtype, padded_lowres, B, shape, C, padding, weights, bias,
                        preds_out, preds_f32, stream);
}

static int linear_predict(int kind, int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B,
                          const int64_t shape[3], int64_t C, int32_t padding, const float* weights, const float* bias,
                          void* preds_out, float* preds_f32, kmp_stream_t stream) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(padded_lowres && weights && bias && preds_out && shape && padding >= 0, "bad argument");
  KMP_REQUIRE(B >= 0 && C >= 1, "bad batch or channel count");
  LinSrc s{};
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) {
      s.S[a] = 1; s.cext[a] = 1; s.Lc[a] = 1;
      continue;
    }
    const int64_t S = shape[a - (3 - nsp)];
    const int64_t cells = S - 2 * padding - 1;
    KMP_REQUIRE(cells >= 1, "window has no cells");
    s.S[a] = S;
    s.cext[a] = cells;
    s.Lc[a] = cells;
  }
  s.mult = 0;
  return dispatch_int_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    return launch_linear<T>((const T*)padded_lowres, s, nsp, padding, B, C, weights, bias, (T*)preds_out, preds_f32,
                            (hipStream_t)stream, kind);
  });
}
