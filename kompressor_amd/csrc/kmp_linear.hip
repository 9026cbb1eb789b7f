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
#include "kmp_wave.h"

namespace kmp {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// astype(T) of an MFMA result: for 8- / 16-bit samples the clamp-then-convert form of the
// saturating hardware conversion (kmp_wave.h cvt_sat_mfma: NaN -> 0, truncation, saturation --
// cast_f32's semantics in 3 VALU instead of its f64 path with branches)
template <typename T>
__device__ __forceinline__ T lin_cast(float v) {
  if constexpr (sizeof(T) <= 2) return (T)wv::cvt_sat_mfma<T>(v);
  else return cast_f32<T>(v);
}

struct LinSrc {
  int64_t S[3];   // source spatial extents
  int32_t mult;   // 2: highres (lowres node j = sample 2*sym(j)), 1: lowres, 0: padded window
  int64_t L[3], E[3];
  int64_t cbeg[3], cext[3];  // box of cells to compute
  int64_t Lc[3];             // cells of the full grid (output indexing)
  int32_t simple;            // every node index needs at most one reflection per sym (launch_linear)
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

// A lane's cell neighbourhood as element offsets into the source, per axis (KK = 2p + 2 nodes
// each): feature n = (dz, dy, dx) in the reference's order is src[base + oz[dz] + oy[dy] + ox[dx]]
// -- the index arithmetic of lin_feature done once per cell instead of once per feature.
template <int NSP, int KK, typename I>
struct Nbhd {
  I base, oz[NSP == 3 ? KK : 1], oy[KK], ox[KK];
  __device__ __forceinline__ void init(const LinSrc& s, int p, int64_t C, I b, I c, I cz, I cy, I cx) {
    const I Cc = (I)C, sy = (I)s.S[2] * Cc, sz = (I)s.S[1] * sy;
    base = b * ((I)s.S[0] * sz) + c;
    auto src = [&](int64_t j, int a) -> I {  // source index of padded node j along axis a
      if (s.mult == 0) return (I)j;
      if constexpr (sizeof(I) == 4) {
        if (s.simple) {  // kernel argument: a uniform branch; 32-bit, select-only reflections
          const int L = (int)s.L[a], E = (int)s.E[a];
          int v = (int)j;
          v = v < 0 ? -1 - v : (v >= L ? 2 * L - 1 - v : v);
          v = v >= E ? 2 * E - 1 - v : v;
          return (I)(s.mult * v);
        }
      }
      return (I)(s.mult * sym_index(sym_index(j, s.L[a]), s.E[a]));
    };
#pragma unroll
    for (int d = 0; d < KK; ++d) {
      ox[d] = src(cx - (s.mult ? p : 0) + d, 2) * Cc;
      oy[d] = src(cy - (s.mult ? p : 0) + d, 1) * sy;
      if constexpr (NSP == 3) oz[d] = src(cz - (s.mult ? p : 0) + d, 0) * sz;
    }
    if constexpr (NSP != 3) oz[0] = 0;
  }
  // feature n's offset (n compile-time after unrolling)
  __device__ __forceinline__ I at(int n) const {
    const int dz = NSP == 3 ? n / (KK * KK) : 0, dy = (n / KK) % KK, dx = n % KK;
    return base + oz[dz] + oy[dy] + ox[dx];
  }
};

// The row decomposition (b, cell in box, c) of the flattened rows, by multiply-high division
struct LinFlat {
  uint32_t dC_m, dC_s, d2_m, d2_s, d1_m, d1_s, d0_m, d0_s;
  uint32_t C, e2, e1, e0;
};
static inline void lf_div(int64_t d64, uint32_t& m, uint32_t& sh) {
  const uint32_t d = (uint32_t)(d64 < 1 ? 1 : d64);
  uint32_t s = 0;
  while (s < 32 && (1ull << s) < d) ++s;
  m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  sh = s;
}
static inline LinFlat make_linflat(const LinSrc& s, int64_t C) {
  LinFlat f{};
  lf_div(C, f.dC_m, f.dC_s);
  lf_div(s.cext[2], f.d2_m, f.d2_s);
  lf_div(s.cext[1], f.d1_m, f.d1_s);
  lf_div(s.cext[0], f.d0_m, f.d0_s);
  f.C = (uint32_t)C; f.e2 = (uint32_t)s.cext[2]; f.e1 = (uint32_t)s.cext[1]; f.e0 = (uint32_t)s.cext[0];
  return f;
}
template <typename I>
__device__ __forceinline__ void lin_unflat(int64_t row, const LinFlat& f, const LinSrc& s, int64_t C, I& b, I& z, I& y,
                                           I& x, I& c) {
  if constexpr (sizeof(I) == 4) {
    uint32_t u = (uint32_t)row, q;
    q = (__umulhi(u, f.dC_m) + u) >> f.dC_s; c = (I)(u - q * f.C); u = q;
    q = (__umulhi(u, f.d2_m) + u) >> f.d2_s; x = (I)(u - q * f.e2); u = q;
    q = (__umulhi(u, f.d1_m) + u) >> f.d1_s; y = (I)(u - q * f.e1); u = q;
    q = (__umulhi(u, f.d0_m) + u) >> f.d0_s; z = (I)(u - q * f.e0); b = (I)q;
  } else {
    int64_t bb, zz, yy, xx, cc;
    unflat5(row, s.cext[0], s.cext[1], s.cext[2], C, bb, zz, yy, xx, cc);
    b = bb; z = zz; y = yy; x = xx; c = cc;
  }
  z += (I)s.cbeg[0];
  y += (I)s.cbeg[1];
  x += (I)s.cbeg[2];
}

// One wave per 32-row tile; rows = (b, cell in box, c) flattened.  Writes preds[cell * cst + k *
// kst + c] (launch_linear: interleaved or planar) in T and optionally the f32 values.  KK = 2p + 2 at compile time (p <= 2:
// the neighbourhood offsets per lane once, the N/2 steps unrolled) or 0 (any p: lin_feature).
template <typename T, int NSP, int KK, typename I>
__global__ void __launch_bounds__(256) linear_mfma_kernel(const T* __restrict__ src, LinSrc s, LinFlat lf, int p,
                                                          int64_t B, int64_t C, const float* __restrict__ W,
                                                          const float* __restrict__ bias, int N, int K,
                                                          T* __restrict__ out, float* __restrict__ out_f32,
                                                          int64_t rows, int64_t cst, int64_t kst) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int j = lane & 31;  // output column this lane feeds (B operand) and holds (D)
  const int h = lane >> 5;  // k within the 2-wide step
  const float bj = j < K ? bias[j] : 0.0f;
  // the lane's weights of every step, loaded once for all its tiles when they fit in registers
  constexpr int NN0 = KK > 0 ? (NSP == 3 ? KK * KK * KK : KK * KK) : 2;
  constexpr bool WREG = KK > 0 && NN0 / 2 <= 32;
  float wreg[WREG ? NN0 / 2 : 1];
  if constexpr (WREG) {
#pragma unroll
    for (int st = 0; st < NN0 / 2; ++st) wreg[st] = j < K ? W[(2 * st + h) * K + j] : 0.0f;
  }
  for (int64_t tile = wave; tile * 32 < rows; tile += nwaves) {
    // this lane's A row (cell)
    const int64_t row = tile * 32 + (lane & 31);
    const bool row_ok = row < rows;
    I b, z, y, x, c;
    lin_unflat<I>(row_ok ? row : 0, lf, s, C, b, z, y, x, c);
    f32x16 acc;
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = bj;  // every row of column j starts at b[j]
    if constexpr (KK > 0) {
      Nbhd<NSP, KK, I> nb;
      nb.init(s, p, C, b, c, z, y, x);
      constexpr int NN = NSP == 3 ? KK * KK * KK : KK * KK;
      if constexpr (NN / 2 > 32) {
        // 3D p = 2 (108 steps): unrolled per z plane only -- fully unrolled, the compiler hoisted
        // every gather (310 VGPRs, one wave a SIMD).  Same steps in the same order.
        constexpr int PL = KK * KK / 2;  // steps per z plane
#pragma unroll 1
        for (int dz = 0; dz < KK; ++dz) {
          I zo = nb.oz[0];
#pragma unroll
          for (int d = 1; d < KK; ++d) zo = dz == d ? nb.oz[d] : zo;
#pragma unroll
          for (int q = 0; q < PL; ++q) {
            const int dy = (2 * q) / KK, dx = (2 * q) % KK;  // features 2q, 2q + 1 of the plane
            const I o = nb.base + zo + nb.oy[dy] + (h ? nb.ox[dx + 1] : nb.ox[dx]);
            const float a = row_ok ? (float)src[o] : 0.0f;
            const int st = dz * PL + q;
            const float w = j < K ? W[(2 * st + h) * K + j] : 0.0f;
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w, acc, 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int st = 0; st < NN / 2; ++st) {
          // features 2st and 2st + 1 share dz, dy (KK even): the lane's is 2st + h
          const I o0 = nb.at(2 * st), o1 = nb.at(2 * st + 1);
          const float a = row_ok ? (float)src[h ? o1 : o0] : 0.0f;
          const float w = WREG ? wreg[WREG ? st : 0] : (j < K ? W[(2 * st + h) * K + j] : 0.0f);
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w, acc, 0, 0, 0);
        }
      }
    } else {
      const int64_t bz = b, zz = z, yy = y, xx = x, cc = c;
      for (int st = 0; st < N / 2; ++st) {
        const int n = 2 * st + h;
        const float a = row_ok ? lin_feature(src, s, NSP, p, bz, cc, C, zz, yy, xx, n) : 0.0f;
        const float w = j < K ? W[n * K + j] : 0.0f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, w, acc, 0, 0, 0);
      }
    }
    // the output offset of each row, held by the row's own lane: cell * cst + c (+ k * kst)
    const int64_t cell = (((int64_t)b * s.Lc[0] + z) * s.Lc[1] + y) * s.Lc[2] + x;
    const int64_t obase = cell * cst + c;
    const int olo = (int)(uint32_t)obase, ohi = sizeof(I) == 4 ? 0 : (int)(obase >> 32);
    // (the shuffles run with every lane active: a lane reading an inactive lane gets no value)
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int r = (q & 3) + 8 * (q >> 2) + 4 * h;
      const int64_t ob = sizeof(I) == 4 ? (int64_t)__shfl(olo, r, 64)
                                        : (int64_t)(uint32_t)__shfl(olo, r, 64) | ((int64_t)__shfl(ohi, r, 64) << 32);
      if (j >= K || tile * 32 + r >= rows) continue;
      const int64_t o = ob + (int64_t)j * kst;
      out[o] = lin_cast<T>(acc[q]);
      if (out_f32) out_f32[o] = acc[q];
    }
  }
}

// KMP_PRED_LINEAR_MFMA (kmp_bf16x2.h): one wave per 16-row tile (rows = (b, cell, c) as above),
// the K outputs in column tiles of 16, per accumulation step (8 features, kmp_bf16x2.h
// step_feature) one v_mfma_f32_16x16x32_bf16 per column tile.  u8 / u16 samples only (the byte
// split is exact for them).  KK as linear_mfma_kernel's: the neighbourhood offsets once per cell,
// the steps unrolled (step-outer: each A fragment feeds every column tile; per column tile the
// accumulation order is unchanged, so the bits are), each lane's 4 features of a step one select
// between the two lane groups'.
template <typename T, int NSP, int KK, typename I>
__global__ void __launch_bounds__(256) linear_bf16x2_kernel(const T* __restrict__ src, LinSrc s, LinFlat lf, int p,
                                                            int64_t B, int64_t C, const float* __restrict__ W,
                                                            const float* __restrict__ bias, int N, int K,
                                                            T* __restrict__ out, float* __restrict__ out_f32,
                                                            int64_t rows, int64_t cst, int64_t kst) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  const int m = lane & 15, g = lane >> 4;
  const int nq = (N + 7) / 8, nct = (K + 15) / 16;
  // the lane's B fragments of every (column tile, step), built once for all its tiles when they
  // fit in 64 registers (the bf16 splits of 4 weights per fragment were redone per tile)
  constexpr int NQ0 = KK > 0 ? ((NSP == 3 ? KK * KK * KK : KK * KK) + 7) / 8 : 1;
  constexpr int NCT0 = NSP == 3 ? 2 : 1;
  constexpr bool BREG = KK > 0 && NCT0 * NQ0 <= 16;
  bx::u32x4 breg[BREG ? NCT0 : 1][BREG ? NQ0 : 1];
  if constexpr (BREG) {
#pragma unroll
    for (int ct = 0; ct < NCT0; ++ct)
#pragma unroll
      for (int t = 0; t < NQ0; ++t) {
        const int k = 16 * ct + m;
        breg[ct][t] = bx::b_fragment(W + (k < K ? k : 0), K, N, NSP, p, t, g, k < K);
      }
  }
  constexpr int NQP = KK > 0 ? ((NSP == 3 ? KK * KK * KK : KK * KK) + 7) / 8 : 1;
  if constexpr (KK > 0 && NQP <= 8) {
    // p <= 1 (<= 8 steps): software-pipelined over the wave's tiles.  The gathers are the latency
    // chain (offsets -> loads -> MFMAs -> stores, with ~3 waves a SIMD), so each iteration issues
    // the next tile's gathers (16 raw values a lane at most) before the current tile's MFMAs and
    // stores.  Same fragments, same MFMA order per column tile as the loop below: same bits.
    constexpr int NN = NSP == 3 ? KK * KK * KK : KK * KK;
    constexpr int NP = (NQP + 1) / 2;  // step pairs (the last one may be a single step)
    const bool up = g >= 2;
    struct In {
      uint32_t raw[NP][4];
      int olo, ohi;
    };
    auto fetch = [&](int64_t tile, In& in) {
      const int64_t row = tile * 16 + m;
      const bool row_ok = row < rows;
      I b, z, y, x, c;
      lin_unflat<I>(row_ok ? row : 0, lf, s, C, b, z, y, x, c);
      Nbhd<NSP, KK, I> nb;
      nb.init(s, p, C, b, c, z, y, x);
      auto feat = [&](int t, int i, int& n) -> I {
        const int n0 = bx::step_feature(NSP, (KK - 2) / 2, NQP, t, 0, i);
        const int n1 = bx::step_feature(NSP, (KK - 2) / 2, NQP, t, 1, i);
        n = (g & 1) ? n1 : n0;
        return (g & 1) ? nb.at(n1 < NN ? n1 : 0) : nb.at(n0 < NN ? n0 : 0);
      };
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int t = 2 * q;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          int nl, nu = 0;
          const I ol = feat(t, i, nl);
          I o = ol;
          int n = nl;
          if (t + 1 < NQP) {  // low half: step t, high half: step t + 1
            const I ou = feat(t + 1, i, nu);
            o = up ? ou : ol;
            n = up ? nu : nl;
          }
          in.raw[q][i] = (row_ok && n < NN) ? (uint32_t)src[o] : 0u;
        }
      }
      const int64_t cell = (((int64_t)b * s.Lc[0] + z) * s.Lc[1] + y) * s.Lc[2] + x;
      const int64_t obase = cell * cst + c;
      in.olo = (int)(uint32_t)obase;
      in.ohi = sizeof(I) == 4 ? 0 : (int)(obase >> 32);
    };
    In cur, nxt;
    int64_t tile = wave;
    if (tile * 16 < rows) fetch(tile, cur);
    for (; tile * 16 < rows; tile += nwaves) {
      if ((tile + nwaves) * 16 < rows) fetch(tile + nwaves, nxt);
      bx::f32x4 acc[NCT0];
#pragma unroll
      for (int ct = 0; ct < NCT0; ++ct) {
        const int k = 16 * ct + m;
        const float bk = k < K ? bias[k] : 0.0f;
        acc[ct] = bx::f32x4{bk, bk, bk, bk};
      }
      auto step = [&](const bx::u32x4& a, int t) {
#pragma unroll
        for (int ct = 0; ct < NCT0; ++ct) {
          const int k = 16 * ct + m;
          if constexpr (BREG) acc[ct] = bx::mfma(a, breg[ct][t], acc[ct]);
          else acc[ct] = bx::mfma(a, bx::b_fragment(W + (k < K ? k : 0), K, N, NSP, p, t, g, k < K), acc[ct]);
        }
      };
#pragma unroll
      for (int q = 0; q < NP; ++q) {
        const int t = 2 * q;
        bx::u32x4 a0, a1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t v = bx::feature_dword(cur.raw[q][i]);
          if (t + 1 < NQP) {  // lanes 32-63 of the first operand trade with lanes 0-31 of the second
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            a0[i] = r[0];
            a1[i] = r[1];
          } else {
            a0[i] = v;
          }
        }
        step(a0, t);
        if (t + 1 < NQP) step(a1, t + 1);
      }
#pragma unroll
      for (int ct = 0; ct < NCT0; ++ct) {
        const int k = 16 * ct + m;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = 4 * g + r;  // (every lane active for the shuffle)
          const int64_t ob = sizeof(I) == 4
                                 ? (int64_t)__shfl(cur.olo, rr, 64)
                                 : (int64_t)(uint32_t)__shfl(cur.olo, rr, 64) | ((int64_t)__shfl(cur.ohi, rr, 64) << 32);
          if (k >= K || tile * 16 + rr >= rows) continue;
          const int64_t o = ob + (int64_t)k * kst;
          out[o] = lin_cast<T>(acc[ct][r]);
          if (out_f32) out_f32[o] = acc[ct][r];
        }
      }
      cur = nxt;
    }
    return;
  }
  for (int64_t tile = wave; tile * 16 < rows; tile += nwaves) {
    const int64_t row = tile * 16 + m;  // this lane's A row (cell)
    const bool row_ok = row < rows;
    I b, z, y, x, c;
    lin_unflat<I>(row_ok ? row : 0, lf, s, C, b, z, y, x, c);
    constexpr int NQ = KK > 0 ? ((NSP == 3 ? KK * KK * KK : KK * KK) + 7) / 8 : 1;
    Nbhd<NSP, (KK > 0 ? KK : 2), I> nb;
    if constexpr (KK > 0) nb.init(s, p, C, b, c, z, y, x);
    const int64_t cell = (((int64_t)b * s.Lc[0] + z) * s.Lc[1] + y) * s.Lc[2] + x;
    const int64_t obase = cell * cst + c;
    const int olo = (int)(uint32_t)obase, ohi = sizeof(I) == 4 ? 0 : (int)(obase >> 32);
    // the lane's output row offsets for the epilogue (every lane active for the shuffle: see
    // linear_mfma_kernel)
    auto store = [&](const bx::f32x4& acc, int k) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = 4 * g + r;
        const int64_t ob = sizeof(I) == 4 ? (int64_t)__shfl(olo, rr, 64)
                                          : (int64_t)(uint32_t)__shfl(olo, rr, 64) | ((int64_t)__shfl(ohi, rr, 64) << 32);
        if (k >= K || tile * 16 + rr >= rows) continue;
        const int64_t o = ob + (int64_t)k * kst;
        out[o] = lin_cast<T>(acc[r]);
        if (out_f32) out_f32[o] = acc[r];
      }
    };
    if constexpr (KK > 0) {
      constexpr int NN = NSP == 3 ? KK * KK * KK : KK * KK;
      // The A fragment depends on (m, g & 1) only, so the two half-waves need the same values:
      // per pair of steps the low half gathers step t, the high half step t + 1, and one
      // permlane32 swap per dword gives every lane both (half the gathers of loading each step
      // in both halves).  Each step's fragment then feeds both column tiles.
      auto feat = [&](int t, int i, int& n) -> I {  // this lane's feature i of step t and its offset
        const int n0 = bx::step_feature(NSP, (KK - 2) / 2, NQ, t, 0, i);
        const int n1 = bx::step_feature(NSP, (KK - 2) / 2, NQ, t, 1, i);
        n = (g & 1) ? n1 : n0;
        return (g & 1) ? nb.at(n1 < NN ? n1 : 0) : nb.at(n0 < NN ? n0 : 0);
      };
      bx::f32x4 acc[NCT0];
#pragma unroll
      for (int ct = 0; ct < NCT0; ++ct) {
        const int k = 16 * ct + m;
        const float bk = k < K ? bias[k] : 0.0f;
        acc[ct] = bx::f32x4{bk, bk, bk, bk};
      }
      auto step = [&](const bx::u32x4& a, int t) {
#pragma unroll
        for (int ct = 0; ct < NCT0; ++ct) {
          const int k = 16 * ct + m;
          if constexpr (BREG) acc[ct] = bx::mfma(a, breg[ct][t], acc[ct]);
          else acc[ct] = bx::mfma(a, bx::b_fragment(W + (k < K ? k : 0), K, N, NSP, p, t, g, k < K), acc[ct]);
        }
      };
      const bool up = g >= 2;
#pragma unroll
      for (int t = 0; t < NQ; t += 2) {
        bx::u32x4 a0, a1;
        if (t + 1 < NQ) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            int nl, nu;
            const I ol = feat(t, i, nl), ou = feat(t + 1, i, nu);
            const int n = up ? nu : nl;
            const uint32_t v = bx::feature_dword((row_ok && n < NN) ? (uint32_t)src[up ? ou : ol] : 0u);
            // lanes 32-63 of the first operand trade with lanes 0-31 of the second
            const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
            a0[i] = r[0];
            a1[i] = r[1];
          }
          step(a0, t);
          step(a1, t + 1);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            int n;
            const I o = feat(t, i, n);
            a0[i] = bx::feature_dword((row_ok && n < NN) ? (uint32_t)src[o] : 0u);
          }
          step(a0, t);
        }
      }
#pragma unroll
      for (int ct = 0; ct < NCT0; ++ct) store(acc[ct], 16 * ct + m);
    } else {
      const int64_t bz = b, zz = z, yy = y, xx = x, cc = c;
      for (int ct = 0; ct < nct; ++ct) {
        const int k = 16 * ct + m;  // this lane's B / D column
        const bool col_ok = k < K;
        const float bk = col_ok ? bias[k] : 0.0f;
        bx::f32x4 acc = {bk, bk, bk, bk};
        for (int t = 0; t < nq; ++t) {  // accumulation steps (kmp_bf16x2.h step_feature)
          bx::u32x4 a;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int n = bx::step_feature(NSP, p, nq, t, g & 1, i);
            const uint32_t v = (row_ok && n < N) ? (uint32_t)lin_feature(src, s, NSP, p, bz, cc, C, zz, yy, xx, n) : 0u;
            a[i] = bx::feature_dword(v);
          }
          acc = bx::mfma(a, bx::b_fragment(W + (col_ok ? k : 0), K, N, NSP, p, t, g, col_ok), acc);
        }
        store(acc, k);
      }
    }
  }
}

// KMP_PRED_LINEAR on the vector ALUs: each thread keeps R = 4 consecutive cells of a row and
// runs the reference's chain for every (cell, k) literally -- acc = b[k]; acc = fmaf(f[n], W[n, k],
// acc) for n = 0, 1, ... -- so it is the oracle's arithmetic by construction, as the f32 MFMA is.
// The weights are staged in LDS per workgroup (broadcast reads); a (dz, dy) row of R + KK - 1
// nodes is read once for the R cells.  The 32 x 32 f32 MFMA tile spent 64 cycles per 2 features x
// 32 outputs (19 or 5 used) and ran latency-bound at ~1 wave of work per tile; this does K fmas per
// feature and cell at 16 lanes a cycle with no fragment traffic.
constexpr int kValuR = 4;

template <typename I>
__device__ __forceinline__ I node_off(const LinSrc& s, int64_t j, int a) {
  if (s.mult == 0) return (I)j;
  if constexpr (sizeof(I) == 4) {
    if (s.simple) {  // one reflection per sym (launch_linear's check)
      const int L = (int)s.L[a], E = (int)s.E[a];
      int v = (int)j;
      v = v < 0 ? -1 - v : (v >= L ? 2 * L - 1 - v : v);
      v = v >= E ? 2 * E - 1 - v : v;
      return (I)(s.mult * v);
    }
  }
  return (I)(s.mult * sym_index(sym_index(j, s.L[a]), s.E[a]));
}

// R consecutive samples as one (unaligned) store
template <typename T, int R>
__device__ __forceinline__ void store_run(T* p, const T (&v)[R]) {
  static_assert(R == 4, "store_run: 4 samples");
  if constexpr (sizeof(T) == 1) {
    typedef uint32_t u32a1 __attribute__((aligned(1)));
    *(u32a1*)p = (uint32_t)v[0] | ((uint32_t)v[1] << 8) | ((uint32_t)v[2] << 16) | ((uint32_t)v[3] << 24);
  } else if constexpr (sizeof(T) == 2) {
    typedef uint32_t u32x2a1 __attribute__((ext_vector_type(2), aligned(1)));
    *(u32x2a1*)p = u32x2a1{(uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2] | ((uint32_t)v[3] << 16)};
  } else {
    typedef uint32_t u32x4a1 __attribute__((ext_vector_type(4), aligned(1)));
    *(u32x4a1*)p = u32x4a1{(uint32_t)v[0], (uint32_t)v[1], (uint32_t)v[2], (uint32_t)v[3]};
  }
}

template <typename T, int NSP, int KK, int KO>
__global__ void __launch_bounds__(256) linear_valu_kernel(const T* __restrict__ src, LinSrc s, LinFlat lf, int p,
                                                          int64_t C, const float* __restrict__ W,
                                                          const float* __restrict__ bias, T* __restrict__ out,
                                                          float* __restrict__ out_f32, int64_t nthreads, int64_t nxq,
                                                          int64_t cst, int64_t kst) {
  constexpr int R = kValuR, NX = R + KK - 1;
  using I = int32_t;
  const I Cc = (I)C, sy = (I)s.S[2] * Cc, sz = (I)s.S[1] * sy;
  const int sh = s.mult ? p : 0;
  const int64_t xend = s.cbeg[2] + s.cext[2];        // cells [cbeg, xend) along x
  const int64_t jmax = xend - 1 - sh + (KK - 1);     // the last node a valid cell reads
  // the weights in LDS: every lane reads the same word (a broadcast); as scalar loads the compiler
  // hoisted a row's KK x KO weights into SGPRs and spilled
  constexpr int NW = (NSP == 3 ? KK * KK * KK : KK * KK) * KO;
  __shared__ float wl[NW];
  for (int i = threadIdx.x; i < NW; i += blockDim.x) wl[i] = W[i];
  __syncthreads();
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < nthreads;
       t += (int64_t)gridDim.x * blockDim.x) {
    // (b, z, y, xq, c), c fastest: the LinFlat of a box whose x extent is nxq groups
    uint32_t u = (uint32_t)t, q;
    q = (__umulhi(u, lf.dC_m) + u) >> lf.dC_s; const I c = (I)(u - q * lf.C); u = q;
    q = (__umulhi(u, lf.d2_m) + u) >> lf.d2_s; const I xq = (I)(u - q * lf.e2); u = q;
    q = (__umulhi(u, lf.d1_m) + u) >> lf.d1_s; const I y = (I)(u - q * lf.e1) + (I)s.cbeg[1]; u = q;
    q = (__umulhi(u, lf.d0_m) + u) >> lf.d0_s; const I z = (I)(u - q * lf.e0) + (I)s.cbeg[0];
    const I b = (I)q;
    const I x0 = (I)s.cbeg[2] + R * xq;
    const I base = b * ((I)s.S[0] * sz) + c;
    I ox[NX], oy[KK], oz[NSP == 3 ? KK : 1];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      int64_t j = (int64_t)x0 - sh + i;
      j = j > jmax ? jmax : j;  // past the box's last cell: any in-range node (not stored)
      ox[i] = node_off<I>(s, j, 2) * Cc;
    }
#pragma unroll
    for (int d = 0; d < KK; ++d) {
      oy[d] = node_off<I>(s, (int64_t)y - sh + d, 1) * sy;
      if constexpr (NSP == 3) oz[d] = node_off<I>(s, (int64_t)z - sh + d, 0) * sz;
    }
    // accumulators as pairs of cells (2r, 2r + 1): one packed fma (v_pk_fma_f32, an IEEE fma per
    // half) per pair, output and feature
    f32x2 acc[R / 2][KO];
#pragma unroll
    for (int k = 0; k < KO; ++k) {
      const float bk = bias[k];
#pragma unroll
      for (int r = 0; r < R / 2; ++r) acc[r][k] = f32x2{bk, bk};
    }
    // one (dz, dy) row of nodes per iteration, in feature order (a runtime loop: the code stays
    // small and the row's loads are the only ones in flight)
    constexpr int NROW = (NSP == 3 ? KK : 1) * KK;
#pragma unroll 1
    for (int row = 0; row < NROW; ++row) {
      const int dz = row / KK, dy = row - dz * KK;
      I zo = NSP == 3 ? oz[0] : 0, yo = oy[0];
#pragma unroll
      for (int d = 1; d < KK; ++d) {
        if constexpr (NSP == 3) zo = dz == d ? oz[d] : zo;
        yo = dy == d ? oy[d] : yo;
      }
      const I rb = base + zo + yo;
      float f[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) f[i] = (float)src[rb + ox[i]];
      f32x2 fp[NX - 1];  // fp[i] = (f[i], f[i + 1]): cells 2r, 2r + 1 at offset dx read fp[2r + dx]
#pragma unroll
      for (int i = 0; i + 1 < NX; ++i) fp[i] = f32x2{f[i], f[i + 1]};
      const float* wr = wl + row * KK * KO;
#pragma unroll
      for (int dx = 0; dx < KK; ++dx) {
#pragma unroll
        for (int k = 0; k < KO; ++k) {
          const float w = wr[dx * KO + k];
#pragma unroll
          for (int r = 0; r < R / 2; ++r)
            acc[r][k] = __builtin_elementwise_fma(fp[2 * r + dx], f32x2{w, w}, acc[r][k]);
        }
      }
    }
    // 32-bit output offsets (launch_linear's i32 condition covers the output array)
    const int ob0 = (int)((((int64_t)b * s.Lc[0] + z) * s.Lc[1] + y) * s.Lc[2] + x0) * (int)cst + c;
    const int ks = (int)kst, cs = (int)cst;
    const int nv = (int)(xend - x0 < R ? xend - x0 : R);  // valid cells of the group
    if (out_f32 == nullptr && cs == 1 && nv == R) {
      // planar, one channel: the R cells of an output are consecutive -- one store
#pragma unroll
      for (int k = 0; k < KO; ++k) {
        T v[R];
#pragma unroll
        for (int r = 0; r < R; ++r) v[r] = lin_cast<T>(acc[r / 2][k][r & 1]);
        store_run<T, R>(out + ob0 + k * ks, v);
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        if (r >= nv) break;
#pragma unroll
        for (int k = 0; k < KO; ++k) {
          const float v = acc[r / 2][k][r & 1];
          out[ob0 + r * cs + k * ks] = lin_cast<T>(v);
          if (out_f32) out_f32[ob0 + r * cs + k * ks] = v;
        }
      }
    }
  }
}

template <typename T>
static int launch_linear(const T* src, const LinSrc& s, int nsp, int p, int64_t B, int64_t C, const float* W,
                         const float* bias, T* out, float* out_f32, hipStream_t stream, int kind = KMP_PRED_LINEAR,
                         bool planar = false) {
  const int k = 2 * p + 2;
  const int N = nsp == 3 ? k * k * k : k * k;
  const int K = nsp == 3 ? 19 : 5;
  const int64_t rows = B * s.cext[0] * s.cext[1] * s.cext[2] * C;
  if (rows == 0) return KMP_OK;
  // preds [B, Lc..., K, C] (kmp_linear_predict), or planar [K, B, Lc..., C] (the generic codec's
  // cells: a map's channel of neighbouring cells is then contiguous)
  const int64_t cst = planar ? C : K * C, kst = planar ? B * s.Lc[0] * s.Lc[1] * s.Lc[2] * C : C;
  // 32-bit rows, source and output offsets when all stay below 2^31
  const int64_t lim = (int64_t)1 << 31;
  const bool i32 = rows < lim && B * s.S[0] * s.S[1] * s.S[2] * C < lim && B * s.Lc[0] * s.Lc[1] * s.Lc[2] * K * C < lim;
  // one reflection per sym for every node index the box can touch: j in [cbeg - p, cbeg + cext + p]
  // within [-L, 2L), and sym(., L) < L <= 2E (else the general sym_index)
  LinSrc sv = s;
  sv.simple = 1;
  for (int a = 3 - nsp; a < 3; ++a)
    if (!(s.cbeg[a] - p >= -s.L[a] && s.cbeg[a] + s.cext[a] + p < 2 * s.L[a] && s.L[a] <= 2 * s.E[a])) sv.simple = 0;
  if (kind == KMP_PRED_LINEAR_MFMA) {
    if constexpr (std::is_same<T, uint8_t>::value || std::is_same<T, uint16_t>::value) {
      // persistent waves, one resident round (the variant's occupancy x CUs): each wave builds its
      // B fragments once (thousands of instructions, the bf16 splits of the weights), so one wave
      // per tile or two spent most of the time there
      const int64_t need = ceil_div(ceil_div(rows, 16), 4);
      const LinFlat lf = make_linflat(s, C);
      auto go = [&](auto nsp_c, auto kk_c, auto i_tag) {
        auto kern = linear_bf16x2_kernel<T, decltype(nsp_c)::value, decltype(kk_c)::value, decltype(i_tag)>;
        static int resident = 0;  // per variant: blocks per CU x CUs
        if (resident == 0) {
          int per_cu = 0, dev = 0, cus = 0;
          if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess || per_cu < 1) per_cu = 2;
          if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1)
            cus = 256;
          resident = per_cu * cus;
        }
        const int64_t blocks = need < resident ? need : resident;
        kern<<<(unsigned)blocks, 256, 0, stream>>>(src, sv, lf, p, B, C, W, bias, N, K, out, out_f32, rows, cst, kst);
      };
      auto with_kk = [&](auto nsp_c, auto i_tag) {
        if (p == 0) go(nsp_c, std::integral_constant<int, 2>{}, i_tag);
        else if (p == 1) go(nsp_c, std::integral_constant<int, 4>{}, i_tag);
        else if (p == 2) go(nsp_c, std::integral_constant<int, 6>{}, i_tag);
        else go(nsp_c, std::integral_constant<int, 0>{}, int64_t{});
      };
      auto with_i = [&](auto nsp_c) {
        if (i32) with_kk(nsp_c, int32_t{});
        else with_kk(nsp_c, int64_t{});
      };
      if (nsp == 3) with_i(std::integral_constant<int, 3>{});
      else with_i(std::integral_constant<int, 2>{});
      return check_launch("linear_bf16x2");
    }
    return fail(KMP_ERR_UNSUPPORTED, "the matrix-core LinearPredictor (bf16x2) takes uint8 / uint16 samples");
  }
  if (i32 && p <= 2 && !opt(OPT_LINEAR_F32_MFMA, 0)) {  // the fma-chain kernel (linear_valu_kernel)
    const int64_t nxq = ceil_div(s.cext[2], (int64_t)kValuR);
    const int64_t nthreads = B * s.cext[0] * s.cext[1] * nxq * C;
    if (nthreads < ((int64_t)1 << 31)) {
      LinSrc sq = s;
      sq.cext[2] = nxq;
      const LinFlat lf = make_linflat(sq, C);
      int64_t blocks = ceil_div(nthreads, 256);
      if (blocks > 65536) blocks = 65536;
      auto go = [&](auto nsp_c, auto kk_c) {
        constexpr int NSP_ = decltype(nsp_c)::value;
        linear_valu_kernel<T, NSP_, decltype(kk_c)::value, NSP_ == 3 ? 19 : 5>
            <<<(unsigned)blocks, 256, 0, stream>>>(src, sv, lf, p, C, W, bias, out, out_f32, nthreads, nxq, cst, kst);
      };
      auto with_kk = [&](auto nsp_c) {
        if (p == 0) go(nsp_c, std::integral_constant<int, 2>{});
        else if (p == 1) go(nsp_c, std::integral_constant<int, 4>{});
        else go(nsp_c, std::integral_constant<int, 6>{});
      };
      if (nsp == 3) with_kk(std::integral_constant<int, 3>{});
      else with_kk(std::integral_constant<int, 2>{});
      return check_launch("linear_valu");
    }
  }
  int64_t waves = ceil_div(rows, 32);
  int64_t blocks = ceil_div(waves, 4);
  if (blocks > 65536) blocks = 65536;
  const LinFlat lf = make_linflat(s, C);
  auto go = [&](auto nsp_c, auto kk_c, auto i_tag) {
    linear_mfma_kernel<T, decltype(nsp_c)::value, decltype(kk_c)::value, decltype(i_tag)>
        <<<(unsigned)blocks, 256, 0, stream>>>(src, sv, lf, p, B, C, W, bias, N, K, out, out_f32, rows, cst, kst);
  };
  auto with_kk = [&](auto nsp_c, auto i_tag) {
    if (p == 0) go(nsp_c, std::integral_constant<int, 2>{}, i_tag);
    else if (p == 1) go(nsp_c, std::integral_constant<int, 4>{}, i_tag);
    else if (p == 2) go(nsp_c, std::integral_constant<int, 6>{}, i_tag);
    else go(nsp_c, std::integral_constant<int, 0>{}, int64_t{});
  };
  auto with_i = [&](auto nsp_c) {
    if (i32) with_kk(nsp_c, int32_t{});
    else with_kk(nsp_c, int64_t{});
  };
  if (nsp == 3) with_i(std::integral_constant<int, 3>{});
  else with_i(std::integral_constant<int, 2>{});
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
                          pred->kind, true);
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
