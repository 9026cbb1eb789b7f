// kmp_bf16x2.h -- the LinearPredictor's matrix-core arithmetic (KMP_PRED_LINEAR_MFMA), shared by
// every kernel that evaluates it (kmp_linear.hip: any shape / padding, the callback path and the
// generic codec; kmp_codec_linear3m.hip: the fused p = 0 volume codec), so all of them produce
// bit-identical predictions and a volume encoded by one path decodes losslessly through another.
//
// pred[cell, k] = b[k] + sum_n f_n * W[n, k]  (the north star's 1e-5 FP contract, not the f32
// fma chain of KMP_PRED_LINEAR):
//   * a u8 / u16 feature f = 256 * hi + lo splits into two bf16-exact bytes (hi, lo <= 255);
//   * a weight splits into w1 = bf16(w), w2 = bf16(w - w1) (round to nearest even), so
//     |w - w1 - w2| <= 2^-18 |w|; the hi parts take 256 * w1, 256 * w2 (exact: a power of two);
//   * features are taken in steps of 8; per step ONE v_mfma_f32_16x16x32_bf16 with
//         K = 32 = [hi_0, lo_0, ..., hi_7, lo_7 | the same 16] x [u1 of the step | u2 of the step],
//     accumulated from the bias in step order: acc = b[k]; acc = mfma(A_0, B_0, acc); ...
//     (features past N and padded columns are zeros).  Step t, lane half h, element i takes feature
//     step_feature(nsp, p, t, h, i) of the reference's order (features_from_lowres,
//     volume/utils.py:199-210: n = dz (2p+2)^2 + dy (2p+2) + dx):
//       - the volume p = 1 neighbourhood (4 x 4 x 4 nodes): step t = 2 dy + e holds node row dy of
//         the planes dz = 2 e + h, nodes dx = i -- one node row per step and plane pair, so a kernel
//         walking the node rows of a plane block reads each row's fragment once and applies it to
//         the four cell rows that share it (dy = 0 .. 3 of rows Y .. Y-3; kmp_codec_linear3pm.hip);
//       - every other neighbourhood: 8 consecutive features per chunk q (4 h + i within it), the
//         even chunks first, then the odd ones (chunk_at);
//   * then the sample dtype's truncating, saturating cast (XLA astype).
// Error: <= 2^-18 sum|f w| from the split plus the f32 accumulation inside the MFMA, well within
// 1e-5 of sum|f w| + |b| (tests/test_gpu_linear.py).  An MFMA output element depends only on its
// A row, B column and C value, so the lane / tile position of a cell or channel does not matter.
//
// Fragment maps (cdna_hip_programming.md §3): lane l = 16 g + m holds A[row m][k = 8g + j] and
// B[k = 8g + j][col m], j = 0..7, as 4 dwords of bf16 pairs (element 2i in the low half); C/D:
// col m, rows 4g .. 4g + 3.  So lane group g carries features 4(g & 1) .. 4(g & 1) + 3 of the
// chunk, against u1 (g < 2) or u2 (g >= 2).
#pragma once

#include "kmp_common.h"

namespace kmp {
namespace bx {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// the i-th chunk (of nq) in accumulation order: 0, 2, 4, ..., then 1, 3, 5, ...
__host__ __device__ constexpr int chunk_at(int i, int nq) {
  return i < (nq + 1) / 2 ? 2 * i : 2 * (i - (nq + 1) / 2) + 1;
}

// the feature (reference order) of accumulation step t (of nq = ceil(N / 8)), lane half h, element i
__host__ __device__ constexpr int step_feature(int nsp, int p, int nq, int t, int h, int i) {
  return (nsp == 3 && p == 1) ? (2 * (t & 1) + h) * 16 + (t >> 1) * 4 + i : 8 * chunk_at(t, nq) + 4 * h + i;
}

// f32 -> bf16 bits, round to nearest even (NaN stays NaN)
__host__ __device__ __forceinline__ uint32_t bf16_rne(float f) {
  uint32_t u;
  __builtin_memcpy(&u, &f, 4);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
__host__ __device__ __forceinline__ float bf16_f32(uint32_t h) {
  const uint32_t u = h << 16;
  float f;
  __builtin_memcpy(&f, &u, 4);
  return f;
}

// The two bf16 terms of a weight, part = 0 / 1, and the hi-byte feature's scaled copy (hi = 1).
__host__ __device__ __forceinline__ uint32_t weight_part(float w, int part, int hi) {
  const uint32_t w1 = bf16_rne(w);
  const uint32_t v = part == 0 ? w1 : bf16_rne(w - bf16_f32(w1));
  return hi ? bf16_rne(bf16_f32(v) * 256.0f) : v;
}

// A feature's fragment dword: bf16(hi) in the low half, bf16(lo) in the high half.  For a byte b,
// f32(b)'s upper half IS bf16(b) (8 significant bits at most).
__device__ __forceinline__ uint32_t feature_dword(uint32_t v) {
  const uint32_t fh = __float_as_uint((float)(v >> 8)), fl = __float_as_uint((float)(v & 0xffu));
  return __builtin_amdgcn_perm(fl, fh, 0x07060302u);  // {fh[31:16], fl[31:16]} -> low, high
}

// B fragment of accumulation step t for the lane of group g, column weights Wcol[n * ldw] (n < N,
// else 0): element j of K = 8g + j -> feature step_feature(nsp, p, nq, t, g & 1, j >> 1), byte j & 1
// (0 = hi), term g >> 1
__device__ __forceinline__ u32x4 b_fragment(const float* Wcol, int ldw, int N, int nsp, int p, int t, int g,
                                            bool valid) {
  const int nq = (N + 7) / 8;
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int n = step_feature(nsp, p, nq, t, g & 1, i);
    const float w = (valid && n < N) ? Wcol[(int64_t)n * ldw] : 0.0f;
    r[i] = weight_part(w, g >> 1, 1) | (weight_part(w, g >> 1, 0) << 16);
  }
  return r;
}

__device__ __forceinline__ f32x4 mfma(const u32x4& a, const u32x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0,
                                                 0, 0);
}

// 4 MFMA results -> 4 samples of T (u8 / u16) packed little-endian in the low 4 * sizeof(T) bytes,
// with the sample dtype's cast (XLA astype: truncate, NaN and negatives 0, saturate), clamped to
// [0, hi] first (hi = the dtype's maximum, or 0 for a result the caller wants zeroed): v_med3_f32
// takes NaN to min3 = 0, so the float -> u32 conversion only ever sees in-range values (defined
// C++; the same values as cast_f32 in kmp_common.h)
template <typename T>
__device__ __forceinline__ uint2 cast_pack4(const f32x4& v, float hi) {
  uint32_t u[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) u[j] = (uint32_t)__builtin_amdgcn_fmed3f(v[j], 0.0f, hi);
  if constexpr (sizeof(T) == 2) {
    return make_uint2(u[0] | (u[1] << 16), u[2] | (u[3] << 16));
  } else {
    return make_uint2(u[0] | (u[1] << 8) | (u[2] << 16) | (u[3] << 24), 0u);
  }
}

// u16 without a clamp instruction: v_cvt_u32_f32 (truncates; NaN and negatives 0; saturates) and
// v_cvt_pk_u16_u32 (saturates to 65535) are XLA's astype to uint16 exactly -- 6 instead of 10 VALU
// per 4 samples.  The conversion is inline asm because a C++ float -> unsigned conversion of an
// out-of-range value is undefined; the asm reads an MFMA's D, a hazard hipcc does not pad inside an
// asm string: s_nop 7 = the 8 wait states of a 4-pass XDL write -> VALU read on gfx950 (the
// 16-cycle v_mfma_f32_16x16x32_bf16; an 8-pass one needs 12)
__device__ __forceinline__ uint2 cast_pack4_u16(const f32x4& v) {
  uint32_t u0, u1, u2, u3;
  asm("s_nop 7\n\tv_cvt_u32_f32 %0, %4\n\tv_cvt_u32_f32 %1, %5\n\tv_cvt_u32_f32 %2, %6\n\tv_cvt_u32_f32 %3, %7"
      : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
  return make_uint2(__builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_u16(u0, u1)),
                    __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_u16(u2, u3)));
}

// the same without the hazard pad, for a caller that has issued at least 8 other MFMAs (each at least
// one wait state) since the last MFMA writing ``v``, with a scheduling barrier in between so the
// compiler cannot move this above them
__device__ __forceinline__ uint2 cast_pack4_u16_late(const f32x4& v) {
  uint32_t u0, u1, u2, u3;
  asm("v_cvt_u32_f32 %0, %4\n\tv_cvt_u32_f32 %1, %5\n\tv_cvt_u32_f32 %2, %6\n\tv_cvt_u32_f32 %3, %7"
      : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
  return make_uint2(__builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_u16(u0, u1)),
                    __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_u16(u2, u3)));
}

// u8 (XLA astype(uint8)) into the u16 channel table: the same saturating conversions, then one packed
// min with 255 -- 7 instead of 10 VALU per 4 samples (cast_pack4<uint16_t>(v, 255.f): med3 + cvt each)
typedef unsigned short bx_u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 cast_pack4_u8_tab(uint32_t u0, uint32_t u1, uint32_t u2, uint32_t u3) {
  const bx_u16x2 lim = {255, 255};
  const bx_u16x2 a = __builtin_bit_cast(bx_u16x2, __builtin_amdgcn_cvt_pk_u16(u0, u1));
  const bx_u16x2 b = __builtin_bit_cast(bx_u16x2, __builtin_amdgcn_cvt_pk_u16(u2, u3));
  return make_uint2(__builtin_bit_cast(uint32_t, __builtin_elementwise_min(a, lim)),
                    __builtin_bit_cast(uint32_t, __builtin_elementwise_min(b, lim)));
}
__device__ __forceinline__ uint2 cast_pack4_u8(const f32x4& v) {
  uint32_t u0, u1, u2, u3;
  asm("s_nop 7\n\tv_cvt_u32_f32 %0, %4\n\tv_cvt_u32_f32 %1, %5\n\tv_cvt_u32_f32 %2, %6\n\tv_cvt_u32_f32 %3, %7"
      : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
  return cast_pack4_u8_tab(u0, u1, u2, u3);
}
__device__ __forceinline__ uint2 cast_pack4_u8_late(const f32x4& v) {
  uint32_t u0, u1, u2, u3;
  asm("v_cvt_u32_f32 %0, %4\n\tv_cvt_u32_f32 %1, %5\n\tv_cvt_u32_f32 %2, %6\n\tv_cvt_u32_f32 %3, %7"
      : "=&v"(u0), "=&v"(u1), "=&v"(u2), "=&v"(u3)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
  return cast_pack4_u8_tab(u0, u1, u2, u3);
}

}  // namespace bx
}  // namespace kmp
