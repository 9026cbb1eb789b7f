// kmp_bits.h -- register-level bit machinery shared by the container kernels (kmp_pack.hip: the
// fixed-width bit-plane format, kmp_rice.hip: the block-adaptive Rice format).  A lane owns 8
// consecutive W-bit samples (one 8 / 16 / 32-byte load), 8 lanes a 64-sample block, a wave step
// 8 blocks.  Bit-planes are formed without ballots: 8x8 bit transposes in registers per sample
// byte, then an 8x8 BYTE transpose across the block's 8 lanes (DPP), after which lane j holds the
// 64-bit planes 8p + j.
#pragma once

#include "kmp_common.h"

namespace kmp {
namespace pk {

constexpr int kBlock = 64;         // samples per block == lanes per wave
constexpr int kChunk = 1024;       // blocks per scan chunk (256 chunks for a 32 MiB u16 map)
constexpr int kScanThreads = 256;  // 4 blocks per thread

template <int W>
__device__ __forceinline__ uint32_t zigzag(uint32_t v) {
  if constexpr (W == 32) {
    const int32_t s = (int32_t)v;
    return (uint32_t)((s << 1) ^ (s >> 31));
  } else {
    const int32_t s = (int32_t)(v << (32 - W)) >> (32 - W);  // sign-extend the W-bit sample
    return (uint32_t)((s << 1) ^ (s >> 31)) & ((1u << W) - 1u);
  }
}
template <int W>
__device__ __forceinline__ uint32_t unzigzag(uint32_t z) {
  const uint32_t v = (z >> 1) ^ (0u - (z & 1u));
  if constexpr (W == 32) return v;
  else return v & ((1u << W) - 1u);
}

template <int W>
__device__ __forceinline__ uint32_t load_sample(const void* x, int64_t i) {
  if constexpr (W == 8) return ((const uint8_t*)x)[i];
  else if constexpr (W == 16) return ((const uint16_t*)x)[i];
  else return ((const uint32_t*)x)[i];
}
template <int W>
__device__ __forceinline__ void store_sample(void* x, int64_t i, uint32_t v) {
  if constexpr (W == 8) ((uint8_t*)x)[i] = (uint8_t)v;
  else if constexpr (W == 16) ((uint16_t*)x)[i] = (uint16_t)v;
  else ((uint32_t*)x)[i] = v;
}

// ---- lane layout: 8 consecutive samples per lane, 8 lanes per block, 8 blocks per wave step ----
// A lane's 8 samples are W/4 32-bit words (2, 4 or 8).  Planes are formed without ballots: the
// lane's samples are bit-transposed in registers (8x8 bit transposes, one per sample byte), which
// gives, per 8-plane group p, the byte of planes 8p .. 8p+7 this lane contributes (bit k = its
// sample k); an 8x8 BYTE transpose across the block's 8 lanes (DPP) then leaves lane j holding the
// whole 64-bit plane 8p+j.  Zigzag is applied in the plane domain (z-plane 0 = the sign plane,
// z-plane b = s-plane b-1 ^ sign plane).  About 12 VALU instructions per block for 16-bit samples,
// against ~80 for one ballot per plane.
template <int W>
struct Sw {
  static constexpr int NW = W / 4;  // 32-bit words per lane (8 samples)
  static constexpr int NP = W / 8;  // 8-plane groups (64-bit words as lo / hi)
};
typedef uint32_t u32x2a1 __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32x4a1 __attribute__((ext_vector_type(4), aligned(1)));

template <int W>
__device__ __forceinline__ void load8s(const void* x, int64_t n, int64_t i0, uint32_t (&w)[Sw<W>::NW]) {
  const char* p = (const char*)x + i0 * (W / 8);
  if (i0 + 8 <= n) {
    if constexpr (W == 8) {
      const u32x2a1 v = *(const u32x2a1*)p;
      w[0] = v[0]; w[1] = v[1];
    } else {
#pragma unroll
      for (int q = 0; q < W / 16; ++q) {
        const u32x4a1 v = *(const u32x4a1*)(p + 16 * q);
        w[4 * q] = v[0]; w[4 * q + 1] = v[1]; w[4 * q + 2] = v[2]; w[4 * q + 3] = v[3];
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < Sw<W>::NW; ++k) w[k] = 0u;
  for (int e = 0; e < 8; ++e) {
    if (i0 + e >= n) break;
    w[(e * W) / 32] |= load_sample<W>(x, i0 + e) << ((e * W) % 32);
  }
}
template <int W>
__device__ __forceinline__ void store8s(void* x, int64_t n, int64_t i0, const uint32_t (&w)[Sw<W>::NW]) {
  char* p = (char*)x + i0 * (W / 8);
  if (i0 + 8 <= n) {
    if constexpr (W == 8) {
      *(u32x2a1*)p = u32x2a1{w[0], w[1]};
    } else {
#pragma unroll
      for (int q = 0; q < W / 16; ++q) *(u32x4a1*)(p + 16 * q) = u32x4a1{w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]};
    }
    return;
  }
  for (int e = 0; e < 8; ++e) {
    if (i0 + e >= n) break;
    const uint32_t v = W == 32 ? w[e] : (w[(e * W) / 32] >> ((e * W) % 32)) & ((1u << (W & 31)) - 1u);
    store_sample<W>(x, i0 + e, v);
  }
}

__device__ __forceinline__ uint32_t perm(uint32_t hi, uint32_t lo, uint32_t sel) {  // bytes 0-3 lo, 4-7 hi
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// 8x8 bit transpose of the 64-bit (lo, hi): bit 8r + c <-> bit 8c + r
__device__ __forceinline__ void tr8x8(uint32_t& lo, uint32_t& hi) {
  uint32_t t;
  t = (lo ^ (lo >> 7)) & 0x00AA00AAu; lo ^= t ^ (t << 7);
  t = (hi ^ (hi >> 7)) & 0x00AA00AAu; hi ^= t ^ (t << 7);
  t = (lo ^ (lo >> 14)) & 0x0000CCCCu; lo ^= t ^ (t << 14);
  t = (hi ^ (hi >> 14)) & 0x0000CCCCu; hi ^= t ^ (t << 14);
  t = (lo ^ (hi << 4)) & 0xF0F0F0F0u; lo ^= t; hi ^= t >> 4;
}

// samples -> X[p] (byte k = byte p of sample k) and back
template <int W>
__device__ __forceinline__ void gather_bytes(const uint32_t (&w)[Sw<W>::NW], uint32_t (&X)[Sw<W>::NP][2]) {
  if constexpr (W == 8) {
    X[0][0] = w[0]; X[0][1] = w[1];
  } else if constexpr (W == 16) {
    X[0][0] = perm(w[1], w[0], 0x06040200u); X[0][1] = perm(w[3], w[2], 0x06040200u);
    X[1][0] = perm(w[1], w[0], 0x07050301u); X[1][1] = perm(w[3], w[2], 0x07050301u);
  } else {
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
      for (int h = 0; h < 2; ++h)
        X[p][h] = perm(w[4 * h + 1], w[4 * h], 0x0c0c0000u | ((4u + p) << 8) | p) |
                  perm(w[4 * h + 3], w[4 * h + 2], ((4u + p) << 24) | ((uint32_t)p << 16) | 0x0c0cu);
  }
}
template <int W>
__device__ __forceinline__ void scatter_bytes(const uint32_t (&X)[Sw<W>::NP][2], uint32_t (&w)[Sw<W>::NW]) {
  if constexpr (W == 8) {
    w[0] = X[0][0]; w[1] = X[0][1];
  } else if constexpr (W == 16) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      w[2 * h] = perm(X[1][h], X[0][h], 0x05010400u);
      w[2 * h + 1] = perm(X[1][h], X[0][h], 0x07030602u);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int h = k >> 2, b = k & 3;
      w[k] = perm(X[1][h], X[0][h], 0x0c0c0000u | ((4u + b) << 8) | b) |
             perm(X[3][h], X[2][h], ((4u + b) << 24) | ((uint32_t)b << 16) | 0x0c0cu);
    }
  }
}

template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  // bound_ctrl: a read past the row gives 0 (no copy of the old value; the move can fold into its
  // consumer).  Every caller discards the lanes whose source lies past the row
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, true);
}

// 8x8 BYTE transpose across lanes j = lane & 7 (row j = the lane's (lo, hi)): afterwards lane j
// holds column j.  Three exchange stages (lane distance 4, 2, 1), each swapping the off-diagonal
// sub-blocks: lanes with bit d clear keep columns with bit d clear and take the partner's.
__device__ __forceinline__ void xtr8(uint32_t& lo, uint32_t& hi, int j) {
  {  // d = 4: 32-bit halves (row_shl:4 reads lane l+4, row_shr:4 lane l-4; both stay in the 8)
    const uint32_t up = dpp<0x104>(lo), dn = dpp<0x114>(hi);
    if (j & 4) lo = dn;
    else hi = up;
  }
  {  // d = 2: 16-bit units (quad_perm [2,3,0,1])
    const bool odd = j & 2;
    const uint32_t recv = dpp<0x4E>(perm(hi, lo, odd ? 0x05040100u : 0x07060302u));
    lo = perm(recv, lo, odd ? 0x03020504u : 0x05040100u);
    hi = perm(recv, hi, odd ? 0x03020706u : 0x07060100u);
  }
  {  // d = 1: bytes (quad_perm [1,0,3,2])
    const bool odd = j & 1;
    const uint32_t recv = dpp<0xB1>(perm(hi, lo, odd ? 0x06040200u : 0x07050301u));
    lo = perm(recv, lo, odd ? 0x03050104u : 0x05020400u);
    hi = perm(recv, hi, odd ? 0x03070106u : 0x07020600u);
  }
}


struct Ws {  // workspace carve-up of a block-size scan
  uint32_t* local;
  uint64_t* sums;
  uint64_t* cbase;
  uint64_t* total;
};
Ws carve(void* ws, int64_t nb);
// exclusive scan of per-block sizes (uint8) into Ws.local / Ws.cbase; the total at Ws.total
int scan(const uint8_t* sizes, int64_t nb, const Ws& w, hipStream_t s);
// a wave step = 8 blocks, 4 waves per workgroup
unsigned waves_grid(int64_t nb);
int sample_bits(int dtype);

}  // namespace pk
}  // namespace kmp
