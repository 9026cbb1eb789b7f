// kmp_wave.h -- register-level helpers shared by the barrier-free wave kernels
// (kmp_codec_wave3d.hip, kmp_codec_wave2d.hip): streaming vector loads / stores, element
// (un)packing of 8- and 16-byte row segments, the padded-node index map, and cross-lane shuffles.
#pragma once

#include "kmp_codec.h"

namespace kmp {
namespace wv {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint4 ld16(const void* p) {
  const u32x4 v = __builtin_nontemporal_load((const u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ld8(const void* p) {
  const u32x2 v = __builtin_nontemporal_load((const u32x2*)p);
  return make_uint2(v.x, v.y);
}
// default-policy loads: for bytes another workgroup re-reads soon (z-halo node rows), which must
// stay in L2 rather than stream past it
__device__ __forceinline__ uint4 ld16c(const void* p) { return *(const uint4*)p; }
__device__ __forceinline__ uint2 ld8c(const void* p) { return *(const uint2*)p; }
__device__ __forceinline__ void st16(void* p, uint4 v) {
  u32x4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, (u32x4*)p);
}
__device__ __forceinline__ void st8(void* p, uint2 v) {
  u32x2 w = {v.x, v.y};
  __builtin_nontemporal_store(w, (u32x2*)p);
}

// STC: a default-policy (MALL-allocating) store, for outputs the next kernel reads; otherwise the
// streaming (non-temporal) st8
template <bool STC>
__device__ __forceinline__ void stp8(void* p, uint2 v) {
  if constexpr (STC) *(uint2*)p = v;
  else st8(p, v);
}

template <typename T>
__device__ __forceinline__ uint32_t el16(const uint4& v, int e) {  // element e of 16 bytes
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  if constexpr (sizeof(T) == 2) return (w[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
  else return (w[e >> 2] >> ((e & 3) * 8)) & 0xffu;
}
template <typename T>
__device__ __forceinline__ uint32_t el8(const uint2& v, int e) {  // element e of 8 bytes
  const uint32_t w[2] = {v.x, v.y};
  if constexpr (sizeof(T) == 2) return (w[e >> 1] >> ((e & 1) * 16)) & 0xffffu;
  else return (w[e >> 2] >> ((e & 3) * 8)) & 0xffu;
}
template <typename T, int VX>
__device__ __forceinline__ uint2 pack8(const uint32_t (&v)[VX]) {
  if constexpr (sizeof(T) == 2) {
    return make_uint2((v[0] & 0xffffu) | (v[1] << 16), (v[2] & 0xffffu) | (v[3] << 16));
  } else {
    return make_uint2((v[0] & 0xffu) | ((v[1] & 0xffu) << 8) | ((v[2] & 0xffu) << 16) | (v[3] << 24),
                      (v[4] & 0xffu) | ((v[5] & 0xffu) << 8) | ((v[6] & 0xffu) << 16) | (v[7] << 24));
  }
}
template <typename T, int VX>
__device__ __forceinline__ uint4 pack16(const uint32_t (&ev)[VX], const uint32_t (&od)[VX]) {  // interleave
  if constexpr (sizeof(T) == 2) {
    return make_uint4((ev[0] & 0xffffu) | (od[0] << 16), (ev[1] & 0xffffu) | (od[1] << 16),
                      (ev[2] & 0xffffu) | (od[2] << 16), (ev[3] & 0xffffu) | (od[3] << 16));
  } else {
    uint32_t w[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
      w[q] = (ev[2 * q] & 0xffu) | ((od[2 * q] & 0xffu) << 8) | ((ev[2 * q + 1] & 0xffu) << 16) | (od[2 * q + 1] << 24);
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// Per-lane 4-cell segments of 8- or 16-bit samples (kernels whose lane owns VX = 4 cells of a row
// for either dtype: kmp_codec_linear3pm.hip, kmp_codec_linear3dp.hip): a highres row segment is the 8
// samples of the cells' two highres columns (16 B for u16, 8 B for u8), a lowres / map segment the 4
// cells (8 B / 4 B); ld*c = default-policy loads, the others streaming.
template <typename T> using HSeg = typename std::conditional<sizeof(T) == 2, uint4, uint2>::type;
template <typename T> using MSeg = typename std::conditional<sizeof(T) == 2, uint2, uint32_t>::type;
template <typename T> __device__ __forceinline__ HSeg<T> ldH(const T* p) {
  if constexpr (sizeof(T) == 2) return ld16(p);
  else return ld8(p);
}
template <typename T> __device__ __forceinline__ HSeg<T> ldHc(const T* p) {
  if constexpr (sizeof(T) == 2) return ld16c(p);
  else return ld8c(p);
}
template <typename T> __device__ __forceinline__ MSeg<T> ldM(const T* p) {
  if constexpr (sizeof(T) == 2) return ld8(p);
  else return __builtin_nontemporal_load((const uint32_t*)p);
}
template <typename T> __device__ __forceinline__ MSeg<T> ldMc(const T* p) {
  if constexpr (sizeof(T) == 2) return ld8c(p);
  else return *(const uint32_t*)p;
}
template <typename T> __device__ __forceinline__ void stH(T* p, const HSeg<T>& v) {
  if constexpr (sizeof(T) == 2) st16(p, v);
  else st8(p, v);
}
template <typename T> __device__ __forceinline__ void stM(T* p, const MSeg<T>& v) {
  if constexpr (sizeof(T) == 2) st8(p, v);
  else __builtin_nontemporal_store(v, (uint32_t*)p);
}
template <typename T> __device__ __forceinline__ uint32_t elH(const HSeg<T>& v, int e) {  // sample e < 8
  if constexpr (sizeof(T) == 2) return el16<T>(v, e);
  else return el8<T>(v, e);
}
template <typename T> __device__ __forceinline__ uint32_t elM(const MSeg<T>& v, int i) {  // cell i < 4
  if constexpr (sizeof(T) == 2) return el8<T>(v, i);
  else return (v >> (8 * i)) & 0xffu;
}
template <typename T> __device__ __forceinline__ MSeg<T> packM(const uint32_t (&v)[4]) {
  if constexpr (sizeof(T) == 2) return pack8<T, 4>(v);
  else return (v[0] & 0xffu) | ((v[1] & 0xffu) << 8) | ((v[2] & 0xffu) << 16) | (v[3] << 24);
}
template <typename T> __device__ __forceinline__ HSeg<T> packH(const uint32_t (&ev)[4], const uint32_t (&od)[4]) {
  if constexpr (sizeof(T) == 2) return pack16<T, 4>(ev, od);
  else
    return make_uint2((ev[0] & 0xffu) | ((od[0] & 0xffu) << 8) | ((ev[1] & 0xffu) << 16) | (od[1] << 24),
                      (ev[2] & 0xffu) | ((od[2] & 0xffu) << 8) | ((ev[3] & 0xffu) << 16) | (od[3] << 24));
}
__device__ __forceinline__ int lsrc1(int r, int L, int E);

__device__ __forceinline__ int lsrc(int r, int L, int E) {
  // stored node index of padded node r along an axis (even reflect pad: node E -> E - 1).  Within one
  // reflection of the axis (-L <= r < 2L, and L <= 2E: m < L <= 2E below) that is lsrc1's
  // division-free form; the integer divisions (VALU reciprocal sequences with quarter-rate multiplies,
  // even for uniform r) run only for indices further out
  if (r >= -L && r < 2 * L && L <= 2 * E) return lsrc1(r, L, E);
  // periodic folds by subtraction, not %: a division's reciprocal setup depends only on L / E, so
  // the compiler hoists it out of this rare branch into every kernel's prologue
  int m = r;
  while (m < 0) m += 2 * L;
  while (m >= 2 * L) m -= 2 * L;
  m = m < L ? m : 2 * L - 1 - m;
  while (m >= 2 * E) m -= 2 * E;
  return m < E ? m : 2 * E - 1 - m;
}

// validity of cells X-1+q (q = 0..VX) for a lane whose VX nodes X..X+VX-1 lie inside the stored
// row (the wave kernels' geometry: Ex = txn * VX).  Since Lc = L - 1 >= E - 1, cells X .. X+VX-2
// always exist: only q = 0 (X = 0) and q = VX (the row's last cell) can be missing -- stated so
// that the compiler keeps 2 lane masks, not VX + 1 (the C3 kernel spilled them to VGPR lanes)
template <int VX>
__device__ __forceinline__ void cells_valid(bool (&vx)[VX + 1], int X, int Lcx) {
#pragma unroll
  for (int q = 0; q <= VX; ++q) vx[q] = q == 0 ? X >= 1 : (q == VX ? X + VX - 1 < Lcx : true);
}

// lsrc for indices within one reflection of the axis (-L <= r < 2L): no integer division
__device__ __forceinline__ int lsrc1(int r, int L, int E) {
  int m = r < 0 ? -1 - r : r;
  m = m >= L ? 2 * L - 1 - m : m;
  return m >= E ? 2 * E - 1 - m : m;
}

// astype(uint8 / uint16) of an f32 (XLA: truncate toward zero, saturate, NaN -> 0):
// v_cvt_u32_f32 truncates and saturates to [0, 2^32-1] with NaN -> 0, then clamp to the dtype
template <typename T>
__device__ __forceinline__ uint32_t cvt_sat(float v) {
  uint32_t u;
  asm("v_cvt_u32_f32 %0, %1" : "=v"(u) : "v"(v));
  constexpr uint32_t hi = sizeof(T) == 2 ? 0xffffu : 0xffu;
  return u < hi ? u : hi;
}

// cvt_sat for a value an MFMA just wrote: the same result from compiler-visible instructions
// (clamp, then an in-range conversion), because the compiler's hazard recognizer does not look
// inside inline asm -- an asm read of an MFMA destination can issue before the result is written
// (seen: linear3dm decode with the asm form read stale accumulators).  fmaxf(NaN, 0) = 0, and
// [0, max] truncates like the saturating conversion.
template <typename T>
__device__ __forceinline__ uint32_t cvt_sat_mfma(float v) {
  constexpr float hi = sizeof(T) == 2 ? 65535.0f : 255.0f;
  return (uint32_t)__builtin_fminf(__builtin_fmaxf(v, 0.0f), hi);
}

// Lane l reads lane l + d (shdn) / l - d (shup); out-of-range lanes keep their own value.  A
// distance known to be 1 after inlining is one DPP move (wave_shl:1 / wave_shr:1, whole-wave
// shifts on CDNA) instead of an LDS-crossbar ds_bpermute with its address computation.
__device__ __forceinline__ uint32_t shdn(uint32_t v, int d) {
  if (__builtin_constant_p(d) && d == 1) return __builtin_amdgcn_update_dpp(v, v, 0x130, 0xf, 0xf, false);
  return (uint32_t)__shfl_down((int)v, d, 64);
}
__device__ __forceinline__ uint32_t shup(uint32_t v, int d) {
  if (__builtin_constant_p(d) && d == 1) return __builtin_amdgcn_update_dpp(v, v, 0x138, 0xf, 0xf, false);
  return (uint32_t)__shfl_up((int)v, d, 64);
}

}  // namespace wv
}  // namespace kmp
