// kmp_categorical.hip -- the categorical rank coder of utils.py:58-111 without a sort.
//
// The reference ranks the logits of each element by ``argsort(pred)[..., ::-1]`` (stable
// ascending argsort, cast to the value dtype, reversed) and codes a value as the index of its
// class in that order.  The descending rank of class i is
//     pos(i) = L - 1 - #{ j : l[j] < l[i]  or  (l[j] == l[i] and j < i) }
// (stability: equal logits keep index order ascending, so reversed the higher index ranks first).
//   encode: min over classes i with (dtype)i == gt of pos(i)   (argmax of the match; 0 if none)
//   decode: the class i with pos(i) == clamp(enc, 0, L-1), cast to the dtype
// One wavefront per element: the 64 lanes stage the element's logits in LDS and each counts a
// 1/64 share of the comparisons, reduced with cross-lane adds.  NaN sorts after every number
// (numpy / XLA argsort order).
#include "kmp_common.h"

namespace kmp {

constexpr int kCatWaves = 4;
constexpr int kCatStage = 1024;  // logits staged in LDS per wave (longer rows read global memory)

__device__ __forceinline__ bool cat_less(float a, float b) {  // a sorts before b
  const bool na = a != a, nb = b != b;
  return (!na && nb) || a < b;
}
__device__ __forceinline__ bool cat_equal(float a, float b) { return a == b || (a != a && b != b); }

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ int64_t class_mod() {  // classes alias modulo 2^bits of the value dtype
  if constexpr (sizeof(T) == 1) return 256;
  else if constexpr (sizeof(T) == 2) return 65536;
  else return (int64_t)1 << 32;
}

template <typename T, int DIR>
__global__ void __launch_bounds__(64 * kCatWaves) categorical_kernel(const float* __restrict__ logits, int64_t n,
                                                                      int64_t L, const T* __restrict__ x,
                                                                      T* __restrict__ out) {
  __shared__ float stage[kCatWaves][kCatStage];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* st = stage[w];
  const bool staged = L <= kCatStage;
  for (int64_t e = (int64_t)blockIdx.x * kCatWaves + w; e < n; e += (int64_t)gridDim.x * kCatWaves) {
    const float* row = logits + e * L;
    if (staged) {
      for (int64_t j = lane; j < L; j += 64) st[j] = row[j];
      __builtin_amdgcn_wave_barrier();
    }
    auto lv = [&](int64_t j) -> float { return staged ? st[j] : row[j]; };
    // ascending stable position of class i, computed by the whole wave
    auto pos_asc = [&](int64_t i) -> int64_t {
      const float li = lv(i);
      int cnt = 0;
      for (int64_t j = lane; j < L; j += 64) {
        const float lj = lv(j);
        cnt += (cat_less(lj, li) || (cat_equal(lj, li) && j < i)) ? 1 : 0;
      }
      return wave_sum(cnt);
    };
    if (DIR == KMP_ENCODE) {
      const int64_t g = (int64_t)(std::is_signed<T>::value ? (int64_t)x[e] : (int64_t)(uint64_t)x[e]);
      int64_t best = -1;
      if (g >= 0)
        for (int64_t i = g; i < L; i += class_mod<T>()) {
          const int64_t p = L - 1 - pos_asc(i);
          best = (best < 0 || p < best) ? p : best;
        }
      if (lane == 0) out[e] = (T)(best < 0 ? 0 : best);
    } else {
      int64_t k = (int64_t)(std::is_signed<T>::value ? (int64_t)x[e] : (int64_t)(uint64_t)x[e]);
      k = k < 0 ? 0 : (k >= L ? L - 1 : k);
      // each lane tests its own candidate classes; exactly one class has descending rank k
      for (int64_t i0 = 0; i0 < L; i0 += 64) {
        const int64_t i = i0 + lane;
        bool hit = false;
        if (i < L) {
          const float li = lv(i);
          int64_t cnt = 0;
          for (int64_t j = 0; j < L; ++j) {
            const float lj = lv(j);
            cnt += (cat_less(lj, li) || (cat_equal(lj, li) && j < i)) ? 1 : 0;
          }
          hit = (L - 1 - cnt) == k;
        }
        if (hit) out[e] = (T)i;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}


// ---- decode by a wave-wide bitonic sort (L <= 64 * E) ----------------------------------------
// The descending rank of class i is #{j : key_j > key_i or (key_j == key_i and j > i)}, i.e. the
// position of the combined 64-bit key (key_i << 32 | i) in DESCENDING order of all combined keys.
// key is the float mapped to an order-preserving uint32 (-0 -> +0, every NaN -> 0xffffffff: NaN
// after every number, NaNs equal -- the cat_less / cat_equal order).  The wave sorts its E
// combined keys per lane (blocked layout, element p = lane * E + e) with a bitonic network --
// in-register compare-exchange for partner distances < E, xor shuffles above -- and reads the
// class at position k.  O(L log^2 L) per element instead of the counting kernel's O(L^2).
__device__ __forceinline__ uint32_t order_key(float f) {
  if (f != f) return 0xffffffffu;
  uint32_t u = __float_as_uint(f == 0.0f ? 0.0f : f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
  const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, 64);
  const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}

template <typename T, int E>
__global__ void __launch_bounds__(64 * kCatWaves) categorical_decode_sort_kernel(const float* __restrict__ logits,
                                                                                int64_t n, int64_t L,
                                                                                const T* __restrict__ x,
                                                                                T* __restrict__ out) {
  constexpr int NE = 64 * E;
  __shared__ uint32_t pos_idx[kCatWaves][NE];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t el = (int64_t)blockIdx.x * kCatWaves + w; el < n; el += (int64_t)gridDim.x * kCatWaves) {
    const float* row = logits + el * L;
    uint64_t v[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = lane * E + e;
      v[e] = i < L ? (((uint64_t)order_key(row[i]) << 32) | (uint32_t)i) : 0ull;  // padding sorts last
    }
    // bitonic network, descending overall
#pragma unroll
    for (int k = 2; k <= NE; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
        if (j < E) {
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int pe = e ^ j;
            if (pe > e) {
              const int p = lane * E + e;
              const bool desc = (p & k) == 0;  // this block sorts descending
              const uint64_t a = v[e], b = v[pe];
              const bool sw = desc ? (a < b) : (a > b);
              v[e] = sw ? b : a;
              v[pe] = sw ? a : b;
            }
          }
        } else {
          const int m = j / E;  // partner lane distance
#pragma unroll
          for (int e = 0; e < E; ++e) {
            const int p = lane * E + e;
            const uint64_t o = shfl_xor64(v[e], m);
            const bool lower = (p & j) == 0;  // p < partner
            const bool desc = (p & k) == 0;
            // keep the larger of the pair at the lower position in a descending block
            const bool keep_max = (lower == desc);
            v[e] = keep_max ? (v[e] > o ? v[e] : o) : (v[e] < o ? v[e] : o);
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < E; ++e) pos_idx[w][lane * E + e] = (uint32_t)v[e];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (lane == 0) {
      int64_t k = (int64_t)(std::is_signed<T>::value ? (int64_t)x[el] : (int64_t)(uint64_t)x[el]);
      k = k < 0 ? 0 : (k >= L ? L - 1 : k);
      out[el] = (T)pos_idx[w][k];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
}

}  // namespace kmp

using namespace kmp;

extern "C" int kmp_categorical(int32_t direction, const float* logits, int64_t n, int64_t L, int32_t dtype,
                               const void* x, void* out, kmp_stream_t stream) {
  KMP_REQUIRE(direction == KMP_ENCODE || direction == KMP_DECODE, "bad direction");
  KMP_REQUIRE(n >= 0 && L >= 1, "bad element or class count");
  if (n == 0) return KMP_OK;
  KMP_REQUIRE(logits && x && out, "null pointer");
  int64_t g = (n + kCatWaves - 1) / kCatWaves;
  const unsigned grid = (unsigned)(g > 65536 ? 65536 : g);
  return dispatch_int_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    if (direction == KMP_ENCODE)
      categorical_kernel<T, KMP_ENCODE><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L, (const T*)x,
                                                                                          (T*)out);
    else if (L <= 64)
      categorical_decode_sort_kernel<T, 1><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else if (L <= 128)
      categorical_decode_sort_kernel<T, 2><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else if (L <= 256)
      categorical_decode_sort_kernel<T, 4><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else if (L <= 512)
      categorical_decode_sort_kernel<T, 8><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else
      categorical_kernel<T, KMP_DECODE><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L, (const T*)x,
                                                                                          (T*)out);
    return check_launch("categorical");
  });
}
