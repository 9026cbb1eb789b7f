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
constexpr uint32_t kCatSmallRank = 8;  // decode: ranks below this peel maxima instead of a radix select

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


// ---- decode by a wave-wide radix select (L <= 64 * E) -----------------------------------------
// The descending rank of class i is #{j : key_j > key_i or (key_j == key_i and j > i)}, where key
// is the float mapped to an order-preserving uint32 (-0 -> +0, every NaN -> 0xffffffff: NaN after
// every number, NaNs equal -- the cat_less / cat_equal order).  Lane l holds classes e * 64 + l.
// The class of rank k: the largest threshold T with #{key >= T} >= k + 1, found bit by bit from
// the top (32 rounds of E ballots + popcounts), is the (k+1)-th largest key; among the classes
// with key == T the answer is the (k - #{key > T})-th highest index.  O(32 E) per element instead
// of a sorting network's O(L log^2 L).
__device__ __forceinline__ uint32_t order_key(float f) {
  if (f != f) return 0xffffffffu;
  uint32_t u = __float_as_uint(f == 0.0f ? 0.0f : f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <typename T, int E>
__global__ void __launch_bounds__(64 * kCatWaves) categorical_decode_select_kernel(const float* __restrict__ logits,
                                                                                  int64_t n, int64_t L,
                                                                                  const T* __restrict__ x,
                                                                                  T* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int64_t el = (int64_t)blockIdx.x * kCatWaves + w; el < n; el += (int64_t)gridDim.x * kCatWaves) {
    const float* row = logits + el * L;
    uint32_t key[E];
    bool ok[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int i = e * 64 + lane;
      ok[e] = i < L;
      key[e] = ok[e] ? order_key(row[i]) : 0u;
    }
    int64_t kk = (int64_t)(std::is_signed<T>::value ? (int64_t)x[el] : (int64_t)(uint64_t)x[el]);
    const uint32_t k = (uint32_t)(kk < 0 ? 0 : (kk >= L ? L - 1 : kk));
    auto count = [&](auto pred) {  // wave-uniform #{valid classes with pred(key)}
      uint32_t c = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) c += __popcll(__ballot(ok[e] && pred(key[e])));
      return c;
    };
    uint32_t t = 0, m = 0;
    if (k < kCatSmallRank) {
      // small ranks (a good predictor's usual case): peel the k + 1 largest keys one at a time;
      // t = the (k+1)-th largest key, m = how many classes with key t rank before the answer
      uint64_t above = 1ull << 32;   // keys >= above are used up
      uint32_t taken = 0;            // classes peeled so far
      while (true) {
        uint32_t best = 0;
        bool any = false;
#pragma unroll
        for (int e = 0; e < E; ++e)
          if (ok[e] && (uint64_t)key[e] < above) { best = key[e] > best || !any ? key[e] : best; any = true; }
        const bool lane_any = any;
        uint32_t wmax = lane_any ? best : 0u;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) wmax = max(wmax, (uint32_t)__shfl_xor((int)wmax, off, 64));
        const uint32_t ties = count([&](uint32_t v) { return v == wmax; });
        if (taken + ties > k) {
          t = wmax;
          m = k - taken;
          break;
        }
        taken += ties;
        above = wmax;
      }
    } else {
#pragma unroll 4
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t cand = t | (1u << bit);
        if (count([&](uint32_t v) { return v >= cand; }) >= k + 1) t = cand;
      }
      m = k - count([&](uint32_t v) { return v > t; });
    }
    int64_t cls = 0;
#pragma unroll
    for (int e = E - 1; e >= 0; --e) {  // m-th highest class index with key == t
      uint64_t word = __ballot(ok[e] && key[e] == t);
      const uint32_t c = (uint32_t)__popcll(word);
      if (m < c) {
        for (uint32_t s = 0; s < m; ++s) word &= ~(1ull << (63 - __clzll(word)));
        cls = e * 64 + (63 - __clzll(word));
        break;
      }
      m -= c;
    }
    if (lane == 0) out[el] = (T)cls;
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
      categorical_decode_select_kernel<T, 1><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else if (L <= 128)
      categorical_decode_select_kernel<T, 2><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else if (L <= 256)
      categorical_decode_select_kernel<T, 4><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else if (L <= 512)
      categorical_decode_select_kernel<T, 8><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L,
                                                                                             (const T*)x, (T*)out);
    else
      categorical_kernel<T, KMP_DECODE><<<grid, 64 * kCatWaves, 0, (hipStream_t)stream>>>(logits, n, L, (const T*)x,
                                                                                          (T*)out);
    return check_launch("categorical");
  });
}
