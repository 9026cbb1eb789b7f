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
#include <cstdlib>

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


// ---- 16-byte vector form (L % 4 == 0, L <= 256 * E4, rows 16-B aligned) -----------------------
// Lane l holds classes s * 256 + 4 l + q (q = 0..3) of slot s as one float4: one 16-B load per lane
// and slot instead of four 4-B loads; classes past L are loaded as NaN.  Each wave walks one
// contiguous range of elements (loop control and addressing on the scalar unit) with a ring of
// kCatPF rows -- and their values, in a VGPR -- in registers, refilling a slot as soon as it is
// ranked.  (A value read as a uniform scalar load was waited out at the load: every element paid a
// memory latency, 260 / 390 us per 1 M x 256 encode / decode; with the value in the ring 190 /
// 380 us.)  Instruction issue per element is what bounds this kernel, so:
//   encode: #{j : l_j < l_i, or l_j == l_i and j < i} from two float compares per class (NaN rows
//   of the reference order handled by a uniform branch; padding NaNs never count), the j < i part
//   as a scalar lane mask.
//   decode: order_key integers; rank 0 by one wave max; otherwise a 256-bin histogram (LDS
//   atomics) of the 8 highest bits in which the keys differ (DPP OR-reduce), a DPP prefix scan
//   over the bins to pick the one that holds rank k (its lane by one ballot, the bin inside the
//   lane on the scalar unit), and a bitwise radix select inside that bin, stopping as soon as the
//   key range [t, hi) that holds rank k contains one key.  Then the m-th highest class index with
//   a key in [t, hi) -- when the last bin holds one key, its class straight from the bin's
//   owner slot (written beside the histogram), otherwise from ballots.  Ranks and ranges are 32-bit
//   scalar arithmetic throughout (VALU issue is the bound: r3 SQ counters, 130 VALU per element).
constexpr int kCatPF = 4;  // 8 measured no faster (r3s54: decode 394-397 vs 376-385 us)
// Decode ranks below kCatPeel take k + 1 wave max-reductions (~20 VALU each) instead of the radix
// select (a histogram round is ~35 VALU, one to three rounds per element): a good predictor's ranks
// (bench_rows decode_small_ranks, ranks < 4) stay on the peel.
constexpr int kCatPeel = 4;
// per wave: the 256 bins, then the owner slots (bins[kCatOwn + d])
constexpr int kCatOwn = 320;
typedef float cat_f32x4 __attribute__((ext_vector_type(4)));

template <int E4>
struct CatRow {
  cat_f32x4 v[E4];
  uint32_t xv;  // the element's value (gt / enc), raw 32-bit pattern, in a VGPR
};

// Rows and values are read through buffer resources over the wave's range (soffset = the element's
// byte offset, on the scalar unit; voffset = the lane's constant offset), so no per-element
// address arithmetic runs on the VALU, whose issue bounds this kernel.  The value is read as the
// aligned dword that holds it (cat_xval shifts it out when the element is ranked), through a
// divergent zero voffset (zero0 below): a wave-uniform load would be moved to a scalar register
// and waited out right at the load instead of when the element is ranked PF elements later.
template <typename T, int E4, bool FULL>
__device__ __forceinline__ void cat_load(__amdgpu_buffer_rsrc_t rows, uint32_t roff, __amdgpu_buffer_rsrc_t xs,
                                         uint32_t xoff, int64_t L, int lane, uint32_t zero0, CatRow<E4>& r) {
  const float qnan = __builtin_nanf("");
#pragma unroll
  for (int s = 0; s < E4; ++s) {
    const int c4 = s * 64 + lane;
    r.v[s] = FULL || 4 * c4 < L
                 ? __builtin_bit_cast(cat_f32x4, __builtin_amdgcn_raw_buffer_load_b128(rows, (uint32_t)c4 * 16u, roff, 2))
                 : (cat_f32x4){qnan, qnan, qnan, qnan};
  }
  r.xv = __builtin_amdgcn_raw_buffer_load_b32(xs, zero0, xoff, 0);
}
template <typename T>
__device__ __forceinline__ int64_t cat_xval(const T* xe, uint32_t word) {  // xe: the element's value
  if constexpr (sizeof(T) == 4) {
    return std::is_signed<T>::value ? (int64_t)(int32_t)word : (int64_t)word;
  } else {
    static_assert(!std::is_signed<T>::value, "sub-dword value dtypes are unsigned");
    const uint32_t sh = (uint32_t)((uintptr_t)xe & 3) * 8;
    return (int64_t)((word >> sh) & ((1u << (8 * sizeof(T))) - 1));
  }
}

// DPP steps (row_shr:1,2,4,8 inside rows of 16, then row_bcast:15 / row_bcast:31 across rows):
// an inclusive scan over the 64 lanes; lane 63 holds the whole-wave reduction.
template <typename Op>
__device__ __forceinline__ uint32_t wave_scan_dpp(uint32_t x, uint32_t id, Op op) {
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x111, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x112, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x114, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x118, 0xf, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x142, 0xa, 0xf, false));
  x = op(x, (uint32_t)__builtin_amdgcn_update_dpp((int)id, (int)x, 0x143, 0xc, 0xf, false));
  return x;
}
__device__ __forceinline__ uint32_t wave_max_dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane(
      (int)wave_scan_dpp(x, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; }), 63);
}
__device__ __forceinline__ uint32_t wave_or_dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_dpp(x, 0u, [](uint32_t a, uint32_t b) { return a | b; }), 63);
}

__device__ __forceinline__ uint32_t order_key_fast(float f) {  // == order_key
  const float z = f + 0.0f;  // -0 -> +0 (round to nearest), NaN stays NaN
  const uint32_t u = __float_as_uint(z);
  const uint32_t k = u ^ ((uint32_t)((int32_t)u >> 31) | 0x80000000u);
  return z != z ? 0xffffffffu : k;
}

// max(a - b, 0) on the scalar unit (the compiler's form is a clamped VALU subtract and a readback)
__device__ __forceinline__ int s_floor_sub(int a, int b) {
  int r;
  asm("s_sub_i32 %0, %1, %2\n\ts_max_i32 %0, %0, 0" : "=&s"(r) : "s"(a), "s"(b) : "scc");
  return r;
}

__device__ __forceinline__ uint64_t lanes_below(int nl) {  // mask of lanes 0 .. nl-1
  return nl <= 0 ? 0ull : nl >= 64 ? ~0ull : ((1ull << nl) - 1);
}

// ---- decode: keys, rank, radix select ----------------------------------------------------------
// Every logit in [+0, +inf] (softmax output, the reference's categorical predictor): the float bits
// are already order-preserving -- no work per key when every class exists (FULL), + 1 to keep key 0
// for padding otherwise -- instead of order_key's six operations.  -0, negatives and NaN (bits
// above +inf) take order_key.  lmax: the lane's largest key.
template <int E4, bool FULL>
__device__ __forceinline__ void cat_dec_keys(const CatRow<E4>& cur, int64_t L, int lane, uint32_t (&key)[E4][4],
                                             bool (&ok)[E4][4], uint32_t& lmax) {
  uint32_t mx = 0;
#pragma unroll
  for (int s = 0; s < E4; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      ok[s][q] = FULL || s * 256 + 4 * lane + q < L;
      mx = max(mx, ok[s][q] ? __float_as_uint(cur.v[s][q]) : 0u);
    }
  if (__ballot(mx > 0x7f800000u) == 0) {  // wave-uniform
#pragma unroll
    for (int s = 0; s < E4; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        key[s][q] = FULL ? __float_as_uint(cur.v[s][q]) : ok[s][q] ? __float_as_uint(cur.v[s][q]) + 1u : 0u;
    lmax = FULL ? mx : mx + 1u;  // (an empty lane's 1 is below the wave's largest valid key)
  } else {
    lmax = 0;
#pragma unroll
    for (int s = 0; s < E4; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        key[s][q] = ok[s][q] ? order_key_fast(cur.v[s][q]) : 0u;  // padding keys 0
        lmax = max(lmax, key[s][q]);
      }
  }
}

// the rank, clamped to [0, L) in 32-bit scalar arithmetic (xv holds a T value; L <= 512 here)
template <typename T>
__device__ __forceinline__ uint32_t cat_dec_k(int64_t xv, int64_t L) {
  const uint32_t k = std::is_signed<T>::value ? (uint32_t)max((int32_t)xv, 0) : (uint32_t)xv;
  return min(k, (uint32_t)L - 1u);
}

// the lane's OR of (key ^ k0) over its valid keys: the wave's OR has its top bit where keys first differ
template <int E4>
__device__ __forceinline__ uint32_t cat_dif(const uint32_t (&key)[E4][4], const bool (&ok)[E4][4], uint32_t k0) {
  uint32_t dif = 0;
#pragma unroll
  for (int s = 0; s < E4; ++s)
#pragma unroll
    for (int q = 0; q < 4; ++q) dif |= ok[s][q] ? key[s][q] ^ k0 : 0u;
  return dif;
}

// the m-th highest class index among the keys whose ballots are w (ties: lanes from the highest,
// within a lane q from 3 down)
template <int E4>
__device__ __forceinline__ int cat_dec_walk(const uint64_t (&w)[E4][4], uint32_t m) {
#pragma unroll
  for (int s = E4 - 1; s >= 0; --s) {
    uint32_t tot = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) tot += (uint32_t)__popcll(w[s][q]);
    if (m >= tot) {
      m -= tot;
      continue;
    }
    if (tot == 1u) {  // one key: its lane and slot, no walk
      int c = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) c = w[s][q] ? 4 * __builtin_ctzll(w[s][q]) + q : c;
      return s * 256 + c;
    }
    uint64_t lanes = w[s][0] | w[s][1] | w[s][2] | w[s][3];
    while (true) {
      const int l = 63 - __clzll(lanes);
      int q = 3;
      for (; q >= 0; --q)
        if ((w[s][q] >> l) & 1) {
          if (m == 0) break;
          --m;
        }
      if (q >= 0) return s * 256 + 4 * l + q;
      lanes &= ~(1ull << l);
    }
  }
  return 0;
}

template <typename T, int DIR, int E4, bool FULL>
__device__ __forceinline__ T cat_rank(const CatRow<E4>& cur, int64_t L, int lane, uint32_t* bins,
                                      int64_t xv) {  // the element's code (wave-uniform)
  if constexpr (DIR == KMP_ENCODE) {
    const int64_t g = xv;
    int64_t best = -1;
    if (g >= 0)
      for (int64_t i = g; i < L; i += class_mod<T>()) {
        const int ii = (int)i, si = ii >> 8, ln = (ii & 255) >> 2, qi = ii & 3;
        float fv = 0.f;
#pragma unroll
        for (int ss = 0; ss < E4; ++ss)
          if (ss == si) fv = qi == 0 ? cur.v[ss].x : qi == 1 ? cur.v[ss].y : qi == 2 ? cur.v[ss].z : cur.v[ss].w;
        const float li = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fv), ln));
        uint32_t asc = 0;
        bool fast = li == li;
        if (fast) {  // #{l_j < l_i} and #{l_j <= l_i} per lane in one word, summed by a DPP scan
          uint32_t c = 0;
#pragma unroll
          for (int s = 0; s < E4; ++s)
#pragma unroll
            for (int q = 0; q < 4; ++q) c += (cur.v[s][q] < li ? 1u : 0u) + (cur.v[s][q] <= li ? 0x10000u : 0u);
          c = (uint32_t)__builtin_amdgcn_readlane(
              (int)wave_scan_dpp(c, 0u, [](uint32_t a, uint32_t b) { return a + b; }), 63);
          asc = c & 0xffffu;
          fast = (c >> 16) == asc + 1;  // class i is its only tie
        }
        if (!fast) {  // ties (ordered by class index) or a NaN logit
          asc = 0;
#pragma unroll
        for (int s = 0; s < E4; ++s)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lj = cur.v[s][q];
            // lanes whose class s * 256 + 4 lane + q is below ii
            const uint64_t before = lanes_below((ii - s * 256 - q + 3) >> 2);
            uint64_t hit;
            if (li == li) hit = __ballot(lj < li) | (__ballot(lj == li) & before);
            else hit = __ballot(lj == lj) | (__ballot(lj != lj) & before);  // NaN sorts after numbers
            asc += __popcll(hit);
          }
        }
        const int64_t p = L - 1 - (int64_t)asc;
        best = (best < 0 || p < best) ? p : best;
      }
    return (T)(best < 0 ? 0 : best);
  } else {
    uint32_t key[E4][4];
    bool ok[E4][4];
    uint32_t lmax;
    cat_dec_keys<E4, FULL>(cur, L, lane, key, ok, lmax);
    const uint32_t k = cat_dec_k<T>(xv, L);
    if (k < (uint32_t)kCatPeel) {
      // the largest key, its ties; while those are all above rank k, the largest key below it.
      // "Largest key below wmax" as one add and one max per key: key + c (c = -wmax) wraps the keys
      // below wmax above every other (padding keys 0 included, which never win: k < L valid keys).
      uint64_t w[E4][4];  // ballots of the keys equal to the answer's
      uint32_t taken = 0, wmax = wave_max_dpp(lmax);
      while (true) {
        uint32_t ties = 0;
#pragma unroll
        for (int s = 0; s < E4; ++s)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            w[s][q] = __ballot(key[s][q] == wmax);
            ties += (uint32_t)__popcll(w[s][q]);
          }
        if (taken + ties > k) return (T)cat_dec_walk<E4>(w, k - taken);
        taken += ties;
        const uint32_t c = 0u - wmax;
        uint32_t best = 0;
#pragma unroll
        for (int s = 0; s < E4; ++s)
#pragma unroll
          for (int q = 0; q < 4; ++q) best = max(best, key[s][q] + c);
        wmax = wave_max_dpp(best) - c;
      }
    }
    // radix select on digits of up to 8 bits from the top of the bits in which the keys differ
    // (P of them below the common prefix): per round a 256-bin LDS histogram of the digit over the
    // keys in the current range (bin = digit, one bit-field extract per key), a DPP scan over the
    // bins in descending digit order, the bin that holds rank k; the range narrows to that bin.
    // Stops when the bin holds one key or the digits run out (ties).  Every key also writes its
    // class into the owner slot of its bin (same address register, immediate offset): when the final
    // bin holds one key, that slot names the class -- one LDS read, no ballots.  Keys outside the
    // range skip their atomics (an exec-masked branch).  Measured and not kept (round 5,
    // profiles/round5/ab_categorical_r5c.txt): branch-free rounds -- bins counted down from the
    // range's top key so out-of-range keys land past the range or in per-lane trash bins, the bin
    // inside the lane selected on the VALU -- and two elements per wave with interleaved scans: SALU
    // below VALU (8.8 k vs 13.3 k per wave) but 323 vs 308 us for uniform ranks; the VALU the
    // unconditional rounds add costs more than the branches cost the scalar unit
    uint32_t* own = bins + kCatOwn;
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)key[0][0]);  // class 0 exists
    const uint32_t dif = wave_or_dpp(cat_dif<E4>(key, ok, k0));
    const int P = dif == 0 ? 0 : 32 - __clz((int)dif);
    int sh = s_floor_sub(P, 8), wd = P - sh;  // digit = bits [sh, sh + wd)
    uint32_t t = P >= 32 ? 0u : (k0 >> P) << P;
    uint32_t c_hi = 0, cnt, dig;  // c_hi: keys above the range
    // the bin that holds rank k: its digit, its count; keys above it into c_hi
    auto pick_bin = [&](uint32_t dm) {
      __builtin_amdgcn_wave_barrier();
      // bins in ascending digit order; lane l takes digits 255 - 4 l down to 252 - 4 l
      const uint4 bu = *(const uint4*)(bins + 4 * (63 - lane));
      const uint32_t tot = bu.x + bu.y + bu.z + bu.w;
      const uint32_t incl = wave_scan_dpp(tot, 0u, [](uint32_t a, uint32_t c) { return a + c; });
      const uint32_t r = k - c_hi;
      const int ls = (int)__builtin_ctzll(__ballot(r < incl));  // the first lane past r (incl ascends)
      // inside that lane, on the scalar unit: the bin whose cumulative range holds r
      uint32_t cb = (uint32_t)__builtin_amdgcn_readlane((int)(incl - tot), ls);
      const uint32_t b0 = (uint32_t)__builtin_amdgcn_readlane((int)bu.w, ls);
      const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)bu.z, ls);
      const uint32_t b2 = (uint32_t)__builtin_amdgcn_readlane((int)bu.y, ls);
      const uint32_t b3 = (uint32_t)__builtin_amdgcn_readlane((int)bu.x, ls);
      uint32_t q = 0;
      cnt = b0;
      if (r >= cb + b0) {
        cb += b0; cnt = b1; q = 1;
        if (r >= cb + b1) {
          cb += b1; cnt = b2; q = 2;
          if (r >= cb + b2) { cb += b2; cnt = b3; q = 3; }
        }
      }
      c_hi += cb;
      dig = (255u - (uint32_t)(4 * ls) - q) & dm;
      t |= dig << sh;
    };
    *(uint4*)(bins + 4 * lane) = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < E4; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (ok[s][q]) {
          const uint32_t d = __builtin_amdgcn_ubfe(key[s][q], (uint32_t)sh, (uint32_t)wd);
          atomicAdd(bins + d, 1u);
          own[d] = (uint32_t)(s * 256 + 4 * lane + q);
        }
    pick_bin((1u << wd) - 1u);
    while (cnt > 1u && sh != 0) {
      const int nsh = s_floor_sub(sh, 8);
      wd = sh - nsh;
      sh = nsh;
      const uint32_t dm = (1u << wd) - 1u;
      __builtin_amdgcn_wave_barrier();  // the zeroing must not overtake the last round's reads
      *(uint4*)(bins + 4 * lane) = make_uint4(0, 0, 0, 0);
      __builtin_amdgcn_wave_barrier();
      // keys in the range [t, t + 2^(sh + wd)): (key >> sh) - (t >> sh) <= dm, and that is the digit
      const uint32_t lo = t >> sh;
#pragma unroll
      for (int s = 0; s < E4; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t d = (key[s][q] >> sh) - lo;
          if (ok[s][q] && d <= dm) {
            atomicAdd(bins + d, 1u);
            own[d] = (uint32_t)(s * 256 + 4 * lane + q);
          }
        }
      pick_bin(dm);
    }
    // the final round's writes precede this read in the wave's LDS order
    if (cnt == 1u) return (T)__builtin_amdgcn_readfirstlane((int)own[dig]);
    // ties: the (k - c_hi)-th highest class index among the keys in [tlo, t | span]; padding keys
    // (0) are below every valid key (>= 1), so without FULL the range starts at 1 at the least
    const uint32_t span = (1u << sh) - 1u;  // sh <= 24
    const uint32_t tlo = FULL || t > 0 ? t : 1u, ext = (t | span) - tlo;
    uint64_t w[E4][4];
#pragma unroll
    for (int s = 0; s < E4; ++s)
#pragma unroll
      for (int q = 0; q < 4; ++q) w[s][q] = __ballot(key[s][q] - tlo <= ext);
    return (T)cat_dec_walk<E4>(w, k - c_hi);
  }
}

template <typename T, int DIR, int E4, int PF, bool FULL>
__global__ void __launch_bounds__(64 * kCatWaves) categorical_vec_kernel(const float* __restrict__ logits, int64_t n,
                                                                          int64_t L, const T* __restrict__ x,
                                                                          T* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t bins_all[kCatWaves][2 * kCatOwn];  // bins, owner slots
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));  // wave-uniform
  uint32_t* bins = bins_all[wv];
  // each wave codes one contiguous range of elements
  const int64_t nw = (int64_t)gridDim.x * kCatWaves;
  const int64_t per = (n + nw - 1) / nw;
  const int64_t b = ((int64_t)blockIdx.x * kCatWaves + wv) * per;
  const int64_t end = b + per < n ? b + per : n;
  if (b >= end) return;
  // Element b + j sits in ring[j % PF]: it is ranked in place and its slot reloaded right after,
  // so no register copies tie a wait to the newest load, and every load of the main loop is issued
  // (the loop stops PF elements before the range's end) so the outstanding count at each use is
  // the same PF - 1.  Row, value and code pointers advance on the scalar unit.
  const uint32_t zero0 = (threadIdx.x >> 6) - (uint32_t)wv;  // 0, but not provably wave-uniform
  // the wave's rows and the dwords that hold its values (the host keeps a range's rows < 2^31 bytes)
  const uint32_t rstride = (uint32_t)L * 4u;
  const __amdgpu_buffer_rsrc_t rows = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(logits + b * L), (short)0, (int)((uint32_t)(end - b) * rstride), 0x00020000);
  const uintptr_t xb = (uintptr_t)(x + b) & ~(uintptr_t)3;
  const __amdgpu_buffer_rsrc_t xs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xb, (short)0, (int)((((uintptr_t)(x + end - 1) & ~(uintptr_t)3) + 4) - xb), 0x00020000);
  auto xoff = [&](const T* xe) { return (uint32_t)(((uintptr_t)xe & ~(uintptr_t)3) - xb); };
  uint32_t ro = 0;
  const T* xp = x + b;
  T* op = out + b;
  int64_t e = b;
  CatRow<E4> ring[PF];
  auto rank = [&](int u, const T* xe) {
    const uint32_t xw = (uint32_t)__builtin_amdgcn_readfirstlane((int)ring[u].xv);
    return cat_rank<T, DIR, E4, FULL>(ring[u], L, lane, bins, cat_xval<T>(xe, xw));
  };
  auto load = [&](int u, int j) {  // element e + j into ring[u]
    cat_load<T, E4, FULL>(rows, ro + (uint32_t)j * rstride, xs, xoff(xp + j), L, lane, zero0, ring[u]);
  };
  const bool main = b + 2 * PF <= end;
  if (main) {
#pragma unroll
    for (int u = 0; u < PF; ++u) load(u, u);
    do {
#pragma unroll
      for (int u = 0; u < PF; ++u) {
        const T code = rank(u, xp + u);
        if (lane == 0) op[u] = code;
        load(u, u + PF);
      }
      ro += PF * rstride;
      xp += PF;
      op += PF;
      e += PF;
    } while (e + 2 * PF <= end);
  } else {
#pragma unroll
    for (int u = 0; u < PF; ++u)
      if (e + u < end) load(u, u);
  }
  // the range's last elements (PF to 2 PF - 1 after the main loop, fewer without it): ring[u]
  // holds element e + u; reload a slot only while elements remain
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (e + u < end) {
      const T code = rank(u, xp + u);
      if (lane == 0) op[u] = code;
      if (e + u + PF < end) load(u, u + PF);
    }
#pragma unroll
  for (int u = 0; u < PF - 1; ++u)
    if (e + PF + u < end) {
      const T code = rank(u, xp + PF + u);
      if (lane == 0) op[PF + u] = code;
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
  // vector form: 8 waves per SIMD over the chip, each walking its elements one load ahead
  const bool vec = L % 4 == 0 && L <= 512 && ((uintptr_t)logits & 15) == 0;
  // a wave's rows (buffer resource, 32-bit offsets) stay below 2^31 bytes: more waves for huge n
  const int64_t per_max = ((int64_t)1 << 31) / (L * 4) - 1;
  const int64_t g_min = (n + per_max * kCatWaves - 1) / (per_max * kCatWaves);
  const unsigned vgrid = (unsigned)std::max<int64_t>(g > 2048 ? 2048 : g, g_min);
  return dispatch_int_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    if (vec) {
      constexpr int PF = kCatPF;
      hipStream_t st = (hipStream_t)stream;
      // FULL: L == 256 E4, no padding classes (no per-class masks)
      auto go = [&](auto kern) { kern<<<vgrid, 64 * kCatWaves, 0, st>>>(logits, n, L, (const T*)x, (T*)out); };
      if (direction == KMP_ENCODE && L <= 256)
        L == 256 ? go(categorical_vec_kernel<T, KMP_ENCODE, 1, PF, true>) : go(categorical_vec_kernel<T, KMP_ENCODE, 1, PF, false>);
      else if (direction == KMP_ENCODE)
        L == 512 ? go(categorical_vec_kernel<T, KMP_ENCODE, 2, PF, true>) : go(categorical_vec_kernel<T, KMP_ENCODE, 2, PF, false>);
      else if (L <= 256)
        L == 256 ? go(categorical_vec_kernel<T, KMP_DECODE, 1, PF, true>) : go(categorical_vec_kernel<T, KMP_DECODE, 1, PF, false>);
      else
        L == 512 ? go(categorical_vec_kernel<T, KMP_DECODE, 2, PF, true>) : go(categorical_vec_kernel<T, KMP_DECODE, 2, PF, false>);
      return check_launch("categorical_vec");
    }
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
