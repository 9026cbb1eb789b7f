// kmp_rice.hip -- block-adaptive Rice coding of coded maps (the entropy
// stage the reference does not have -- encode returns residual arrays, volume/encode_decode.py:56
// -- so the format is the build's own; its specification is oracle/rice.py, byte for byte).
//
// Samples are zigzag-mapped W-bit residuals z.  Per 64-sample block the Rice parameter k
// minimises the block's 32-bit word count 2k + ceil((64 + sum_i (z_i >> k)) / 32); the block
// stores k low bit-planes of z (64 bits each) and then the unary parts (q_i = z_i >> k zeros and
// a one per sample), zero padded to a 32-bit word.  Side information: params[b] = k + 1 (0 = an
// all-zero block, no payload) and bw[b] = the block's payload words.
//
// Lane layout as kmp_pack.hip (kmp_bits.h): 8 consecutive samples per lane, 8 lanes per block,
// 8 blocks per wave step, grid-stride over wave steps.  Launches:
//   rice_plan_kernel   z-planes in registers -> per-plane popcounts (SWAR, DPP-reduced over the
//                      block's lanes) -> S_k by Horner (S_k = 2 S_{k+1} + count_k) -> k*, bw
//   scan               exclusive scan of bw (kmp_pack.hip's two scan kernels) -> word offsets
//   rice_pack_kernel   the k* low planes (the bit-plane transposes of the planes format) + the
//                      unary part: a DPP prefix of the lanes' unary lengths, one ds_or per
//                      sample's terminator bit into a per-block LDS stream, copied out as words
//   rice_unpack_kernel lane j loads planes 8p + j < k and transposes back to the samples' low
//                      bits; the unary part: the lane finds the end of terminator 8j - 1 (a
//                      popcount walk + a binary-search select in one word), then reads its 8
//                      quotients off a 64-bit window of the stream with ctz (a word-by-word walk
//                      when the 8 codes are longer than 64 bits)
// All three are VALU-bound, not latency-bound: the SQ counters give VALU instructions x 4 cycles
// (wave64 on a 16-lane SIMD) / 1024 SIMDs = the kernel time (profiles/round2/rice_kernels.log), and
// U steps per wave with their loads batched (U = 2, 4, 8) measured no faster.
#include "kmp_bits.h"

namespace kmp {
namespace rc {

using namespace pk;

constexpr uint32_t kSumCap = 1u << 20;  // S_k past this can never be the optimum (see plan)

template <int W>
__device__ __forceinline__ uint32_t sample_of(const uint32_t (&w)[Sw<W>::NW], int e) {
  if constexpr (W == 8) return (w[e >> 2] >> (8 * (e & 3))) & 0xffu;
  else if constexpr (W == 16) return (w[e >> 1] >> (16 * (e & 1))) & 0xffffu;
  else return w[e];
}
template <int W>
__device__ __forceinline__ void set_sample(uint32_t (&w)[Sw<W>::NW], int e, uint32_t v) {
  if constexpr (W == 8) w[e >> 2] |= (v & 0xffu) << (8 * (e & 3));
  else if constexpr (W == 16) w[e >> 1] |= (v & 0xffffu) << (16 * (e & 1));
  else w[e] = v;
}

// z-planes of the lane's 8 samples: byte b of Z[p] (lo, hi) = bits of z-plane 8p + b (before the
// cross-lane transpose); the zigzag is applied in the plane domain as in kmp_pack.hip
template <int W>
__device__ __forceinline__ void zplanes(const uint32_t (&w)[Sw<W>::NW], uint32_t (&Z)[Sw<W>::NP][2]) {
  constexpr int NP = Sw<W>::NP;
  uint32_t X[NP][2];
  gather_bytes<W>(w, X);
#pragma unroll
  for (int p = 0; p < NP; ++p) tr8x8(X[p][0], X[p][1]);
  const uint32_t sg = perm(X[NP - 1][1], X[NP - 1][1], 0x07070707u);
#pragma unroll
  for (int i = 2 * NP - 1; i >= 0; --i) {
    const uint32_t cur = X[i >> 1][i & 1];
    const uint32_t prev = i ? X[(i - 1) >> 1][(i - 1) & 1] : 0u;
    Z[i >> 1][i & 1] = __builtin_amdgcn_alignbit(cur, prev, 24) ^ sg;
  }
}

__device__ __forceinline__ uint32_t bytes_popcount(uint32_t v) {  // 4 byte-wise popcounts (each <= 8)
  v = v - ((v >> 1) & 0x55555555u);
  v = (v & 0x33333333u) + ((v >> 2) & 0x33333333u);
  return (v + (v >> 4)) & 0x0f0f0f0fu;
}

// sum over the block's 8 lanes (every lane of the group ends with the total)
__device__ __forceinline__ uint32_t group8_sum(uint32_t v, int lane) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  const uint32_t up = dpp<0x104>(v), dn = dpp<0x114>(v);  // full exec (see kmp_pack.hip widths_kernel)
  return v + ((lane & 4) ? dn : up);
}

// inclusive prefix over the block's 8 lanes (j = lane & 7)
__device__ __forceinline__ uint32_t group8_incl(uint32_t v, int j) {
  uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);  // row_shr:1
  if (j & 7) v += t;
  t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);  // row_shr:2
  if ((j & 7) >= 2) v += t;
  t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);  // row_shr:4
  if ((j & 7) >= 4) v += t;
  return v;
}

// position of the t-th (0-based) set bit of x (t < popcount(x))
__device__ __forceinline__ int select32(uint32_t x, uint32_t t) {
  int pos = 0;
  uint32_t c = __builtin_popcount(x & 0xffffu);
  if (t >= c) { t -= c; x >>= 16; pos += 16; }
  c = __builtin_popcount(x & 0xffu);
  if (t >= c) { t -= c; x >>= 8; pos += 8; }
  c = __builtin_popcount(x & 0xfu);
  if (t >= c) { t -= c; x >>= 4; pos += 4; }
  c = __builtin_popcount(x & 0x3u);
  if (t >= c) { t -= c; x >>= 2; pos += 2; }
  c = x & 1u;
  if (t >= c) pos += 1;
  return pos;
}

// per block: k* and the payload words (params / bw), from the per-plane popcounts
template <int W>
__global__ void __launch_bounds__(256) rice_plan_kernel(const void* __restrict__ x, int64_t n,
                                                      uint8_t* __restrict__ params, uint8_t* __restrict__ bw,
                                                      int64_t nb) {
  constexpr int NP = Sw<W>::NP;
  const int lane = threadIdx.x & 63;
  const int64_t nstep = (nb + 7) / 8;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    uint32_t w[Sw<W>::NW];
    load8s<W>(x, n, st * 512 + (int64_t)lane * 8, w);
    uint32_t Z[NP][2];
    zplanes<W>(w, Z);
    uint32_t cnt[2 * NP];  // byte b of cnt[i]: the block's count of ones in z-plane 4i + b
#pragma unroll
    for (int i = 0; i < 2 * NP; ++i) cnt[i] = group8_sum(bytes_popcount(Z[i >> 1][i & 1]), lane);
    // S_k = sum_i (z_i >> k) = 2 S_{k+1} + count_k; words(k) = 2k + ceil((64 + S_k) / 32).  An S_k
    // past kSumCap costs more than 2W + 2 words (the k = W - 1 cost bound), so capping it keeps the
    // argmin exact (ties: the smallest k, as the descending loop keeps the last <=)
    // (W <= 16: S_0 <= 64 (2^16 - 1) needs no cap.)  The argmin as one min per k over the key
    // 32 words(k) + k = ((S_k + 95) & ~31) + 65 k: the fewest words, ties to the smallest k
    uint32_t S = 0, key = 0xffffffffu;
#pragma unroll
    for (int k = W - 1; k >= 0; --k) {
      const uint32_t c = (cnt[k >> 2] >> (8 * (k & 3))) & 0xffu;
      S = 2u * S + c;
      if constexpr (W > 16) S = min(S, kSumCap);
      key = min(key, ((S + 95u) & ~31u) + 65u * (uint32_t)k);
    }
    const uint32_t best = key >> 5;
    const int kbest = (int)(key & 31u);
    const bool zero = S == 0;  // S_0 == sum of z: an all-zero block
    const int64_t blk = st * 8 + (lane >> 3);
    if ((lane & 7) == 0 && blk < nb) {
      params[blk] = zero ? 0 : (uint8_t)(kbest + 1);
      bw[blk] = zero ? 0 : (uint8_t)best;
    }
  }
}

template <int W>
__global__ void __launch_bounds__(256) rice_pack_kernel(const void* __restrict__ x, int64_t n,
                                                      const uint8_t* __restrict__ params,
                                                      const uint32_t* __restrict__ local,
                                                      const uint64_t* __restrict__ cbase, int64_t nb,
                                                      uint32_t* __restrict__ payload) {
  constexpr int NP = Sw<W>::NP;
  constexpr int UMAX = 2 * W + 2;
  __shared__ uint32_t stream_lds[4][8][UMAX];
  const int lane = threadIdx.x & 63, j = lane & 7, g = lane >> 3;
  uint32_t* ustream = stream_lds[threadIdx.x >> 6][g];
  const int64_t nstep = (nb + 7) / 8;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t blk = st * 8 + g;
    uint32_t w[Sw<W>::NW];
    load8s<W>(x, n, st * 512 + (int64_t)lane * 8, w);
    int param = 0;
    uint64_t off = 0;
    if (blk < nb) {
      param = params[blk];
      off = cbase[blk / kChunk] + local[blk];
    }
    const int k = param > 0 ? min(param - 1, W - 1) : 0;
    // low planes: lane j stores z-planes 8p + j < k
    uint32_t Z[NP][2];
    zplanes<W>(w, Z);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      xtr8(Z[p][0], Z[p][1], j);
      const int b = 8 * p + j;
      if (param > 0 && b < k) {
        KMP_DCHECK(off + 2 * b + 1 < off + 2 * W + 2, "plane %d past the block", b);
        payload[off + 2 * b] = Z[p][0];
        payload[off + 2 * b + 1] = Z[p][1];
      }
    }
    // unary part: lane's quotients, their total, the prefix over the block's lanes
    uint32_t q[8], len = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      q[e] = zigzag<W>(sample_of<W>(w, e)) >> k;
      len += q[e] + 1u;
    }
    const uint32_t incl = group8_incl(len, j);
    const uint32_t tot = (uint32_t)__shfl((int)incl, (g << 3) | 7, 64);  // the block's unary bits
    const uint32_t uw = (tot + 31u) >> 5;
    // zero the block's uw stream words (all a terminator can land in: pos < tot), OR in one
    // terminator per sample, copy the words out
    for (uint32_t i = j; i < uw && i < (uint32_t)UMAX; i += 8) ustream[i] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    uint32_t pos = incl - len;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      pos += q[e];
      if (param > 0 && pos < 32u * min(uw, (uint32_t)UMAX)) atomicOr(&ustream[pos >> 5], 1u << (pos & 31));
      pos += 1u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    if (param > 0) {
      const uint64_t ubase = off + 2u * (uint32_t)k;
      for (uint32_t i = j; i < uw && i < (uint32_t)UMAX; i += 8) payload[ubase + i] = ustream[i];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();  // the next step's zeroing must not overtake these reads
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

template <int W>
__global__ void __launch_bounds__(256) rice_unpack_kernel(const uint32_t* __restrict__ payload, int64_t n,
                                                        const uint8_t* __restrict__ params,
                                                        const uint8_t* __restrict__ bw,
                                                        const uint32_t* __restrict__ local,
                                                        const uint64_t* __restrict__ cbase, int64_t nb,
                                                        void* __restrict__ out) {
  constexpr int NP = Sw<W>::NP;
  constexpr int SPAN = 8 * (2 * W + 2);  // payload words of a wave step's 8 blocks, at most
  __shared__ uint32_t span_lds[4][SPAN];
  const int lane = threadIdx.x & 63, j = lane & 7;
  uint32_t* const wspan = span_lds[(threadIdx.x >> 6) & 3];
  const int64_t nstep = (nb + 7) / 8;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t blk = st * 8 + (lane >> 3);
    int param = 0, words = 0;
    uint64_t off = 0;
    if (blk < nb) {
      param = params[blk];
      words = min((int)bw[blk], 2 * W + 2);  // a corrupt bw never steers a read past the span
      off = cbase[blk / kChunk] + local[blk];
    }
    // the step's 8 blocks are consecutive in the payload: stage their words [start, end) in LDS
    // with coalesced loads, so the low planes and the unary walk below read LDS, not memory
    const uint64_t start = __shfl(off, 0, 64);
    uint64_t end = blk < nb ? off + (uint64_t)words : start;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const uint64_t o = __shfl_xor(end, d, 64);
      end = o > end ? o : end;
    }
    const int cnt = (int)min<uint64_t>(end - start, (uint64_t)SPAN);
    for (int i = lane; i < cnt; i += 64) wspan[i] = payload[start + i];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    const uint32_t* const bp = wspan + (off - start);  // this lane's block in LDS
    const int k = param > 0 ? min(param - 1, W - 1) : 0;
    const int uw = param > 0 ? max(words - 2 * k, 0) : 0;  // a corrupt bw never steers a read past the block
    // low bits: planes 8p + j < k, transposed back to the lane's 8 samples
    uint32_t Z[NP][2];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int b = 8 * p + j;
      const bool have = param > 0 && b < k && 2 * b + 1 < words;
      Z[p][0] = have ? bp[2 * b] : 0u;
      Z[p][1] = have ? bp[2 * b + 1] : 0u;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      xtr8(Z[p][0], Z[p][1], j);
      tr8x8(Z[p][0], Z[p][1]);
    }
    uint32_t lowv[Sw<W>::NW];
    scatter_bytes<W>(Z, lowv);
    // unary part: start after terminator 8j - 1, then 8 quotients by ctz
    const uint32_t* us = bp + 2 * k;
    uint32_t q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = 0u;
    if (param > 0 && uw > 0) {
      uint32_t pos = 0;  // stream position where sample 8j's code starts
      if (j > 0) {
        const uint32_t r = 8u * j - 1u;  // 0-based rank of the terminator ending sample 8j - 1
        uint32_t acc = 0, word = 0;
        int wi = 0;
        for (; wi < uw; ++wi) {
          word = us[wi];
          const uint32_t c = __builtin_popcount(word);
          if (acc + c > r) break;
          acc += c;
        }
        pos = wi < uw ? 32u * wi + select32(word, r - acc) + 1u : 32u * uw;
      }
      int wi = (int)(pos >> 5);
      // the 64 stream bits from ``pos`` (three words funnel-shifted); when they hold the lane's 8
      // terminators -- a mean quotient below 7 at the block's k, nearly always -- the quotients are
      // 8 branch-free ctz steps, otherwise the word-by-word walk below
      const uint32_t sh = pos & 31u;
      const uint32_t a = wi < uw ? us[wi] : 0u, b = wi + 1 < uw ? us[wi + 1] : 0u, c = wi + 2 < uw ? us[wi + 2] : 0u;
      uint64_t win = ((uint64_t)__builtin_amdgcn_alignbit(c, b, sh) << 32) | __builtin_amdgcn_alignbit(b, a, sh);
      if (__builtin_popcountll(win) >= 8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t t = (uint32_t)__builtin_ctzll(win);
          q[e] = t;
          win = (win >> t) >> 1;
        }
      } else {
        // ``cur``: the stream bits from position ``base`` up to the end of word ``wi``
        uint32_t cur = wi < uw ? us[wi] >> sh : 0u;
        uint32_t base = pos;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          while (cur == 0u && wi + 1 < uw) {  // only zeros left in this word: continue in the next
            ++wi;
            cur = us[wi];
            base = 32u * wi;
          }
          if (cur == 0u) break;  // a corrupt stream with fewer than 64 terminators
          const uint32_t t = __builtin_ctz(cur);
          q[e] = base + t - pos;  // the zeros between the code's start and its terminator
          pos = base + t + 1u;
          cur = t == 31u ? 0u : cur >> (t + 1u);
          base = pos;
        }
      }
    }
    uint32_t wout[Sw<W>::NW];
#pragma unroll
    for (int i = 0; i < Sw<W>::NW; ++i) wout[i] = 0u;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t z = param > 0 ? (q[e] << k) | sample_of<W>(lowv, e) : 0u;
      set_sample<W>(wout, e, unzigzag<W>(z));
    }
    store8s<W>(out, n, st * 512 + (int64_t)lane * 8, wout);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();  // the next step's staging must not overtake these reads
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

// side information a blob may hold (one workgroup; written next to the scan's total): planes --
// widths <= W; rice -- k < W, an all-zero block has no payload, a coded block holds its 2k plane
// words and >= 2 unary words, at most 2W + 2 in all.  The count of violating blocks is read back
// with the payload length before any unpack kernel runs.
// Side-information check over all blocks: a thread tests 8 consecutive blocks (one 8-byte load
// per side array when both are 8-byte aligned), a wave sums its count and adds it to *bad_out
// (zeroed by the launcher) with one vector atomic when it is non-zero.  Was one 1024-thread
// workgroup reading a byte per block: 103 us for the 524288 blocks of a 32 MiB u16 map.
template <bool ALIGNED>
__global__ void __launch_bounds__(256) side_check_kernel(int format, int W, const uint8_t* __restrict__ a,
                                                       const uint8_t* __restrict__ b, int64_t nb,
                                                       unsigned long long* __restrict__ bad_out) {
  const int64_t i0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  uint32_t bad = 0;
  if (i0 < nb) {
    uint8_t av[8], bv[8];
    if (ALIGNED && i0 + 8 <= nb) {
      *(uint2*)av = *(const uint2*)(a + i0);
      *(uint2*)bv = format ? *(const uint2*)(b + i0) : make_uint2(0, 0);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // past the end: a zero block with no payload, which is valid
        av[j] = i0 + j < nb ? a[i0 + j] : 0;
        bv[j] = format && i0 + j < nb ? b[i0 + j] : 0;
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (format == 0) {
        bad += av[j] > W;
      } else {
        const int k = (int)av[j] - 1, words = bv[j];
        bad += av[j] == 0 ? (words != 0) : (k >= W || words < 2 * k + 2 || words > 2 * W + 2);
      }
    }
  }
  for (int d = 32; d >= 1; d >>= 1) bad += __shfl_xor(bad, d, 64);
  if ((threadIdx.x & 63) == 0 && bad) atomicAdd(bad_out, (unsigned long long)bad);
}

}  // namespace rc
}  // namespace kmp

using namespace kmp;

extern "C" {

int kmp_rice_plan(int32_t dtype, const void* x, int64_t n, uint8_t* params, uint8_t* bw, void* workspace,
                  kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "rice: unsupported dtype");
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || (x && params && bw)), "rice: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  hipStream_t s = (hipStream_t)stream;
  if (nb > 0) {
    if (W == 8) rc::rice_plan_kernel<8><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, params, bw, nb);
    else if (W == 16) rc::rice_plan_kernel<16><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, params, bw, nb);
    else rc::rice_plan_kernel<32><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, params, bw, nb);
    if (int st = check_launch("rice_plan")) return st;
  }
  return pk::scan(bw, nb, pk::carve(workspace, nb), s);
}

int kmp_rice_pack(int32_t dtype, const void* x, int64_t n, const uint8_t* params, const void* workspace,
                  uint32_t* payload, kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "rice: unsupported dtype");
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || (x && params && payload)), "rice: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  if (nb == 0) return KMP_OK;
  const pk::Ws w = pk::carve((void*)workspace, nb);
  hipStream_t s = (hipStream_t)stream;
  if (W == 8) rc::rice_pack_kernel<8><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, params, w.local, w.cbase, nb, payload);
  else if (W == 16) rc::rice_pack_kernel<16><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, params, w.local, w.cbase, nb, payload);
  else rc::rice_pack_kernel<32><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, params, w.local, w.cbase, nb, payload);
  return check_launch("rice_pack");
}

int kmp_unpack_check(int32_t format, int32_t dtype, const uint8_t* side_a, const uint8_t* side_b, int64_t n,
                     void* workspace, kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "unpack_check: unsupported dtype");
  KMP_REQUIRE(format == 0 || format == 1, "unpack_check: format must be 0 (planes) or 1 (rice)");
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || (side_a && (format == 0 || side_b))), "unpack_check: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  unsigned long long* bad = (unsigned long long*)((char*)workspace + kmp_pack_total_offset(n) + 8);
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(bad, 0, sizeof(*bad), s) != hipSuccess) return fail(KMP_ERR_LAUNCH, "unpack_check: memset");
  if (nb == 0) return KMP_OK;
  const unsigned grid = (unsigned)ceil_div(nb, (int64_t)8 * 256);
  if ((((uintptr_t)side_a | (uintptr_t)side_b) & 7) == 0)
    rc::side_check_kernel<true><<<grid, 256, 0, s>>>(format, W, side_a, side_b, nb, bad);
  else
    rc::side_check_kernel<false><<<grid, 256, 0, s>>>(format, W, side_a, side_b, nb, bad);
  return check_launch("unpack_check");
}

int kmp_rice_unpack(int32_t dtype, const uint32_t* payload, int64_t n, const uint8_t* params, const uint8_t* bw,
                    const void* workspace, void* out, kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "rice: unsupported dtype");
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || (payload && params && bw && out)), "rice: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  if (nb == 0) return KMP_OK;
  const pk::Ws w = pk::carve((void*)workspace, nb);
  hipStream_t s = (hipStream_t)stream;
  if (W == 8) rc::rice_unpack_kernel<8><<<pk::waves_grid(nb), 256, 0, s>>>(payload, n, params, bw, w.local, w.cbase, nb, out);
  else if (W == 16) rc::rice_unpack_kernel<16><<<pk::waves_grid(nb), 256, 0, s>>>(payload, n, params, bw, w.local, w.cbase, nb, out);
  else rc::rice_unpack_kernel<32><<<pk::waves_grid(nb), 256, 0, s>>>(payload, n, params, bw, w.local, w.cbase, nb, out);
  return check_launch("rice_unpack");
}

}  // extern "C"
