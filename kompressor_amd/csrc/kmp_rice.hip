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

typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

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

// the lane's 8 samples all in [-128, 127] as signed W-bit values (their z < 256)
template <int W>
__device__ __forceinline__ bool byte_residuals(const uint32_t (&w)[Sw<W>::NW]) {
  uint32_t hb = 0;
  if constexpr (W == 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t t = __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, w[i]) + (u16x2){0x80, 0x80});
      hb |= t & 0xff00ff00u;
    }
  } else if constexpr (W == 32) {
#pragma unroll
    for (int i = 0; i < 8; ++i) hb |= (w[i] + 0x80u) & 0xffffff00u;
  }
  return hb == 0;
}

// zplanes when every sample is in [-128, 127]: plane group 0 only (its sign plane is plane 7, which
// equals every higher s-plane), the others zero
template <int W>
__device__ __forceinline__ void zplanes_lo(const uint32_t (&w)[Sw<W>::NW], uint32_t (&Z)[Sw<W>::NP][2]) {
  constexpr int NP = Sw<W>::NP;
  static_assert(W == 16 || W == 32, "8-bit samples have one plane group");
  uint32_t X0, X1;
  if constexpr (W == 16) {
    X0 = perm(w[1], w[0], 0x06040200u);
    X1 = perm(w[3], w[2], 0x06040200u);
  } else {
    X0 = perm(w[1], w[0], 0x0c0c0400u) | perm(w[3], w[2], 0x04000c0cu);
    X1 = perm(w[5], w[4], 0x0c0c0400u) | perm(w[7], w[6], 0x04000c0cu);
  }
  tr8x8(X0, X1);
  const uint32_t sg = perm(X1, X1, 0x07070707u);
  Z[0][0] = __builtin_amdgcn_alignbit(X0, 0u, 24) ^ sg;
  Z[0][1] = __builtin_amdgcn_alignbit(X1, X0, 24) ^ sg;
#pragma unroll
  for (int p = 1; p < NP; ++p) Z[p][0] = Z[p][1] = 0u;
}

// lane j of a block's 8-lane group ends with sum_{m=j..7} x_m 2^(m-j) (row_shl:d reads lane l+d;
// a lane whose partner lies past the group adds nothing)
__device__ __forceinline__ uint32_t group8_suffix2(uint32_t x, int j) {
  uint32_t t = dpp<0x101>(x);
  if (j < 7) x += t << 1;
  t = dpp<0x102>(x);
  if (j < 6) x += t << 2;
  t = dpp<0x104>(x);
  if (j < 4) x += t << 4;
  return x;
}

// the value of the group's lane 0 / lane 7 on all its 8 lanes: row_newbcast of the second group's
// lane (row lane 8 / 15) to the whole row of 16, then of the first group's (row lane 0 / 7) to banks
// 0-1 (lanes 0-7) only -- two DPP moves, no select
__device__ __forceinline__ uint32_t group8_first(uint32_t x, int) {
  const int b = __builtin_amdgcn_update_dpp(0, (int)x, 0x158, 0xf, 0xf, false);  // row_newbcast:8
  return (uint32_t)__builtin_amdgcn_update_dpp(b, (int)x, 0x150, 0xf, 0x3, false);  // row_newbcast:0, lanes 0-7
}
__device__ __forceinline__ uint32_t group8_last(uint32_t x, int) {
  const int b = __builtin_amdgcn_update_dpp(0, (int)x, 0x15F, 0xf, 0xf, false);  // row_newbcast:15
  return (uint32_t)__builtin_amdgcn_update_dpp(b, (int)x, 0x157, 0xf, 0x3, false);  // row_newbcast:7, lanes 0-7
}

// sum / minimum over the group (every lane of the group ends with it): the quad's by two quad_perm
// steps, then the other quad's by row_half_mirror (lane i of a half row reads lane 7 - i, which lies
// in the other quad of the same group) -- three DPP operations, no select
__device__ __forceinline__ uint32_t group8_sum(uint32_t v, int) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  return v + dpp<0x141>(v);
}
__device__ __forceinline__ uint32_t group8_min(uint32_t v, int) {
  v = min(v, dpp<0xB1>(v));
  v = min(v, dpp<0x4E>(v));
  return min(v, dpp<0x141>(v));
}

// inclusive prefix over the block's 8 lanes: the inclusive scan over the row of 16 (row_shr 1, 2,
// 4, 8 with zeros shifted in at the row's start: one DPP add each, no per-lane masks), then lanes
// 8-15 take off the first group's total (row lane 7's prefix, row_newbcast:7).  The last step is a
// broadcast and a select, not a bank-masked DPP subtract: that form (v_subrev_u32_dpp, banks 2-3)
// left lanes 8-15 unsubtracted on the GPU
__device__ __forceinline__ uint32_t group8_incl(uint32_t v, int j8) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
  const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x157, 0xf, 0xf, false);  // row_newbcast:7
  return j8 ? v - t : v;
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

// ---- the Rice bundle (format v2): every array of a call in one single-pass encode launch and
// one decode launch per sample width ----
//
// Work unit: a TILE of 256 blocks (16384 samples): one 256-thread workgroup, each wave 8 steps of
// 8 blocks in the lane layout above (fewer, larger tiles: the look-back chain is per tile).  Tiles of all arrays form one sequence (array after array); a tile's
// payload words follow its predecessor's, so the bundle holds ONE payload region and per array a
// table of tile offsets (u64 word offsets) that lets the decoder start every tile independently.
//
// Encode (rice_bundle_encode_kernel), reading the samples ONCE: per block k* and its word count
// from the bit-plane popcounts (the plan above, in registers), the block's exclusive prefix inside
// the wave (scan over the 8 groups) and the workgroup (LDS), the tile's start by a decoupled
// look-back over the tiles before it (a tile publishes its aggregate, then its inclusive prefix;
// the first wave reads 64 predecessors per round trip; tiles are numbered by an atomic ticket in
// start order, so every tile a tile waits on has started -- no deadlock), then the payload written from the same registers.  Was: plan kernel
// (reads the map), two scan launches, pack kernel (reads the map again) per array.
//
// Decode (rice_bundle_decode_kernel): the tile offset from the table, the blocks' offsets by the
// same in-workgroup prefix over the stored bw, the unpack below.  Every read is bounded by the tile
// / payload extents, and the side information is checked in the same pass (k < W, bw within
// [2k + 2, 2W + 2], a zero block without payload, the tile's words meeting the next tile's offset);
// a tile that fails decodes as zeros and is counted, so a corrupt bundle raises on the host after
// the one synchronisation instead of steering a read outside the blob.
constexpr int kTileSteps = 8;                     // decode: wave steps (of 8 blocks) per wave and tile
constexpr int kTileBlocks = 4 * 8 * kTileSteps;    // 256 blocks = 16384 samples per tile
constexpr int kEncWaves = 4, kEncSteps = 8;        // encode: as the decode (8 waves of 4 steps: 5 % slower)
static_assert(kEncWaves * 8 * kEncSteps == kTileBlocks, "encode tile shape");
constexpr uint64_t kFlagAgg = 1ull << 62, kFlagPre = 2ull << 62, kValMask = (1ull << 62) - 1;

struct RArr {        // device copy of kmp_rice_array
  const void* x;     // encode input / decode output
  int64_t n, nb, ntile, tile0;
  int64_t side_off, toff_off, rec_off;
};
constexpr int kMaxArr = 32;
struct RArrs {
  RArr a[kMaxArr];
  int count;
};

// the array of global tile g (uniform)
__device__ __forceinline__ int array_of(const RArrs& A, int64_t g) {
  int a = 0;
  while (a + 1 < A.count && g >= A.a[a + 1].tile0) ++a;
  return a;
}

// exclusive prefix of v over the 8 block groups of a wave (v is the same on a group's 8 lanes, so
// shifts by whole groups keep every lane of a group equal); *tot = the wave's total.  Three DPP adds
// (row_shr:8 inside each row of 16, then row_bcast:15 / row_bcast:31 across rows) instead of three
// ds_bpermute round trips
__device__ __forceinline__ uint32_t wave_groups_excl(uint32_t v, int lane, uint32_t* tot) {
  uint32_t x = v;
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  *tot = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  (void)lane;
  return x - v;
}


// q[e] = zigzag(sample e) >> k for the lane's 8 samples; 16-bit samples two at a time (packed
// 16-bit shifts: zigzag = (s << 1) ^ (s >> 15) per half)
template <int W>
__device__ __forceinline__ void quotients(const uint32_t (&w)[Sw<W>::NW], int k, uint32_t (&q)[8]) {
  if constexpr (W == 16) {
    const u16x2 kk = {(unsigned short)k, (unsigned short)k};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const s16x2 sv = __builtin_bit_cast(s16x2, w[i]);
      const u16x2 z = __builtin_bit_cast(u16x2, (s16x2)(sv << (s16x2){1, 1})) ^
                      __builtin_bit_cast(u16x2, (s16x2)(sv >> (s16x2){15, 15}));
      const uint32_t qw = __builtin_bit_cast(uint32_t, (u16x2)(z >> kk));
      q[2 * i] = qw & 0xffffu;
      q[2 * i + 1] = qw >> 16;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = zigzag<W>(sample_of<W>(w, e)) >> k;
  }
}

// 8- and 16-bit samples at 4 waves per SIMD (amdgpu_waves_per_eu: at most 128 VGPRs, 16-bit samples
// spill 28 bytes): 170 vs 180 us per C3 bundle at 3 waves (137 VGPRs),
// profiles/round4/ab_rice_waves4_r4r1.log; 32-bit samples need more registers than that
template <int W>
__global__ void __launch_bounds__(64 * kEncWaves) __attribute__((amdgpu_waves_per_eu(W <= 16 ? 4 : 1))) rice_bundle_encode_kernel(RArrs A, int64_t tile_begin, int64_t tiles_total,
                                                               uint8_t* __restrict__ blob, int64_t payload_off,
                                                               uint64_t* __restrict__ state,
                                                               unsigned* __restrict__ ticket) {
  constexpr int NP = Sw<W>::NP, NW = Sw<W>::NW;
  constexpr int UMAX = 2 * W + 2;
  constexpr int S = kEncSteps;
  __shared__ uint32_t stage[kEncWaves][8 * S * UMAX];  // each wave's payload words, in payload order
  __shared__ uint32_t wsum[kEncWaves];
  __shared__ uint64_t s_excl;
  __shared__ int64_t s_tile;
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, j = lane & 7, g8 = lane >> 3;
  if (tid == 0) s_tile = (int64_t)atomicAdd(ticket, 1u);
  __syncthreads();
  const int64_t g = tile_begin + s_tile;
  const int a = array_of(A, g);
  const RArr& R = A.a[a];
  const int64_t t = g - R.tile0;
  const int64_t blk0 = t * kTileBlocks + wv * 8 * S;  // the wave's first block; step s: blk0 + 8 s + g8
  uint8_t* params = blob + R.side_off;
  uint8_t* bw = params + ((R.nb + 7) & ~(int64_t)7);
  // ---- pass 1: per step, the block's z-planes (lane j: planes 8p + j after the byte transpose,
  // kept for pass 2), k* and its word count; the samples stay in registers for pass 2 ----
  uint32_t w[S][NW];
  uint32_t Zt[S][NP][2];
  uint32_t pb[S];  // the block's k + 1 (6 bits) | its exclusive word offset inside the wave << 6
  uint32_t wtot = 0;
#pragma unroll
  for (int st = 0; st < S; ++st) load8s<W>(R.x, R.n, (blk0 + 8 * st + g8) * 64 + j * 8, w[st]);
  // the wave's whole stage zeroed once while the loads are in flight (UMAX / 2 coalesced 8-byte
  // stores per lane), so pass 2 ORs the unary codes into it with no per-step zeroing and no LDS
  // wait between a step's zeroing and its ORs
  uint8_t* const pside = params + blk0 + g8;
  uint8_t* const wside = bw + blk0 + g8;
  uint32_t* const wl = stage[wv];
  // the stage holds 8 S UMAX words per wave = S UMAX / 16 rounds of 64 lanes x 8 bytes: exact only
  // when S UMAX is a multiple of 16, or the tail words would keep stale bits under the unary ORs
  static_assert((S * UMAX) % 16 == 0, "stage zeroing must cover the whole stage");
#pragma unroll
  for (int t = 0; t < S * UMAX / 16; ++t) ((uint2*)wl)[lane + 64 * t] = make_uint2(0u, 0u);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
  for (int st = 0; st < S; ++st) {
    const int64_t blk = blk0 + 8 * st + g8;
    const bool has = blk < R.nb;
    // S_k = sum_i (z_i >> k) = sum_{b >= k} count_b 2^(b - k) for this lane's k = 8p + j: a doubling
    // suffix sum of the plane counts over the group, plus S_{8(p+1)} (group lane 0) << (8 - j).
    // Equal to the Horner recurrence S_k = 2 S_{k+1} + count_k of the oracle (capped at kSumCap
    // for 32-bit samples: min(S_k, cap), which is what the capped recurrence yields)
    uint32_t key = 0xffffffffu;
    bool lo = false;
    if constexpr (NP > 1) {
      lo = __all(byte_residuals<W>(w[st]));
      if (lo) {
        // every sample of the wave step in [-128, 127] (the usual residual map): z < 256, so the
        // z-planes from 8 up are zero -- transpose and count plane group 0 only; the sign plane
        // is plane 7; the keys of k >= 8 are those of S_k = 0
        zplanes_lo<W>(w[st], Zt[st]);
        xtr8(Zt[st][0][0], Zt[st][0][1], j);
        const uint32_t sk = group8_suffix2(__builtin_popcount(Zt[st][0][0]) + __builtin_popcount(Zt[st][0][1]), j);
        key = min(((sk + 95u) & ~31u) + 65u * (uint32_t)j, 64u + 65u * (uint32_t)(8 + j));
      }
    }
    if (!lo) {
      zplanes<W>(w[st], Zt[st]);
#pragma unroll
      for (int p = 0; p < NP; ++p) xtr8(Zt[st][p][0], Zt[st][p][1], j);
      uint32_t above = 0;
#pragma unroll
      for (int p = NP - 1; p >= 0; --p) {
        const uint32_t c = __builtin_popcount(Zt[st][p][0]) + __builtin_popcount(Zt[st][p][1]);
        uint32_t sk = group8_suffix2(c, j);
        if (p < NP - 1) sk += above << (8 - j);
        if constexpr (W > 16) sk = min(sk, kSumCap);
        key = min(key, ((sk + 95u) & ~31u) + 65u * (uint32_t)(8 * p + j));
        if (p > 0) above = group8_first(sk, j);
      }
    }
    key = group8_min(key, j);
    // key == 64 <=> k = 0 with 2 words <=> S_0 == 0: an all-zero block
    const bool zero = key == 64u || !has;
    const uint32_t prm = zero ? 0u : (key & 31u) + 1u;
    const uint32_t words = zero ? 0u : key >> 5;
    if (j == 0 && has) {
      pside[8 * st] = (uint8_t)prm;  // immediate offsets from one lane pointer per array
      wside[8 * st] = (uint8_t)words;
    }
    uint32_t stot;
    pb[st] = prm | ((wtot + wave_groups_excl(words, lane, &stot)) << 6);
    wtot += stot;
  }
  // ---- the tile's start: workgroup sum; wave 0 publishes the aggregate and issues the first
  // look-back reads, which are in flight while every wave stages its payload in LDS ----
  if (lane == 0) wsum[wv] = wtot;
  __syncthreads();
  uint32_t agg = 0, wbase = 0;
#pragma unroll
  for (int q = 0; q < kEncWaves; ++q) {
    wbase += q < wv ? wsum[q] : 0u;
    agg += wsum[q];
  }
  // decoupled look-back by the whole first wave: lane l reads the state of tile base - l, so each
  // memory round trip covers 64 predecessors (a thread walking them one by one serialised the chain
  // at ~0.5 us per tile; 256 per round trip measured slower: more registers).  The states are the
  // only data exchanged, so relaxed agent-scope atomics suffice
  int64_t base = g - 1;
  uint64_t v = 0;
  if (wv == 0) {
    if (lane == 0) __hip_atomic_store(&state[g], (g == 0 ? kFlagPre : kFlagAgg) | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int64_t i = base - lane;
    if (g > 0) v = i >= 0 ? __hip_atomic_load(&state[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagPre;
  }
  // ---- pass 2: each step's block payloads staged in LDS at their wave-local word offsets: the k
  // low planes, then the unary part (one LDS or per 32 bits of a lane's codes into the zeroed stage) ----
#pragma unroll
  for (int st = 0; st < S; ++st) {
    const int param = (int)(pb[st] & 63u);
    const uint32_t off = pb[st] >> 6;
    const int k = param > 0 ? param - 1 : 0;
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int b = 8 * p + j;
      if (param > 0 && b < k) {
        wl[off + 2 * b] = Zt[st][p][0];
        wl[off + 2 * b + 1] = Zt[st][p][1];
      }
    }
    uint32_t q[8];
    quotients<W>(w[st], k, q);
    // r[e]: bit of sample e's terminator relative to the lane's first code
    uint32_t r[8];
    r[0] = q[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) r[e] = r[e - 1] + q[e] + 1u;
    const uint32_t len = r[7] + 1u;
    const uint32_t incl = group8_incl(len, lane & 8);
    const uint32_t uw = (group8_last(incl, j) + 31u) >> 5;
    uint32_t* const us = wl + off + 2 * k;
    const uint32_t pos0 = incl - len;
    if (param > 0) {
      if (len <= 32u) {  // the lane's 8 codes in one 32-bit mask: at most 2 LDS ors
        uint32_t m = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) m |= 1u << r[e];
        const uint32_t wd = pos0 >> 5;
        const uint64_t mm = (uint64_t)m << (pos0 & 31u);
        atomicOr(&us[wd], (uint32_t)mm);
        if ((uint32_t)(mm >> 32)) atomicOr(&us[wd + 1], (uint32_t)(mm >> 32));
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t pos = pos0 + r[e];
          if (pos < 32u * min(uw, (uint32_t)UMAX)) atomicOr(&us[pos >> 5], 1u << (pos & 31));
        }
      }
    }
  }
  // ---- wave 0 completes the look-back ----
  if (wv == 0) {
    uint64_t excl = 0;
    if (g > 0) {
      while (true) {
        while (__any((v >> 62) == 0)) {  // a predecessor has not published yet: re-read those
          __builtin_amdgcn_s_sleep(1);
          if ((v >> 62) == 0) v = __hip_atomic_load(&state[base - lane], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint64_t pre = __ballot((v >> 62) == 2);  // tiles whose inclusive prefix is known
        const int lp = pre ? __builtin_ctzll(pre) : 64;  // the nearest one
        uint64_t c = lane <= lp ? (v & kValMask) : 0;  // aggregates after it, and its prefix
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) c += __shfl_xor(c, d, 64);
        excl += c;
        if (pre) break;
        base -= 64;
        const int64_t i = base - lane;
        v = i >= 0 ? __hip_atomic_load(&state[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : kFlagPre;
      }
      if (lane == 0) __hip_atomic_store(&state[g], kFlagPre | (excl + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_excl = excl;
      ((uint64_t*)(blob + R.toff_off))[t] = excl;
      uint64_t* rec = (uint64_t*)(blob + R.rec_off);
      if (t == 0) rec[0] = excl;
      if (t == R.ntile - 1) {
        rec[1] = excl + agg;
        for (int64_t b = R.nb; b < ((R.nb + 7) & ~(int64_t)7); ++b) params[b] = bw[b] = 0;  // the side arrays' padding
      }
      if (g == tiles_total - 1) {  // the bundle's payload words and byte size (header fields 56, 64)
        ((uint64_t*)blob)[7] = excl + agg;
        ((uint64_t*)blob)[8] = (uint64_t)payload_off + (((excl + agg) * 4 + 7) & ~7ull);
        if ((excl + agg) & 1) ((uint32_t*)(blob + payload_off))[excl + agg] = 0u;  // the payload's padding to 8 bytes
      }
    }
  }
  __syncthreads();
  // ---- the wave's payload words are contiguous: one coalesced copy out of LDS ----
  uint32_t* const dst = (uint32_t*)(blob + payload_off) + (s_excl + wbase);
  for (uint32_t i = lane; i < wtot; i += 64) dst[i] = wl[i];
}

// the lane's 8 samples from their quotients and low bits: unzigzag((q << k) | low); 16-bit samples
// two at a time (for a valid stream q << k < 2^16, so the packed shift loses nothing)
template <int W>
__device__ __forceinline__ void samples_from_codes(const uint32_t (&q)[8], int k, const uint32_t (&lowv)[Sw<W>::NW],
                                                   bool coded, uint32_t (&wout)[Sw<W>::NW]) {
  if constexpr (W == 16) {
    const u16x2 kk = {(unsigned short)k, (unsigned short)k};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const u16x2 qv = __builtin_bit_cast(u16x2, (q[2 * i] & 0xffffu) | (q[2 * i + 1] << 16));
      const u16x2 z = (u16x2)(qv << kk) | __builtin_bit_cast(u16x2, lowv[i]);
      const u16x2 v = (u16x2)(z >> (u16x2){1, 1}) ^ (u16x2)((u16x2){0, 0} - (z & (u16x2){1, 1}));
      wout[i] = coded ? __builtin_bit_cast(uint32_t, v) : 0u;
    }
  } else {
#pragma unroll
    for (int i = 0; i < Sw<W>::NW; ++i) wout[i] = 0u;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const uint32_t z = coded ? (q[e] << k) | sample_of<W>(lowv, e) : 0u;
      set_sample<W>(wout, e, unzigzag<W>(z));
    }
  }
}

template <int W>
__global__ void __launch_bounds__(256) rice_bundle_decode_kernel(RArrs A, int64_t tile_begin,
                                                               const uint8_t* __restrict__ blob,
                                                               int64_t payload_off, uint64_t payload_words,
                                                               unsigned long long* __restrict__ bad_out) {
  constexpr int NP = Sw<W>::NP, NW = Sw<W>::NW;
  constexpr int SPAN = 8 * (2 * W + 2);  // payload words of a wave step's 8 blocks, at most
  constexpr int S = kTileSteps;
  __shared__ uint32_t span_lds[4][S * SPAN];  // each wave's payload words (contiguous in the payload)
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t wbad[4];
  const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, j = lane & 7, g8 = lane >> 3;
  const int64_t g = tile_begin + blockIdx.x;
  const int a = array_of(A, g);
  const RArr& R = A.a[a];
  const int64_t t = g - R.tile0;
  const int64_t blk0 = t * kTileBlocks + wv * 8 * S;
  const uint8_t* params = blob + R.side_off;
  const uint8_t* bwp = params + ((R.nb + 7) & ~(int64_t)7);
  // ---- the side information of the wave's S steps, checked; per-block offsets in the wave ----
  int prm[S], wds[S];
  uint32_t bex[S], stp[S];
  uint32_t wtot = 0;
  bool bad = false;
#pragma unroll
  for (int st = 0; st < S; ++st) {
    const int64_t blk = blk0 + 8 * st + g8;
    const bool has = blk < R.nb;
    prm[st] = has ? params[blk] : 0;
    wds[st] = has ? bwp[blk] : 0;
  }
#pragma unroll
  for (int st = 0; st < S; ++st) {
    const int kk = prm[st] - 1;
    const bool b = prm[st] == 0 ? wds[st] != 0 : (kk >= W || wds[st] < 2 * kk + 2 || wds[st] > 2 * W + 2);
    bad |= b;
    if (b) wds[st] = 0;  // keeps the offsets of the good blocks in bounds
    uint32_t stot;
    bex[st] = wave_groups_excl((uint32_t)wds[st], lane, &stot);
    stp[st] = wtot;
    wtot += stot;
  }
  const bool wave_bad = __any(bad);
  if (lane == 0) {
    wsum[wv] = wtot;
    wbad[wv] = wave_bad;
  }
  __syncthreads();
  const uint64_t* toff = (const uint64_t*)(blob + R.toff_off);
  const uint64_t* rec = (const uint64_t*)(blob + R.rec_off);
  const uint64_t start = toff[t];
  const uint64_t end = t + 1 < R.ntile ? toff[t + 1] : rec[1];
  const uint32_t agg = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  const bool tile_bad = wbad[0] || wbad[1] || wbad[2] || wbad[3] || start > payload_words || end > payload_words ||
                        start + agg != end || (t == 0 && start != rec[0]);
  if (tile_bad && tid == 0) atomicAdd(bad_out, 1ull);
  uint32_t wbase = 0;
  for (int q = 0; q < wv; ++q) wbase += wsum[q];
  // ---- the wave's payload words (all S steps: one contiguous span) staged in LDS at once, 8
  // loads per lane in flight (a span per step paid one memory latency per step) ----
  uint32_t* const wspan = span_lds[wv];
  {
    const uint32_t* src = (const uint32_t*)(blob + payload_off) + (start + wbase);
    const int cnt = tile_bad ? 0 : (int)min(wtot, (uint32_t)(S * SPAN));
    for (int i0 = 0; i0 < cnt; i0 += 64 * 8) {
      uint32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u + lane;
        v[u] = i < cnt ? src[i] : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + 64 * u + lane;
        if (i < cnt) wspan[i] = v[u];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  // ---- per step: unpack the 8 blocks (fully unrolled: the steps' side information, offsets and
  // uniform branch conditions resolve per step at compile time instead of in a runtime loop --
  // 157-159 -> 142-143 us per C3 bundle, profiles/round5/ab_rice_decode_unroll_r5k2.txt) ----
#pragma unroll
  for (int st = 0; st < S; ++st) {
    int param = tile_bad ? 0 : prm[st];
    const int words = tile_bad ? 0 : wds[st];
    const uint32_t* const bp = wspan + (tile_bad ? 0 : stp[st] + bex[st]);
    const int k = param > 0 ? param - 1 : 0;
    const int uw = param > 0 ? words - 2 * k : 0;
    uint32_t Z[NP][2];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int b = 8 * p + j;
      const bool hv = param > 0 && b < k;
      Z[p][0] = hv ? bp[2 * b] : 0u;
      Z[p][1] = hv ? bp[2 * b + 1] : 0u;
    }
    // every block of the wave step with k <= 8 (the usual residual map): plane groups from 1 up
    // hold no stored planes (all zero), so only group 0 is transposed back
    const bool lo8 = __all(param <= 9);
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      if (p > 0 && lo8) continue;
      xtr8(Z[p][0], Z[p][1], j);
      tr8x8(Z[p][0], Z[p][1]);
    }
    uint32_t lowv[NW];
    scatter_bytes<W>(Z, lowv);
    const uint32_t* us = bp + 2 * k;
    uint32_t q[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) q[e] = 0u;
    // lane j's first code follows terminator 8j - 1.  Streams of at most 8 words (the usual case):
    // lane m holds word m and its popcount c_m; with the group's inclusive counts cum_m, the word
    // holding terminator 8j - 1 is #{m : cum_m >> 3 < j}, counted for all j at once as nibble j of
    // a group sum (lane m adds 1 to the nibbles j > cum_m >> 3); then one select in that word.
    // No loop and no LDS round trip per word (a walk word by word measured slower)
    uint32_t pos8 = 0;
    const bool short_stream = __all(!(param > 0) || uw <= 8);
    if (short_stream) {
      const uint32_t wm = (param > 0 && j < uw) ? us[j] : 0u;
      const uint32_t cm = __builtin_popcount(wm);
      const uint32_t cum = group8_incl(cm, lane & 8);
      const uint32_t d = cum >> 3;
      const uint32_t f = d >= 7u ? 0u : 0x11111110u & (~0u << (4u * (d + 1u)));
      const uint32_t F = group8_sum(f, j);
      const uint32_t wi = (F >> (4 * j)) & 15u;  // j > 0
      const int src = (lane & ~7) | (int)min(wi, 7u);
      const uint32_t wsel = (uint32_t)__shfl((int)wm, src, 64);
      const uint32_t before = (uint32_t)__shfl((int)(cum - cm), src, 64);
      pos8 = j == 0 ? 0u : wi < 8u && wi < (uint32_t)uw ? 32u * wi + select32(wsel, 8u * j - 1u - before) + 1u
                                                         : 32u * (uint32_t)uw;
    }
    if (param > 0 && uw > 0) {
      uint32_t pos = pos8;
      if (!short_stream && j > 0) {
        const uint32_t r = 8u * j - 1u;
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
      const uint32_t sh = pos & 31u;
      const uint32_t a0 = wi < uw ? us[wi] : 0u, b0 = wi + 1 < uw ? us[wi + 1] : 0u;
      uint32_t x = __builtin_amdgcn_alignbit(b0, a0, sh);
      if (__builtin_popcount(x) >= 8) {  // the lane's 8 codes within 32 bits (the common case)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t tz = (uint32_t)__builtin_ctz(x);
          q[e] = tz;
          x = (x >> tz) >> 1;
        }
      } else {
        const uint32_t c0 = wi + 2 < uw ? us[wi + 2] : 0u;
        uint64_t win = ((uint64_t)__builtin_amdgcn_alignbit(c0, b0, sh) << 32) | x;
        if (__builtin_popcountll(win) >= 8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t tz = (uint32_t)__builtin_ctzll(win);
            q[e] = tz;
            win = (win >> tz) >> 1;
          }
        } else {
          uint32_t cur = wi < uw ? us[wi] >> sh : 0u;
          uint32_t base = pos;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            while (cur == 0u && wi + 1 < uw) {
              ++wi;
              cur = us[wi];
              base = 32u * wi;
            }
            if (cur == 0u) break;  // a corrupt stream with fewer than 64 terminators
            const uint32_t tz = __builtin_ctz(cur);
            q[e] = base + tz - pos;
            pos = base + tz + 1u;
            cur = tz == 31u ? 0u : cur >> (tz + 1u);
            base = pos;
          }
        }
      }
    }
    uint32_t wout[NW];
    samples_from_codes<W>(q, k, lowv, param > 0, wout);
    const int64_t blk = blk0 + 8 * st + g8;
    if (blk < R.nb) store8s<W>((void*)R.x, R.n, blk * 64 + j * 8, wout);
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

int64_t kmp_rice_tiles(int64_t n) { return n > 0 ? ceil_div(kmp_pack_blocks(n), (int64_t)rc::kTileBlocks) : 0; }

static int rice_arrays(const kmp_rice_array* arrays, int32_t count, int64_t tile_begin, rc::RArrs& A,
                       int64_t& tiles) {
  KMP_REQUIRE(arrays && count >= 1 && count <= rc::kMaxArr, "rice bundle: 1 .. 32 arrays per call");
  A.count = count;
  tiles = 0;
  for (int i = 0; i < count; ++i) {
    const kmp_rice_array& s = arrays[i];
    KMP_REQUIRE(s.n >= 0 && (s.n == 0 || s.samples), "rice bundle: bad array");
    KMP_REQUIRE(s.side_off >= 0 && s.toff_off % 8 == 0 && s.rec_off % 8 == 0, "rice bundle: bad layout");
    rc::RArr& r = A.a[i];
    r.x = s.samples;
    r.n = s.n;
    r.nb = kmp_pack_blocks(s.n);
    r.ntile = kmp_rice_tiles(s.n);
    r.tile0 = tile_begin + tiles;
    r.side_off = s.side_off;
    r.toff_off = s.toff_off;
    r.rec_off = s.rec_off;
    tiles += r.ntile;
  }
  return KMP_OK;
}

int kmp_rice_bundle_encode(int32_t dtype, const kmp_rice_array* arrays, int32_t count, int64_t tile_begin,
                           int64_t tiles_total, uint8_t* bundle, int64_t payload_off, void* workspace,
                           kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "rice bundle: unsupported dtype");
  KMP_REQUIRE(bundle && workspace && payload_off % 8 == 0 && tile_begin >= 0 && tiles_total >= 0,
              "rice bundle: bad argument");
  rc::RArrs A{};
  int64_t tiles = 0;
  if (int st = rice_arrays(arrays, count, tile_begin, A, tiles)) return st;
  KMP_REQUIRE(tile_begin + tiles <= tiles_total, "rice bundle: tiles past the total");
  uint64_t* state = (uint64_t*)workspace;
  unsigned* ticket = (unsigned*)(state + tiles_total);
  hipStream_t s = (hipStream_t)stream;
  if (tile_begin == 0 && hipMemsetAsync(state, 0, (size_t)tiles_total * 8, s) != hipSuccess)
    return fail(KMP_ERR_LAUNCH, "rice bundle: memset");
  if (hipMemsetAsync(ticket, 0, sizeof(unsigned), s) != hipSuccess) return fail(KMP_ERR_LAUNCH, "rice bundle: memset");
  if (tiles == 0) return KMP_OK;
  KMP_REQUIRE(tiles < ((int64_t)1 << 31), "rice bundle: too many tiles in one call");
  if (W == 8) rc::rice_bundle_encode_kernel<8><<<(unsigned)tiles, 64 * rc::kEncWaves, 0, s>>>(A, tile_begin, tiles_total, bundle, payload_off, state, ticket);
  else if (W == 16) rc::rice_bundle_encode_kernel<16><<<(unsigned)tiles, 64 * rc::kEncWaves, 0, s>>>(A, tile_begin, tiles_total, bundle, payload_off, state, ticket);
  else rc::rice_bundle_encode_kernel<32><<<(unsigned)tiles, 64 * rc::kEncWaves, 0, s>>>(A, tile_begin, tiles_total, bundle, payload_off, state, ticket);
  return check_launch("rice_bundle_encode");
}

int64_t kmp_rice_bundle_workspace_bytes(int64_t tiles_total) { return 8 * tiles_total + 8; }

int kmp_rice_bundle_decode(int32_t dtype, const kmp_rice_array* arrays, int32_t count, int64_t tile_begin,
                           const uint8_t* bundle, int64_t payload_off, uint64_t payload_words,
                           unsigned long long* bad, kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "rice bundle: unsupported dtype");
  KMP_REQUIRE(bundle && bad && payload_off % 8 == 0 && tile_begin >= 0, "rice bundle: bad argument");
  rc::RArrs A{};
  int64_t tiles = 0;
  if (int st = rice_arrays(arrays, count, tile_begin, A, tiles)) return st;
  if (tiles == 0) return KMP_OK;
  KMP_REQUIRE(tiles < ((int64_t)1 << 31), "rice bundle: too many tiles in one call");
  hipStream_t s = (hipStream_t)stream;
  if (W == 8) rc::rice_bundle_decode_kernel<8><<<(unsigned)tiles, 256, 0, s>>>(A, tile_begin, bundle, payload_off, payload_words, bad);
  else if (W == 16) rc::rice_bundle_decode_kernel<16><<<(unsigned)tiles, 256, 0, s>>>(A, tile_begin, bundle, payload_off, payload_words, bad);
  else rc::rice_bundle_decode_kernel<32><<<(unsigned)tiles, 256, 0, s>>>(A, tile_begin, bundle, payload_off, payload_words, bad);
  return check_launch("rice_bundle_decode");
}

}  // extern "C"
