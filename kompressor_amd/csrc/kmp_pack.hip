// kmp_pack.hip -- bit-plane packing of coded maps (the reference stops at
// residual arrays, volume/encode_decode.py:56, so the bytes never shrink; this is the build's
// container payload, no reference counterpart -- its spec is oracle/packing.py).
//
// A coded map is a flat array of W-bit samples (W = 8, 16, 32).  Residuals of a good predictor are
// small signed values modulo 2^W, so each sample is zigzag-mapped (z = (s << 1) ^ (s >> (W-1)) of
// its signed W-bit reading: 0, -1, 1, -2 ... -> 0, 1, 2, 3 ...), and every block of 64 samples is
// stored as `width` 64-bit bit-planes, width = the bit length of the block's largest z (0 for an
// all-zero block).  On a 64-lane wavefront one block is one wave, and bit-plane i of the block is
// exactly ``ballot((z >> i) & 1)``: packing is `width` ballots, unpacking `width` uniform words
// read by every lane -- no cross-lane bit shuffling at all.
//
// Launches: widths -> per-chunk exclusive scan of the widths (4096 blocks per workgroup) -> scan
// of the chunk sums (one workgroup) -> pack / unpack.  The payload offset of block b, in 64-bit
// words, is chunk_base[b / 4096] + local[b].  Every kernel moves the samples as one 16-byte
// vector per lane: a wave covers SPL = 128 / W blocks per step (16 B = SPL samples per lane), so
// it has one load in flight per SPL blocks instead of one 2-byte load per block; pack / unpack
// turn that layout into one-sample-per-lane (the ballot layout) through 1 KB of LDS per wave.
#include "kmp_common.h"

namespace kmp {
namespace pk {

constexpr int kBlock = 64;         // samples per block == lanes per wave
constexpr int kChunk = 4096;       // blocks per scan chunk
constexpr int kScanThreads = 256;  // 16 blocks per thread
constexpr int kPackHeadMax = 128;  // header bytes a kmp_pack_header call can write

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

// 16 bytes of samples per lane: lanes g*LPB .. g*LPB+LPB-1 of a wave step hold block g (SPL blocks)
template <int W>
struct Lay {
  static constexpr int SPL = 128 / W;       // samples per lane == blocks per wave step
  static constexpr int LPB = kBlock / SPL;  // lanes per block
};
typedef uint32_t u32x4a1 __attribute__((ext_vector_type(4), aligned(1)));

template <int W>
__device__ __forceinline__ u32x4v load16(const void* x, int64_t n, int64_t i0) {  // samples i0 .. i0+SPL-1
  constexpr int SPL = Lay<W>::SPL;
  if (i0 + SPL <= n) return *(const u32x4a1*)((const char*)x + i0 * (W / 8));
  u32x4v v = {0u, 0u, 0u, 0u};
  for (int e = 0; e < SPL; ++e) {
    if (i0 + e >= n) break;
    const uint32_t s = load_sample<W>(x, i0 + e);
    v[(e * W) / 32] |= s << ((e * W) % 32);
  }
  return v;
}
template <int W>
__device__ __forceinline__ uint32_t elem(const u32x4v& v, int e) {
  if constexpr (W == 32) return v[e];
  else return (v[(e * W) / 32] >> ((e * W) % 32)) & ((1u << W) - 1u);
}

// wave step: widths of SPL consecutive blocks (OR within the lane, then across its LPB lanes)
template <int W>
__global__ void __launch_bounds__(256) widths_kernel(const void* __restrict__ x, int64_t n, uint8_t* __restrict__ widths,
                                                   int64_t nb) {
  constexpr int SPL = Lay<W>::SPL, LPB = Lay<W>::LPB;
  const int lane = threadIdx.x & 63;
  const int64_t nstep = (nb + SPL - 1) / SPL;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const u32x4v v = load16<W>(x, n, st * SPL * kBlock + (int64_t)lane * SPL);
    uint32_t o = 0;
#pragma unroll
    for (int e = 0; e < SPL; ++e) o |= zigzag<W>(elem<W>(v, e));
#pragma unroll
    for (int d = 1; d < LPB; d <<= 1) o |= (uint32_t)__shfl_xor((int)o, d, 64);
    const int64_t blk = st * SPL + lane / LPB;
    if (lane % LPB == 0 && blk < nb) widths[blk] = (uint8_t)(o ? 32 - __clz(o) : 0);
  }
}

// exclusive scan of the widths inside each chunk of kChunk blocks; chunk totals to ``sums``
__global__ void __launch_bounds__(kScanThreads) scan_local_kernel(const uint8_t* __restrict__ widths, int64_t nb,
                                                                 uint32_t* __restrict__ local,
                                                                 uint64_t* __restrict__ sums) {
  constexpr int PER = kChunk / kScanThreads;
  __shared__ uint32_t part[kScanThreads];
  const int64_t base = (int64_t)blockIdx.x * kChunk + (int64_t)threadIdx.x * PER;
  uint32_t w[PER], s = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    w[j] = base + j < nb ? widths[base + j] : 0u;
    s += w[j];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < kScanThreads; d <<= 1) {  // Hillis-Steele inclusive scan of the thread sums
    const uint32_t add = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0u;
    __syncthreads();
    part[threadIdx.x] += add;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;  // exclusive
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    if (base + j < nb) local[base + j] = run;
    run += w[j];
  }
  if (threadIdx.x == kScanThreads - 1) sums[blockIdx.x] = part[threadIdx.x];
}

// exclusive scan of the chunk sums (one workgroup, sequential over tiles of 1024); total words
__global__ void __launch_bounds__(1024) scan_chunks_kernel(const uint64_t* __restrict__ sums, int64_t nchunk,
                                                          uint64_t* __restrict__ cbase, uint64_t* __restrict__ total) {
  __shared__ uint64_t part[1024];
  uint64_t carry = 0;
  for (int64_t t0 = 0; t0 < nchunk; t0 += 1024) {
    const int64_t i = t0 + threadIdx.x;
    const uint64_t v = i < nchunk ? sums[i] : 0ull;
    part[threadIdx.x] = v;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const uint64_t add = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0ull;
      __syncthreads();
      part[threadIdx.x] += add;
      __syncthreads();
    }
    if (i < nchunk) cbase[i] = carry + part[threadIdx.x] - v;
    const uint64_t tile = part[1023];
    __syncthreads();
    carry += tile;
  }
  if (threadIdx.x == 0) *total = carry;
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l), hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// wave step: SPL blocks; samples land in LDS as 16 B per lane and are re-read one per lane per
// block; lane j < SPL fetches block j's width and offset, broadcast with readlane
template <int W>
__global__ void __launch_bounds__(256) pack_kernel(const void* __restrict__ x, int64_t n,
                                                 const uint8_t* __restrict__ widths, const uint32_t* __restrict__ local,
                                                 const uint64_t* __restrict__ cbase, int64_t nb,
                                                 uint64_t* __restrict__ payload) {
  constexpr int SPL = Lay<W>::SPL;
  __shared__ u32x4v stage[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nstep = (nb + SPL - 1) / SPL;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t blk0 = st * SPL;
    const u32x4v v = load16<W>(x, n, blk0 * kBlock + (int64_t)lane * SPL);
    uint32_t wj = 0;
    uint64_t oj = 0;
    if (lane < SPL && blk0 + lane < nb) {
      wj = widths[blk0 + lane];
      oj = cbase[(blk0 + lane) / kChunk] + local[blk0 + lane];
    }
    stage[wv][lane] = v;
    wave_lds_sync();
    const unsigned char* sb = (const unsigned char*)stage[wv];
    for (int g = 0; g < SPL; ++g) {
      if (blk0 + g >= nb) break;  // uniform
      const int w = (int)__builtin_amdgcn_readlane(wj, g);
      const uint64_t off = readlane64(oj, g);
      uint32_t smp;
      if constexpr (W == 8) smp = sb[g * 64 + lane];
      else if constexpr (W == 16) smp = ((const uint16_t*)sb)[g * 64 + lane];
      else smp = ((const uint32_t*)sb)[g * 64 + lane];
      const uint32_t z = zigzag<W>(smp);
      uint64_t mine = 0;
      for (int b = 0; b < w; ++b) {  // bit-plane b of the block, kept by lane b
        const uint64_t plane = __ballot((z >> b) & 1u);
        mine = lane == b ? plane : mine;
      }
      if (lane < w) payload[off + lane] = mine;
    }
    wave_lds_sync();
  }
}

// wave step: SPL blocks; every block's planes are loaded up front (lane b holds plane b), each
// sample is rebuilt from readlane-broadcast planes into LDS, then stored as 16 B per lane
template <int W>
__global__ void __launch_bounds__(256) unpack_kernel(const uint64_t* __restrict__ payload, int64_t n,
                                                   const uint8_t* __restrict__ widths,
                                                   const uint32_t* __restrict__ local,
                                                   const uint64_t* __restrict__ cbase, int64_t nb, void* __restrict__ out) {
  constexpr int SPL = Lay<W>::SPL;
  __shared__ u32x4v stage[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t nstep = (nb + SPL - 1) / SPL;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t blk0 = st * SPL;
    uint32_t wj = 0;
    uint64_t oj = 0;
    if (lane < SPL && blk0 + lane < nb) {
      wj = widths[blk0 + lane];
      oj = cbase[(blk0 + lane) / kChunk] + local[blk0 + lane];
    }
    uint64_t mine[SPL];
#pragma unroll
    for (int g = 0; g < SPL; ++g) {
      const int w = (int)__builtin_amdgcn_readlane(wj, g);  // 0 past the last block
      mine[g] = lane < w ? payload[readlane64(oj, g) + lane] : 0ull;
    }
    unsigned char* sb = (unsigned char*)stage[wv];
#pragma unroll
    for (int g = 0; g < SPL; ++g) {
      const int w = (int)__builtin_amdgcn_readlane(wj, g);
      uint32_t z = 0;
      for (int b = 0; b < w; ++b) z |= (uint32_t)(readlane64(mine[g], b) >> lane & 1u) << b;
      const uint32_t v = unzigzag<W>(z);
      if constexpr (W == 8) sb[g * 64 + lane] = (uint8_t)v;
      else if constexpr (W == 16) ((uint16_t*)sb)[g * 64 + lane] = (uint16_t)v;
      else ((uint32_t*)sb)[g * 64 + lane] = v;
    }
    wave_lds_sync();
    const u32x4v v = stage[wv][lane];
    const int64_t i0 = blk0 * kBlock + (int64_t)lane * SPL;
    if (i0 + SPL <= n) {
      *(u32x4a1*)((char*)out + i0 * (W / 8)) = v;
    } else {
      for (int e = 0; e < SPL; ++e) {
        if (i0 + e >= n) break;
        store_sample<W>(out, i0 + e, elem<W>(v, e));
      }
    }
    wave_lds_sync();
  }
}

// container header from kernel arguments (no host-to-device copy): bytes [0, len), zeros over
// [zfrom, zto), and the scan's total word count (u64) at ``words_at`` when >= 0
struct HeadBytes {
  uint8_t b[kPackHeadMax];
};
__global__ void __launch_bounds__(128) header_kernel(uint8_t* __restrict__ dst, HeadBytes h, int len, int64_t zfrom,
                                                    int64_t zto, const uint64_t* __restrict__ total, int64_t words_at) {
  for (int i = threadIdx.x; i < len; i += 128) dst[i] = h.b[i];
  for (int64_t i = zfrom + threadIdx.x; i < zto; i += 128) dst[i] = 0;
  if (words_at >= 0 && threadIdx.x < 8) dst[words_at + threadIdx.x] = (uint8_t)(*total >> (8 * threadIdx.x));
}

template <int W>
static inline unsigned waves_grid(int64_t nb) {
  int64_t g = ceil_div(ceil_div(nb, (int64_t)Lay<W>::SPL), 4);  // a wave step = SPL blocks, 4 waves per workgroup
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

static int sample_bits(int dtype) {
  switch (dtype) {
    case KMP_U8: return 8;
    case KMP_U16: return 16;
    case KMP_I32: case KMP_U32: case KMP_F32: return 32;
    default: return 0;
  }
}

struct Ws {  // workspace carve-up
  uint32_t* local;
  uint64_t* sums;
  uint64_t* cbase;
  uint64_t* total;
};
static Ws carve(void* ws, int64_t nb) {
  const int64_t nchunk = ceil_div(nb, kChunk);
  char* p = (char*)ws;
  Ws w;
  w.local = (uint32_t*)p;
  p += ceil_div(nb * 4, 8) * 8;
  w.sums = (uint64_t*)p;
  p += nchunk * 8;
  w.cbase = (uint64_t*)p;
  p += nchunk * 8;
  w.total = (uint64_t*)p;
  return w;
}

static int scan(const uint8_t* widths, int64_t nb, const Ws& w, hipStream_t s) {
  const int64_t nchunk = ceil_div(nb, kChunk);
  if (nchunk > 0) {
    scan_local_kernel<<<(unsigned)nchunk, kScanThreads, 0, s>>>(widths, nb, w.local, w.sums);
    if (int st = check_launch("pack_scan")) return st;
  }
  scan_chunks_kernel<<<1, 1024, 0, s>>>(w.sums, nchunk, w.cbase, w.total);
  return check_launch("pack_scan");
}

}  // namespace pk
}  // namespace kmp

using namespace kmp;

extern "C" {

int64_t kmp_pack_blocks(int64_t n) { return n > 0 ? ceil_div(n, pk::kBlock) : 0; }

int64_t kmp_pack_workspace_bytes(int64_t n) {
  const int64_t nb = kmp_pack_blocks(n), nchunk = ceil_div(nb, pk::kChunk);
  return ceil_div(nb * 4, 8) * 8 + nchunk * 16 + 8;
}

int64_t kmp_pack_total_offset(int64_t n) {
  const int64_t nb = kmp_pack_blocks(n), nchunk = ceil_div(nb, pk::kChunk);
  return ceil_div(nb * 4, 8) * 8 + nchunk * 16;
}

int kmp_pack_plan(int32_t dtype, const void* x, int64_t n, uint8_t* widths, void* workspace, kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "pack: unsupported dtype");
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || (x && widths)), "pack: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  const pk::Ws w = pk::carve(workspace, nb);
  hipStream_t s = (hipStream_t)stream;
  if (nb > 0) {
    if (W == 8) pk::widths_kernel<8><<<pk::waves_grid<8>(nb), 256, 0, s>>>(x, n, widths, nb);
    else if (W == 16) pk::widths_kernel<16><<<pk::waves_grid<16>(nb), 256, 0, s>>>(x, n, widths, nb);
    else pk::widths_kernel<32><<<pk::waves_grid<32>(nb), 256, 0, s>>>(x, n, widths, nb);
    if (int st = check_launch("pack_widths")) return st;
  }
  return pk::scan(widths, nb, w, s);
}

int kmp_pack_header(uint8_t* dst, const uint8_t* bytes, int32_t len, int64_t zero_from, int64_t zero_to,
                    const void* workspace, int64_t n, int64_t words_at, kmp_stream_t stream) {
  KMP_REQUIRE(dst && len >= 0 && len <= pk::kPackHeadMax && (len == 0 || bytes), "pack_header: bad header");
  KMP_REQUIRE(zero_from >= 0 && zero_to - zero_from <= 4096, "pack_header: bad zero range");
  KMP_REQUIRE(words_at < 0 || workspace, "pack_header: no workspace");
  pk::HeadBytes h{};
  for (int i = 0; i < len; ++i) h.b[i] = bytes[i];
  const uint64_t* total = words_at >= 0 ? pk::carve((void*)workspace, kmp_pack_blocks(n)).total : nullptr;
  pk::header_kernel<<<1, 128, 0, (hipStream_t)stream>>>(dst, h, len, zero_from, zero_to, total, words_at);
  return check_launch("pack_header");
}

int kmp_unpack_plan(const uint8_t* widths, int64_t n, void* workspace, kmp_stream_t stream) {
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || widths), "unpack: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  return pk::scan(widths, nb, pk::carve(workspace, nb), (hipStream_t)stream);
}

int kmp_pack(int32_t dtype, const void* x, int64_t n, const uint8_t* widths, const void* workspace, uint64_t* payload,
             kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "pack: unsupported dtype");
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || (x && widths && payload)), "pack: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  if (nb == 0) return KMP_OK;
  const pk::Ws w = pk::carve((void*)workspace, nb);
  hipStream_t s = (hipStream_t)stream;
  if (W == 8) pk::pack_kernel<8><<<pk::waves_grid<8>(nb), 256, 0, s>>>(x, n, widths, w.local, w.cbase, nb, payload);
  else if (W == 16) pk::pack_kernel<16><<<pk::waves_grid<16>(nb), 256, 0, s>>>(x, n, widths, w.local, w.cbase, nb, payload);
  else pk::pack_kernel<32><<<pk::waves_grid<32>(nb), 256, 0, s>>>(x, n, widths, w.local, w.cbase, nb, payload);
  return check_launch("pack");
}

int kmp_unpack(int32_t dtype, const uint64_t* payload, int64_t n, const uint8_t* widths, const void* workspace,
               void* out, kmp_stream_t stream) {
  const int W = pk::sample_bits(dtype);
  KMP_REQUIRE(W > 0, "unpack: unsupported dtype");
  KMP_REQUIRE(n >= 0 && workspace && (n == 0 || (payload && widths && out)), "unpack: bad argument");
  const int64_t nb = kmp_pack_blocks(n);
  if (nb == 0) return KMP_OK;
  const pk::Ws w = pk::carve((void*)workspace, nb);
  hipStream_t s = (hipStream_t)stream;
  if (W == 8) pk::unpack_kernel<8><<<pk::waves_grid<8>(nb), 256, 0, s>>>(payload, n, widths, w.local, w.cbase, nb, out);
  else if (W == 16) pk::unpack_kernel<16><<<pk::waves_grid<16>(nb), 256, 0, s>>>(payload, n, widths, w.local, w.cbase, nb, out);
  else pk::unpack_kernel<32><<<pk::waves_grid<32>(nb), 256, 0, s>>>(payload, n, widths, w.local, w.cbase, nb, out);
  return check_launch("unpack");
}

}  // extern "C"
