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
// Launches: widths (one wave per block) -> per-chunk exclusive scan of the widths (4096 blocks
// per workgroup) -> scan of the chunk sums (one workgroup) -> pack / unpack (one wave per block).
// The payload offset of block b, in 64-bit words, is chunk_base[b / 4096] + local[b].
#include "kmp_common.h"

namespace kmp {
namespace pk {

constexpr int kBlock = 64;         // samples per block == lanes per wave
constexpr int kChunk = 4096;       // blocks per scan chunk
constexpr int kScanThreads = 256;  // 16 blocks per thread

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
  return W == 32 ? v : v & ((1u << W) - 1u);
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

// one wave per block: width = bit length of the OR of the block's zigzag values
template <int W>
__global__ void __launch_bounds__(256) widths_kernel(const void* __restrict__ x, int64_t n, uint8_t* __restrict__ widths,
                                                   int64_t nb) {
  const int lane = threadIdx.x & 63;
  for (int64_t blk = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; blk < nb;
       blk += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t i = blk * kBlock + lane;
    uint32_t z = i < n ? zigzag<W>(load_sample<W>(x, i)) : 0u;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) z |= (uint32_t)__shfl_xor((int)z, d, 64);
    if (lane == 0) widths[blk] = (uint8_t)(z ? 32 - __clz(z) : 0);
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

template <int W>
__global__ void __launch_bounds__(256) pack_kernel(const void* __restrict__ x, int64_t n,
                                                 const uint8_t* __restrict__ widths, const uint32_t* __restrict__ local,
                                                 const uint64_t* __restrict__ cbase, int64_t nb,
                                                 uint64_t* __restrict__ payload) {
  const int lane = threadIdx.x & 63;
  for (int64_t blk = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; blk < nb;
       blk += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t i = blk * kBlock + lane;
    const uint32_t z = i < n ? zigzag<W>(load_sample<W>(x, i)) : 0u;
    const int w = widths[blk];
    const uint64_t off = cbase[blk / kChunk] + local[blk];
    uint64_t mine = 0;
    for (int b = 0; b < w; ++b) {  // bit-plane b of the block, kept by lane b
      const uint64_t plane = __ballot((z >> b) & 1u);
      mine = lane == b ? plane : mine;
    }
    if (lane < w) payload[off + lane] = mine;
  }
}

template <int W>
__global__ void __launch_bounds__(256) unpack_kernel(const uint64_t* __restrict__ payload, int64_t n,
                                                   const uint8_t* __restrict__ widths,
                                                   const uint32_t* __restrict__ local,
                                                   const uint64_t* __restrict__ cbase, int64_t nb, void* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  for (int64_t blk = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; blk < nb;
       blk += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int w = widths[blk];
    const uint64_t off = cbase[blk / kChunk] + local[blk];
    const uint64_t mine = lane < w ? payload[off + lane] : 0ull;  // lane b holds bit-plane b
    uint32_t z = 0;
    for (int b = 0; b < w; ++b) {
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)mine, b, 64);
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(mine >> 32), b, 64);
      const uint32_t bit = lane < 32 ? (lo >> lane) & 1u : (hi >> (lane - 32)) & 1u;
      z |= bit << b;
    }
    const int64_t i = blk * kBlock + lane;
    if (i < n) store_sample<W>(out, i, unzigzag<W>(z));
  }
}

static inline unsigned waves_grid(int64_t nb) {
  int64_t g = ceil_div(nb, 4);  // 4 waves per 256-thread workgroup
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
    if (W == 8) pk::widths_kernel<8><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, widths, nb);
    else if (W == 16) pk::widths_kernel<16><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, widths, nb);
    else pk::widths_kernel<32><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, widths, nb);
    if (int st = check_launch("pack_widths")) return st;
  }
  return pk::scan(widths, nb, w, s);
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
  if (W == 8) pk::pack_kernel<8><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, widths, w.local, w.cbase, nb, payload);
  else if (W == 16) pk::pack_kernel<16><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, widths, w.local, w.cbase, nb, payload);
  else pk::pack_kernel<32><<<pk::waves_grid(nb), 256, 0, s>>>(x, n, widths, w.local, w.cbase, nb, payload);
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
  if (W == 8) pk::unpack_kernel<8><<<pk::waves_grid(nb), 256, 0, s>>>(payload, n, widths, w.local, w.cbase, nb, out);
  else if (W == 16) pk::unpack_kernel<16><<<pk::waves_grid(nb), 256, 0, s>>>(payload, n, widths, w.local, w.cbase, nb, out);
  else pk::unpack_kernel<32><<<pk::waves_grid(nb), 256, 0, s>>>(payload, n, widths, w.local, w.cbase, nb, out);
  return check_launch("unpack");
}

}  // extern "C"
