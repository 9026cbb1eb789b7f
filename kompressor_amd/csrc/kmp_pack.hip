// kmp_pack.hip -- bit-plane packing of coded maps (the reference stops at
// residual arrays, volume/encode_decode.py:56, so the bytes never shrink; this is the build's
// container payload, no reference counterpart -- its spec is oracle/packing.py).
//
// A coded map is a flat array of W-bit samples (W = 8, 16, 32).  Residuals of a good predictor are
// small signed values modulo 2^W, so each sample is zigzag-mapped (z = (s << 1) ^ (s >> (W-1)) of
// its signed W-bit reading: 0, -1, 1, -2 ... -> 0, 1, 2, 3 ...), and every block of 64 samples is
// stored as `width` 64-bit bit-planes, width = the bit length of the block's largest z (0 for an
// all-zero block).  Plane b of a block is the 64-bit word whose bit s is bit b of sample s.
//
// Launches: widths -> per-chunk exclusive scan of the widths (kChunk blocks per workgroup) -> scan
// of the chunk sums (one workgroup) -> pack / unpack.  The payload offset of block b, in 64-bit
// words, is chunk_base[b / kChunk] + local[b].  Every kernel gives a lane 8 consecutive samples
// (one 8 / 16 / 32-byte load), so a wave step covers 8 blocks; pack / unpack build the planes with
// register bit transposes and a cross-lane byte transpose (see ``xtr8``), no LDS, no ballots --
// the ballot-per-plane form was VALU-bound at 7 instructions per plane.
#include "kmp_bits.h"

namespace kmp {
namespace pk {

constexpr int kPackHeadMax = 128;  // header bytes a kmp_pack_header call can write

// per block OR of the zigzag samples -> width; lane 8g+0 writes block g's
template <int W>
__global__ void __launch_bounds__(256) widths_kernel(const void* __restrict__ x, int64_t n, uint8_t* __restrict__ widths,
                                                   int64_t nb) {
  const int lane = threadIdx.x & 63;
  const int64_t nstep = (nb + 7) / 8;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    uint32_t w[Sw<W>::NW];
    load8s<W>(x, n, st * 512 + (int64_t)lane * 8, w);
    // OR of the zigzag samples without forming them: z = ((s ^ m) << 1) | (m & 1), m = the sign
    // replicated, so OR z = (OR (s ^ m)) << 1 | (any sample negative)
    uint32_t acc = 0, neg = 0;
#pragma unroll
    for (int k = 0; k < Sw<W>::NW; ++k) {
      uint32_t m;
      if constexpr (W == 8) m = perm(w[k], w[k] << 8, 0x0b090a08u);  // sign bits 7 / 15 / 23 / 31 per byte
      else if constexpr (W == 16) m = (uint32_t)((int32_t)(w[k] << 16) >> 31 & 0xffff) | (uint32_t)((int32_t)w[k] >> 31 << 16);
      else m = (uint32_t)((int32_t)w[k] >> 31);
      acc |= w[k] ^ m;
      neg |= m;
    }
    if constexpr (W == 8) acc |= (acc >> 16) | (acc >> 8) | (acc >> 24);
    else if constexpr (W == 16) acc |= acc >> 16;
    uint32_t o = ((acc & ((W == 32) ? 0xffffffffu : ((1u << (W & 31)) - 1u))) << 1) | (neg ? 1u : 0u);
    o |= dpp<0xB1>(o);
    o |= dpp<0x4E>(o);
    const uint32_t up = dpp<0x104>(o), dn = dpp<0x114>(o);  // both in full exec: DPP reads of lanes
    o |= (lane & 4) ? dn : up;                                 // masked off by a branch return ``old``
    const int64_t blk = st * 8 + (lane >> 3);
    if ((lane & 7) == 0 && blk < nb) widths[blk] = (uint8_t)(o ? 32 - __clz(o) : 0);
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

// wave step: 8 blocks; lane j of block g stores planes 8p + j < width, contiguous per block
template <int W>
__global__ void __launch_bounds__(256) pack_kernel(const void* __restrict__ x, int64_t n,
                                                 const uint8_t* __restrict__ widths, const uint32_t* __restrict__ local,
                                                 const uint64_t* __restrict__ cbase, int64_t nb,
                                                 uint64_t* __restrict__ payload) {
  constexpr int NP = Sw<W>::NP;
  const int lane = threadIdx.x & 63, j = lane & 7;
  const int64_t nstep = (nb + 7) / 8;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t blk = st * 8 + (lane >> 3);
    uint32_t w[Sw<W>::NW];
    load8s<W>(x, n, st * 512 + (int64_t)lane * 8, w);
    int wd = 0;
    uint64_t off = 0;
    if (blk < nb) {
      wd = widths[blk];
      off = cbase[blk / kChunk] + local[blk];
    }
    uint32_t X[NP][2];
    gather_bytes<W>(w, X);
#pragma unroll
    for (int p = 0; p < NP; ++p) tr8x8(X[p][0], X[p][1]);  // byte b of X[p]: s-plane 8p + b
    // zigzag on planes: z-plane 0 = sign plane (s-plane W-1), z-plane b = s-plane b-1 ^ sign
    const uint32_t sg = perm(X[NP - 1][1], X[NP - 1][1], 0x07070707u);
    uint32_t Z[NP][2];
#pragma unroll
    for (int i = 2 * NP - 1; i >= 0; --i) {
      const uint32_t cur = X[i >> 1][i & 1];
      const uint32_t prev = i ? X[(i - 1) >> 1][(i - 1) & 1] : 0u;
      Z[i >> 1][i & 1] = __builtin_amdgcn_alignbit(cur, prev, 24) ^ sg;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      xtr8(Z[p][0], Z[p][1], j);
      if (8 * p + j < wd) payload[off + 8 * p + j] = ((uint64_t)Z[p][1] << 32) | Z[p][0];
    }
  }
}

// wave step: 8 blocks; the inverse of pack_kernel (both transposes are their own inverses)
template <int W>
__global__ void __launch_bounds__(256) unpack_kernel(const uint64_t* __restrict__ payload, int64_t n,
                                                   const uint8_t* __restrict__ widths,
                                                   const uint32_t* __restrict__ local,
                                                   const uint64_t* __restrict__ cbase, int64_t nb, void* __restrict__ out) {
  constexpr int NP = Sw<W>::NP;
  const int lane = threadIdx.x & 63, j = lane & 7;
  const int64_t nstep = (nb + 7) / 8;
  for (int64_t st = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; st < nstep;
       st += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int64_t blk = st * 8 + (lane >> 3);
    int wd = 0;
    uint64_t off = 0;
    if (blk < nb) {
      wd = min((int)widths[blk], W);  // a width past the sample size never steers a read (the host
      off = cbase[blk / kChunk] + local[blk];  // also rejects such blobs before launching)
    }
    uint32_t Z[NP][2];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const uint64_t v = 8 * p + j < wd ? payload[off + 8 * p + j] : 0ull;
      Z[p][0] = (uint32_t)v;
      Z[p][1] = (uint32_t)(v >> 32);
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) xtr8(Z[p][0], Z[p][1], j);  // byte b of Z[p]: z-plane 8p + b
    const uint32_t sg = perm(Z[0][0], Z[0][0], 0x00000000u);
    uint32_t X[NP][2];
#pragma unroll
    for (int i = 0; i < 2 * NP; ++i) {
      const uint32_t cur = Z[i >> 1][i & 1];
      const uint32_t next = i + 1 < 2 * NP ? Z[(i + 1) >> 1][(i + 1) & 1] : 0u;
      X[i >> 1][i & 1] = __builtin_amdgcn_alignbit(next, cur, 8) ^ sg;
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) tr8x8(X[p][0], X[p][1]);
    uint32_t w[Sw<W>::NW];
    scatter_bytes<W>(X, w);
    store8s<W>(out, n, st * 512 + (int64_t)lane * 8, w);
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

unsigned waves_grid(int64_t nb) {
  int64_t g = ceil_div(ceil_div(nb, (int64_t)8), 4);  // a wave step = 8 blocks, 4 waves per workgroup
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

int sample_bits(int dtype) {
  switch (dtype) {
    case KMP_U8: return 8;
    case KMP_U16: return 16;
    case KMP_I32: case KMP_U32: case KMP_F32: return 32;
    default: return 0;
  }
}

Ws carve(void* ws, int64_t nb) {
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

int scan(const uint8_t* widths, int64_t nb, const Ws& w, hipStream_t s) {
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
  return ceil_div(nb * 4, 8) * 8 + nchunk * 16 + 16;  // + the scan's total and kmp_unpack_check's count
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
