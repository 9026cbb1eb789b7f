// kmp_crc.hip -- CRC-32 (zlib / IEEE 802.3: reflected polynomial 0xEDB88320, init and final xor
// 0xFFFFFFFF) of a device byte buffer, equal to zlib.crc32 of the same bytes.  The container's
// integrity check (container.py: one CRC per file) runs here instead of on one
// host core (1.97 GB/s for a C3 bundle, profiles/round4).
//
// Arithmetic over GF(2)[x] mod P in zlib's reflected representation (bit 31 = x^0):
//   * raw(M)       = the CRC register after M from 0 (no conditioning); linear in M;
//   * raw(A || B)  = raw(A) * x^(8|B|)  ^  raw(B);
//   * crc(M)       = raw(M) ^ (0xFFFFFFFF * x^(8|M|)) ^ 0xFFFFFFFF.
// Layout: a wave owns a region of kSteps x 1 KiB; in step j lane l reads the 16 bytes at
// j KiB + 16 l (one coalesced 1 KiB load per wave-instruction) and advances its register by
// acc <- slice16(acc * x^(8 (1024 - 16)), bytes) -- slice-by-16 tables in LDS plus a 4-table
// multiply by the constant -- so each lane holds the raw CRC of its strided sub-sequence.  The
// lane registers combine as acc_l * x^(8 * 16 (63 - l)) (XOR over the wave), the regions as
// region_w * x^(8 R (W - 1 - w)) (an atomic XOR per wave into the result).  The buffer is zero-
// padded at the END to whole regions (k bytes): raw(M || 0^k) = raw(M) * x^(8k), undone by
// x^(-8k); wave 0 adds the conditioning term.  No host work besides one memset, no sync.
#include "kmp_common.h"

namespace kmp {
namespace crc {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kOne = 0x80000000u;   // x^0
constexpr uint32_t kXinv = 0xDB710641u;  // x^-1 mod P  (x * kXinv == 1)
constexpr int kLanes = 64;
constexpr int kStep = kLanes * 16;       // bytes per wave step
constexpr int kSteps = 32;
constexpr int64_t kRegion = (int64_t)kStep * kSteps;  // bytes per wave (32 KiB)
constexpr int kWaves = 4;                // per workgroup

__host__ __device__ constexpr uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = kOne, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    if (m == 0) break;
    b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
  }
  return p;
}

struct Tables {
  uint32_t t[16][256];  // slice-by-16
  uint32_t k[4][256];   // multiply by x^(8 (kStep - 16)), byte by byte
  uint32_t x2n[64];     // x^(2^n)
  uint32_t xi2n[64];    // x^(-8 * 2^n)
  uint32_t lane[kLanes];  // x^(8 * 16 * (63 - l))
};

constexpr Tables make_tables() {
  Tables T{};
  for (int i = 0; i < 256; ++i) {
    uint32_t c = (uint32_t)i;
    for (int b = 0; b < 8; ++b) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
    T.t[0][i] = c;
  }
  for (int s = 1; s < 16; ++s)
    for (int i = 0; i < 256; ++i) T.t[s][i] = (T.t[s - 1][i] >> 8) ^ T.t[0][T.t[s - 1][i] & 0xff];
  uint32_t p = kOne >> 1;  // x^1
  for (int n = 0; n < 64; ++n) {
    T.x2n[n] = p;
    p = multmodp(p, p);
  }
  uint32_t q = kXinv;
  for (int i = 0; i < 3; ++i) q = multmodp(q, q);  // x^-8
  for (int n = 0; n < 64; ++n) {
    T.xi2n[n] = q;
    q = multmodp(q, q);
  }
  // x^(8 e) by squares: bits of e against x^(2^(n + 3))
  auto x8 = [&T](uint64_t e) {
    uint32_t r = kOne;
    for (int n = 3; e; e >>= 1, ++n)
      if (e & 1) r = multmodp(T.x2n[n & 63], r);
    return r;
  };
  const uint32_t K = x8(kStep - 16);
  for (int b = 0; b < 4; ++b)
    for (int v = 0; v < 256; ++v) T.k[b][v] = multmodp(K, (uint32_t)v << (8 * b));
  for (int l = 0; l < kLanes; ++l) T.lane[l] = x8((uint64_t)16 * (kLanes - 1 - l));
  return T;
}

__device__ constexpr Tables kTables = make_tables();

__device__ __forceinline__ uint32_t x8pow(const Tables& T, uint64_t e) {  // x^(8 e)
  uint32_t r = kOne;
  for (int n = 3; e; e >>= 1, ++n)
    if (e & 1) r = multmodp(T.x2n[n & 63], r);
  return r;
}
__device__ __forceinline__ uint32_t xinv8pow(const Tables& T, uint64_t e) {  // x^(-8 e)
  uint32_t r = kOne;
  for (int n = 0; e; e >>= 1, ++n)
    if (e & 1) r = multmodp(T.xi2n[n & 63], r);
  return r;
}

__global__ void __launch_bounds__(64 * kWaves) crc32_kernel(const uint8_t* __restrict__ data, int64_t n_arg,
                                                            const int64_t* __restrict__ n_dev, uint32_t* out) {
  __shared__ uint32_t st[16][256];
  __shared__ uint32_t sk[4][256];
  for (int i = threadIdx.x; i < 16 * 256; i += blockDim.x) (&st[0][0])[i] = (&kTables.t[0][0])[i];
  for (int i = threadIdx.x; i < 4 * 256; i += blockDim.x) (&sk[0][0])[i] = (&kTables.k[0][0])[i];
  __syncthreads();
  const int64_t n = n_dev ? min(max(*n_dev, (int64_t)0), n_arg) : n_arg;  // never past the buffer
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int64_t W = n > 0 ? (n + kRegion - 1) / kRegion : 1;
  if (w >= W) return;
  const int64_t base = w * kRegion;
  uint32_t acc = 0;
  for (int j = 0; j < kSteps; ++j) {
    const int64_t off = base + (int64_t)j * kStep + 16 * lane;
    uint32_t d[4];
    if (off + 16 <= n) {
      const uint4 v = *(const uint4*)(data + off);
      d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
    } else {  // the zero padding past the end (and the one chunk that straddles it)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const int64_t i = off + 4 * q + b;
          if (i < n) word |= (uint32_t)data[i] << (8 * b);
        }
        d[q] = word;
      }
    }
    // acc * x^(8 (kStep - 16)), then slice-by-16 over the 16 bytes
    uint32_t c = sk[0][acc & 0xff] ^ sk[1][(acc >> 8) & 0xff] ^ sk[2][(acc >> 16) & 0xff] ^ sk[3][acc >> 24];
    c ^= d[0];
    acc = st[15][c & 0xff] ^ st[14][(c >> 8) & 0xff] ^ st[13][(c >> 16) & 0xff] ^ st[12][c >> 24] ^
          st[11][d[1] & 0xff] ^ st[10][(d[1] >> 8) & 0xff] ^ st[9][(d[1] >> 16) & 0xff] ^ st[8][d[1] >> 24] ^
          st[7][d[2] & 0xff] ^ st[6][(d[2] >> 8) & 0xff] ^ st[5][(d[2] >> 16) & 0xff] ^ st[4][d[2] >> 24] ^
          st[3][d[3] & 0xff] ^ st[2][(d[3] >> 8) & 0xff] ^ st[1][(d[3] >> 16) & 0xff] ^ st[0][d[3] >> 24];
  }
  // the wave's region: lane registers at their distances from the region's end
  uint32_t r = multmodp(kTables.lane[lane], acc);
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) r ^= (uint32_t)__shfl_xor((int)r, m, 64);
  if (lane == 0) {
    const int64_t pad = W * kRegion - n;                // zero bytes appended
    const int64_t e = kRegion * (W - 1 - w) - pad;      // this region's distance from the true end
    uint32_t v = multmodp(e >= 0 ? x8pow(kTables, (uint64_t)e) : xinv8pow(kTables, (uint64_t)(-e)), r);
    if (w == 0) v ^= multmodp(x8pow(kTables, (uint64_t)n), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
    atomicXor(out, v);
  }
}

}  // namespace crc

extern "C" {

int kmp_crc32(const uint8_t* data, int64_t n_max, const int64_t* n_dev, uint32_t* crc_out, kmp_stream_t stream) {
  KMP_REQUIRE(n_max >= 0 && crc_out && (n_max == 0 || data), "crc32: bad argument");
  KMP_REQUIRE(((uintptr_t)data & 15) == 0, "crc32: data must be 16-byte aligned");
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(crc_out, 0, sizeof(uint32_t), s) != hipSuccess) return fail(KMP_ERR_LAUNCH, "crc32: memset");
  const int64_t regions = n_max > 0 ? (n_max + crc::kRegion - 1) / crc::kRegion : 1;
  const int64_t blocks = (regions + crc::kWaves - 1) / crc::kWaves;
  KMP_REQUIRE(blocks < ((int64_t)1 << 31), "crc32: buffer too large");
  crc::crc32_kernel<<<(unsigned)blocks, 64 * crc::kWaves, 0, s>>>(data, n_max, n_dev, crc_out);
  return check_launch("crc32");
}

}  // extern "C"

}  // namespace kmp
