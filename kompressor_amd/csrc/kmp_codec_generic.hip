// kmp_codec_generic.hip -- the fused encode/decode for ANY shape, channel count, padding and
// integer dtype: two launches per direction.
//
//   1. predictor apply: one value per cell (MEAN) or K per cell (LINEAR) into a workspace
//      [K, B, Lc..., C] (channel planes) -- the reference's features_from_lowres + mean/astype
//      (tests/volume/test_encode_decode.py:46-51) without materialising the features;
//   2. residual pass: per output block position o, read the 2^d highres block at 2o, aggregate
//      the cell predictions exactly as maps_from_predictions does (kmp_aggregate.h), apply the
//      coder and write lowres + every map in its trimmed shape (encode), or the inverse
//      (decode: interleave into highres, highres_from_lowres_and_maps + trim).
//
// Lowres node j of the padded volume along an axis is source sample 2*sym(j, E) (encode: even
// reflect pad volume/utils.py:226-237) or sym(j, E) of the trimmed lowres (decode: symmetric
// pad_lowres volume/utils.py:240-244); the neighbourhood padding adds sym(., L)
// (pad_neighborhood volume/utils.py:213-218).  Costs ~1.25x the HBM bytes of the one-pass
// fast kernels (kmp_codec_fast3d.hip); used whenever those are not eligible.
#include "kmp_codec.h"
#include "kmp_aggregate.h"
#include "kmp_wave.h"

namespace kmp {

constexpr int kGThreads = 256;

static inline unsigned ggrid(int64_t n) {
  int64_t g = ceil_div(n, kGThreads);
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

struct Src {
  int64_t S[3];  // source extents (highres n for encode, trimmed lowres E for decode)
  int32_t mult;  // 2 (encode: lowres node j <- highres 2j) or 1 (decode)
};

// Cell mean, float32 sum in feature order (z-major, y, x) / N, XLA cast (the reference test
// predictor).  Exact (order-independent) for uint8 with p <= 4 and uint16 with p <= 2.
struct Frame {
  int64_t begin[3], ext[3];
};

// Unsigned 32-bit division by a runtime constant as multiply-high + add + shift (the host computes
// the magic number): n / d for n < 2^31.  The generic kernels' per-element index split was four
// integer divisions (~40 VALU each, emulated); this is 3 VALU per division.
struct FDiv {
  uint32_t d, m, s;
};
static inline FDiv fdiv(int64_t d64) {
  const uint32_t d = (uint32_t)(d64 < 1 ? 1 : d64);
  uint32_t s = 0;
  while (s < 32 && (1ull << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return FDiv{d, (uint32_t)m, s};
}
__device__ __forceinline__ uint32_t fdiv_q(uint32_t n, const FDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// The index space of a frame: t -> (b, i0, i1, i2, c), c fastest (as unflat5)
struct Flat {
  FDiv dC, d2, d1, d0;
};
static inline Flat make_flat(const int64_t (&ext)[3], int64_t C) {
  return Flat{fdiv(C), fdiv(ext[2]), fdiv(ext[1]), fdiv(ext[0])};
}
template <typename I>
__device__ __forceinline__ void unflat_i(int64_t t, const Flat& F, const int64_t (&ext)[3], int64_t C, I& b, I& i0,
                                         I& i1, I& i2, I& c) {
  if constexpr (sizeof(I) == 4) {  // t < 2^31 (the host's choice of I)
    uint32_t u = (uint32_t)t, q;
    q = fdiv_q(u, F.dC); c = (I)(u - q * F.dC.d); u = q;
    q = fdiv_q(u, F.d2); i2 = (I)(u - q * F.d2.d); u = q;
    q = fdiv_q(u, F.d1); i1 = (I)(u - q * F.d1.d); u = q;
    q = fdiv_q(u, F.d0); i0 = (I)(u - q * F.d0.d); b = (I)q;
  } else {
    int64_t bb, z, y, x, cc;
    unflat5(t, ext[0], ext[1], ext[2], C, bb, z, y, x, cc);
    b = bb; i0 = z; i1 = y; i2 = x; c = cc;
  }
}

// astype(T) of the aggregation / mean: the saturating hardware conversion for 8- / 16-bit samples
// (cvt_sat, kmp_wave.h), the exact restatement otherwise
template <typename T>
__device__ __forceinline__ T gcast(float v) {
  if constexpr (std::is_same<T, uint8_t>::value || std::is_same<T, uint16_t>::value) return (T)wv::cvt_sat<T>(v);
  else return cast_f32<T>(v);
}

// astype(T) of an f32 LinearPredictor value (kmp_linear.hip lin_cast: the clamp-then-convert form
// of the saturating conversion for 8- / 16-bit samples, cast_f32 otherwise)
template <typename T>
__device__ __forceinline__ T lin_cast_t(float v) {
  if constexpr (sizeof(T) <= 2) return (T)wv::cvt_sat_mfma<T>(v);
  else return cast_f32<T>(v);
}

// the 7 (3) maps' lattice parities (z, y, x) and contributions at compile time (kmp_aggregate.h)
template <int NSP>
__device__ __forceinline__ constexpr int gpar(int k, int a) {
  constexpr int8_t t3[7][3] = {{1, 1, 0}, {1, 0, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
  constexpr int8_t t2[3][3] = {{0, 1, 0}, {0, 0, 1}, {0, 1, 1}};
  return NSP == 3 ? t3[k][a] : t2[k][a];
}

// Lowres node source index along an axis: mult * sym(sym(j, L), E) (even reflect pad, then the
// neighbourhood's symmetric pad)
__device__ __forceinline__ int64_t node_src(int64_t j, int64_t L, int64_t E, int mult) {
  return mult * sym_index(sym_index(j, L), E);
}

// ``cf`` is the box of cells to compute (a region launch needs cells [begin-1, end) only);
// results land at their global position in ``cells`` [B, Lc..., C].  KK = 2p + 2 at compile time
// (p <= 2: the node offsets per axis in registers, the (2p+2)^d loads unrolled) or 0 (any p).
template <typename T, int NSP, int KK, typename I>
__global__ void __launch_bounds__(kGThreads) cell_mean_kernel(const T* __restrict__ src, Src s, Geo g, int64_t B,
                                                            int64_t C, int p, Frame cf, Flat F, T* __restrict__ cells,
                                                            int64_t total) {
  const int k = KK ? KK : 2 * p + 2;
  const int kz = NSP == 3 ? k : 1;
  const int pz = NSP == 3 ? p : 0;
  const float inv_n = (float)(kz * k * k);
  const I Cc = (I)C, sy = (I)s.S[2] * Cc, sz = (I)s.S[1] * sy, sb = (I)s.S[0] * sz;
  const I cy = (I)g.Lc[2] * Cc, cz = (I)g.Lc[1] * cy, cb = (I)g.Lc[0] * cz;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    I b, z, y, x, c;
    unflat_i<I>(t, F, cf.ext, C, b, z, y, x, c);
    z += (I)cf.begin[0];
    y += (I)cf.begin[1];
    x += (I)cf.begin[2];
    const I base = b * sb + c;
    float sum = 0.0f;
    if constexpr (KK > 0) {
      I ox[KK], oy[KK];
#pragma unroll
      for (int d = 0; d < KK; ++d) {
        ox[d] = (I)node_src(x - p + d, g.L[2], g.E[2], s.mult) * Cc;
        oy[d] = (I)node_src(y - p + d, g.L[1], g.E[1], s.mult) * sy;
      }
#pragma unroll
      for (int dz = 0; dz < (NSP == 3 ? KK : 1); ++dz) {
        const I zo = base + (NSP == 3 ? (I)node_src(z - pz + dz, g.L[0], g.E[0], s.mult) * sz : 0);
#pragma unroll
        for (int dy = 0; dy < KK; ++dy)
#pragma unroll
          for (int dx = 0; dx < KK; ++dx) sum += (float)src[zo + oy[dy] + ox[dx]];
      }
    } else {
      for (int dz = 0; dz < kz; ++dz) {
        const I zo = base + (NSP == 3 ? (I)node_src(z - pz + dz, g.L[0], g.E[0], s.mult) * sz : 0);
        for (int dy = 0; dy < k; ++dy) {
          const I yo = zo + (I)node_src(y - p + dy, g.L[1], g.E[1], s.mult) * sy;
          for (int dx = 0; dx < k; ++dx) sum += (float)src[yo + (I)node_src(x - p + dx, g.L[2], g.E[2], s.mult) * Cc];
        }
      }
    }
    cells[b * cb + z * cz + y * cy + x * Cc + c] = gcast<T>(sum / inv_n);
  }
}

// The cell mean, R = 4 consecutive cells of a row per thread: each (dz, dy) row of R + KK - 1 nodes
// is read once for the 4 cells (28 loads for 4 cells at p = 1 instead of 4 x 64).  EXACT (8- /
// 16-bit samples with N x max sample < 2^24: u8 at p <= 4, u16 at p <= 2): the reference's
// in-order float sum is the integer sum, formed by sliding windows; otherwise each cell's float
// sum is accumulated in the reference's feature order (z-major, y, x), exactly cell_mean_kernel's.
constexpr int kMeanR = 4;

template <typename T, int NSP, int KK, bool EXACT>
__global__ void __launch_bounds__(kGThreads) cell_mean_row_kernel(const T* __restrict__ src, Src s, Geo g, int64_t C,
                                                                int p, Frame cf, Flat F, T* __restrict__ cells,
                                                                int64_t total) {
  constexpr int R = kMeanR, NX = R + KK - 1;
  using I = int32_t;
  const float n_f = (float)((NSP == 3 ? KK : 1) * KK * KK);
  const I Cc = (I)C, sy = (I)s.S[2] * Cc, sz = (I)s.S[1] * sy, sb = (I)s.S[0] * sz;
  const I cy = (I)g.Lc[2] * Cc, cz = (I)g.Lc[1] * cy, cb = (I)g.Lc[0] * cz;
  const int pz = NSP == 3 ? p : 0;
  const I xend = (I)(cf.begin[2] + cf.ext[2]);
  const int64_t jmax = xend - 1 - p + (KK - 1);  // the last node a valid cell reads
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ext_q[3] = {cf.ext[0], cf.ext[1], (cf.ext[2] + R - 1) / R};
    I b, z, y, xq, c;
    unflat_i<I>(t, F, ext_q, C, b, z, y, xq, c);
    z += (I)cf.begin[0];
    y += (I)cf.begin[1];
    const I x0 = (I)cf.begin[2] + R * xq;
    const I base = b * sb + c;
    I ox[NX], oy[KK], oz[NSP == 3 ? KK : 1];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      int64_t j = (int64_t)x0 - p + i;
      j = j > jmax ? jmax : j;
      ox[i] = (I)node_src(j, g.L[2], g.E[2], s.mult) * Cc;
    }
#pragma unroll
    for (int d = 0; d < KK; ++d) {
      oy[d] = (I)node_src(y - p + d, g.L[1], g.E[1], s.mult) * sy;
      if constexpr (NSP == 3) oz[d] = (I)node_src(z - pz + d, g.L[0], g.E[0], s.mult) * sz;
    }
    uint32_t sum[R];
    float fsum[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      sum[r] = 0u;
      fsum[r] = 0.0f;
    }
    constexpr int ZU = NSP == 3 && KK <= 4 ? KK : 1;  // 3D p = 2: a runtime z loop (all 324 loads
                                                    // hoisted took 267 VGPRs)
#pragma unroll ZU
    for (int dz = 0; dz < (NSP == 3 ? KK : 1); ++dz) {
      I zo = NSP == 3 ? oz[0] : 0;
#pragma unroll
      for (int d = 1; d < (NSP == 3 ? KK : 1); ++d) zo = dz == d ? oz[d] : zo;
#pragma unroll
      for (int dy = 0; dy < KK; ++dy) {
        const I rb = base + zo + oy[dy];
        if constexpr (EXACT) {
          uint32_t v[NX];
#pragma unroll
          for (int i = 0; i < NX; ++i) v[i] = (uint32_t)src[rb + ox[i]];
          uint32_t w = 0u;
#pragma unroll
          for (int i = 0; i < KK; ++i) w += v[i];
          sum[0] += w;
#pragma unroll
          for (int r = 1; r < R; ++r) {
            w += v[r + KK - 1] - v[r - 1];
            sum[r] += w;
          }
        } else {
          float v[NX];
#pragma unroll
          for (int i = 0; i < NX; ++i) v[i] = (float)src[rb + ox[i]];
#pragma unroll
          for (int dx = 0; dx < KK; ++dx)
#pragma unroll
            for (int r = 0; r < R; ++r) fsum[r] += v[r + dx];
        }
      }
    }
    const I ob = b * cb + z * cz + y * cy + x0 * Cc + c;
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (x0 + r < xend) cells[ob + r * Cc] = gcast<T>((EXACT ? (float)sum[r] : fsum[r]) / n_f);
  }
}

// Per output position o (and channel): the lowres node and the 7 (3) maps.  The cell values the
// maps aggregate are read once: the 2^d cells o - {0,1}^d (MeanPredictor: one value per cell), or
// each contribution's channel (LinearPredictor: K per cell, planar: channel ch of every cell in
// plane ch, kmp_linear.hip launch_linear); missing cells (past the cell box) are skipped exactly as
// maps_from_predictions does, in the reference's channel order.
template <typename T, int NSP, bool PERCH, typename I>
struct GenCells {
  const T* cells;
  I base, sx, sy, sz;  // cells[base - dz sz - dy sy - dx sx + ch kp]
  I kp;                // LinearPredictor: the channel plane stride
  bool v[2][2][2];     // cell o - (dz, dy, dx) exists
  T m[2][2][2];        // MeanPredictor: the cell means

  __device__ __forceinline__ void init(const T* c_, I b, I oz, I oy, I ox, I c, const Geo& g, I Cc, I kp_) {
    cells = c_;
    kp = kp_;
    sx = Cc;
    sy = (I)g.Lc[2] * Cc;
    sz = (I)g.Lc[1] * sy;
    base = b * ((I)g.Lc[0] * sz) + oz * sz + oy * sy + ox * sx + c;
    const bool vz[2] = {oz < (I)g.Lc[0], oz >= 1}, vy[2] = {oy < (I)g.Lc[1], oy >= 1},
               vx[2] = {ox < (I)g.Lc[2], ox >= 1};
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          v[dz][dy][dx] = (NSP == 3 || dz == 0) && vz[dz] && vy[dy] && vx[dx];
          if (!PERCH) m[dz][dy][dx] = v[dz][dy][dx] ? cells[base - dz * sz - dy * sy - dx * sx] : T(0);
        }
  }
  __device__ __forceinline__ T get(int dz, int dy, int dx, int ch) const {
    if constexpr (PERCH) return cells[base - dz * sz - dy * sy - dx * sx + (I)ch * kp];
    else return m[dz][dy][dx];
  }
  // map k's prediction (maps_from_predictions for one element)
  __device__ __forceinline__ T pred(int k) const {
    Contrib c[4];
    const int nc = map_contribs(NSP, k, c);
    if (k == center_map(NSP)) return get(0, 0, 0, c[0].ch);
    float s = 0.0f;
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i >= nc) break;
      if (v[c[i].dz][c[i].dy][c[i].dx]) {
        s += (float)get(c[i].dz, c[i].dy, c[i].dx, c[i].ch);
        ++cnt;
      }
    }
    if (cnt == 4) s *= 0.25f;
    else if (cnt == 2) s *= 0.5f;
    return gcast<T>(s);
  }
};

template <typename T, int CODER, bool PERCH, int NSP, typename I>
__global__ void __launch_bounds__(kGThreads) encode_generic_kernel(const T* __restrict__ hi, Geo g, int64_t B,
                                                                 int64_t C, const T* __restrict__ cells, int K,
                                                                 T* __restrict__ lowres, MapPtrs maps, Frame f, Flat F,
                                                                 int64_t total) {
  using TO = typename coder_out<CODER>::type;
  constexpr int NM = NSP == 3 ? 7 : 3;
  const I Cc = (I)C;
  const I hy = (I)g.n[2] * Cc, hz = (I)g.n[1] * hy, hb = (I)g.n[0] * hz;
  const I ly = (I)g.E[2] * Cc, lz = (I)g.E[1] * ly, lb = (I)g.E[0] * lz;
  const I kp = (I)(B * g.Lc[0] * g.Lc[1] * g.Lc[2] * C);  // LinearPredictor: channel plane stride
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    I b, oz, oy, ox, c;
    unflat_i<I>(t, F, f.ext, C, b, oz, oy, ox, c);
    oz += (I)f.begin[0];
    oy += (I)f.begin[1];
    ox += (I)f.begin[2];
    const I h0 = b * hb + (2 * oz) * hz + (2 * oy) * hy + (2 * ox) * Cc + c;
    if (oz < (I)g.E[0] && oy < (I)g.E[1] && ox < (I)g.E[2]) lowres[b * lb + oz * lz + oy * ly + ox * Cc + c] = hi[h0];
    GenCells<T, NSP, PERCH, I> gc;
    gc.init(cells, b, oz, oy, ox, c, g, Cc, kp);
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      const int p0 = gpar<NSP>(k, 0), p1 = gpar<NSP>(k, 1), p2 = gpar<NSP>(k, 2);
      const I e0 = (I)(p0 ? g.Lc[0] : g.E[0]), e1 = (I)(p1 ? g.Lc[1] : g.E[1]), e2 = (I)(p2 ? g.Lc[2] : g.E[2]);
      if (oz >= e0 || oy >= e1 || ox >= e2) continue;
      const T pred = gc.pred(k);
      const T gt = hi[h0 + p0 * hz + p1 * hy + p2 * Cc];
      ((TO*)maps.p[k])[((b * e0 + oz) * e1 + oy) * e2 * Cc + ox * Cc + c] = code_encode<CODER>(to_i32(pred), to_i32(gt));
    }
  }
}

template <typename T, int CODER, bool PERCH, int NSP, typename I>
__global__ void __launch_bounds__(kGThreads) decode_generic_kernel(const T* __restrict__ lowres, CMapPtrs maps, Geo g,
                                                                 int64_t B, int64_t C, const T* __restrict__ cells,
                                                                 int K, T* __restrict__ hi, Frame f, Flat F,
                                                                 int64_t total) {
  using TO = typename coder_out<CODER>::type;
  constexpr int NM = NSP == 3 ? 7 : 3;
  const I Cc = (I)C;
  const I hy = (I)g.n[2] * Cc, hz = (I)g.n[1] * hy, hb = (I)g.n[0] * hz;
  const I ly = (I)g.E[2] * Cc, lz = (I)g.E[1] * ly, lb = (I)g.E[0] * lz;
  const I kp = (I)(B * g.Lc[0] * g.Lc[1] * g.Lc[2] * C);  // LinearPredictor: channel plane stride
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    I b, oz, oy, ox, c;
    unflat_i<I>(t, F, f.ext, C, b, oz, oy, ox, c);
    oz += (I)f.begin[0];
    oy += (I)f.begin[1];
    ox += (I)f.begin[2];
    const I h0 = b * hb + (2 * oz) * hz + (2 * oy) * hy + (2 * ox) * Cc + c;
    if (oz < (I)g.E[0] && oy < (I)g.E[1] && ox < (I)g.E[2]) hi[h0] = lowres[b * lb + oz * lz + oy * ly + ox * Cc + c];
    GenCells<T, NSP, PERCH, I> gc;
    gc.init(cells, b, oz, oy, ox, c, g, Cc, kp);
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      const int p0 = gpar<NSP>(k, 0), p1 = gpar<NSP>(k, 1), p2 = gpar<NSP>(k, 2);
      const I e0 = (I)(p0 ? g.Lc[0] : g.E[0]), e1 = (I)(p1 ? g.Lc[1] : g.E[1]), e2 = (I)(p2 ? g.Lc[2] : g.E[2]);
      if (oz >= e0 || oy >= e1 || ox >= e2) continue;
      const T pred = gc.pred(k);
      const TO enc = ((const TO*)maps.p[k])[((b * e0 + oz) * e1 + oy) * e2 * Cc + ox * Cc + c];
      hi[h0 + p0 * hz + p1 * hy + p2 * Cc] = (T)code_decode<CODER>(to_i32(pred), to_i32(enc));
    }
  }
}

// ---- the generic codec with one channel: a thread owns 4 consecutive output columns of a row ----
// The per-element kernels above move 2-byte values (u16) one per thread; with C == 1 (the common
// case outside the one-pass kernels: odd or wide rows, p >= 3) a thread here reads the 8 highres
// samples of each of its 2^d rows as one unaligned vector access (element-wise only in a row's
// last partial group), the cells around its outputs once, and writes each map's 4 values together.
typedef uint32_t g32x2a1 __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t g32x4a1 __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t g32a1 __attribute__((aligned(1)));
typedef uint8_t g8x4 __attribute__((ext_vector_type(4)));
typedef uint8_t g8x4a1 __attribute__((ext_vector_type(4), aligned(1)));

// N consecutive samples (N x sizeof(T) a multiple of 4 bytes) as unaligned dword vector accesses
template <typename T, int N>
__device__ __forceinline__ void g_loadn(const T* p, uint32_t (&v)[N]) {
  constexpr int NW = N * (int)sizeof(T) / 4;
  static_assert(N * sizeof(T) % 4 == 0, "g_loadn: whole dwords");
  uint32_t w[NW];
  const char* c = (const char*)p;
  constexpr int N4 = NW / 4 * 4;  // dwordx4 pieces, then one x2 and / or one x1
#pragma unroll
  for (int i = 0; i < N4; i += 4) {
    const g32x4a1 t = *(const g32x4a1*)(c + 4 * i);
    w[i] = t[0]; w[i + 1] = t[1]; w[i + 2] = t[2]; w[i + 3] = t[3];
  }
  if constexpr (NW - N4 >= 2) {
    const g32x2a1 t = *(const g32x2a1*)(c + 4 * N4);
    w[N4] = t[0]; w[N4 + 1] = t[1];
  }
  if constexpr ((NW - N4) % 2) w[NW - 1] = *(const g32a1*)(c + 4 * (NW - 1));
  constexpr int PER = 4 / (int)(sizeof(T) < 4 ? sizeof(T) : 4);
  constexpr uint32_t MASK = sizeof(T) == 1 ? 0xffu : (sizeof(T) == 2 ? 0xffffu : 0xffffffffu);
#pragma unroll
  for (int e = 0; e < N; ++e) v[e] = (w[e / PER] >> (8 * sizeof(T) * (e % PER))) & MASK;
}
template <typename T, int N>
__device__ __forceinline__ void g_storen(T* p, const uint32_t (&v)[N]) {
  constexpr int NW = N * (int)sizeof(T) / 4;
  static_assert(N * sizeof(T) % 4 == 0, "g_storen: whole dwords");
  constexpr int PER = 4 / (int)(sizeof(T) < 4 ? sizeof(T) : 4);
  constexpr uint32_t MASK = sizeof(T) == 1 ? 0xffu : (sizeof(T) == 2 ? 0xffffu : 0xffffffffu);
  uint32_t w[NW];
#pragma unroll
  for (int i = 0; i < NW; ++i) w[i] = 0u;
#pragma unroll
  for (int e = 0; e < N; ++e) w[e / PER] |= (v[e] & MASK) << (8 * sizeof(T) * (e % PER));
  char* c = (char*)p;
  constexpr int N4 = NW / 4 * 4;
#pragma unroll
  for (int i = 0; i < N4; i += 4) *(g32x4a1*)(c + 4 * i) = g32x4a1{w[i], w[i + 1], w[i + 2], w[i + 3]};
  if constexpr (NW - N4 >= 2) *(g32x2a1*)(c + 4 * N4) = g32x2a1{w[N4], w[N4 + 1]};
  if constexpr ((NW - N4) % 2) *(g32a1*)(c + 4 * (NW - 1)) = w[NW - 1];
}

// (b, oz, oy, xq) of a flat thread index over B x ext0 x ext1 x nxq (xq: a group of 4 columns)
struct Row4 {
  FDiv dq, d1, d0;
};

// CC channels (1..4, interleaved): a thread owns 4 output positions x CC channels of a row, so
// its highres rows are 8 x CC consecutive samples, its lowres / map values 4 x CC, its cells 5 x CC
// FK > 0 (images, one channel, f32 LinearPredictor with KK = FK = 2p + 2 <= 4): no cells array --
// the thread computes the 2 x 5 cells around its outputs itself, from a (FK + 1) x (FK + 4) patch
// of lowres nodes, with the reference's fma chain (linear_valu_kernel's arithmetic: same bits).
// Each cell is computed by ~2.5 threads; the cells pass (a write and a re-read of 5 predictions a
// cell) is gone.
template <typename T, int CODER, bool PERCH, int NSP, int CC, bool DEC, int FK = 0>
__global__ void __launch_bounds__(kGThreads) codec_row4_kernel(const T* __restrict__ src, CMapPtrs imaps, Geo g,
                                                             const T* __restrict__ cells, int64_t B, T* __restrict__ dst,
                                                             MapPtrs omaps, Frame f, Row4 R, int64_t nxq,
                                                             int64_t total, Src ns = Src{}, const float* W = nullptr,
                                                             const float* bias = nullptr, int p = 0) {
  static_assert(FK == 0 || (NSP == 2 && CC == 1 && PERCH), "fused cells: images, one channel, LinearPredictor");
  constexpr int FKO = 5, FN = FK * FK;  // outputs / features of a 2D cell
  __shared__ float wl[FK > 0 ? FN * FKO + FKO : 1];
  if constexpr (FK > 0) {
    for (int i = threadIdx.x; i < FN * FKO + FKO; i += blockDim.x) wl[i] = i < FN * FKO ? W[i] : bias[i - FN * FKO];
    __syncthreads();
  }
  using I = int32_t;
  using TO = typename coder_out<CODER>::type;
  constexpr int NM = NSP == 3 ? 7 : 3;
  constexpr int NZ = NSP == 3 ? 2 : 1;
  constexpr int NH = 8 * CC, NO = 4 * CC;  // samples of a highres row segment / of an output group
  const I hy = (I)g.n[2] * CC, hz = (I)g.n[1] * hy, hb = (I)g.n[0] * hz;
  const I ly = (I)g.E[2] * CC, lz = (I)g.E[1] * ly, lb = (I)g.E[0] * lz;
  const I cy = (I)g.Lc[2] * CC, cz = (I)g.Lc[1] * cy, cb = (I)g.Lc[0] * cz;
  const I kp = (I)B * cb;  // LinearPredictor: channel plane stride (planar cells)
  const I end2 = (I)(f.begin[2] + f.ext[2]);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    I b, oz, oy, xq;
    {
      uint32_t u = (uint32_t)t, q;
      q = fdiv_q(u, R.dq); xq = (I)(u - q * R.dq.d); u = q;
      q = fdiv_q(u, R.d1); oy = (I)(u - q * R.d1.d); u = q;
      q = fdiv_q(u, R.d0); oz = (I)(u - q * R.d0.d); b = (I)q;
    }
    oz += (I)f.begin[0];
    oy += (I)f.begin[1];
    const I ox0 = (I)f.begin[2] + 4 * xq;
    const int nout = (int)(end2 - ox0 < 4 ? end2 - ox0 : 4);
    // ---- the cells around the 4 outputs: (oz - dz, oy - dy, ox0 - 1 + j), j = 0..4 ----
    const I cbase = b * cb + oz * cz + oy * cy + ox0 * CC;  // cell (oz, oy, ox0), channel 0
    bool cv[2][2][5];
    T cm[2][2][5][CC];
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        const bool rowok = (NSP == 3 || dz == 0) && oz - dz >= 0 && oz - dz < (I)g.Lc[0] && oy - dy >= 0 &&
                           oy - dy < (I)g.Lc[1];
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          const I x = ox0 - 1 + j;
          cv[dz][dy][j] = rowok && x >= 0 && x < (I)g.Lc[2];
#pragma unroll
          for (int ch = 0; ch < CC; ++ch)
            if (!PERCH) cm[dz][dy][j][ch] = cv[dz][dy][j] ? cells[cbase - dz * cz - dy * cy + (j - 1) * CC + ch] : T(0);
        }
      }
    // map k's contribution channel kch of the cell (oz - dz, oy - dy, ox0 + i - dx), sample channel ch
    // FK > 0: the cells (oy - dy, ox0 - 1 + j), channels kch, computed here
    T pc[FK > 0 ? 2 : 1][FK > 0 ? 5 : 1][FKO];
    if constexpr (FK > 0) {
      constexpr int NRW = FK + 1, NCL = FK + 4;  // node patch: rows oy - 1 - p .., cols ox0 - 1 - p ..
      const I sr = DEC ? (I)g.E[2] : (I)g.n[2];
      const I sb = DEC ? (I)(g.E[0] * g.E[1] * g.E[2]) : (I)(g.n[0] * g.n[1] * g.n[2]);
      I col[NCL];
#pragma unroll
      for (int c2 = 0; c2 < NCL; ++c2) col[c2] = (I)node_src((int64_t)ox0 - 1 - p + c2, g.L[2], g.E[2], ns.mult);
      float nd[NRW][NCL];
#pragma unroll
      for (int r2 = 0; r2 < NRW; ++r2) {
        const I rb = b * sb + (I)node_src((int64_t)oy - 1 - p + r2, g.L[1], g.E[1], ns.mult) * sr;
#pragma unroll
        for (int c2 = 0; c2 < NCL; ++c2) nd[r2][c2] = (float)src[rb + col[c2]];
      }
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int j = 0; j < 5; ++j) {
          float acc[FKO];
#pragma unroll
          for (int k = 0; k < FKO; ++k) acc[k] = wl[FN * FKO + k];
#pragma unroll
          for (int fy = 0; fy < FK; ++fy)
#pragma unroll
            for (int fx = 0; fx < FK; ++fx) {
              const float fv = nd[1 - dy + fy][j + fx];
#pragma unroll
              for (int k = 0; k < FKO; ++k) acc[k] = __builtin_fmaf(fv, wl[(fy * FK + fx) * FKO + k], acc[k]);
            }
#pragma unroll
          for (int k = 0; k < FKO; ++k) pc[dy][j][k] = lin_cast_t<T>(acc[k]);
        }
    }
    auto cell = [&](int i, int dz, int dy, int dx, int kch, int ch) -> T {
      if constexpr (FK > 0) return pc[dy][i + 1 - dx][kch];
      else if constexpr (PERCH) return cells[cbase - dz * cz - dy * cy + (i - dx) * CC + ch + (I)kch * kp];
      else return cm[dz][dy][i + 1 - dx][ch];
    };
    auto pred = [&](int k, int i, int ch) -> uint32_t {
      Contrib c[4];
      const int nc = map_contribs(NSP, k, c);
      if (k == center_map(NSP)) return (uint32_t)to_i32(cell(i, 0, 0, 0, c[0].ch, ch));
      float sacc = 0.0f;
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (q >= nc) break;
        if (cv[c[q].dz][c[q].dy][i + 1 - c[q].dx]) {
          sacc += (float)cell(i, c[q].dz, c[q].dy, c[q].dx, c[q].ch, ch);
          ++cnt;
        }
      }
      if (cnt == 4) sacc *= 0.25f;
      else if (cnt == 2) sacc *= 0.5f;
      return (uint32_t)to_i32(gcast<T>(sacc));
    };
    if constexpr (!DEC) {
      // ---- encode: the 8 x CC samples of each of the 2^d highres rows, then lowres + maps ----
      uint32_t hv[NZ][2][NH];
#pragma unroll
      for (int pz = 0; pz < NZ; ++pz)
#pragma unroll
        for (int py = 0; py < 2; ++py) {
          const I hz_ = 2 * oz + pz, hy_ = 2 * oy + py;
          const bool rowok = hz_ < (I)g.n[0] && hy_ < (I)g.n[1];
          const T* rp = src + b * hb + hz_ * hz + hy_ * hy + 2 * ox0 * CC;
          if (rowok && 2 * ox0 + 8 <= (I)g.n[2]) {
            g_loadn<T, NH>(rp, hv[pz][py]);
          } else {
#pragma unroll
            for (int e = 0; e < NH; ++e) hv[pz][py][e] = (rowok && 2 * ox0 + e / CC < (I)g.n[2]) ? (uint32_t)rp[e] : 0u;
          }
        }
      if (oz < (I)g.E[0] && oy < (I)g.E[1]) {
        uint32_t lv[NO];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ch = 0; ch < CC; ++ch) lv[i * CC + ch] = hv[0][0][2 * i * CC + ch];
        T* lp = dst + b * lb + oz * lz + oy * ly + ox0 * CC;
        const int n = (int)((I)g.E[2] - ox0 < nout ? (I)g.E[2] - ox0 : nout);
        if (n == 4) g_storen<T, NO>(lp, lv);
        else
#pragma unroll
          for (int e = 0; e < NO; ++e)
            if (e / CC < n) lp[e] = (T)lv[e];
      }
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        const int p0 = gpar<NSP>(k, 0), p1 = gpar<NSP>(k, 1), p2 = gpar<NSP>(k, 2);
        const I e0 = (I)(p0 ? g.Lc[0] : g.E[0]), e1 = (I)(p1 ? g.Lc[1] : g.E[1]), e2 = (I)(p2 ? g.Lc[2] : g.E[2]);
        if (oz >= e0 || oy >= e1) continue;
        const int n = (int)(e2 - ox0 < nout ? e2 - ox0 : nout);
        if (n <= 0) continue;
        uint32_t ov[NO];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int ch = 0; ch < CC; ++ch)
            ov[i * CC + ch] = (uint32_t)code_encode<CODER>((int32_t)pred(k, i, ch),
                                                           to_i32((T)hv[NSP == 3 ? p0 : 0][p1][(2 * i + p2) * CC + ch]));
        TO* mp = (TO*)omaps.p[k] + (((b * e0 + oz) * e1 + oy) * e2 + ox0) * CC;
        if (n == 4) g_storen<TO, NO>(mp, ov);
        else
#pragma unroll
          for (int e = 0; e < NO; ++e)
            if (e / CC < n) mp[e] = (TO)ov[e];
      }
    } else {
      // ---- decode: lowres + maps into the 8 x CC samples of each highres row ----
      uint32_t hv[NZ][2][8][CC];
      bool hok[NZ][2][8];
#pragma unroll
      for (int pz = 0; pz < NZ; ++pz)
#pragma unroll
        for (int py = 0; py < 2; ++py)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
#pragma unroll
            for (int ch = 0; ch < CC; ++ch) hv[pz][py][e][ch] = 0u;
            hok[pz][py][e] = false;
          }
      if (oz < (I)g.E[0] && oy < (I)g.E[1]) {
        const T* lp = src + b * lb + oz * lz + oy * ly + ox0 * CC;
        const int n = (int)((I)g.E[2] - ox0 < nout ? (I)g.E[2] - ox0 : nout);
        uint32_t lv[NO];
        if (n == 4) g_loadn<T, NO>(lp, lv);
        else
#pragma unroll
          for (int e = 0; e < NO; ++e) lv[e] = e / CC < n ? (uint32_t)lp[e] : 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int ch = 0; ch < CC; ++ch) hv[0][0][2 * i][ch] = lv[i * CC + ch];
          hok[0][0][2 * i] = i < n;
        }
      }
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        const int p0 = gpar<NSP>(k, 0), p1 = gpar<NSP>(k, 1), p2 = gpar<NSP>(k, 2);
        const I e0 = (I)(p0 ? g.Lc[0] : g.E[0]), e1 = (I)(p1 ? g.Lc[1] : g.E[1]), e2 = (I)(p2 ? g.Lc[2] : g.E[2]);
        if (oz >= e0 || oy >= e1) continue;
        const int n = (int)(e2 - ox0 < nout ? e2 - ox0 : nout);
        if (n <= 0) continue;
        const TO* mp = (const TO*)imaps.p[k] + (((b * e0 + oz) * e1 + oy) * e2 + ox0) * CC;
        uint32_t mv[NO];
        if (n == 4) g_loadn<TO, NO>(mp, mv);
        else
#pragma unroll
          for (int e = 0; e < NO; ++e) mv[e] = e / CC < n ? (uint32_t)mp[e] : 0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
          for (int ch = 0; ch < CC; ++ch)
            hv[NSP == 3 ? p0 : 0][p1][2 * i + p2][ch] =
                (uint32_t)(T)code_decode<CODER>((int32_t)pred(k, i, ch), (int32_t)(TO)mv[i * CC + ch]);
          hok[NSP == 3 ? p0 : 0][p1][2 * i + p2] = i < n;
        }
      }
#pragma unroll
      for (int pz = 0; pz < NZ; ++pz)
#pragma unroll
        for (int py = 0; py < 2; ++py) {
          const I hz_ = 2 * oz + pz, hy_ = 2 * oy + py;
          if (hz_ >= (I)g.n[0] || hy_ >= (I)g.n[1]) continue;
          T* rp = dst + b * hb + hz_ * hz + hy_ * hy + 2 * ox0 * CC;
          bool all = true;
#pragma unroll
          for (int e = 0; e < 8; ++e) all = all && hok[pz][py][e];
          uint32_t row[NH];
#pragma unroll
          for (int e = 0; e < 8; ++e)
#pragma unroll
            for (int ch = 0; ch < CC; ++ch) row[e * CC + ch] = hv[pz][py][e][ch];
          if (all) g_storen<T, NH>(rp, row);
          else
#pragma unroll
            for (int e = 0; e < NH; ++e)
              if (hok[pz][py][e / CC]) rp[e] = (T)row[e];
        }
    }
  }
}

// ------------------------------------------------------------------------------------------
// Host side of the generic path
// ------------------------------------------------------------------------------------------
int64_t generic_workspace_bytes(int dtype, int nsp, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred) {
  const bool lin = pred && (pred->kind == KMP_PRED_LINEAR || pred->kind == KMP_PRED_LINEAR_MFMA);
  const int K = lin ? (nsp == 3 ? 19 : 5) : 1;
  int64_t need = B * g.Lc[0] * g.Lc[1] * g.Lc[2] * K * C * dtype_size(dtype);
  if (lin && B > 0) {  // the fused LinearPredictor kernels keep a reordered copy of W [N, K] there
    const int64_t nb = 2 * pred->padding + 2, N = nsp == 3 ? nb * nb * nb : nb * nb;
    int64_t wbytes = N * K * (int64_t)sizeof(float);
    // the matrix-core kernels' B fragments (3 column tiles x 8 chunks x 64 lanes x 16 B) + biases
    // + linear3pm's dummy store slots (64 lanes x 16 B)
    constexpr int64_t kMfmaWs = 3 * 8 * 64 * 16 + 3 * 64 * 4 + 64 * 16;
    if (pred->kind == KMP_PRED_LINEAR_MFMA) wbytes = wbytes > kMfmaWs ? wbytes : kMfmaWs;
    need = need > wbytes ? need : wbytes;
  }
  return need;
}

static Frame make_frame(int nsp, const Geo& g, const kmp_region* region) {
  Frame f{};
  for (int a = 0; a < 3; ++a) {
    int64_t lo = 0, hi = g.E[a];
    if (region && a >= 3 - nsp) {
      lo = region->begin[a] < 0 ? 0 : region->begin[a];
      hi = region->end[a] > g.E[a] ? g.E[a] : region->end[a];
    }
    f.begin[a] = lo;
    f.ext[a] = hi > lo ? hi - lo : 0;
  }
  return f;
}

// Cells a frame of outputs depends on: [begin-1, end) clipped to [0, Lc).
static Frame cell_frame(const Geo& g, const Frame& f) {
  Frame cf{};
  for (int a = 0; a < 3; ++a) {
    int64_t lo = f.begin[a] - 1, hi = f.begin[a] + f.ext[a];
    lo = lo < 0 ? 0 : lo;
    hi = hi > g.Lc[a] ? g.Lc[a] : hi;
    cf.begin[a] = lo;
    cf.ext[a] = (f.ext[a] > 0 && hi > lo) ? hi - lo : 0;
  }
  return cf;
}

// 32-bit element indexing when every array the generic kernels address (highres, cells, lowres,
// maps: all at most the padded highres size x K) and the index space stay below 2^31
static bool fits32(const Geo& g, int64_t B, int64_t C, int K) {
  const int64_t lim = (int64_t)1 << 31;
  const int64_t hi = B * (g.n[0] + 1) * (g.n[1] + 1) * (g.n[2] + 1) * C;
  const int64_t cells = B * g.L[0] * g.L[1] * g.L[2] * K * C;
  return B > 0 && hi < lim && cells < lim;
}

template <typename T>
static int run_predictor(const T* src, const Src& s, const Geo& g, int nsp, int64_t B, int64_t C,
                         const kmp_predictor* pred, const Frame& f, T* cells, hipStream_t stream) {
  const Frame cf = cell_frame(g, f);
  const int64_t ncell = B * cf.ext[0] * cf.ext[1] * cf.ext[2] * C;
  if (ncell == 0) return KMP_OK;
  if (pred->kind == KMP_PRED_MEAN) {
    const bool i32 = fits32(g, B, C, 1);
    const int p = pred->padding, kk = 2 * p + 2;
    const int64_t nn = (nsp == 3 ? kk : 1) * (int64_t)kk * kk;
    const int64_t top = std::is_same<T, uint8_t>::value ? 255 : (std::is_same<T, uint16_t>::value ? 65535 : -1);
    if (i32 && p <= 3) {  // cell_mean_row_kernel: exact integer sums when they are, else in-order floats
      const bool exact = top > 0 && nn * top < ((int64_t)1 << 24);
      const int64_t ext_q[3] = {cf.ext[0], cf.ext[1], ceil_div(cf.ext[2], (int64_t)kMeanR)};
      const Flat Fq = make_flat(ext_q, C);
      const int64_t nq = B * ext_q[0] * ext_q[1] * ext_q[2] * C;
      auto go = [&](auto nsp_c, auto kk_c) {
        constexpr int NSP = decltype(nsp_c)::value, KK = decltype(kk_c)::value;
        if (exact) cell_mean_row_kernel<T, NSP, KK, true><<<ggrid(nq), kGThreads, 0, stream>>>(src, s, g, C, p, cf, Fq, cells, nq);
        else cell_mean_row_kernel<T, NSP, KK, false><<<ggrid(nq), kGThreads, 0, stream>>>(src, s, g, C, p, cf, Fq, cells, nq);
      };
      auto with_kk = [&](auto nsp_c) {
        if (p == 0) go(nsp_c, std::integral_constant<int, 2>{});
        else if (p == 1) go(nsp_c, std::integral_constant<int, 4>{});
        else if (p == 2) go(nsp_c, std::integral_constant<int, 6>{});
        else go(nsp_c, std::integral_constant<int, 8>{});
      };
      if (nsp == 3) with_kk(std::integral_constant<int, 3>{});
      else with_kk(std::integral_constant<int, 2>{});
      return check_launch("cell_mean");
    }
    const Flat F = make_flat(cf.ext, C);
    auto go = [&](auto nsp_c, auto i_tag) {
      constexpr int NSP = decltype(nsp_c)::value;
      using I = decltype(i_tag);
#define KMP_CM(KK) cell_mean_kernel<T, NSP, KK, I><<<ggrid(ncell), kGThreads, 0, stream>>>(src, s, g, B, C, p, cf, F, cells, ncell)
      if (p == 0) KMP_CM(2);
      else if (p == 1) KMP_CM(4);
      else if (p == 2) KMP_CM(6);
      else KMP_CM(0);
#undef KMP_CM
    };
    if (nsp == 3) {
      if (i32) go(std::integral_constant<int, 3>{}, int32_t{});
      else go(std::integral_constant<int, 3>{}, int64_t{});
    } else {
      if (i32) go(std::integral_constant<int, 2>{}, int32_t{});
      else go(std::integral_constant<int, 2>{}, int64_t{});
    }
    return check_launch("cell_mean");
  }
  const int64_t cbeg[3] = {cf.begin[0], cf.begin[1], cf.begin[2]}, cext[3] = {cf.ext[0], cf.ext[1], cf.ext[2]};
  return linear_cells<T>(src, s.S, s.mult, g, nsp, B, C, pred, cbeg, cext, cells, stream);
}

// Images with one channel and the f32 LinearPredictor at p <= 1: the row kernel computes its cells
// itself (codec_row4_kernel FK > 0; at p = 2 the 7 x 10 node patch and 36 x 5 weights outgrow the
// registers); KMP_DISABLE_LINEAR_FUSED=1 keeps the two-pass path
static bool fuse_lin2d(int nsp, int64_t C, const Geo& g, int64_t B, const kmp_predictor* pred) {
  return nsp == 2 && C == 1 && pred->kind == KMP_PRED_LINEAR && pred->padding <= 1 && pred->weights && pred->bias &&
         fits32(g, B, C, 5) && !opt(OPT_DISABLE_LINEAR_FUSED, 0);
}
template <typename F>
static void with_fk(int p, F&& f) {
  if (p == 0) f(std::integral_constant<int, 2>{});
  else f(std::integral_constant<int, 4>{});
}

// the row kernel's compile-time channel count (1..4; 3D takes 1..2 -- with 3-4 channels its
// 7 maps' values outgrow the registers and spill)
template <typename F>
static void with_cc(int64_t C, F&& f) {
  if (C == 1) f(std::integral_constant<int, 1>{});
  else if (C == 2) f(std::integral_constant<int, 2>{});
  else if (C == 3) f(std::integral_constant<int, 3>{});
  else f(std::integral_constant<int, 4>{});
}

// the encode / decode kernel of (NSP, PERCH, I) for this call
template <bool DEC, typename T, int CODER, typename Launch>
static void gen_dispatch(int nsp, bool perch, bool i32, Launch&& launch) {
  auto with_i = [&](auto nsp_c, auto perch_c) {
    if (i32) launch(nsp_c, perch_c, int32_t{});
    else launch(nsp_c, perch_c, int64_t{});
  };
  using N3 = std::integral_constant<int, 3>;
  using N2 = std::integral_constant<int, 2>;
  using PT = std::true_type;
  using PF = std::false_type;
  if (nsp == 3) {
    if (perch) with_i(N3{}, PT{});
    else with_i(N3{}, PF{});
  } else {
    if (perch) with_i(N2{}, PT{});
    else with_i(N2{}, PF{});
  }
}

template <typename T, int CODER>
static int encode_generic_t(const T* hi, const Geo& g, int nsp, int64_t B, int64_t C, const kmp_predictor* pred,
                            T* lowres, const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  const int64_t need = generic_workspace_bytes(dtype_code<T>(), nsp, g, B, C, pred);
  if ((int64_t)ws_bytes < need || (!ws && need > 0))
    return fail(KMP_ERR_ARG, "encode: workspace too small (" + std::to_string(ws_bytes) + " < " + std::to_string(need) + ")");
  Src s{{g.n[0], g.n[1], g.n[2]}, 2};
  T* cells = (T*)ws;
  Frame f = make_frame(nsp, g, region);
  const int64_t total = B * f.ext[0] * f.ext[1] * f.ext[2] * C;
  if (fuse_lin2d(nsp, C, g, B, pred)) {  // images, f32 LinearPredictor: the cells computed in the row kernel
    if (total == 0) return KMP_OK;
    const int64_t nxq = ceil_div(f.ext[2], 4), n4 = B * f.ext[0] * f.ext[1] * nxq;
    const Row4 R{fdiv(nxq), fdiv(f.ext[1]), fdiv(f.ext[0])};
    with_fk(pred->padding, [&](auto fk_c) {
      codec_row4_kernel<T, CODER, true, 2, 1, false, decltype(fk_c)::value><<<ggrid(n4), kGThreads, 0, stream>>>(
          hi, CMapPtrs{}, g, nullptr, B, lowres, maps, f, R, nxq, n4, s, pred->weights, pred->bias, pred->padding);
    });
    return check_launch("encode_generic");
  }
  if (int st = run_predictor<T>(hi, s, g, nsp, B, C, pred, f, cells, stream)) return st;
  if (total == 0) return KMP_OK;
  const bool perch = pred->kind != KMP_PRED_MEAN;
  const int K = perch ? (nsp == 3 ? 19 : 5) : 1;
  if (C <= (nsp == 3 ? 2 : 4) && fits32(g, B, C, K)) {  // 4 output positions (x C) a thread
    const int64_t nxq = ceil_div(f.ext[2], 4), n4 = B * f.ext[0] * f.ext[1] * nxq;
    const Row4 R{fdiv(nxq), fdiv(f.ext[1]), fdiv(f.ext[0])};
    gen_dispatch<false, T, CODER>(nsp, perch, true, [&](auto nsp_c, auto perch_c, auto) {
      with_cc(C, [&](auto cc_c) {
        constexpr int NSP = decltype(nsp_c)::value, CC = decltype(cc_c)::value;
        if constexpr (NSP == 2 || CC <= 2)  // (3D with 3-4 channels: the per-element kernel, see above)
          codec_row4_kernel<T, CODER, decltype(perch_c)::value, NSP, CC, false>
              <<<ggrid(n4), kGThreads, 0, stream>>>(hi, CMapPtrs{}, g, cells, B, lowres, maps, f, R, nxq, n4);
      });
    });
    return check_launch("encode_generic");
  }
  const Flat F = make_flat(f.ext, C);
  gen_dispatch<false, T, CODER>(nsp, perch, fits32(g, B, C, K), [&](auto nsp_c, auto perch_c, auto i_tag) {
    encode_generic_kernel<T, CODER, decltype(perch_c)::value, decltype(nsp_c)::value, decltype(i_tag)>
        <<<ggrid(total), kGThreads, 0, stream>>>(hi, g, B, C, cells, K, lowres, maps, f, F, total);
  });
  return check_launch("encode_generic");
}

template <typename T, int CODER>
static int decode_generic_t(const T* lowres, const CMapPtrs& maps, const Geo& g, int nsp, int64_t B, int64_t C,
                            const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  const int64_t need = generic_workspace_bytes(dtype_code<T>(), nsp, g, B, C, pred);
  if ((int64_t)ws_bytes < need || (!ws && need > 0))
    return fail(KMP_ERR_ARG, "decode: workspace too small (" + std::to_string(ws_bytes) + " < " + std::to_string(need) + ")");
  Src s{{g.E[0], g.E[1], g.E[2]}, 1};
  T* cells = (T*)ws;
  Frame f = make_frame(nsp, g, region);
  const int64_t total = B * f.ext[0] * f.ext[1] * f.ext[2] * C;
  if (fuse_lin2d(nsp, C, g, B, pred)) {
    if (total == 0) return KMP_OK;
    const int64_t nxq = ceil_div(f.ext[2], 4), n4 = B * f.ext[0] * f.ext[1] * nxq;
    const Row4 R{fdiv(nxq), fdiv(f.ext[1]), fdiv(f.ext[0])};
    with_fk(pred->padding, [&](auto fk_c) {
      codec_row4_kernel<T, CODER, true, 2, 1, true, decltype(fk_c)::value><<<ggrid(n4), kGThreads, 0, stream>>>(
          lowres, maps, g, nullptr, B, hi, MapPtrs{}, f, R, nxq, n4, s, pred->weights, pred->bias, pred->padding);
    });
    return check_launch("decode_generic");
  }
  if (int st = run_predictor<T>(lowres, s, g, nsp, B, C, pred, f, cells, stream)) return st;
  if (total == 0) return KMP_OK;
  const bool perch = pred->kind != KMP_PRED_MEAN;
  const int K = perch ? (nsp == 3 ? 19 : 5) : 1;
  if (C <= (nsp == 3 ? 2 : 4) && fits32(g, B, C, K)) {  // 4 output positions (x C) a thread
    const int64_t nxq = ceil_div(f.ext[2], 4), n4 = B * f.ext[0] * f.ext[1] * nxq;
    const Row4 R{fdiv(nxq), fdiv(f.ext[1]), fdiv(f.ext[0])};
    gen_dispatch<true, T, CODER>(nsp, perch, true, [&](auto nsp_c, auto perch_c, auto) {
      with_cc(C, [&](auto cc_c) {
        constexpr int NSP = decltype(nsp_c)::value, CC = decltype(cc_c)::value;
        if constexpr (NSP == 2 || CC <= 2)
          codec_row4_kernel<T, CODER, decltype(perch_c)::value, NSP, CC, true>
              <<<ggrid(n4), kGThreads, 0, stream>>>(lowres, maps, g, cells, B, hi, MapPtrs{}, f, R, nxq, n4);
      });
    });
    return check_launch("decode_generic");
  }
  const Flat F = make_flat(f.ext, C);
  gen_dispatch<true, T, CODER>(nsp, perch, fits32(g, B, C, K), [&](auto nsp_c, auto perch_c, auto i_tag) {
    decode_generic_kernel<T, CODER, decltype(perch_c)::value, decltype(nsp_c)::value, decltype(i_tag)>
        <<<ggrid(total), kGThreads, 0, stream>>>(lowres, maps, g, B, C, cells, K, hi, f, F, total);
  });
  return check_launch("decode_generic");
}

// Natural coder per dtype: (u8, U8), (u16, U16), (i32, RAW), (u32, U32).
template <typename F>
static int dispatch_natural(int dtype, int coder, F&& f) {
  if (dtype == KMP_U8 && coder == KMP_CODER_U8) return f(uint8_t{}, std::integral_constant<int, KMP_CODER_U8>{});
  if (dtype == KMP_U16 && coder == KMP_CODER_U16) return f(uint16_t{}, std::integral_constant<int, KMP_CODER_U16>{});
  if (dtype == KMP_I32 && coder == KMP_CODER_RAW) return f(int32_t{}, std::integral_constant<int, KMP_CODER_RAW>{});
  if (dtype == KMP_U32 && coder == KMP_CODER_U32) return f(uint32_t{}, std::integral_constant<int, KMP_CODER_U32>{});
  return fail(KMP_ERR_UNSUPPORTED, "fused codec supports (uint8, U8), (uint16, U16), (int32, RAW), (uint32, U32); got dtype " +
                                       std::to_string(dtype) + " coder " + std::to_string(coder));
}

static int check_predictor(const kmp_predictor* pred, int dtype) {
  KMP_REQUIRE(pred, "null predictor");
  KMP_REQUIRE(pred->padding >= 0, "negative padding");
  KMP_REQUIRE(pred->kind == KMP_PRED_MEAN || pred->kind == KMP_PRED_LINEAR || pred->kind == KMP_PRED_LINEAR_MFMA,
              "unknown predictor kind");
  if (pred->kind != KMP_PRED_MEAN) KMP_REQUIRE(pred->weights && pred->bias, "linear predictor needs weights and bias");
  if (pred->kind == KMP_PRED_LINEAR_MFMA)
    KMP_REQUIRE(dtype == KMP_U8 || dtype == KMP_U16, "the matrix-core LinearPredictor takes uint8 / uint16 samples");
  return KMP_OK;
}

int codec_encode(int nsp, int dtype, const void* highres, int64_t B, const int64_t* shape, int64_t C,
                 const kmp_predictor* pred, int coder, void* lowres_out, void* const* maps_out, int32_t* dims_out,
                 const kmp_region* region, void* ws, size_t ws_bytes, hipStream_t stream) {
  KMP_REQUIRE(B >= 0 && C >= 1, "bad batch or channel count");
  for (int a = 0; a < nsp; ++a) KMP_REQUIRE(shape[a] >= 2, "spatial dims must be >= 2 (>= 3 after even padding)");
  if (int st = check_predictor(pred, dtype)) return st;
  Geo g = make_geo_from_highres(nsp, shape);
  if (dims_out)
    for (int a = 0; a < nsp; ++a) dims_out[a] = g.dims[a + 3 - nsp];
  KMP_REQUIRE(highres && lowres_out && maps_out, "null pointer");
  MapPtrs maps{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(maps_out[k], "null map pointer");
    maps.p[k] = maps_out[k];
  }
  if (B == 0) return KMP_OK;
  return dispatch_natural(dtype, coder, [&](auto tag, auto coder_c) {
    using T = decltype(tag);
    constexpr int CODER = decltype(coder_c)::value;
    int st = try_fast_encode<T>(nsp, (const T*)highres, g, B, C, pred, (T*)lowres_out, maps, region, ws, ws_bytes,
                                stream);
    if (st != KMP_ERR_UNSUPPORTED) return st;
    return encode_generic_t<T, CODER>((const T*)highres, g, nsp, B, C, pred, (T*)lowres_out, maps, region, ws,
                                      ws_bytes, stream);
  });
}

int codec_decode(int nsp, int dtype, const void* lowres, const void* const* maps_in, int64_t B, const int64_t* E,
                 int64_t C, const int32_t* dims, const kmp_predictor* pred, int coder, void* highres_out,
                 const kmp_region* region, void* ws, size_t ws_bytes, hipStream_t stream) {
  KMP_REQUIRE(B >= 0 && C >= 1 && dims, "bad batch/channel count or dims");
  for (int a = 0; a < nsp; ++a) {
    KMP_REQUIRE(dims[a] == 0 || dims[a] == 1, "dims must be 0 or 1");
    KMP_REQUIRE(E[a] >= 1 && E[a] + dims[a] >= 2, "lowres too small");
  }
  if (int st = check_predictor(pred, dtype)) return st;
  Geo g = make_geo_from_lowres(nsp, E, dims);
  KMP_REQUIRE(lowres && maps_in && highres_out, "null pointer");
  CMapPtrs maps{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(maps_in[k], "null map pointer");
    maps.p[k] = maps_in[k];
  }
  if (B == 0) return KMP_OK;
  return dispatch_natural(dtype, coder, [&](auto tag, auto coder_c) {
    using T = decltype(tag);
    constexpr int CODER = decltype(coder_c)::value;
    int st = try_fast_decode<T>(nsp, (const T*)lowres, maps, g, B, C, pred, (T*)highres_out, region, ws, ws_bytes,
                                stream);
    if (st != KMP_ERR_UNSUPPORTED) return st;
    return decode_generic_t<T, CODER>((const T*)lowres, maps, g, nsp, B, C, pred, (T*)highres_out, region, ws,
                                      ws_bytes, stream);
  });
}

}  // namespace kmp

using namespace kmp;

extern "C" {

int kmp_volume_encode(int32_t dtype, const void* highres, int64_t B, int64_t D, int64_t H, int64_t W, int64_t C,
                      const kmp_predictor* predictor, int32_t coder, void* lowres_out, void* const maps_out[7],
                      int32_t dims_out[3], const kmp_region* region, void* workspace, size_t workspace_bytes,
                      kmp_stream_t stream) {
  const int64_t shape[3] = {D, H, W};
  return codec_encode(3, dtype, highres, B, shape, C, predictor, coder, lowres_out, maps_out, dims_out, region,
                      workspace, workspace_bytes, (hipStream_t)stream);
}

int kmp_volume_decode(int32_t dtype, const void* lowres, const void* const maps[7], int64_t B, int64_t Ed, int64_t Eh,
                      int64_t Ew, int64_t C, const int32_t dims[3], const kmp_predictor* predictor, int32_t coder,
                      void* highres_out, const kmp_region* region, void* workspace, size_t workspace_bytes,
                      kmp_stream_t stream) {
  const int64_t E[3] = {Ed, Eh, Ew};
  return codec_decode(3, dtype, lowres, maps, B, E, C, dims, predictor, coder, highres_out, region, workspace,
                      workspace_bytes, (hipStream_t)stream);
}

int64_t kmp_volume_workspace_bytes(int32_t dtype, int64_t B, int64_t D, int64_t H, int64_t W, int64_t C,
                                   const kmp_predictor* predictor) {
  const int64_t shape[3] = {D, H, W};
  Geo g = make_geo_from_highres(3, shape);
  return generic_workspace_bytes(dtype, 3, g, B, C, predictor);
}

int kmp_image_encode(int32_t dtype, const void* highres, int64_t B, int64_t H, int64_t W, int64_t C,
                     const kmp_predictor* predictor, int32_t coder, void* lowres_out, void* const maps_out[3],
                     int32_t dims_out[2], const kmp_region* region, void* workspace, size_t workspace_bytes,
                     kmp_stream_t stream) {
  const int64_t shape[2] = {H, W};
  return codec_encode(2, dtype, highres, B, shape, C, predictor, coder, lowres_out, maps_out, dims_out, region,
                      workspace, workspace_bytes, (hipStream_t)stream);
}

int kmp_image_decode(int32_t dtype, const void* lowres, const void* const maps[3], int64_t B, int64_t Eh, int64_t Ew,
                     int64_t C, const int32_t dims[2], const kmp_predictor* predictor, int32_t coder,
                     void* highres_out, const kmp_region* region, void* workspace, size_t workspace_bytes,
                     kmp_stream_t stream) {
  const int64_t E[2] = {Eh, Ew};
  return codec_decode(2, dtype, lowres, maps, B, E, C, dims, predictor, coder, highres_out, region, workspace,
                      workspace_bytes, (hipStream_t)stream);
}

int64_t kmp_image_workspace_bytes(int32_t dtype, int64_t B, int64_t H, int64_t W, int64_t C,
                                  const kmp_predictor* predictor) {
  const int64_t shape[2] = {H, W};
  Geo g = make_geo_from_highres(2, shape);
  return generic_workspace_bytes(dtype, 2, g, B, C, predictor);
}

}  // extern "C"
