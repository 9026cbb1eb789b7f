// kmp_primitives.hip -- the geometry primitives of the reference API as gfx950 kernels.
//
// These back the generic ``predictions_fn`` callback path (a caller's predictor composes
// features_from_lowres / maps_from_predictions / coders exactly as in the reference) and the
// standalone re-exports of volume/__init__.py:31-35 and image/__init__.py:31-35.  They are
// HBM-bound gathers/scatters: one thread per output element group, 64-bit index math,
// grid-stride loops, 256-thread workgroups.  The fused one-pass codec lives in kmp_codec*.hip.
#include <mutex>

#include "kmp_aggregate.h"

namespace kmp {

static thread_local std::string g_last_error;
static thread_local const char* g_last_launch = "";

void set_error(const std::string& msg) { g_last_error = msg; }
int fail(int status, const std::string& msg) {
  g_last_error = msg;
  return status;
}
int check_launch(const char* what) {
  g_last_launch = what;
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(KMP_ERR_LAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  return KMP_OK;
}

constexpr int kThreads = 256;

static inline unsigned grid_for(int64_t n) {
  int64_t g = ceil_div(n, kThreads);
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// Every kernel below is instantiated with a 32-bit index type when all the arrays it touches
// have fewer than 2^30 elements (64-bit multiplies and divisions are multi-instruction sequences
// on gfx950), and with I otherwise.
template <typename I>
struct IdxT {
  I b, i0, i1, i2, c;
};
// Decompose a flat index over [B, e0, e1, e2, C].
template <typename I>
__device__ __forceinline__ IdxT<I> unflat_t(I t, I e0, I e1, I e2, I C) {
  IdxT<I> r;
  if constexpr (sizeof(I) == 4) {
    uint32_t u = (uint32_t)t;
    if (C == 1) {
      r.c = 0;
    } else {
      r.c = (I)(u % (uint32_t)C);
      u /= (uint32_t)C;
    }
    r.i2 = (I)(u % (uint32_t)e2); u /= (uint32_t)e2;
    r.i1 = (I)(u % (uint32_t)e1); u /= (uint32_t)e1;
    r.i0 = (I)(u % (uint32_t)e0);
    r.b = (I)(u / (uint32_t)e0);
  } else {
    unflat5(t, e0, e1, e2, C, r.b, r.i0, r.i1, r.i2, r.c);
  }
  return r;
}
template <typename I>
__device__ __forceinline__ I sym_idx(I i, I n) {  // sym_index in the kernel's index type
  if (i >= 0 && i < n) return i;
  if (i >= -n && i < 2 * n) return i < 0 ? -1 - i : 2 * n - 1 - i;
  I m = i % (2 * n);
  if (m < 0) m += 2 * n;
  return m < n ? m : 2 * n - 1 - m;
}

// ------------------------------------------------------------------------------------------
// Parity (de)interleave: lowres_from_highres, maps_from_highres, highres_from_lowres_and_maps
// ------------------------------------------------------------------------------------------
struct Ext3 {
  int64_t e[3];
};
template <typename I>
struct E3 {
  I e[3];
};
template <typename I>
static inline E3<I> e3(const Ext3& x) {
  return E3<I>{{(I)x.e[0], (I)x.e[1], (I)x.e[2]}};
}

// out_k[b, o, c] = in[b, 2*o + par_k, c] for every class k whose pointer is set and whose
// extent contains o.  Class 0 = all-even (lowres), classes 1..7 (1..3) = maps.
template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) deinterleave_kernel(const T* __restrict__ in, I B, E3<I> n,
                                                              I C, int nsp, MapPtrs outs, void* lowres,
                                                              I total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  // frame = ceil(n/2) per axis (dummy axes: 1)
  const I f0 = (n.e[0] + 1) / 2, f1 = (n.e[1] + 1) / 2, f2 = (n.e[2] + 1) / 2;
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, f0, f1, f2, C);
    auto src = [&](int pz, int py, int px) -> T {
      const I z = 2 * q.i0 + pz, y = 2 * q.i1 + py, x = 2 * q.i2 + px;
      return in[(((q.b * n.e[0] + z) * n.e[1] + y) * n.e[2] + x) * C + q.c];
    };
    if (lowres) {
      T* o = (T*)lowres;
      o[(((q.b * f0 + q.i0) * f1 + q.i1) * f2 + q.i2) * C + q.c] = src(0, 0, 0);
    }
    for (int k = 0; k < nmaps; ++k) {
      if (!outs.p[k]) continue;
      int par[3];
      map_parity(nsp, k, par);
      // extent of class: parity 1 -> floor(n/2), parity 0 -> ceil(n/2); dummy axis -> 1
      I e[3];
      const I idx[3] = {q.i0, q.i1, q.i2};
      bool ok = true;
      for (int a = 0; a < 3; ++a) {
        e[a] = (a < 3 - nsp) ? 1 : (par[a] ? n.e[a] / 2 : (n.e[a] + 1) / 2);
        ok = ok && idx[a] < e[a];
      }
      if (!ok) continue;
      T* o = (T*)outs.p[k];
      o[(((q.b * e[0] + q.i0) * e[1] + q.i1) * e[2] + q.i2) * C + q.c] = src(par[0], par[1], par[2]);
    }
  }
}

// out[b, 2*o + par_k, c] = class_k[b, o, c]; out extent 2L-1 per axis.  Class extents follow
// highres_from_lowres_and_maps: lowres L, maps (par ? L-1 : L).
template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) interleave_kernel(const T* __restrict__ lowres, CMapPtrs maps,
                                                            I B, E3<I> L, I C, int nsp, T* __restrict__ out,
                                                            I total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  const I h0 = 2 * L.e[0] - 1, h1 = 2 * L.e[1] - 1, h2 = 2 * L.e[2] - 1;
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, L.e[0], L.e[1], L.e[2], C);
    auto dst = [&](int pz, int py, int px) -> T& {
      const I z = 2 * q.i0 + pz, y = 2 * q.i1 + py, x = 2 * q.i2 + px;
      return out[(((q.b * h0 + z) * h1 + y) * h2 + x) * C + q.c];
    };
    dst(0, 0, 0) = lowres[t];
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      I e[3];
      const I idx[3] = {q.i0, q.i1, q.i2};
      bool ok = true;
      for (int a = 0; a < 3; ++a) {
        e[a] = (a < 3 - nsp) ? 1 : (par[a] ? L.e[a] - 1 : L.e[a]);
        ok = ok && idx[a] < e[a];
      }
      if (!ok) continue;
      const T* m = (const T*)maps.p[k];
      dst(par[0], par[1], par[2]) = m[(((q.b * e[0] + q.i0) * e[1] + q.i1) * e[2] + q.i2) * C + q.c];
    }
  }
}

// ------------------------------------------------------------------------------------------
// targets_from_highres: [B, cells..., K, C], K = 19 (5); cells = (n-1)/2 per axis.
// Offsets (relative to 2*cell) per target in reference order, volume/utils.py:40-72.
// ------------------------------------------------------------------------------------------
__constant__ int8_t c_targets3[19][3] = {
    {1, 1, 0}, {1, 1, 2}, {1, 0, 1}, {1, 2, 1}, {0, 1, 1}, {2, 1, 1}, {1, 1, 1},  // L R U D F B C
    {1, 0, 0}, {1, 0, 2}, {1, 2, 2}, {1, 2, 0},                                 // z0..z3
    {0, 1, 0}, {0, 1, 2}, {2, 1, 2}, {2, 1, 0},                                 // y0..y3
    {0, 0, 1}, {0, 2, 1}, {2, 2, 1}, {2, 0, 1}};                                // x0..x3
__constant__ int8_t c_targets2[5][2] = {{1, 0}, {1, 2}, {0, 1}, {2, 1}, {1, 1}};  // image/utils.py:40-44

template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) targets_kernel(const T* __restrict__ in, I B, E3<I> n, I C,
                                                         int nsp, T* __restrict__ out, I total) {
  const int K = nsp == 3 ? 19 : 5;
  const I c0 = nsp == 3 ? (n.e[0] - 1) / 2 : 1, c1 = (n.e[1] - 1) / 2, c2 = (n.e[2] - 1) / 2;
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, c0, c1, c2, C);
    const I cell = ((q.b * c0 + q.i0) * c1 + q.i1) * c2 + q.i2;
    for (int k = 0; k < K; ++k) {
      int dz, dy, dx;
      if (nsp == 3) { dz = c_targets3[k][0]; dy = c_targets3[k][1]; dx = c_targets3[k][2]; }
      else { dz = 0; dy = c_targets2[k][0]; dx = c_targets2[k][1]; }
      const I z = nsp == 3 ? 2 * q.i0 + dz : 0, y = 2 * q.i1 + dy, x = 2 * q.i2 + dx;
      out[(cell * K + k) * C + q.c] = in[(((q.b * n.e[0] + z) * n.e[1] + y) * n.e[2] + x) * C + q.c];
    }
  }
}

// features_from_lowres: [B, S-2p-1..., N, C], N = (2p+2)^d, offsets z-major then y, x.
template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) features_kernel(const T* __restrict__ in, I B, E3<I> S, I C,
                                                          int nsp, int p, T* __restrict__ out, I total) {
  const int k = 2 * p + 2;
  const int kz = nsp == 3 ? k : 1;
  const int N = kz * k * k;
  const I c0 = nsp == 3 ? S.e[0] - 2 * p - 1 : 1, c1 = S.e[1] - 2 * p - 1, c2 = S.e[2] - 2 * p - 1;
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, c0, c1, c2, C);
    const I cell = ((q.b * c0 + q.i0) * c1 + q.i1) * c2 + q.i2;
    int f = 0;
    for (int dz = 0; dz < kz; ++dz)
      for (int dy = 0; dy < k; ++dy)
        for (int dx = 0; dx < k; ++dx, ++f) {
          const I z = q.i0 + dz, y = q.i1 + dy, x = q.i2 + dx;
          out[(cell * N + f) * C + q.c] = in[(((q.b * S.e[0] + z) * S.e[1] + y) * S.e[2] + x) * C + q.c];
        }
  }
}

// C == 1, 32-bit indices, compile-time neighbourhood: one cell per thread, its N features
// gathered into registers and written as 16-byte vectors (or one 4 / 8-byte store when the whole
// cell is smaller); the output is 16-byte aligned.
template <typename T, int NSP, int P>
__global__ void __launch_bounds__(kThreads) features_vec_kernel(const T* __restrict__ in, int32_t S0, int32_t S1,
                                                              int32_t S2, T* __restrict__ out, int32_t cells) {
  constexpr int K = 2 * P + 2, KZ = NSP == 3 ? K : 1, N = KZ * K * K;
  constexpr int NB = N * (int)sizeof(T);
  constexpr int SB = NB >= 16 ? 16 : NB;  // store width: 16 bytes, or the whole cell when smaller
  static_assert(NB % SB == 0 && (SB == 16 || SB == 8 || SB == 4), "whole stores per cell");
  using SV = typename std::conditional<SB == 16, uint4, typename std::conditional<SB == 8, uint2, uint32_t>::type>::type;
  const int32_t c0 = NSP == 3 ? S0 - 2 * P - 1 : 1, c1 = S1 - 2 * P - 1, c2 = S2 - 2 * P - 1;
  for (int32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < cells; t += gridDim.x * blockDim.x) {
    uint32_t q = (uint32_t)t;
    const int32_t x = q % (uint32_t)c2; q /= (uint32_t)c2;
    const int32_t y = q % (uint32_t)c1; q /= (uint32_t)c1;
    const int32_t z = q % (uint32_t)c0;
    const int32_t b = q / (uint32_t)c0;
    const T* base = in + ((b * S0 + z) * S1 + y) * S2 + x;
    T f[N];
#pragma unroll
    for (int dz = 0; dz < KZ; ++dz)
#pragma unroll
      for (int dy = 0; dy < K; ++dy)
#pragma unroll
        for (int dx = 0; dx < K; ++dx) f[(dz * K + dy) * K + dx] = base[(dz * S1 + dy) * S2 + dx];
    SV* o = (SV*)(out + (int64_t)t * N);
#pragma unroll
    for (int v = 0; v < NB / SB; ++v) {
      SV w;
      __builtin_memcpy(&w, (const char*)f + v * SB, SB);
      o[v] = w;
    }
  }
}

// u8 / u16, C == 1, 32-bit indices: the f32 sum of at most 4 integer predictions is exact, so the
// reference's scale-and-truncate is an integer shift (the values of aggregate_map).
template <typename T, int NSP>
__global__ void __launch_bounds__(kThreads) maps_from_predictions_int_kernel(const T* __restrict__ preds, int32_t Lcz,
                                                                           int32_t Lcy, int32_t Lcx, MapPtrs outs,
                                                                           int32_t total) {
  constexpr int NM = NSP == 3 ? 7 : 3, K = NSP == 3 ? 19 : 5;
  const int32_t f0 = NSP == 3 ? Lcz + 1 : 1, f1 = Lcy + 1, f2 = Lcx + 1, cz = NSP == 3 ? Lcz : 1;
  for (int32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    uint32_t q = (uint32_t)t;
    const int32_t ox = q % (uint32_t)f2; q /= (uint32_t)f2;
    const int32_t oy = q % (uint32_t)f1; q /= (uint32_t)f1;
    const int32_t oz = q % (uint32_t)f0;
    const int32_t b = q / (uint32_t)f0;
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      int par[3];
      map_parity(NSP, k, par);
      const int32_t e0 = NSP == 3 ? (par[0] ? Lcz : Lcz + 1) : 1, e1 = par[1] ? Lcy : Lcy + 1, e2 = par[2] ? Lcx : Lcx + 1;
      if (oz >= e0 || oy >= e1 || ox >= e2) continue;
      Contrib c[4];
      const int nc = map_contribs(NSP, k, c);
      uint32_t s = 0, cnt = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i >= nc) break;
        const int32_t z = oz - c[i].dz, y = oy - c[i].dy, x = ox - c[i].dx;
        if (z >= 0 && z < cz && y >= 0 && y < Lcy && x >= 0 && x < Lcx) {
          s += preds[(((b * cz + z) * Lcy + y) * Lcx + x) * K + c[i].ch];
          ++cnt;
        }
      }
      ((T*)outs.p[k])[((b * e0 + oz) * e1 + oy) * e2 + ox] = (T)(k == center_map(NSP) ? s : s >> (cnt >> 1));
    }
  }
}

// ------------------------------------------------------------------------------------------
// maps_from_predictions: float32 aggregation of [B, cells..., K, C] predictions.
// ------------------------------------------------------------------------------------------
template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) maps_from_predictions_kernel(const T* __restrict__ preds, I B,
                                                                       E3<I> cells, I C, int nsp, MapPtrs outs,
                                                                       I total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  const int K = nsp == 3 ? 19 : 5;
  // frame = cells + 1 per spatial axis
  const I f0 = nsp == 3 ? cells.e[0] + 1 : 1, f1 = cells.e[1] + 1, f2 = cells.e[2] + 1;
  const I Lcz = cells.e[0], Lcy = cells.e[1], Lcx = cells.e[2];
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, f0, f1, f2, C);
    auto get = [&](int64_t z64, int64_t y64, int64_t x64, int ch) -> T {
      const I z = (I)z64, y = (I)y64, x = (I)x64;
      return preds[(((((q.b * Lcz + z) * Lcy + y) * Lcx + x) * K) + ch) * C + q.c];
    };
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      I e[3];
      const I idx[3] = {q.i0, q.i1, q.i2};
      bool ok = true;
      for (int a = 0; a < 3; ++a) {
        e[a] = (a < 3 - nsp) ? 1 : (par[a] ? cells.e[a] : cells.e[a] + 1);
        ok = ok && idx[a] < e[a];
      }
      if (!ok) continue;
      T* o = (T*)outs.p[k];
      o[(((q.b * e[0] + q.i0) * e[1] + q.i1) * e[2] + q.i2) * C + q.c] =
          aggregate_map<T>(nsp, k, (int64_t)q.i0, (int64_t)q.i1, (int64_t)q.i2, (int64_t)Lcz, (int64_t)Lcy, (int64_t)Lcx, get);
    }
  }
}

// LDS-staged form (C == 1, < 2^30 elements).  A workgroup owns YB frame rows x XO frame columns
// of ZC consecutive output planes, for all maps, and rolls along z: cell plane z (rows y0-1 ..
// y0+YB-1, cells ox0-1 .. ox0+XO-1: YB+1 contiguous runs of cells x K channels in HBM) is staged
// into an LDS ring of two planes with 16-byte loads (row pitch rounded to 16 B, so every LDS
// store is aligned), and plane z+1 is fetched into registers while plane z's outputs aggregate
// from LDS.  HBM reads are (YB+1)/YB x (ZC+1)/ZC of the predictions; the per-element kernel
// above reads the channel-interleaved cells with a 19-element lane stride instead (~19 cache
// lines per load instruction).  Arithmetic is the same: integer shifts for u8 / u16, the
// reference's f32 channel-order sum + scale + truncation otherwise.
constexpr int kMfpCpt = 8;  // 16-byte chunks per thread per staged plane (host-checked)

__device__ __forceinline__ void divmod_small(int32_t i, int32_t n, float rcp, int32_t& q, int32_t& r) {
  q = (int32_t)((float)i * rcp);  // i < 2^21: off by at most one
  r = i - q * n;
  if (r < 0) { --q; r += n; } else if (r >= n) { ++q; r -= n; }
}

template <typename T, int NSP>
__global__ void __launch_bounds__(kThreads) maps_from_predictions_lds_kernel(
    const T* __restrict__ preds, int32_t Lcz, int32_t Lcy, int32_t Lcx, MapPtrs outs, int32_t YB, int32_t XO,
    int32_t ZC, int32_t nzc, int32_t nyb, int32_t nxb, int32_t RP, int32_t nchunk, float rcp_nchunk,
    int64_t total_elems) {
  constexpr int NM = NSP == 3 ? 7 : 3, K = NSP == 3 ? 19 : 5;
  constexpr int V = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* lds = (T*)smem;
  int32_t w = (int32_t)blockIdx.x;
  const int32_t xb = w % nxb; w /= nxb;
  const int32_t yb = w % nyb; w /= nyb;
  const int32_t zc = w % nzc;
  const int32_t b = w / nzc;
  const int32_t y0 = yb * YB, ox0 = xb * XO;
  const int32_t xc0 = ox0 > 0 ? ox0 - 1 : 0;
  const int32_t xc1 = (ox0 + XO - 1 < Lcx - 1) ? ox0 + XO - 1 : Lcx - 1;  // last staged cell
  const int32_t nxc_k = (xc1 - xc0 + 1) * K;                                // staged elements per row
  const int32_t cz = NSP == 3 ? Lcz : 1;
  const int32_t fz = NSP == 3 ? Lcz + 1 : 1;
  const int32_t oz0 = zc * ZC, oz1 = (oz0 + ZC < fz) ? oz0 + ZC : fz;  // output planes [oz0, oz1)
  const int32_t slice_work = (YB + 1) * nchunk;

  u32x4v buf[kMfpCpt];
  auto fetch = [&](int32_t z) {  // cell plane z -> registers
#pragma unroll
    for (int c = 0; c < kMfpCpt; ++c) {
      buf[c] = u32x4v{0u, 0u, 0u, 0u};
      const int32_t i = threadIdx.x + c * kThreads;
      if (i >= slice_work) continue;
      int32_t r, ch;
      divmod_small(i, nchunk, rcp_nchunk, r, ch);
      const int32_t y = y0 - 1 + r;
      if (y < 0 || y >= Lcy || ch * V >= nxc_k) continue;
      const int64_t g = ((((int64_t)b * cz + z) * Lcy + y) * Lcx + xc0) * K + (int64_t)ch * V;
      if (g + V <= total_elems) {
        buf[c] = *(const u32x4u*)(preds + g);
      } else {
        T* bt = (T*)&buf[c];
        for (int e = 0; e < V && g + e < total_elems; ++e) bt[e] = preds[g + e];
      }
    }
  };
  auto put = [&](int32_t z) {  // registers -> ring slot z & 1
    T* base = lds + (z & 1) * (YB + 1) * RP;
#pragma unroll
    for (int c = 0; c < kMfpCpt; ++c) {
      const int32_t i = threadIdx.x + c * kThreads;
      if (i >= slice_work) continue;
      int32_t r, ch;
      divmod_small(i, nchunk, rcp_nchunk, r, ch);
      *(u32x4v*)(base + r * RP + ch * V) = buf[c];
    }
  };
  auto at = [&](int32_t z, int32_t r, int32_t x, int ch) -> T {  // cell (z, y0-1+r, x), channel ch
    return lds[((z & 1) * (YB + 1) + r) * RP + (x - xc0) * K + ch];
  };

  // prologue: cell plane oz0 - 1 (3D, when it exists) and oz0
  if (NSP == 3 && oz0 >= 1) {
    fetch(oz0 - 1);
    put(oz0 - 1);
  }
  if (oz0 < cz) {
    fetch(oz0);
    put(oz0);
  }
  __syncthreads();

  for (int32_t oz = oz0; oz < oz1; ++oz) {
    const bool more = oz + 1 < oz1 && oz + 1 < cz;
    if (more) fetch(oz + 1);  // in flight while plane oz aggregates
    for (int32_t i = threadIdx.x; i < YB * XO; i += kThreads) {
      const int32_t xo = i % XO, r = i / XO;
      const int32_t oy = y0 + r, ox = ox0 + xo;
      if (oy > Lcy || ox > Lcx) continue;
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        int par[3];
        map_parity(NSP, k, par);
        const int32_t e0 = NSP == 3 ? (par[0] ? Lcz : Lcz + 1) : 1, e1 = par[1] ? Lcy : Lcy + 1,
                      e2 = par[2] ? Lcx : Lcx + 1;
        if (oz >= e0 || oy >= e1 || ox >= e2) continue;
        Contrib c[4];
        const int nc = map_contribs(NSP, k, c);
        T v;
        if constexpr (sizeof(T) <= 2 && !std::is_same<T, float>::value) {
          uint32_t sum = 0, cnt = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (j >= nc) break;
            const int32_t z = oz - c[j].dz, y = oy - c[j].dy, x = ox - c[j].dx;
            if (z >= 0 && z < cz && y >= 0 && y < Lcy && x >= 0 && x < Lcx) {
              sum += at(z, r + 1 - c[j].dy, x, c[j].ch);
              ++cnt;
            }
          }
          v = (T)(k == center_map(NSP) ? sum : sum >> (cnt >> 1));
        } else if (k == center_map(NSP)) {
          v = at(oz, r + 1, ox, c[0].ch);
        } else {
          float sum = 0.0f;
          int cnt = 0;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (j >= nc) break;
            const int32_t z = oz - c[j].dz, y = oy - c[j].dy, x = ox - c[j].dx;
            if (z >= 0 && z < cz && y >= 0 && y < Lcy && x >= 0 && x < Lcx) {
              sum += (float)at(z, r + 1 - c[j].dy, x, c[j].ch);
              ++cnt;
            }
          }
          if (cnt == 4) sum *= 0.25f;
          else if (cnt == 2) sum *= 0.5f;
          v = cast_f32<T>(sum);
        }
        ((T*)outs.p[k])[((b * e0 + oz) * e1 + oy) * e2 + ox] = v;
      }
    }
    if (!more) break;  // uniform
    __syncthreads();  // plane oz - 1's slot is free
    put(oz + 1);
    __syncthreads();
  }
}

// Fused mean predictor on a padded window (u8 / u16, C == 1): the z-rolling LDS aggregation of
// maps_from_predictions_lds_kernel with the staged cell plane computed on the fly -- cell
// (z, y, x) = astype(T)(f32 sum of its (2p+2)^d window nodes / N), exactly cell_mean_padded --
// so the cell means are written once (as the C map, straight from LDS) and never re-read from
// HBM; the two element kernels below (cell means, then maps) stay for the other layouts.
constexpr int kMpCpt = 4;  // cells per thread per staged plane (host-checked)

template <typename T, int NSP>
__global__ void __launch_bounds__(kThreads) mean_predict_lds_kernel(
    const T* __restrict__ win, E3<int32_t> S, int p, int32_t Lcz, int32_t Lcy, int32_t Lcx, MapPtrs outs, int32_t YB,
    int32_t XO, int32_t ZC, int32_t nzc, int32_t nyb, int32_t nxb, int32_t RP) {
  constexpr int NM = NSP == 3 ? 7 : 3;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* lds = (uint32_t*)smem;  // [2 slots][YB + 1 rows][RP] cell means
  int32_t w = (int32_t)blockIdx.x;
  const int32_t xb = w % nxb; w /= nxb;
  const int32_t yb = w % nyb; w /= nyb;
  const int32_t zc = w % nzc;
  const int32_t b = w / nzc;
  const int32_t y0 = yb * YB, ox0 = xb * XO;
  const int32_t xc0 = ox0 > 0 ? ox0 - 1 : 0;
  const int32_t xc1 = (ox0 + XO - 1 < Lcx - 1) ? ox0 + XO - 1 : Lcx - 1;
  const int32_t ncx = xc1 - xc0 + 1;
  const int32_t cz = NSP == 3 ? Lcz : 1;
  const int32_t fz = NSP == 3 ? Lcz + 1 : 1;
  const int32_t oz0 = zc * ZC, oz1 = (oz0 + ZC < fz) ? oz0 + ZC : fz;
  const int kk = 2 * p + 2, kz = NSP == 3 ? kk : 1;
  const float nn = (float)(kz * kk * kk);
  const int32_t slice = (YB + 1) * ncx;
  const float rcp = 1.0f / (float)ncx;

  uint32_t buf[kMpCpt];
  auto fetch = [&](int32_t z) {  // cell means of cell plane z -> registers
#pragma unroll
    for (int c = 0; c < kMpCpt; ++c) {
      buf[c] = 0;
      const int32_t i = threadIdx.x + c * kThreads;
      if (i >= slice) continue;
      int32_t r, x;
      divmod_small(i, ncx, rcp, r, x);
      const int32_t y = y0 - 1 + r;
      if (y < 0 || y >= Lcy) continue;
      float sum = 0.0f;  // f32 sum in feature order (exact here: < 2^24)
      for (int dz = 0; dz < kz; ++dz)
        for (int dy = 0; dy < kk; ++dy) {
          const T* row = win + ((b * S.e[0] + z + dz) * S.e[1] + y + dy) * S.e[2] + xc0 + x;
          for (int dx = 0; dx < kk; ++dx) sum += (float)row[dx];
        }
      buf[c] = (uint32_t)cast_f32<T>(sum / nn);
    }
  };
  auto put = [&](int32_t z) {
    uint32_t* base = lds + (z & 1) * (YB + 1) * RP;
#pragma unroll
    for (int c = 0; c < kMpCpt; ++c) {
      const int32_t i = threadIdx.x + c * kThreads;
      if (i >= slice) continue;
      int32_t r, x;
      divmod_small(i, ncx, rcp, r, x);
      base[r * RP + x] = buf[c];
    }
  };
  auto at = [&](int32_t z, int32_t r, int32_t x) -> uint32_t { return lds[((z & 1) * (YB + 1) + r) * RP + (x - xc0)]; };

  if (NSP == 3 && oz0 >= 1) {
    fetch(oz0 - 1);
    put(oz0 - 1);
  }
  if (oz0 < cz) {
    fetch(oz0);
    put(oz0);
  }
  __syncthreads();

  for (int32_t oz = oz0; oz < oz1; ++oz) {
    const bool more = oz + 1 < oz1 && oz + 1 < cz;
    if (more) fetch(oz + 1);
    for (int32_t i = threadIdx.x; i < YB * XO; i += kThreads) {
      const int32_t xo = i % XO, r = i / XO;
      const int32_t oy = y0 + r, ox = ox0 + xo;
      if (oy > Lcy || ox > Lcx) continue;
#pragma unroll
      for (int k = 0; k < NM; ++k) {
        int par[3];
        map_parity(NSP, k, par);
        const int32_t e0 = NSP == 3 ? (par[0] ? Lcz : Lcz + 1) : 1, e1 = par[1] ? Lcy : Lcy + 1,
                      e2 = par[2] ? Lcx : Lcx + 1;
        if (oz >= e0 || oy >= e1 || ox >= e2) continue;
        Contrib cb[4];
        const int nc = map_contribs(NSP, k, cb);
        uint32_t sum = 0, cnt = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (j >= nc) break;
          const int32_t z = oz - cb[j].dz, y = oy - cb[j].dy, x = ox - cb[j].dx;
          if (z >= 0 && z < cz && y >= 0 && y < Lcy && x >= 0 && x < Lcx) {
            sum += at(z, r + 1 - cb[j].dy, x);
            ++cnt;
          }
        }
        ((T*)outs.p[k])[((b * e0 + oz) * e1 + oy) * e2 + ox] = (T)(k == center_map(NSP) ? sum : sum >> (cnt >> 1));
      }
    }
    if (!more) break;  // uniform
    __syncthreads();
    put(oz + 1);
    __syncthreads();
  }
}

// Words of padding before and after the two LDS cell planes of the mean predictor kernels.
__host__ __device__ __forceinline__ int32_t mp_pad_words(int64_t Lcx) { return (int32_t)(4 * ((Lcx + 4) / 4)); }

// Row mapping of a plane's positions onto the workgroup: a wave covers R = 64 / W rows of W
// consecutive x positions (lane = r * W + x), the 4 waves interleave row groups.  Every lane's
// (row, x) is fixed per call, so the per-position work has no index division, and the
// conditions that depend on the row (first / last row) change only between row groups.
struct RowMap {
  int32_t lr, lx, R;  // this lane's row within the group, its x, rows per wave
  bool lane_ok;
};
__device__ __forceinline__ RowMap row_map(int32_t W) {
  RowMap m;
  const int32_t lane = threadIdx.x & 63;
  m.R = 64 / W;
  m.lr = (int32_t)((float)lane * (1.0f / (float)W));  // lane < 64: exact after the fix-up
  if (m.lr * W > lane) --m.lr;
  else if ((m.lr + 1) * W <= lane) ++m.lr;
  m.lx = lane - m.lr * W;
  m.lane_ok = m.lr < m.R;
  return m;
}

// The 7 maps at the output positions of plane oz from two LDS cell planes (cell plane oz in slot
// s_cur, oz - 1 in s_prev; ``cells`` must have Lcx + 1 readable words before slot 0 and after
// slot 1).  Positions
// ox < Lcx go through the row mapping in x chunks of <= 64; the last column (ox == Lcx, where
// only the three maps with an even x parity exist and only the cells at ox - 1 contribute) is a
// separate pass with one lane per row.
template <typename T, typename O>
__device__ __forceinline__ void mean_maps_plane(const uint32_t* cells, int32_t oz, int64_t b, int32_t Lcz,
                                                int32_t Lcy, int32_t Lcx, const MapPtrs& outs, int s_cur, int s_prev) {
  const int32_t nplanes = Lcz + 1, oyn = Lcy + 1, oxn = Lcx + 1, cplane = Lcy * Lcx;
  const bool z0 = oz < Lcz, z1 = oz >= 1;  // cell planes oz and oz - 1 exist
  O* const o0 = (O*)outs.p[0] + ((b * Lcz + oz) * Lcy) * oxn;       // LR (1,1,0)
  O* const o1 = (O*)outs.p[1] + ((b * Lcz + oz) * oyn) * Lcx;       // UD (1,0,1)
  O* const o2 = (O*)outs.p[2] + ((b * nplanes + oz) * Lcy) * Lcx;   // FB (0,1,1)
  O* const o3 = (O*)outs.p[3] + ((b * Lcz + oz) * Lcy) * Lcx;       // C  (1,1,1)
  O* const o4 = (O*)outs.p[4] + ((b * Lcz + oz) * oyn) * oxn;       // Z  (1,0,0)
  O* const o5 = (O*)outs.p[5] + ((b * nplanes + oz) * Lcy) * oxn;   // Y  (0,1,0)
  O* const o6 = (O*)outs.p[6] + ((b * nplanes + oz) * oyn) * Lcx;   // X  (0,0,1)
  const uint32_t* cur = cells + s_cur * cplane;
  const uint32_t* prev = cells + s_prev * cplane;
  const uint32_t nz = (uint32_t)z0 + z1;
  const int32_t wv = threadIdx.x >> 6;
  for (int32_t xc = 0; xc < Lcx; xc += 64) {
    const RowMap m = row_map(Lcx - xc < 64 ? Lcx - xc : 64);
    const int32_t ox = xc + m.lx;
    const bool x1 = ox >= 1;
    for (int32_t oy0 = wv * m.R; oy0 <= Lcy; oy0 += 4 * m.R) {
      const int32_t oy = oy0 + m.lr;
      if (!m.lane_ok || oy > Lcy) continue;
      const bool y0 = oy < Lcy, y1 = oy >= 1;
      const int32_t q = oy * Lcx + ox;  // cell (oy, ox)
      // c<z><y><x>: cell (oz - z, oy - y, ox - x); 0 where it does not exist.  The reads are
      // unconditional (the cell slots carry Lcx + 1 words of padding on both sides, so every
      // index here stays inside the workgroup's LDS) and masked afterwards: no exec-mask
      // branch per read.
      const uint32_t mz0 = z0 ? ~0u : 0u, mz1 = z1 ? ~0u : 0u;
      const uint32_t my0 = y0 ? ~0u : 0u, my1 = y1 ? ~0u : 0u, mx1 = x1 ? ~0u : 0u;
      const uint32_t c000 = cur[q] & (mz0 & my0), c001 = cur[q - 1] & (mz0 & my0 & mx1);
      const uint32_t c010 = cur[q - Lcx] & (mz0 & my1), c011 = cur[q - Lcx - 1] & (mz0 & my1 & mx1);
      const uint32_t c100 = prev[q] & (mz1 & my0), c101 = prev[q - 1] & (mz1 & my0 & mx1);
      const uint32_t c110 = prev[q - Lcx] & (mz1 & my1);
      const uint32_t nx = 1u + x1, ny = (uint32_t)y0 + y1;
      const int32_t px = oy * oxn + ox, pc = oy * Lcx + ox;
      o6[pc] = (O)((c000 + c010 + c110 + c100) >> ((nz * ny) >> 1));
      if (z0) {
        o1[pc] = (O)((c000 + c010) >> (ny >> 1));
        o4[px] = (O)((c000 + c001 + c011 + c010) >> ((ny * nx) >> 1));
      }
      if (y0) {
        o2[pc] = (O)((c000 + c100) >> (nz >> 1));
        o5[px] = (O)((c000 + c001 + c101 + c100) >> ((nz * nx) >> 1));
        if (z0) {
          o0[px] = (O)((c000 + c001) >> (nx >> 1));
          o3[pc] = (O)c000;
        }
      }
    }
  }
  // the last column, ox = Lcx: LR, Z, Y from the cells at x = Lcx - 1
  for (int32_t oy = threadIdx.x; oy <= Lcy; oy += kThreads) {
    const bool y0 = oy < Lcy, y1 = oy >= 1;
    const int32_t q = oy * Lcx + Lcx - 1;
    const uint32_t c001 = cur[q] & (z0 && y0 ? ~0u : 0u), c011 = cur[q - Lcx] & (z0 && y1 ? ~0u : 0u);
    const uint32_t c101 = prev[q] & (z1 && y0 ? ~0u : 0u);
    const uint32_t ny = (uint32_t)y0 + y1;
    const int32_t px = oy * oxn + Lcx;
    if (z0) o4[px] = (O)((c001 + c011) >> (ny >> 1));
    if (y0) {
      o5[px] = (O)((c001 + c101) >> (nz >> 1));
      if (z0) o0[px] = (O)c001;
    }
  }
}

// Fused mean predictor, one workgroup per output plane (3D, u8 / u16, C == 1, p <= 2).  The
// 2p+3 window planes that output plane oz reads are copied into LDS as one contiguous byte range
// with 16-byte loads; the two cell planes it aggregates (oz - 1 and oz) are summed there --
// directly for p = 0 (8 nodes), separably for p >= 1 (x sums of 2p+2 nodes first, then the
// (2p+2)^2 box of x sums) -- and each thread then owns output positions (oy, ox) and writes all 7
// maps at that position from the 8 cells around it.  The rolling kernel above fetches every
// node of every cell with its own 2-byte global load; that was its cost (131 -> 93 us for the
// 512 C3 windows).  A z-rolling variant of this kernel (3-slot node ring, next plane prefetched
// in registers, each cell plane summed once) measured slower, 100-108 us: the plane-parallel grid
// hides the load latency as well and has 8x the workgroups.
// PPB output planes per workgroup (1 or 2): with 2, the cell plane between them is summed once
// for both (3 cell planes for 2 outputs instead of 4) -- the kernel is VALU-bound
// (profiles/round2/sq_callback_kernels.txt)
template <typename T, int P, int PPB, typename O = T>
__global__ void __launch_bounds__(kThreads) mean_predict_plane_kernel(
    const T* __restrict__ win, E3<int32_t> S, int32_t Lcz, int32_t Lcy, int32_t Lcx, MapPtrs outs, int32_t xcd_per,
    int32_t nodes_bytes, int32_t xs_bytes) {
  static_assert(PPB == 1 || PPB == 2, "one or two output planes per workgroup");
  constexpr int KK = 2 * P + 2;
  constexpr float NN = (float)(KK * KK * KK);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int32_t nplanes = Lcz + 1, ngrp = (nplanes + PPB - 1) / PPB;
  int32_t blk = (int32_t)blockIdx.x;
  if (xcd_per > 0) {  // consecutive planes of one window on one XCD: shared node planes hit its L2
    const int32_t x = blk % 8, k = blk / 8;
    blk = ((k / xcd_per) * 8 + x) * xcd_per + (k % xcd_per);
  }
  const int32_t oz = (blk % ngrp) * PPB;  // the first output plane; cell slot s is plane oz - 1 + s
  const int64_t b = blk / ngrp;
  const int32_t S1 = S.e[1], S2 = S.e[2], plane = S1 * S2;
  const int32_t zlo = oz >= 1 ? oz - 1 : 0;
  const int32_t zhi = oz + PPB - 1 + KK < S.e[0] ? oz + PPB - 1 + KK : S.e[0];  // node planes [zlo, zhi)

  // ---- node planes -> LDS: the aligned 16-byte blocks covering the byte range; the partial
  // blocks at either end copy only the window's own bytes ----
  const unsigned char* g0 = (const unsigned char*)(win + (b * S.e[0] + zlo) * (int64_t)plane);
  const int32_t shift = (int32_t)((uintptr_t)g0 & 15);
  const int32_t nbytes = (zhi - zlo) * plane * (int32_t)sizeof(T);
  const uint4* src = (const uint4*)(g0 - shift);
  const int32_t nchunk = (nbytes + shift + 15) >> 4;
  for (int32_t i = threadIdx.x; i < nchunk; i += kThreads) {
    const int32_t lo = 16 * i - shift;  // byte range [lo, lo + 16) of the window planes
    if (lo >= 0 && lo + 16 <= nbytes) {
      *(uint4*)(smem + 16 * i) = src[i];
    } else {  // the partial first / last block: only its bytes inside the window, element by element
      for (int32_t k = lo < 0 ? 0 : lo; k < lo + 16 && k < nbytes; k += (int32_t)sizeof(T))
        *(T*)(smem + shift + k) = *(const T*)(g0 + k);
    }
  }
  const T* nodes = (const T*)(smem + shift);  // [z - zlo][y][x]
  uint32_t* xs = (uint32_t*)(smem + nodes_bytes);  // p >= 1: [z - zlo][y][cx] sums over x
  // [slot: z = oz - 1 + slot][cy][cx], PPB + 1 slots, after a pad of >= Lcx + 1 words
  uint32_t* cells = (uint32_t*)(smem + nodes_bytes + xs_bytes) + mp_pad_words(Lcx);
  __syncthreads();

  const int32_t cplane = Lcy * Lcx;
  const float rcx = 1.0f / (float)Lcx;
  if constexpr (P > 0) {
    const int32_t nxs = (zhi - zlo) * S1 * Lcx;
    for (int32_t i = threadIdx.x; i < nxs; i += kThreads) {
      int32_t zy, cx;
      divmod_small(i, Lcx, rcx, zy, cx);
      const T* row = nodes + zy * S2 + cx;  // (z - zlo) * plane + y * S2 == zy * S2
      uint32_t s = 0;
#pragma unroll
      for (int dx = 0; dx < KK; ++dx) s += row[dx];
      xs[i] = s;
    }
    __syncthreads();
  }
  // cell planes oz - 1 .. oz + PPB - 1 (slots 0 .. PPB), rows of all through the row mapping
  const int32_t wv = threadIdx.x >> 6;
  for (int32_t xc = 0; xc < Lcx; xc += 64) {
    const RowMap m = row_map(Lcx - xc < 64 ? Lcx - xc : 64);
    const int32_t cx = xc + m.lx;
    for (int32_t r0 = wv * m.R; r0 < (PPB + 1) * Lcy; r0 += 4 * m.R) {
      const int32_t r = r0 + m.lr;
      const int32_t slot = PPB == 1 ? (int32_t)(r >= Lcy) : (int32_t)(r >= Lcy) + (int32_t)(r >= 2 * Lcy);
      const int32_t cy = r - slot * Lcy;
      const int32_t z = oz - 1 + slot;
      if (!m.lane_ok || r >= (PPB + 1) * Lcy || z < 0 || z >= Lcz) continue;  // (a missing plane is never read)
      uint32_t s = 0;
      if constexpr (P == 0) {
        const T* q = nodes + (z - zlo) * plane + cy * S2 + cx;
        s = (uint32_t)q[0] + q[1] + q[S2] + q[S2 + 1] + q[plane] + q[plane + 1] + q[plane + S2] + q[plane + S2 + 1];
      } else {
#pragma unroll
        for (int dz = 0; dz < KK; ++dz)
#pragma unroll
          for (int dy = 0; dy < KK; ++dy) s += xs[((z - zlo + dz) * S1 + cy + dy) * Lcx + cx];
      }
      cells[slot * cplane + cy * Lcx + cx] = (uint32_t)cast_f32<T>((float)s / NN);  // exact sum (< 2^24)
    }
  }
  __syncthreads();

  mean_maps_plane<T, O>(cells, oz, b, Lcz, Lcy, Lcx, outs, 1, 0);
  if (PPB == 2 && oz + 1 < nplanes) mean_maps_plane<T, O>(cells, oz + 1, b, Lcz, Lcy, Lcx, outs, 2, 1);
}

// ---- p = 0, eight x positions per lane (3D, C == 1, Lcx % 8 == 0) ----
// The same maps as mean_predict_plane_kernel<T, 0, *> with the per-position work cut to adds and
// shifts: the LDS cell planes carry a zero border (row -1 / Lcy, column -1, whole planes -1 /
// Lcz), so a cell that does not exist reads 0 and no read is masked, and each map is a sum of the
// existing cells shifted by log2 of their count (the per-axis flags sz, sy, sx below).  A lane
// owns 8 consecutive x of one row: 2 x 16-byte node-row loads per cell row, 2 ds_read_b128 + 1
// ds_read_b32 per cell row read, one 8-element store per map.  A workgroup computes ZP output
// planes from ZP + 1 cell planes (cell plane oz - 1 is summed by two workgroups).

typedef uint32_t u32x2u __attribute__((ext_vector_type(2), aligned(1)));

// nodes p[0 .. 8] of a window row (unaligned: rows of odd length)
template <typename T>
__device__ __forceinline__ void load_row9(const T* p, uint32_t (&n)[9]) {
  if constexpr (sizeof(T) == 2) {
    const u32x4u v = *(const u32x4u*)p;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      n[2 * k] = v[k] & 0xFFFFu;
      n[2 * k + 1] = v[k] >> 16;
    }
  } else {
    const u32x2u v = *(const u32x2u*)p;
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < 4; ++i) n[4 * k + i] = (v[k] >> (8 * i)) & 0xFFu;
  }
  n[8] = p[8];
}

// 8 map values (each < 2^(8 sizeof(T))) as O at p (element-aligned)
template <typename O>
__device__ __forceinline__ void store_row8(O* p, const uint32_t (&v)[8]) {
  if constexpr (std::is_same<O, float>::value) {
    u32x4u a, b;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a[k] = __float_as_uint((float)v[k]);
      b[k] = __float_as_uint((float)v[4 + k]);
    }
    *(u32x4u*)p = a;
    *(u32x4u*)(p + 4) = b;
  } else if constexpr (sizeof(O) == 2) {
    u32x4u a;
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = v[2 * k] | (v[2 * k + 1] << 16);
    *(u32x4u*)p = a;
  } else {
    u32x2u a;
#pragma unroll
    for (int k = 0; k < 2; ++k) a[k] = v[4 * k] | (v[4 * k + 1] << 8) | (v[4 * k + 2] << 16) | (v[4 * k + 3] << 24);
    *(u32x2u*)p = a;
  }
}

// words of one LDS cell plane: rows -1 .. Lcy, pitch Lcx + 8 (cell x at word x + 4: 16-byte aligned)
__host__ __device__ __forceinline__ int32_t mp8_plane_words(int32_t Lcy, int32_t Lcx) { return (Lcy + 2) * (Lcx + 8); }

template <typename T, typename O>
__global__ void __launch_bounds__(kThreads) mean_predict_p0x8_kernel(const T* __restrict__ win, E3<int32_t> S,
                                                                    int32_t Lcz, int32_t Lcy, int32_t Lcx, MapPtrs outs,
                                                                    int32_t xcd_per, int32_t ZP, int32_t ngrp) {
  extern __shared__ __attribute__((aligned(16))) uint32_t cl[];  // [ZP + 1][Lcy + 2][Lcx + 8]
  int32_t blk = (int32_t)blockIdx.x;
  if (xcd_per > 0) {  // the groups of one window on one XCD (their shared node planes hit its L2)
    const int32_t x = blk % 8, k = blk / 8;
    blk = ((k / xcd_per) * 8 + x) * xcd_per + (k % xcd_per);
  }
  const int32_t b = blk / ngrp, z0 = (blk - b * ngrp) * ZP;  // output planes z0 .. z0 + ZP - 1
  const int32_t RP = Lcx + 8, PW = mp8_plane_words(Lcy, Lcx), NJ = Lcx >> 3;
  const int32_t S1 = S.e[1], S2 = S.e[2];

  // zero border (and the planes outside the window's cells)
  for (int32_t i = threadIdx.x; i < (ZP + 1) * PW / 4; i += kThreads) ((uint4*)cl)[i] = make_uint4(0, 0, 0, 0);
  __syncthreads();

  // cell planes zc = z0 - 1 + s: 8 cells per lane = (8 nodes) >> 3, summed over 4 node rows
  const float rnj = 1.0f / (float)NJ, rlcy = 1.0f / (float)Lcy;
  for (int32_t t = threadIdx.x; t < (ZP + 1) * Lcy * NJ; t += kThreads) {
    int32_t sy, j, s, cy;
    divmod_small(t, NJ, rnj, sy, j);
    divmod_small(sy, Lcy, rlcy, s, cy);
    const int32_t zc = z0 - 1 + s;
    if (zc < 0 || zc >= Lcz) continue;
    uint32_t acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int dz = 0; dz < 2; ++dz)
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        uint32_t n[9];
        load_row9<T>(win + (((int64_t)b * S.e[0] + zc + dz) * S1 + cy + dy) * S2 + 8 * j, n);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += n[i] + n[i + 1];
      }
    uint32_t* dst = cl + s * PW + (cy + 1) * RP + 4 + 8 * j;
    *(uint4*)dst = make_uint4(acc[0] >> 3, acc[1] >> 3, acc[2] >> 3, acc[3] >> 3);
    *(uint4*)(dst + 4) = make_uint4(acc[4] >> 3, acc[5] >> 3, acc[6] >> 3, acc[7] >> 3);
  }
  __syncthreads();

  const int32_t nz = Lcz + 1 - z0 < ZP ? Lcz + 1 - z0 : ZP;  // output planes of this group
  const int32_t oyn = Lcy + 1, oxn = Lcx + 1;
  const float roy = 1.0f / (float)oyn;
  // cells x = 8j - 1 .. 8j + 7 of one LDS row
  auto row9 = [&](const uint32_t* r, int32_t j, uint32_t (&v)[9]) {
    v[0] = r[3 + 8 * j];
    const uint4 a = *(const uint4*)(r + 4 + 8 * j), c = *(const uint4*)(r + 8 + 8 * j);
    v[1] = a.x; v[2] = a.y; v[3] = a.z; v[4] = a.w;
    v[5] = c.x; v[6] = c.y; v[7] = c.z; v[8] = c.w;
  };
  for (int32_t t = threadIdx.x; t < nz * oyn * NJ; t += kThreads) {
    int32_t py, j, pz, oy;
    divmod_small(t, NJ, rnj, py, j);
    divmod_small(py, oyn, roy, pz, oy);
    const int32_t oz = z0 + pz, ox = 8 * j;
    const bool z0f = oz < Lcz, y0f = oy < Lcy;
    const uint32_t sz = (uint32_t)(z0f && oz >= 1), sy = (uint32_t)(y0f && oy >= 1);
    const uint32_t* cur = cl + (pz + 1) * PW;  // cell plane oz
    const uint32_t* prv = cl + pz * PW;        // cell plane oz - 1
    uint32_t a[9], bb[9], c[9], d[9];          // cur row oy, cur row oy - 1, prev row oy, prev row oy - 1
    row9(cur + (oy + 1) * RP, j, a);
    row9(cur + oy * RP, j, bb);
    row9(prv + (oy + 1) * RP, j, c);
    row9(prv + oy * RP, j, d);
    uint32_t m0[8], m1[8], m2[8], m3[8], m4[8], m5[8], m6[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t sx = i > 0 ? 1u : (uint32_t)(ox >= 1);
      const uint32_t lr = a[i + 1] + a[i];
      m0[i] = lr >> sx;                                          // LR (1,1,0)
      m1[i] = (a[i + 1] + bb[i + 1]) >> sy;                      // UD (1,0,1)
      m2[i] = (a[i + 1] + c[i + 1]) >> sz;                       // FB (0,1,1)
      m3[i] = a[i + 1];                                          // C  (1,1,1)
      m4[i] = (lr + bb[i] + bb[i + 1]) >> (sy + sx);             // Z  (1,0,0)
      m5[i] = (lr + c[i] + c[i + 1]) >> (sz + sx);               // Y  (0,1,0)
      m6[i] = (a[i + 1] + bb[i + 1] + c[i + 1] + d[i + 1]) >> (sz + sy);  // X (0,0,1)
    }
    const int32_t zL = b * Lcz + oz, zN = b * (Lcz + 1) + oz;  // plane index in a map of Lcz / Lcz + 1 planes
    store_row8<O>((O*)outs.p[6] + (zN * oyn + oy) * Lcx + ox, m6);
    if (z0f) {
      store_row8<O>((O*)outs.p[1] + (zL * oyn + oy) * Lcx + ox, m1);
      store_row8<O>((O*)outs.p[4] + (zL * oyn + oy) * oxn + ox, m4);
    }
    if (y0f) {
      store_row8<O>((O*)outs.p[2] + (zN * Lcy + oy) * Lcx + ox, m2);
      store_row8<O>((O*)outs.p[5] + (zN * Lcy + oy) * oxn + ox, m5);
      if (z0f) {
        store_row8<O>((O*)outs.p[0] + (zL * Lcy + oy) * oxn + ox, m0);
        store_row8<O>((O*)outs.p[3] + (zL * Lcy + oy) * Lcx + ox, m3);
      }
    }
  }
  // the last column, ox = Lcx: LR, Z, Y from the cells at x = Lcx - 1
  for (int32_t t = threadIdx.x; t < nz * oyn; t += kThreads) {
    int32_t pz, oy;
    divmod_small(t, oyn, roy, pz, oy);
    const int32_t oz = z0 + pz;
    const bool z0f = oz < Lcz, y0f = oy < Lcy;
    const uint32_t sz = (uint32_t)(z0f && oz >= 1), sy = (uint32_t)(y0f && oy >= 1);
    const uint32_t* cur = cl + (pz + 1) * PW + 3 + Lcx;  // x = Lcx - 1
    const uint32_t* prv = cl + pz * PW + 3 + Lcx;
    const uint32_t c001 = cur[(oy + 1) * RP], c011 = cur[oy * RP], c101 = prv[(oy + 1) * RP];
    const int32_t zL = b * Lcz + oz, zN = b * (Lcz + 1) + oz;
    if (z0f) ((O*)outs.p[4])[(zL * oyn + oy) * oxn + Lcx] = (O)((c001 + c011) >> sy);
    if (y0f) {
      ((O*)outs.p[5])[(zN * Lcy + oy) * oxn + Lcx] = (O)((c001 + c101) >> sz);
      if (z0f) ((O*)outs.p[0])[(zL * Lcy + oy) * oxn + Lcx] = (O)c001;
    }
  }
}

// ------------------------------------------------------------------------------------------
// Mean predictor on a padded lowres window (tests/volume/test_encode_decode.py:46-53):
// cell mean = astype(T)(f32 sum of the (2p+2)^d neighbourhood / N), then the map aggregation.
// ------------------------------------------------------------------------------------------
template <typename T, typename I>
__device__ __forceinline__ T cell_mean_padded(const T* __restrict__ in, I b, I cz, I cy, I cx,
                                              I c, E3<I> S, I C, int nsp, int p) {
  const int k = 2 * p + 2;
  const int kz = nsp == 3 ? k : 1;
  float s = 0.0f;
  for (int dz = 0; dz < kz; ++dz)
    for (int dy = 0; dy < k; ++dy)
      for (int dx = 0; dx < k; ++dx)
        s += (float)in[(((b * S.e[0] + cz + dz) * S.e[1] + cy + dy) * S.e[2] + cx + dx) * C + c];
  return cast_f32<T>(s / (float)(kz * k * k));
}

// Two passes: (1) the per-cell means ARE the C map (volume/utils.py:117: channel 6 unscaled; 2D
// channel 4), so they are written there once; (2) every other map aggregates up to 4 of them
// (the f32 scatter-add / scale / truncate of volume/utils.py:83-155, kmp_aggregate.h).
template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) cell_mean_map_kernel(const T* __restrict__ in, I B, E3<I> S,
                                                               I C, int nsp, int p, E3<I> cells,
                                                               T* __restrict__ out, I total) {
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, cells.e[0], cells.e[1], cells.e[2], C);
    out[t] = cell_mean_padded<T, I>(in, q.b, q.i0, q.i1, q.i2, q.c, S, C, nsp, p);
  }
}

// u8 / u16, C == 1, 32-bit indices: the f32 sum of at most 4 cell means is exact there, so the
// scale-and-truncate is an integer shift (the same values as aggregate_map).
template <typename T, int NSP>
__global__ void __launch_bounds__(kThreads) maps_from_cell_means_int_kernel(const T* __restrict__ cm, int32_t Lcz,
                                                                          int32_t Lcy, int32_t Lcx, MapPtrs outs,
                                                                          int32_t total) {
  constexpr int NM = NSP == 3 ? 7 : 3;
  const int32_t f0 = NSP == 3 ? Lcz + 1 : 1, f1 = Lcy + 1, f2 = Lcx + 1;
  for (int32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    uint32_t q = (uint32_t)t;
    const int32_t ox = q % (uint32_t)f2; q /= (uint32_t)f2;
    const int32_t oy = q % (uint32_t)f1; q /= (uint32_t)f1;
    const int32_t oz = q % (uint32_t)f0;
    const int32_t b = q / (uint32_t)f0;
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      if (k == center_map(NSP)) continue;
      int par[3];
      map_parity(NSP, k, par);
      const int32_t e0 = NSP == 3 ? (par[0] ? Lcz : Lcz + 1) : 1, e1 = par[1] ? Lcy : Lcy + 1, e2 = par[2] ? Lcx : Lcx + 1;
      if (oz >= e0 || oy >= e1 || ox >= e2) continue;
      Contrib c[4];
      const int nc = map_contribs(NSP, k, c);
      uint32_t s = 0, cnt = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i >= nc) break;
        const int32_t z = oz - c[i].dz, y = oy - c[i].dy, x = ox - c[i].dx;
        if (z >= 0 && z < (NSP == 3 ? Lcz : 1) && y >= 0 && y < Lcy && x >= 0 && x < Lcx) {
          s += cm[((b * (NSP == 3 ? Lcz : 1) + z) * Lcy + y) * Lcx + x];
          ++cnt;
        }
      }
      ((T*)outs.p[k])[((b * e0 + oz) * e1 + oy) * e2 + ox] = (T)(s >> (cnt >> 1));
    }
  }
}

template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) maps_from_cell_means_kernel(const T* __restrict__ cm, I B,
                                                                      E3<I> cells, I C, int nsp, MapPtrs outs,
                                                                      I total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  const I Lcz = cells.e[0], Lcy = cells.e[1], Lcx = cells.e[2];
  const I f0 = nsp == 3 ? Lcz + 1 : 1, f1 = Lcy + 1, f2 = Lcx + 1;
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, f0, f1, f2, C);
    auto get = [&](int64_t z64, int64_t y64, int64_t x64, int) -> T {
      const I z = (I)z64, y = (I)y64, x = (I)x64;
      return cm[(((q.b * Lcz + z) * Lcy + y) * Lcx + x) * C + q.c];
    };
    for (int k = 0; k < nmaps; ++k) {
      if (k == center_map(nsp)) continue;
      int par[3];
      map_parity(nsp, k, par);
      I e[3];
      const I idx[3] = {q.i0, q.i1, q.i2};
      bool ok = true;
      for (int a = 0; a < 3; ++a) {
        e[a] = (a < 3 - nsp) ? 1 : (par[a] ? cells.e[a] : cells.e[a] + 1);
        ok = ok && idx[a] < e[a];
      }
      if (!ok) continue;
      T* o = (T*)outs.p[k];
      o[(((q.b * e[0] + q.i0) * e[1] + q.i1) * e[2] + q.i2) * C + q.c] =
          aggregate_map<T>(nsp, k, (int64_t)q.i0, (int64_t)q.i1, (int64_t)q.i2, (int64_t)Lcz, (int64_t)Lcy, (int64_t)Lcx, get);
    }
  }
}

// ------------------------------------------------------------------------------------------
// jnp.pad on the spatial axes ('symmetric' / 'reflect'); negative pads crop.
// ------------------------------------------------------------------------------------------
template <typename I>
__device__ __forceinline__ I reflect_index(I i, I n) {
  if (n == 1) return 0;
  const I per = 2 * (n - 1);
  I m = i % per;
  if (m < 0) m += per;
  return m < n ? m : per - m;
}

template <typename T, typename I>
__global__ void __launch_bounds__(kThreads) pad_kernel(const T* __restrict__ in, I B, E3<I> n, I C,
                                                     E3<I> lo, E3<I> out_e, int mode, T* __restrict__ out,
                                                     I total) {
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, out_e.e[0], out_e.e[1], out_e.e[2], C);
    const I o[3] = {q.i0, q.i1, q.i2};
    I s[3];
    for (int a = 0; a < 3; ++a) {
      const I i = o[a] - lo.e[a];
      s[a] = (i >= 0 && i < n.e[a]) ? i : (mode == 0 ? sym_idx<I>(i, n.e[a]) : reflect_index<I>(i, n.e[a]));
    }
    out[t] = in[(((q.b * n.e[0] + s[0]) * n.e[1] + s[1]) * n.e[2] + s[2]) * C + q.c];
  }
}

// ------------------------------------------------------------------------------------------
// Coders (utils.py:28-55), one element per thread.
// ------------------------------------------------------------------------------------------
// 16-byte vector form for operands and result of one element size (the common case: the coder
// of the sample dtype on same-dtype predictions), 16-byte aligned; ``n16`` vectors.
template <int DIR, int CODER, typename TV>
__global__ void __launch_bounds__(kThreads) code_vec_kernel(const u32x4v* __restrict__ pred,
                                                          const u32x4v* __restrict__ x, int64_t n16,
                                                          u32x4v* __restrict__ out) {
  using TO = typename coder_out<CODER>::type;
  constexpr int V = 16 / sizeof(TV);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n16; t += (int64_t)gridDim.x * blockDim.x) {
    const u32x4v pv = __builtin_nontemporal_load(pred + t), xv = __builtin_nontemporal_load(x + t);
    const TV* pp = (const TV*)&pv;
    const TV* xx = (const TV*)&xv;
    u32x4v ov;
    TO* oo = (TO*)&ov;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int32_t p = to_i32(pp[i]), v = to_i32(xx[i]);
      oo[i] = DIR == KMP_ENCODE ? code_encode<CODER>(p, v) : code_decode<CODER>(p, v);
    }
    __builtin_nontemporal_store(ov, out + t);
  }
}

template <int DIR, int CODER, typename TP, typename TX, typename I>
__global__ void __launch_bounds__(kThreads) code_kernel(const TP* __restrict__ pred, const TX* __restrict__ x, I n,
                                                      typename coder_out<CODER>::type* __restrict__ out) {
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < n; t += (I)gridDim.x * blockDim.x) {
    const int32_t p = to_i32(pred[t]);
    const int32_t v = to_i32(x[t]);
    out[t] = DIR == KMP_ENCODE ? code_encode<CODER>(p, v) : code_decode<CODER>(p, v);
  }
}

// ------------------------------------------------------------------------------------------
// Box copy with conversion (slicing / .at[box].set of the chunk driver)
// ------------------------------------------------------------------------------------------
template <typename TO, typename TI>
__device__ __forceinline__ TO convert(TI v) {
  if constexpr (std::is_same<TI, float>::value && !std::is_same<TO, float>::value) return cast_f32<TO>(v);
  else return (TO)v;
}

template <typename TI, typename TO, typename I>
__global__ void __launch_bounds__(kThreads) copy_box_kernel(const TI* __restrict__ in, E3<I> in_e, E3<I> in_off,
                                                          TO* __restrict__ out, E3<I> out_e, E3<I> out_off, E3<I> ext,
                                                          I C, I total) {
  for (I t = blockIdx.x * (I)blockDim.x + threadIdx.x; t < total; t += (I)gridDim.x * blockDim.x) {
    IdxT<I> q = unflat_t<I>(t, ext.e[0], ext.e[1], ext.e[2], C);
    const I si = (((q.b * in_e.e[0] + in_off.e[0] + q.i0) * in_e.e[1] + in_off.e[1] + q.i1) * in_e.e[2] +
                        in_off.e[2] + q.i2) * C + q.c;
    const I so = (((q.b * out_e.e[0] + out_off.e[0] + q.i0) * out_e.e[1] + out_off.e[1] + q.i1) * out_e.e[2] +
                        out_off.e[2] + q.i2) * C + q.c;
    out[so] = convert<TO>(in[si]);
  }
}

// ------------------------------------------------------------------------------------------
// Row kernels (C == 1, < 2^31 elements): one work item = V = 16 / sizeof(T) consecutive outputs
// of one row.  The row decomposition (3 divisions) is paid once per 16 bytes instead of once per
// element, and interior chunks move as one 16-byte load / store per lane.  Rows of these arrays
// have odd lengths (65, 33, ...), so row starts are only element-aligned: the vectors are
// declared byte-aligned and gfx950 serves them as unaligned dwordx4 accesses.  Partial chunks
// and mirrored edges fall back to per-element accesses inside the same item.
// ------------------------------------------------------------------------------------------
// jnp.pad rows: out[b, z, y, x] = in[b, m(z - lz), m(y - ly), m(x - lx)]
template <typename T>
__global__ void __launch_bounds__(kThreads) rows_pad_kernel(const T* __restrict__ in, E3<int32_t> n, E3<int32_t> lo,
                                                          E3<int32_t> oe, int mode, T* __restrict__ out, int32_t nch,
                                                          int32_t items) {
  constexpr int V = Vec16<T>::V;
  auto m = [&](int32_t i, int32_t ext) { return (i >= 0 && i < ext) ? i : (mode == 0 ? sym_idx<int32_t>(i, ext)
                                                                                      : reflect_index<int32_t>(i, ext)); };
  for (int32_t t = blockIdx.x * kThreads + threadIdx.x; t < items; t += gridDim.x * kThreads) {
    const RowItem q = row_item((uint32_t)t, oe.e[0], oe.e[1], nch);
    const int32_t sz = m(q.z - lo.e[0], n.e[0]), sy = m(q.y - lo.e[1], n.e[1]);
    const T* src = in + ((q.b * n.e[0] + sz) * n.e[1] + sy) * n.e[2];
    T* dst = out + ((q.b * oe.e[0] + q.z) * oe.e[1] + q.y) * oe.e[2];
    const int32_t x0 = q.j * V, s0 = x0 - lo.e[2];
    if (x0 + V <= oe.e[2] && s0 >= 0 && s0 + V <= n.e[2]) {
      Vec16<T> v;
      v.load(src + s0);
      v.store(dst + x0);
    } else {
      for (int32_t x = x0; x < x0 + V && x < oe.e[2]; ++x) dst[x] = src[m(x - lo.e[2], n.e[2])];
    }
  }
}

// Parity split of highres rows (lowres_from_highres / maps_from_highres): item = (b, hz, hy)
// highres row (every ``step``-th when only the lowres is wanted), chunk j = highres x in
// [2jV, 2jV + 2V): even x -> class (pz, py, 0), odd x -> class (pz, py, 1).
template <typename T>
__global__ void __launch_bounds__(kThreads) rows_deinterleave_kernel(const T* __restrict__ in, E3<int32_t> n, int nsp,
                                                                   int step, T* lowres, MapPtrs outs, int32_t nch,
                                                                   int32_t items) {
  constexpr int V = Vec16<T>::V;
  const int32_t rz = (n.e[0] + step - 1) / step, ry = (n.e[1] + step - 1) / step;
  for (int32_t t = blockIdx.x * kThreads + threadIdx.x; t < items; t += gridDim.x * kThreads) {
    const RowItem q = row_item((uint32_t)t, rz, ry, nch);
    const int32_t hz = q.z * step, hy = q.y * step;
    const int pz = (nsp == 3) ? (hz & 1) : 0, py = hy & 1;
    T* dst[2] = {nullptr, nullptr};
    int32_t ex[2];
    int32_t ez = nsp == 3 ? (pz ? n.e[0] / 2 : (n.e[0] + 1) / 2) : 1, ey = py ? n.e[1] / 2 : (n.e[1] + 1) / 2;
    ex[0] = (n.e[2] + 1) / 2;
    ex[1] = n.e[2] / 2;
    const int32_t orow = (q.b * ez + (hz >> 1)) * ey + (hy >> 1);
    if (pz == 0 && py == 0 && lowres) dst[0] = (T*)lowres + orow * ex[0];
    if (outs.p[0]) {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        if (k >= (nsp == 3 ? 7 : 3)) break;
        int par[3];
        map_parity(nsp, k, par);
        if (par[0] == pz && par[1] == py) dst[par[2]] = (T*)outs.p[k] + orow * ex[par[2]];
      }
    }
    const T* src = in + ((q.b * n.e[0] + hz) * n.e[1] + hy) * n.e[2];
    const int32_t x0 = q.j * V;
    if (2 * x0 + 2 * V <= n.e[2]) {
      Vec16<T> a, b, ev, od;
      a.load(src + 2 * x0);
      b.load(src + 2 * x0 + V);
#pragma unroll
      for (int i = 0; i < V / 2; ++i) {
        ev.e[i] = a.e[2 * i]; od.e[i] = a.e[2 * i + 1];
        ev.e[V / 2 + i] = b.e[2 * i]; od.e[V / 2 + i] = b.e[2 * i + 1];
      }
      if (dst[0]) ev.store(dst[0] + x0);
      if (dst[1]) od.store(dst[1] + x0);
    } else {
      for (int32_t x = 2 * x0; x < 2 * x0 + 2 * V && x < n.e[2]; ++x)
        if (dst[x & 1]) dst[x & 1][x >> 1] = src[x];
    }
  }
}

// Parity merge (highres_from_lowres_and_maps): item = highres row (b, hz, hy), chunk j = highres x
// in [2jV, 2jV + 2V) from class (pz, py, 0) (lowres when pz = py = 0) and class (pz, py, 1).
template <typename T>
__global__ void __launch_bounds__(kThreads) rows_interleave_kernel(const T* __restrict__ lowres, CMapPtrs maps,
                                                                 E3<int32_t> L, int nsp, T* __restrict__ out,
                                                                 int32_t nch, int32_t items) {
  constexpr int V = Vec16<T>::V;
  const int32_t h0 = 2 * L.e[0] - 1, h1 = 2 * L.e[1] - 1, h2 = 2 * L.e[2] - 1;
  for (int32_t t = blockIdx.x * kThreads + threadIdx.x; t < items; t += gridDim.x * kThreads) {
    const RowItem q = row_item((uint32_t)t, h0, h1, nch);
    const int pz = (nsp == 3) ? (q.z & 1) : 0, py = q.y & 1;
    const T* srcp[2] = {nullptr, nullptr};
    const int32_t ez = nsp == 3 ? (pz ? L.e[0] - 1 : L.e[0]) : 1, ey = py ? L.e[1] - 1 : L.e[1];
    const int32_t ex[2] = {L.e[2], L.e[2] - 1};
    const int32_t irow = (q.b * ez + (q.z >> 1)) * ey + (q.y >> 1);
    if (pz == 0 && py == 0) srcp[0] = lowres + irow * ex[0];
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      if (k >= (nsp == 3 ? 7 : 3)) break;
      int par[3];
      map_parity(nsp, k, par);
      if (par[0] == pz && par[1] == py) srcp[par[2]] = (const T*)maps.p[k] + irow * ex[par[2]];
    }
    T* dst = out + ((q.b * h0 + q.z) * h1 + q.y) * h2;
    const int32_t x0 = q.j * V;
    if (x0 + V <= ex[1]) {
      Vec16<T> ev, od, a, b;
      ev.load(srcp[0] + x0);
      od.load(srcp[1] + x0);
#pragma unroll
      for (int i = 0; i < V / 2; ++i) {
        a.e[2 * i] = ev.e[i]; a.e[2 * i + 1] = od.e[i];
        b.e[2 * i] = ev.e[V / 2 + i]; b.e[2 * i + 1] = od.e[V / 2 + i];
      }
      a.store(dst + 2 * x0);
      b.store(dst + 2 * x0 + V);
    } else {
      for (int32_t x = 2 * x0; x < 2 * x0 + 2 * V && x < h2; ++x) dst[x] = srcp[x & 1][x >> 1];
    }
  }
}

// Same-dtype box copy (slicing / .at[box].set of the chunk driver, trims)
template <typename T>
__global__ void __launch_bounds__(kThreads) rows_copy_kernel(const T* __restrict__ in, E3<int32_t> ie, E3<int32_t> io,
                                                           T* __restrict__ out, E3<int32_t> oe, E3<int32_t> oo,
                                                           E3<int32_t> ext, int32_t nch, int32_t items) {
  constexpr int V = Vec16<T>::V;
  for (int32_t t = blockIdx.x * kThreads + threadIdx.x; t < items; t += gridDim.x * kThreads) {
    const RowItem q = row_item((uint32_t)t, ext.e[0], ext.e[1], nch);
    const T* src = in + ((q.b * ie.e[0] + io.e[0] + q.z) * ie.e[1] + io.e[1] + q.y) * ie.e[2] + io.e[2];
    T* dst = out + ((q.b * oe.e[0] + oo.e[0] + q.z) * oe.e[1] + oo.e[1] + q.y) * oe.e[2] + oo.e[2];
    const int32_t x0 = q.j * V;
    if (x0 + V <= ext.e[2]) {
      Vec16<T> v;
      v.load(src + x0);
      v.store(dst + x0);
    } else {
      for (int32_t x = x0; x < ext.e[2]; ++x) dst[x] = src[x];
    }
  }
}

// ------------------------------------------------------------------------------------------
// C-ABI helpers
// ------------------------------------------------------------------------------------------
static inline Ext3 ext_from(int nsp, const int64_t* shape) {
  Ext3 e;
  for (int a = 0; a < 3; ++a) e.e[a] = (a < 3 - nsp) ? 1 : shape[a - (3 - nsp)];
  return e;
}

// 32-bit kernel indices when every array the launch touches is below 2^30 elements
static inline bool fits32(std::initializer_list<int64_t> counts) {
  for (int64_t c : counts)
    if (c >= ((int64_t)1 << 30)) return false;
  return true;
}
template <typename F>
static int with_index(bool small, F&& f) {
  return small ? f(int32_t{}) : f(int64_t{});
}
static inline int64_t vol(int64_t B, const Ext3& e, int64_t C) { return B * e.e[0] * e.e[1] * e.e[2] * C; }

// the row kernels serve C == 1 arrays below 2^30 elements (KMP_DISABLE_ROWS=1: element kernels)
static bool rows_ok(int64_t C, std::initializer_list<int64_t> counts) {
  return !opt(OPT_DISABLE_ROWS, 0) && C == 1 && fits32(counts);
}
static inline E3<int32_t> e32(const Ext3& x) { return e3<int32_t>(x); }
template <typename T>
static inline int32_t row_chunks(int64_t n) { return (int32_t)ceil_div(n, 16 / (int64_t)sizeof(T)); }

static inline int check_common(int nsp, int64_t B, const int64_t* shape, int64_t C) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(B >= 0 && C >= 1 && shape, "bad batch/channel/shape");
  for (int a = 0; a < nsp; ++a) KMP_REQUIRE(shape[a] >= 0, "negative extent");
  return KMP_OK;
}

}  // namespace kmp

using namespace kmp;

extern "C" {

#ifdef KMP_DEBUG
const char* kmp_version(void) { return "kompressor_hip 0.2.0 (gfx950, debug: device bounds checks)"; }
#else
const char* kmp_version(void) { return "kompressor_hip 0.2.0 (gfx950)"; }
#endif
const char* kmp_last_error(void) { return g_last_error.c_str(); }
const char* kmp_last_launch(void) { return g_last_launch; }

int kmp_device_ok(void) {
  // The real requirement: this library's code object loads on the current device (gfx950).
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    set_error(std::string("no HIP device visible: ") + hipGetErrorString(e));
    return 0;
  }
  hipFuncAttributes attr;
  e = hipFuncGetAttributes(&attr, (const void*)&pad_kernel<uint8_t, int32_t>);
  if (e != hipSuccess) {
    set_error(std::string("libkompressor_hip has no code object for this device (built for gfx950): ") +
              hipGetErrorString(e));
    return 0;
  }
  return 1;
}

int kmp_host_device_pointer(void* host, void** device) {
  KMP_REQUIRE(host && device, "null pointer");
  hipError_t e = hipHostGetDevicePointer(device, host, 0);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(KMP_ERR_UNSUPPORTED, std::string("not device-mapped host memory: ") + hipGetErrorString(e));
  }
  return KMP_OK;
}

int kmp_lowres_from_highres(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3],
                            int64_t C, void* out, kmp_stream_t stream) {
  if (int s = check_common(nsp, B, shape, C)) return s;
  KMP_REQUIRE(in && out, "null pointer");
  Ext3 n = ext_from(nsp, shape);
  const int64_t total = B * ((n.e[0] + 1) / 2) * ((n.e[1] + 1) / 2) * ((n.e[2] + 1) / 2) * C;
  if (total == 0) return KMP_OK;
  MapPtrs none{};
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    if (rows_ok(C, {vol(B, n, C)})) {
      const int32_t nch = row_chunks<T>((n.e[2] + 1) / 2);
      const int64_t items = B * ((n.e[0] + 1) / 2) * ((n.e[1] + 1) / 2) * nch;
      rows_deinterleave_kernel<T><<<grid_for(items), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)in, e32(n), nsp, 2, (T*)out, none, nch, (int32_t)items);
      return check_launch("lowres_from_highres");
    }
    return with_index(fits32({vol(B, n, C)}), [&](auto itag) {
      using I = decltype(itag);
      deinterleave_kernel<T, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)in, (I)B, e3<I>(n), (I)C, nsp, none, out, (I)total);
      return check_launch("lowres_from_highres");
    });
  });
}

int kmp_maps_from_highres(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3], int64_t C,
                          void* const out[7], kmp_stream_t stream) {
  if (int s = check_common(nsp, B, shape, C)) return s;
  KMP_REQUIRE(in && out, "null pointer");
  Ext3 n = ext_from(nsp, shape);
  MapPtrs outs{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(out[k], "null map pointer");
    outs.p[k] = out[k];
  }
  const int64_t total = B * ((n.e[0] + 1) / 2) * ((n.e[1] + 1) / 2) * ((n.e[2] + 1) / 2) * C;
  if (total == 0) return KMP_OK;
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    if (rows_ok(C, {vol(B, n, C)})) {
      const int32_t nch = row_chunks<T>((n.e[2] + 1) / 2);
      const int64_t items = B * n.e[0] * n.e[1] * nch;
      rows_deinterleave_kernel<T><<<grid_for(items), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)in, e32(n), nsp, 1, nullptr, outs, nch, (int32_t)items);
      return check_launch("maps_from_highres");
    }
    return with_index(fits32({vol(B, n, C)}), [&](auto itag) {
      using I = decltype(itag);
      deinterleave_kernel<T, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)in, (I)B, e3<I>(n), (I)C, nsp, outs, nullptr, (I)total);
      return check_launch("maps_from_highres");
    });
  });
}

int kmp_targets_from_highres(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3], int64_t C,
                             void* out, kmp_stream_t stream) {
  if (int s = check_common(nsp, B, shape, C)) return s;
  KMP_REQUIRE(in && out, "null pointer");
  Ext3 n = ext_from(nsp, shape);
  const int64_t c0 = nsp == 3 ? (n.e[0] - 1) / 2 : 1;
  const int64_t total = B * c0 * ((n.e[1] - 1) / 2) * ((n.e[2] - 1) / 2) * C;
  if (total <= 0) return KMP_OK;
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    return with_index(fits32({vol(B, n, C), total * (nsp == 3 ? 19 : 5)}), [&](auto itag) {
      using I = decltype(itag);
      targets_kernel<T, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)in, (I)B, e3<I>(n), (I)C,
                                                                                  nsp, (T*)out, (I)total);
      return check_launch("targets_from_highres");
    });
  });
}

int kmp_highres_from_lowres_and_maps(int32_t nsp, int32_t dtype, const void* lowres, const void* const maps[7],
                                     int64_t B, const int64_t lshape[3], int64_t C, void* out, kmp_stream_t stream) {
  if (int s = check_common(nsp, B, lshape, C)) return s;
  KMP_REQUIRE(lowres && maps && out, "null pointer");
  Ext3 L = ext_from(nsp, lshape);
  CMapPtrs mp{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(maps[k], "null map pointer");
    mp.p[k] = maps[k];
  }
  const int64_t total = B * L.e[0] * L.e[1] * L.e[2] * C;
  if (total == 0) return KMP_OK;
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    const Ext3 H{{2 * L.e[0] - 1, 2 * L.e[1] - 1, 2 * L.e[2] - 1}};
    if (rows_ok(C, {vol(B, H, C)})) {
      const int32_t nch = row_chunks<T>(L.e[2]);
      const int64_t items = B * H.e[0] * H.e[1] * nch;
      rows_interleave_kernel<T><<<grid_for(items), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)lowres, mp, e32(L), nsp, (T*)out, nch, (int32_t)items);
      return check_launch("highres_from_lowres_and_maps");
    }
    return with_index(fits32({vol(B, H, C)}), [&](auto itag) {
      using I = decltype(itag);
      interleave_kernel<T, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)lowres, mp, (I)B,
                                                                                     e3<I>(L), (I)C, nsp, (T*)out,
                                                                                     (I)total);
      return check_launch("highres_from_lowres_and_maps");
    });
  });
}

int kmp_features_from_lowres(int32_t nsp, int32_t dtype, const void* lowres, int64_t B, const int64_t shape[3],
                             int64_t C, int32_t padding, void* out, kmp_stream_t stream) {
  if (int s = check_common(nsp, B, shape, C)) return s;
  KMP_REQUIRE(lowres && out && padding >= 0, "null pointer or negative padding");
  Ext3 S = ext_from(nsp, shape);
  int64_t cells = B * C;
  for (int a = 3 - nsp; a < 3; ++a) {
    KMP_REQUIRE(S.e[a] - 2 * padding - 1 >= 0, "window smaller than the neighbourhood");
    cells *= S.e[a] - 2 * padding - 1;
  }
  if (cells == 0) return KMP_OK;
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    const int k = 2 * padding + 2;
    const bool small = fits32({vol(B, S, C), cells * (nsp == 3 ? k * k * k : k * k)});
    if (small && C == 1 && ((uintptr_t)out & 15) == 0 && padding <= 1 && sizeof(T) <= 2) {
      auto launch = [&](auto kern) {
        kern<<<grid_for(cells), kThreads, 0, (hipStream_t)stream>>>((const T*)lowres, (int32_t)S.e[0], (int32_t)S.e[1],
                                                                    (int32_t)S.e[2], (T*)out, (int32_t)cells);
        return check_launch("features_from_lowres");
      };
      if constexpr (sizeof(T) <= 2) {
        if (nsp == 3) return padding == 0 ? launch(features_vec_kernel<T, 3, 0>) : launch(features_vec_kernel<T, 3, 1>);
        return padding == 0 ? launch(features_vec_kernel<T, 2, 0>) : launch(features_vec_kernel<T, 2, 1>);
      }
    }
    return with_index(small, [&](auto itag) {
      using I = decltype(itag);
      features_kernel<T, I><<<grid_for(cells), kThreads, 0, (hipStream_t)stream>>>((const T*)lowres, (I)B, e3<I>(S),
                                                                                   (I)C, nsp, padding, (T*)out,
                                                                                   (I)cells);
      return check_launch("features_from_lowres");
    });
  });
}

int kmp_maps_from_predictions(int32_t nsp, int32_t dtype, const void* preds, int64_t B, const int64_t cells[3],
                              int64_t C, void* const out[7], kmp_stream_t stream) {
  if (int s = check_common(nsp, B, cells, C)) return s;
  KMP_REQUIRE(preds && out, "null pointer");
  Ext3 ce = ext_from(nsp, cells);
  MapPtrs outs{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(out[k], "null map pointer");
    outs.p[k] = out[k];
  }
  int64_t total = B * C;
  for (int a = 3 - nsp; a < 3; ++a) total *= ce.e[a] + 1;
  if (total == 0) return KMP_OK;
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    const bool small = fits32({vol(B, ce, C) * (nsp == 3 ? 19 : 5), total});
    if (rows_ok(C, {vol(B, ce, C) * (nsp == 3 ? 19 : 5), total})) {
      constexpr int V = 16 / (int)sizeof(T);
      const int K = nsp == 3 ? 19 : 5, NS = nsp == 3 ? 2 : 1;
      const int32_t XO = (int32_t)std::min<int64_t>(ce.e[2] + 1, 64);
      const int32_t YB = std::max(1, std::min(8, kThreads / XO));
      const int32_t nyb = (int32_t)ceil_div(ce.e[1] + 1, YB), nxb = (int32_t)ceil_div(ce.e[2] + 1, XO);
      const int32_t nchunk = (int32_t)ceil_div((int64_t)(XO + 1) * K, V);
      const int32_t RP = nchunk * V;
      // enough workgroups to fill the chip: split the z roll into nzc runs of ZC output planes
      const int64_t fz = nsp == 3 ? ce.e[0] + 1 : 1;
      const int64_t want = ceil_div(4096, B * nyb * nxb);
      const int32_t ZC = (int32_t)ceil_div(fz, std::max<int64_t>(1, std::min<int64_t>(want, fz)));
      const int32_t nzc = (int32_t)ceil_div(fz, ZC);
      const size_t lds = (size_t)NS * (YB + 1) * RP * sizeof(T);
      const int64_t nblk = B * nzc * nyb * nxb;
      if ((int64_t)(YB + 1) * nchunk > kThreads * kMfpCpt) return fail(KMP_ERR_ARG, "maps_from_predictions: tile");
      auto kern = nsp == 3 ? maps_from_predictions_lds_kernel<T, 3> : maps_from_predictions_lds_kernel<T, 2>;
      kern<<<(unsigned)nblk, kThreads, lds, (hipStream_t)stream>>>(
          (const T*)preds, (int32_t)ce.e[0], (int32_t)ce.e[1], (int32_t)ce.e[2], outs, YB, XO, ZC, nzc, nyb, nxb, RP,
          nchunk, 1.0f / (float)nchunk, vol(B, ce, C) * K);
      return check_launch("maps_from_predictions");
    }
    if constexpr (std::is_same<T, uint8_t>::value || std::is_same<T, uint16_t>::value) {
      if (small && C == 1) {
        auto kern = nsp == 3 ? maps_from_predictions_int_kernel<T, 3> : maps_from_predictions_int_kernel<T, 2>;
        kern<<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)preds, (int32_t)ce.e[0], (int32_t)ce.e[1],
                                                                    (int32_t)ce.e[2], outs, (int32_t)total);
        return check_launch("maps_from_predictions");
      }
    }
    return with_index(small, [&](auto itag) {
      using I = decltype(itag);
      maps_from_predictions_kernel<T, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)preds, (I)B, e3<I>(ce), (I)C, nsp, outs, (I)total);
      return check_launch("maps_from_predictions");
    });
  });
}

// out_dtype: the maps' dtype -- the sample dtype, or KMP_F32 (a network-shaped predictor's
// float32 output; the values are the same integers) on the 3D C == 1 LDS kernels.
static int mean_predict_maps_impl(int32_t nsp, int32_t dtype, int32_t out_dtype, const void* padded_lowres, int64_t B,
                                  const int64_t shape[3], int64_t C, int32_t padding, void* const out[7],
                                  kmp_stream_t stream) {
  if (int s = check_common(nsp, B, shape, C)) return s;
  KMP_REQUIRE(out_dtype == dtype || out_dtype == KMP_F32, "map dtype must be the sample dtype or float32");
  KMP_REQUIRE(padded_lowres && out && padding >= 0, "null pointer or negative padding");
  Ext3 S = ext_from(nsp, shape);
  MapPtrs outs{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(out[k], "null map pointer");
    outs.p[k] = out[k];
  }
  int64_t total = B * C, ncell = B * C;
  Ext3 cells{};
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) { cells.e[a] = 1; continue; }
    KMP_REQUIRE(S.e[a] - 2 * padding - 1 >= 1, "window has no cells");
    cells.e[a] = S.e[a] - 2 * padding - 1;
    total *= S.e[a] - 2 * padding;
    ncell *= cells.e[a];
  }
  if (total == 0) return KMP_OK;
  return dispatch_int_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    T* cm = (T*)outs.p[center_map(nsp)];
    const bool small = fits32({vol(B, S, C), total});
    if constexpr (std::is_same<T, uint8_t>::value || std::is_same<T, uint16_t>::value) {
      // one workgroup per output plane when the plane's window planes fit LDS
      const int64_t plane = S.e[1] * S.e[2];
      // PPB output planes per workgroup: 2 where its LDS fits (the cell plane between the two output
      // planes summed once: p = 0 101 -> 94 us, p = 1 300 -> 270 us at 512 C3 windows,
      // profiles/round2/ab_mean_predict_ppb.log), else 1 (e.g. the C3 window at p = 2)
      auto lds_for = [&](int q, int64_t& nb_, int64_t& xs_) {
        nb_ = 16 * (ceil_div((2 * padding + 2 + q) * plane * (int64_t)sizeof(T), 16) + 1);
        xs_ = padding > 0 ? 4 * (2 * padding + 2 + q) * S.e[1] * cells.e[2] : 0;
        return nb_ + xs_ + 4 * (q + 1) * cells.e[1] * cells.e[2] + 8 * mp_pad_words(cells.e[2]);
      };
      int64_t nodes_bytes = 0, xs_bytes = 0;
      int ppb = 2;
      int64_t lds_plane = lds_for(ppb, nodes_bytes, xs_bytes);
      if (ppb == 2 && lds_plane > 64 * 1024) {
        ppb = 1;
        lds_plane = lds_for(ppb, nodes_bytes, xs_bytes);
      }
      const int64_t ngrp = ceil_div(cells.e[0] + 1, (int64_t)ppb);
      const int64_t nblk_plane = B * ngrp;
      const bool f32 = out_dtype == KMP_F32 && !std::is_same<T, float>::value;
      // p = 0, Lcx % 8 == 0: eight x positions per lane (mean_predict_p0x8_kernel), ZP = 3 output
      // planes per workgroup (4 cell planes); 32-bit map offsets
      const int64_t zp8 = std::min<int64_t>(3, cells.e[0] + 1), ngrp8 = ceil_div(cells.e[0] + 1, zp8);
      const int64_t lds8 = 4 * (zp8 + 1) * mp8_plane_words((int32_t)std::min<int64_t>(cells.e[1], 1 << 20),
                                                           (int32_t)std::min<int64_t>(cells.e[2], 1 << 20));
      if (nsp == 3 && C == 1 && padding == 0 && cells.e[2] % 8 == 0 && lds8 <= 64 * 1024 &&
          B * (cells.e[0] + 1) * (cells.e[1] + 1) * (cells.e[2] + 1) < ((int64_t)1 << 31) &&
          B * ngrp8 < ((int64_t)1 << 31) && (zp8 + 1) * cells.e[1] * (cells.e[2] / 8) < ((int64_t)1 << 21)) {
        auto kern = f32 ? mean_predict_p0x8_kernel<T, float> : mean_predict_p0x8_kernel<T, T>;
        kern<<<(unsigned)(B * ngrp8), kThreads, (size_t)lds8, (hipStream_t)stream>>>(
            (const T*)padded_lowres, e32(S), (int32_t)cells.e[0], (int32_t)cells.e[1], (int32_t)cells.e[2], outs,
            B % 8 == 0 ? (int32_t)ngrp8 : 0, (int32_t)zp8, (int32_t)ngrp8);
        return check_launch("mean_predict_p0x8");
      }
      if (nsp == 3 && C == 1 && padding <= 2 && lds_plane <= 64 * 1024 && nblk_plane < ((int64_t)1 << 31) &&
          (cells.e[0] + 1) * (cells.e[1] + 1) * (cells.e[2] + 1) < ((int64_t)1 << 31)) {
        if (f32) {
          auto launch = [&](auto kern) {
            kern<<<(unsigned)nblk_plane, kThreads, (size_t)lds_plane, (hipStream_t)stream>>>(
                (const T*)padded_lowres, e32(S), (int32_t)cells.e[0], (int32_t)cells.e[1], (int32_t)cells.e[2],
                outs, B % 8 == 0 ? (int32_t)ngrp : 0, (int32_t)nodes_bytes, (int32_t)xs_bytes);
            return check_launch(ppb == 2 ? "mean_predict_plane2" : "mean_predict_plane");
          };
          if (ppb == 2) {
            if (padding == 0) return launch(mean_predict_plane_kernel<T, 0, 2, float>);
            if (padding == 1) return launch(mean_predict_plane_kernel<T, 1, 2, float>);
            return launch(mean_predict_plane_kernel<T, 2, 2, float>);
          }
          if (padding == 0) return launch(mean_predict_plane_kernel<T, 0, 1, float>);
          if (padding == 1) return launch(mean_predict_plane_kernel<T, 1, 1, float>);
          return launch(mean_predict_plane_kernel<T, 2, 1, float>);
        }
        auto launch = [&](auto kern) {
          kern<<<(unsigned)nblk_plane, kThreads, (size_t)lds_plane, (hipStream_t)stream>>>(
              (const T*)padded_lowres, e32(S), (int32_t)cells.e[0], (int32_t)cells.e[1], (int32_t)cells.e[2], outs,
              B % 8 == 0 ? (int32_t)ngrp : 0, (int32_t)nodes_bytes, (int32_t)xs_bytes);
          return check_launch(ppb == 2 ? "mean_predict_plane2" : "mean_predict_plane");
        };
        if (ppb == 2) {
          if (padding == 0) return launch(mean_predict_plane_kernel<T, 0, 2>);
          if (padding == 1) return launch(mean_predict_plane_kernel<T, 1, 2>);
          return launch(mean_predict_plane_kernel<T, 2, 2>);
        }
        if (padding == 0) return launch(mean_predict_plane_kernel<T, 0, 1>);
        if (padding == 1) return launch(mean_predict_plane_kernel<T, 1, 1>);
        return launch(mean_predict_plane_kernel<T, 2, 1>);
      }
      if (f32) return fail(KMP_ERR_UNSUPPORTED, "mean_predict_maps: float32 maps need the 3D C == 1 LDS kernels");
      if (rows_ok(C, {vol(B, S, C), total}) && padding <= 1) {
        const int32_t XO = (int32_t)std::min<int64_t>(cells.e[2] + 1, 64);
        const int32_t YB = std::max(1, std::min(8, kThreads / XO));
        const int32_t nyb = (int32_t)ceil_div(cells.e[1] + 1, YB), nxb = (int32_t)ceil_div(cells.e[2] + 1, XO);
        const int32_t RP = XO + 1;
        const int64_t fz = nsp == 3 ? cells.e[0] + 1 : 1;
        const int64_t want = ceil_div(4096, B * nyb * nxb);
        const int32_t ZC = (int32_t)ceil_div(fz, std::max<int64_t>(1, std::min<int64_t>(want, fz)));
        const int32_t nzc = (int32_t)ceil_div(fz, ZC);
        const size_t lds = (size_t)2 * (YB + 1) * RP * sizeof(uint32_t);
        const int64_t nblk = B * nzc * nyb * nxb;
        if ((int64_t)(YB + 1) * RP > kThreads * kMpCpt) return fail(KMP_ERR_ARG, "mean_predict_maps: tile");
        auto kern = nsp == 3 ? mean_predict_lds_kernel<T, 3> : mean_predict_lds_kernel<T, 2>;
        kern<<<(unsigned)nblk, kThreads, lds, (hipStream_t)stream>>>(
            (const T*)padded_lowres, e32(S), padding, (int32_t)cells.e[0], (int32_t)cells.e[1], (int32_t)cells.e[2],
            outs, YB, XO, ZC, nzc, nyb, nxb, RP);
        return check_launch("mean_predict_maps");
      }
    }
    if (out_dtype != dtype) return fail(KMP_ERR_UNSUPPORTED, "mean_predict_maps: float32 maps of this window");
    int st = with_index(small, [&](auto itag) {
      using I = decltype(itag);
      cell_mean_map_kernel<T, I><<<grid_for(ncell), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)padded_lowres, (I)B, e3<I>(S), (I)C, nsp, padding, e3<I>(cells), cm, (I)ncell);
      return check_launch("mean_predict_maps");
    });
    if (st) return st;
    if ((std::is_same<T, uint8_t>::value || std::is_same<T, uint16_t>::value) && C == 1 && total < ((int64_t)1 << 31)) {
      auto k = nsp == 3 ? maps_from_cell_means_int_kernel<T, 3> : maps_from_cell_means_int_kernel<T, 2>;
      k<<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(cm, (int32_t)cells.e[0], (int32_t)cells.e[1],
                                                              (int32_t)cells.e[2], outs, (int32_t)total);
    } else {
      return with_index(small, [&](auto itag) {
        using I = decltype(itag);
        maps_from_cell_means_kernel<T, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(
            cm, (I)B, e3<I>(cells), (I)C, nsp, outs, (I)total);
        return check_launch("mean_predict_maps");
      });
    }
    return check_launch("mean_predict_maps");
  });
}

int kmp_mean_predict_maps(int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B, const int64_t shape[3],
                          int64_t C, int32_t padding, void* const out[7], kmp_stream_t stream) {
  return mean_predict_maps_impl(nsp, dtype, dtype, padded_lowres, B, shape, C, padding, out, stream);
}

int kmp_mean_predict_maps_typed(int32_t nsp, int32_t dtype, int32_t out_dtype, const void* padded_lowres, int64_t B,
                                const int64_t shape[3], int64_t C, int32_t padding, void* const out[7],
                                kmp_stream_t stream) {
  return mean_predict_maps_impl(nsp, dtype, out_dtype, padded_lowres, B, shape, C, padding, out, stream);
}

int kmp_pad(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3], int64_t C,
            const int64_t pad_lo[3], const int64_t pad_hi[3], int32_t mode, void* out, kmp_stream_t stream) {
  if (int s = check_common(nsp, B, shape, C)) return s;
  KMP_REQUIRE(in && out && pad_lo && pad_hi && (mode == 0 || mode == 1), "bad pointer or mode");
  Ext3 n = ext_from(nsp, shape);
  Ext3 lo{}, oe{};
  int64_t total = B * C;
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) { lo.e[a] = 0; oe.e[a] = 1; continue; }
    const int i = a - (3 - nsp);
    lo.e[a] = pad_lo[i];
    oe.e[a] = n.e[a] + pad_lo[i] + pad_hi[i];
    KMP_REQUIRE(oe.e[a] >= 0, "pads remove more than the extent");
    KMP_REQUIRE(n.e[a] > 0 || oe.e[a] == 0, "cannot pad an empty axis");
    total *= oe.e[a];
  }
  if (total == 0) return KMP_OK;
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    if (rows_ok(C, {vol(B, n, C), total})) {
      const int32_t nch = row_chunks<T>(oe.e[2]);
      const int64_t items = B * oe.e[0] * oe.e[1] * nch;
      rows_pad_kernel<T><<<grid_for(items), kThreads, 0, (hipStream_t)stream>>>(
          (const T*)in, e32(n), e32(lo), e32(oe), mode, (T*)out, nch, (int32_t)items);
      return check_launch("pad");
    }
    return with_index(fits32({vol(B, n, C), total}), [&](auto itag) {
      using I = decltype(itag);
      pad_kernel<T, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)in, (I)B, e3<I>(n), (I)C,
                                                                              e3<I>(lo), e3<I>(oe), mode, (T*)out,
                                                                              (I)total);
      return check_launch("pad");
    });
  });
}

int kmp_copy_box(int32_t nsp, int32_t in_dtype, const void* in, const int64_t in_shape[3], const int64_t in_off[3],
                 int32_t out_dtype, void* out, const int64_t out_shape[3], const int64_t out_off[3], int64_t B,
                 int64_t C, const int64_t ext[3], kmp_stream_t stream) {
  if (int s = check_common(nsp, B, in_shape, C)) return s;
  if (int s = check_common(nsp, B, out_shape, C)) return s;
  KMP_REQUIRE(in && out && in_off && out_off && ext, "null pointer");
  Ext3 ie = ext_from(nsp, in_shape), oe = ext_from(nsp, out_shape);
  Ext3 io{}, oo{}, ee{};
  int64_t total = B * C;
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) { io.e[a] = 0; oo.e[a] = 0; ee.e[a] = 1; continue; }
    const int i = a - (3 - nsp);
    io.e[a] = in_off[i]; oo.e[a] = out_off[i]; ee.e[a] = ext[i];
    KMP_REQUIRE(ext[i] >= 0 && in_off[i] >= 0 && out_off[i] >= 0 && in_off[i] + ext[i] <= ie.e[a] &&
                    out_off[i] + ext[i] <= oe.e[a], "box out of bounds");
    total *= ext[i];
  }
  if (total == 0) return KMP_OK;
  return dispatch_any_dtype(in_dtype, [&](auto itag) {
    using TI = decltype(itag);
    return dispatch_any_dtype(out_dtype, [&](auto otag) {
      using TO = decltype(otag);
      if constexpr (std::is_same<TI, TO>::value) {
        if (rows_ok(C, {vol(B, ie, C), vol(B, oe, C)})) {
          const int32_t nch = row_chunks<TI>(ee.e[2]);
          const int64_t items = B * ee.e[0] * ee.e[1] * nch;
          rows_copy_kernel<TI><<<grid_for(items), kThreads, 0, (hipStream_t)stream>>>(
              (const TI*)in, e32(ie), e32(io), (TO*)out, e32(oe), e32(oo), e32(ee), nch, (int32_t)items);
          return check_launch("copy_box");
        }
      }
      return with_index(fits32({vol(B, ie, C), vol(B, oe, C)}), [&](auto itag) {
        using I = decltype(itag);
        copy_box_kernel<TI, TO, I><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(
            (const TI*)in, e3<I>(ie), e3<I>(io), (TO*)out, e3<I>(oe), e3<I>(oo), e3<I>(ee), (I)C, (I)total);
        return check_launch("copy_box");
      });
    });
  });
}

int kmp_code(int32_t direction, int32_t coder, int32_t pred_dtype, const void* pred, int32_t x_dtype, const void* x,
             int64_t n, void* out, kmp_stream_t stream) {
  KMP_REQUIRE(direction == KMP_ENCODE || direction == KMP_DECODE, "bad direction");
  KMP_REQUIRE(n >= 0, "negative count");
  if (n == 0) return KMP_OK;
  KMP_REQUIRE(pred && x && out, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  auto launch = [&](auto dir_c, auto coder_c) {
    constexpr int DIR = decltype(dir_c)::value;
    constexpr int CODER = decltype(coder_c)::value;
    return dispatch_any_dtype(pred_dtype, [&](auto ptag) {
      using TP = decltype(ptag);
      return dispatch_any_dtype(x_dtype, [&](auto xtag) {
        using TX = decltype(xtag);
        using TO = typename coder_out<CODER>::type;
        if constexpr (sizeof(TP) == sizeof(TX) && sizeof(TX) == sizeof(TO) && !std::is_same<TP, float>::value &&
                      !std::is_same<TX, float>::value) {
          constexpr int V = 16 / sizeof(TX);
          if ((((uintptr_t)pred | (uintptr_t)x | (uintptr_t)out) & 15) == 0 && n % V == 0) {
            code_vec_kernel<DIR, CODER, TX><<<grid_for(n / V), kThreads, 0, s>>>(
                (const u32x4v*)pred, (const u32x4v*)x, n / V, (u32x4v*)out);
            return check_launch("code");
          }
        }
        return with_index(fits32({n}), [&](auto itag) {
          using I = decltype(itag);
          code_kernel<DIR, CODER, TP, TX, I><<<grid_for(n), kThreads, 0, s>>>(
              (const TP*)pred, (const TX*)x, (I)n, (typename coder_out<CODER>::type*)out);
          return check_launch("code");
        });
      });
    });
  };
  auto with_coder = [&](auto dir_c) {
    switch (coder) {
      case KMP_CODER_RAW: return launch(dir_c, std::integral_constant<int, KMP_CODER_RAW>{});
      case KMP_CODER_U8: return launch(dir_c, std::integral_constant<int, KMP_CODER_U8>{});
      case KMP_CODER_U16: return launch(dir_c, std::integral_constant<int, KMP_CODER_U16>{});
      case KMP_CODER_U32: return launch(dir_c, std::integral_constant<int, KMP_CODER_U32>{});
      default: return fail(KMP_ERR_ARG, "kmp_code: bad coder");
    }
  };
  return direction == KMP_ENCODE ? with_coder(std::integral_constant<int, KMP_ENCODE>{})
                                 : with_coder(std::integral_constant<int, KMP_DECODE>{});
}

}  // extern "C"
