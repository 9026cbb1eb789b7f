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

// Decompose a flat index over [B, e0, e1, e2, C].
struct Idx5 {
  int64_t b, i0, i1, i2, c;
};
__device__ __forceinline__ Idx5 unflatten5(int64_t t, int64_t e0, int64_t e1, int64_t e2, int64_t C) {
  Idx5 r;
  unflat5(t, e0, e1, e2, C, r.b, r.i0, r.i1, r.i2, r.c);
  return r;
}

// ------------------------------------------------------------------------------------------
// Parity (de)interleave: lowres_from_highres, maps_from_highres, highres_from_lowres_and_maps
// ------------------------------------------------------------------------------------------
struct Ext3 {
  int64_t e[3];
};

// out_k[b, o, c] = in[b, 2*o + par_k, c] for every class k whose pointer is set and whose
// extent contains o.  Class 0 = all-even (lowres), classes 1..7 (1..3) = maps.
template <typename T>
__global__ void __launch_bounds__(kThreads) deinterleave_kernel(const T* __restrict__ in, int64_t B, Ext3 n,
                                                              int64_t C, int nsp, MapPtrs outs, void* lowres,
                                                              int64_t total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  // frame = ceil(n/2) per axis (dummy axes: 1)
  const int64_t f0 = (n.e[0] + 1) / 2, f1 = (n.e[1] + 1) / 2, f2 = (n.e[2] + 1) / 2;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, f0, f1, f2, C);
    auto src = [&](int pz, int py, int px) -> T {
      const int64_t z = 2 * q.i0 + pz, y = 2 * q.i1 + py, x = 2 * q.i2 + px;
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
      int64_t e[3];
      const int64_t idx[3] = {q.i0, q.i1, q.i2};
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
template <typename T>
__global__ void __launch_bounds__(kThreads) interleave_kernel(const T* __restrict__ lowres, CMapPtrs maps,
                                                            int64_t B, Ext3 L, int64_t C, int nsp, T* __restrict__ out,
                                                            int64_t total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  const int64_t h0 = 2 * L.e[0] - 1, h1 = 2 * L.e[1] - 1, h2 = 2 * L.e[2] - 1;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, L.e[0], L.e[1], L.e[2], C);
    auto dst = [&](int pz, int py, int px) -> T& {
      const int64_t z = 2 * q.i0 + pz, y = 2 * q.i1 + py, x = 2 * q.i2 + px;
      return out[(((q.b * h0 + z) * h1 + y) * h2 + x) * C + q.c];
    };
    dst(0, 0, 0) = lowres[t];
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      int64_t e[3];
      const int64_t idx[3] = {q.i0, q.i1, q.i2};
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

template <typename T>
__global__ void __launch_bounds__(kThreads) targets_kernel(const T* __restrict__ in, int64_t B, Ext3 n, int64_t C,
                                                         int nsp, T* __restrict__ out, int64_t total) {
  const int K = nsp == 3 ? 19 : 5;
  const int64_t c0 = nsp == 3 ? (n.e[0] - 1) / 2 : 1, c1 = (n.e[1] - 1) / 2, c2 = (n.e[2] - 1) / 2;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, c0, c1, c2, C);
    const int64_t cell = ((q.b * c0 + q.i0) * c1 + q.i1) * c2 + q.i2;
    for (int k = 0; k < K; ++k) {
      int dz, dy, dx;
      if (nsp == 3) { dz = c_targets3[k][0]; dy = c_targets3[k][1]; dx = c_targets3[k][2]; }
      else { dz = 0; dy = c_targets2[k][0]; dx = c_targets2[k][1]; }
      const int64_t z = nsp == 3 ? 2 * q.i0 + dz : 0, y = 2 * q.i1 + dy, x = 2 * q.i2 + dx;
      out[(cell * K + k) * C + q.c] = in[(((q.b * n.e[0] + z) * n.e[1] + y) * n.e[2] + x) * C + q.c];
    }
  }
}

// features_from_lowres: [B, S-2p-1..., N, C], N = (2p+2)^d, offsets z-major then y, x.
template <typename T>
__global__ void __launch_bounds__(kThreads) features_kernel(const T* __restrict__ in, int64_t B, Ext3 S, int64_t C,
                                                          int nsp, int p, T* __restrict__ out, int64_t total) {
  const int k = 2 * p + 2;
  const int kz = nsp == 3 ? k : 1;
  const int N = kz * k * k;
  const int64_t c0 = nsp == 3 ? S.e[0] - 2 * p - 1 : 1, c1 = S.e[1] - 2 * p - 1, c2 = S.e[2] - 2 * p - 1;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, c0, c1, c2, C);
    const int64_t cell = ((q.b * c0 + q.i0) * c1 + q.i1) * c2 + q.i2;
    int f = 0;
    for (int dz = 0; dz < kz; ++dz)
      for (int dy = 0; dy < k; ++dy)
        for (int dx = 0; dx < k; ++dx, ++f) {
          const int64_t z = q.i0 + dz, y = q.i1 + dy, x = q.i2 + dx;
          out[(cell * N + f) * C + q.c] = in[(((q.b * S.e[0] + z) * S.e[1] + y) * S.e[2] + x) * C + q.c];
        }
  }
}

// ------------------------------------------------------------------------------------------
// maps_from_predictions: float32 aggregation of [B, cells..., K, C] predictions.
// ------------------------------------------------------------------------------------------
template <typename T>
__global__ void __launch_bounds__(kThreads) maps_from_predictions_kernel(const T* __restrict__ preds, int64_t B,
                                                                       Ext3 cells, int64_t C, int nsp, MapPtrs outs,
                                                                       int64_t total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  const int K = nsp == 3 ? 19 : 5;
  // frame = cells + 1 per spatial axis
  const int64_t f0 = nsp == 3 ? cells.e[0] + 1 : 1, f1 = cells.e[1] + 1, f2 = cells.e[2] + 1;
  const int64_t Lcz = cells.e[0], Lcy = cells.e[1], Lcx = cells.e[2];
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, f0, f1, f2, C);
    auto get = [&](int64_t z, int64_t y, int64_t x, int ch) -> T {
      return preds[(((((q.b * Lcz + z) * Lcy + y) * Lcx + x) * K) + ch) * C + q.c];
    };
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      int64_t e[3];
      const int64_t idx[3] = {q.i0, q.i1, q.i2};
      bool ok = true;
      for (int a = 0; a < 3; ++a) {
        e[a] = (a < 3 - nsp) ? 1 : (par[a] ? cells.e[a] : cells.e[a] + 1);
        ok = ok && idx[a] < e[a];
      }
      if (!ok) continue;
      T* o = (T*)outs.p[k];
      o[(((q.b * e[0] + q.i0) * e[1] + q.i1) * e[2] + q.i2) * C + q.c] =
          aggregate_map<T>(nsp, k, q.i0, q.i1, q.i2, Lcz, Lcy, Lcx, get);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Mean predictor on a padded lowres window (tests/volume/test_encode_decode.py:46-53):
// cell mean = astype(T)(f32 sum of the (2p+2)^d neighbourhood / N), then the map aggregation.
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T cell_mean_padded(const T* __restrict__ in, int64_t b, int64_t cz, int64_t cy, int64_t cx,
                                              int64_t c, Ext3 S, int64_t C, int nsp, int p) {
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
template <typename T>
__global__ void __launch_bounds__(kThreads) cell_mean_map_kernel(const T* __restrict__ in, int64_t B, Ext3 S,
                                                               int64_t C, int nsp, int p, Ext3 cells,
                                                               T* __restrict__ out, int64_t total) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, cells.e[0], cells.e[1], cells.e[2], C);
    out[t] = cell_mean_padded<T>(in, q.b, q.i0, q.i1, q.i2, q.c, S, C, nsp, p);
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

template <typename T>
__global__ void __launch_bounds__(kThreads) maps_from_cell_means_kernel(const T* __restrict__ cm, int64_t B,
                                                                      Ext3 cells, int64_t C, int nsp, MapPtrs outs,
                                                                      int64_t total) {
  const int nmaps = nsp == 3 ? 7 : 3;
  const int64_t Lcz = cells.e[0], Lcy = cells.e[1], Lcx = cells.e[2];
  const int64_t f0 = nsp == 3 ? Lcz + 1 : 1, f1 = Lcy + 1, f2 = Lcx + 1;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, f0, f1, f2, C);
    auto get = [&](int64_t z, int64_t y, int64_t x, int) -> T {
      return cm[(((q.b * Lcz + z) * Lcy + y) * Lcx + x) * C + q.c];
    };
    for (int k = 0; k < nmaps; ++k) {
      if (k == center_map(nsp)) continue;
      int par[3];
      map_parity(nsp, k, par);
      int64_t e[3];
      const int64_t idx[3] = {q.i0, q.i1, q.i2};
      bool ok = true;
      for (int a = 0; a < 3; ++a) {
        e[a] = (a < 3 - nsp) ? 1 : (par[a] ? cells.e[a] : cells.e[a] + 1);
        ok = ok && idx[a] < e[a];
      }
      if (!ok) continue;
      T* o = (T*)outs.p[k];
      o[(((q.b * e[0] + q.i0) * e[1] + q.i1) * e[2] + q.i2) * C + q.c] =
          aggregate_map<T>(nsp, k, q.i0, q.i1, q.i2, Lcz, Lcy, Lcx, get);
    }
  }
}

// ------------------------------------------------------------------------------------------
// jnp.pad on the spatial axes ('symmetric' / 'reflect'); negative pads crop.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t reflect_index(int64_t i, int64_t n) {
  if (n == 1) return 0;
  const int64_t per = 2 * (n - 1);
  int64_t m = i % per;
  if (m < 0) m += per;
  return m < n ? m : per - m;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) pad_kernel(const T* __restrict__ in, int64_t B, Ext3 n, int64_t C,
                                                     Ext3 lo, Ext3 out_e, int mode, T* __restrict__ out,
                                                     int64_t total) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, out_e.e[0], out_e.e[1], out_e.e[2], C);
    const int64_t o[3] = {q.i0, q.i1, q.i2};
    int64_t s[3];
    for (int a = 0; a < 3; ++a) {
      const int64_t i = o[a] - lo.e[a];
      s[a] = (i >= 0 && i < n.e[a]) ? i : (mode == 0 ? sym_index(i, n.e[a]) : reflect_index(i, n.e[a]));
    }
    out[t] = in[(((q.b * n.e[0] + s[0]) * n.e[1] + s[1]) * n.e[2] + s[2]) * C + q.c];
  }
}

// ------------------------------------------------------------------------------------------
// Coders (utils.py:28-55), 8 elements per thread when the count allows.
// ------------------------------------------------------------------------------------------
template <int DIR, int CODER, typename TP, typename TX>
__global__ void __launch_bounds__(kThreads) code_kernel(const TP* __restrict__ pred, const TX* __restrict__ x, int64_t n,
                                                      typename coder_out<CODER>::type* __restrict__ out) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
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

template <typename TI, typename TO>
__global__ void __launch_bounds__(kThreads) copy_box_kernel(const TI* __restrict__ in, Ext3 in_e, Ext3 in_off,
                                                          TO* __restrict__ out, Ext3 out_e, Ext3 out_off, Ext3 ext,
                                                          int64_t C, int64_t total) {
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    Idx5 q = unflatten5(t, ext.e[0], ext.e[1], ext.e[2], C);
    const int64_t si = (((q.b * in_e.e[0] + in_off.e[0] + q.i0) * in_e.e[1] + in_off.e[1] + q.i1) * in_e.e[2] +
                        in_off.e[2] + q.i2) * C + q.c;
    const int64_t so = (((q.b * out_e.e[0] + out_off.e[0] + q.i0) * out_e.e[1] + out_off.e[1] + q.i1) * out_e.e[2] +
                        out_off.e[2] + q.i2) * C + q.c;
    out[so] = convert<TO>(in[si]);
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

static inline int check_common(int nsp, int64_t B, const int64_t* shape, int64_t C) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(B >= 0 && C >= 1 && shape, "bad batch/channel/shape");
  for (int a = 0; a < nsp; ++a) KMP_REQUIRE(shape[a] >= 0, "negative extent");
  return KMP_OK;
}

}  // namespace kmp

using namespace kmp;

extern "C" {

const char* kmp_version(void) { return "kompressor_hip 0.1.0 (gfx950)"; }
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
  e = hipFuncGetAttributes(&attr, (const void*)&pad_kernel<uint8_t>);
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
    deinterleave_kernel<T><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)in, B, n, C, nsp, none,
                                                                                   out, total);
    return check_launch("lowres_from_highres");
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
    deinterleave_kernel<T><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)in, B, n, C, nsp, outs,
                                                                                   nullptr, total);
    return check_launch("maps_from_highres");
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
    targets_kernel<T><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)in, B, n, C, nsp, (T*)out,
                                                                              total);
    return check_launch("targets_from_highres");
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
    interleave_kernel<T><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)lowres, mp, B, L, C, nsp,
                                                                                 (T*)out, total);
    return check_launch("highres_from_lowres_and_maps");
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
    features_kernel<T><<<grid_for(cells), kThreads, 0, (hipStream_t)stream>>>((const T*)lowres, B, S, C, nsp, padding,
                                                                               (T*)out, cells);
    return check_launch("features_from_lowres");
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
    maps_from_predictions_kernel<T><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)preds, B, ce, C,
                                                                                            nsp, outs, total);
    return check_launch("maps_from_predictions");
  });
}

int kmp_mean_predict_maps(int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B, const int64_t shape[3],
                          int64_t C, int32_t padding, void* const out[7], kmp_stream_t stream) {
  if (int s = check_common(nsp, B, shape, C)) return s;
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
    cell_mean_map_kernel<T><<<grid_for(ncell), kThreads, 0, (hipStream_t)stream>>>((const T*)padded_lowres, B, S, C,
                                                                                   nsp, padding, cells, cm, ncell);
    if (int st = check_launch("mean_predict_maps")) return st;
    if ((std::is_same<T, uint8_t>::value || std::is_same<T, uint16_t>::value) && C == 1 && total < ((int64_t)1 << 31)) {
      auto k = nsp == 3 ? maps_from_cell_means_int_kernel<T, 3> : maps_from_cell_means_int_kernel<T, 2>;
      k<<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(cm, (int32_t)cells.e[0], (int32_t)cells.e[1],
                                                              (int32_t)cells.e[2], outs, (int32_t)total);
    } else {
      maps_from_cell_means_kernel<T><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>(cm, B, cells, C, nsp, outs,
                                                                                            total);
    }
    return check_launch("mean_predict_maps");
  });
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
    pad_kernel<T><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const T*)in, B, n, C, lo, oe, mode, (T*)out,
                                                                          total);
    return check_launch("pad");
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
      copy_box_kernel<TI, TO><<<grid_for(total), kThreads, 0, (hipStream_t)stream>>>((const TI*)in, ie, io, (TO*)out,
                                                                                      oe, oo, ee, C, total);
      return check_launch("copy_box");
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
        code_kernel<DIR, CODER, TP, TX><<<grid_for(n), kThreads, 0, s>>>(
            (const TP*)pred, (const TX*)x, n, (typename coder_out<CODER>::type*)out);
        return check_launch("code");
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
