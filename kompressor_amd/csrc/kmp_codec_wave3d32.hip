// kmp_codec_wave3d32.hip -- one-pass volume encode / decode for 32-bit samples with the mean
// predictor at p == 0: uint32 (float32 volumes bit-cast, BASELINE config C5, mod-2^32 coder) and
// int32 (the raw coder, utils.py:28-35).
//
// Data movement is kmp_codec_wave3d.hip's plane-block scheme (PL = 2 output planes per
// workgroup, every load up front, neighbours by cross-lane shuffles, tile-per-XCD order) with
// VX = 2 outputs per lane (16 bytes of a highres row = 2 nodes + 2 odd samples).  The arithmetic
// is the reference's float32 one, which for 32-bit samples is NOT exact, so the order is the
// reference's (oracle.predictors.mean_predictions_fn):
//   cell mean = cast(((((((0 + f(n0)) + f(n1)) + ...) + f(n7)) / 8) over the 8 nodes in feature
//               order n = dz*4 + dy*2 + dx (features_from_lowres, volume/utils.py:199-210), f =
//               the float32 conversion, cast = XLA truncating saturating astype;
//   map value  = cast(scale * (((0 + f(m_a)) + f(m_b)) + ...)) over the contributing cells in the
//               reference's channel order (maps_from_predictions, volume/utils.py:83-155; the
//               C map is the raw mean) -- kmp_aggregate.h's contribution lists, with cells outside
//               the grid adding nothing.
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace w32 {

using namespace wv;

struct W32 {
  const void* hi_in;
  void* hi_out;
  const void* lo_in;
  void* lo_out;
  MapPtrs maps;
  int32_t D, H, W;
  int32_t Lz, Ly, Lx, Ez, Ey, Ex, Lcz, Lcy, Lcx;
  int32_t nslab, zbegin, zend;
  int32_t txn, rows, nwv, nyg;
  int32_t xcd_per;
};

// float32 conversion and XLA's truncating saturating astype (NaN -> 0): v_cvt_{u32,i32}_f32
// saturate and map NaN to 0 in hardware
template <typename T>
__device__ __forceinline__ T from_f(float v) {
  T r;
  if constexpr (std::is_same<T, uint32_t>::value) asm("v_cvt_u32_f32 %0, %1" : "=v"(r) : "v"(v));
  else asm("v_cvt_i32_f32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}
template <typename T>
__device__ __forceinline__ float to_f(uint32_t bits) {
  return std::is_same<T, uint32_t>::value ? (float)bits : (float)(int32_t)bits;
}

template <bool DEC>
struct NodeRows {
  using V = typename std::conditional<DEC, uint2, uint4>::type;
  V own, halo;
};
struct OutRows {
  uint4 e1, o0, o1;
  uint2 mv[7];
};

template <bool DEC>
__device__ __forceinline__ uint32_t node(const typename NodeRows<DEC>::V& v, int i) {  // node i of the lane's row
  if constexpr (DEC) return i == 0 ? v.x : v.y;
  else return i == 0 ? v.x : v.z;
}
__device__ __forceinline__ uint32_t odd16(const uint4& v, int i) { return i == 0 ? v.y : v.w; }
__device__ __forceinline__ uint32_t ev16(const uint4& v, int i) { return i == 0 ? v.x : v.z; }

template <typename T, bool DEC, int PL>
__global__ void __launch_bounds__(256) wave3d32_kernel(W32 a) {
  constexpr int VX = 2;
  using NR = NodeRows<DEC>;

  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int tx = lane & (a.txn - 1);
  const int r = lane >> __builtin_ctz(a.txn);
  const int X = tx * VX;
  int blk = (int)blockIdx.x;
  if (a.xcd_per > 0) {
    const int x = blk % 8, k = blk / 8;
    blk = ((k / a.xcd_per) * 8 + x) * a.xcd_per + (k % a.xcd_per);
  }
  const int yg = blk % a.nyg;
  blk /= a.nyg;
  const int pb = blk % a.nslab;
  const int64_t b = blk / a.nslab;
  const int Y0 = (yg * a.nwv + wv) * a.rows;
  if (Y0 >= a.Ey) return;  // a whole idle wave
  const int Y = Y0 + r;
  const bool live = Y < a.Ey;
  const int Yc = live ? Y : a.Ey - 1;
  const int c0 = a.zbegin + pb * PL;
  const int Z1 = a.zend;

  const bool first = r == 0;
  const bool last = r == a.rows - 1 || Y == a.Ey - 1;
  const bool vy1 = Y < a.Lcy;
  const bool vy0 = Y >= 1;
  const bool need_halo = live && ((first && Y0 >= 1) || (last && vy1));
  const int yh = first ? (Y0 >= 1 ? Y0 - 1 : 0) : lsrc(Yc + 1, a.Ly, a.Ey);
  const bool xlast = tx == a.txn - 1;

  const int hplane = a.H * a.W;
  const int lplane = a.Ey * a.Ex;
  const uint32_t* hin = DEC ? nullptr : (const uint32_t*)a.hi_in + b * (int64_t)a.D * hplane;
  uint32_t* hout = DEC ? (uint32_t*)a.hi_out + b * (int64_t)a.D * hplane : nullptr;
  const uint32_t* lin = DEC ? (const uint32_t*)a.lo_in + b * (int64_t)a.Ez * lplane : nullptr;
  const int hx = 2 * X;
  const int ho_own = 2 * Yc * a.W + hx, ho_h = 2 * yh * a.W + hx;
  const int lo_own = Yc * a.Ex + X, lo_h = yh * a.Ex + X;

  const uint32_t* mbase[7];
  int mplane[7];
  bool mok_y[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez, ey = par[1] ? a.Lcy : a.Ey;
    mplane[k] = ey * a.Ex;
    mbase[k] = (const uint32_t*)a.maps.p[k] + b * (int64_t)ez * mplane[k] + Yc * a.Ex + X;
    mok_y[k] = live && (!par[1] || vy1);
  }

  // ---- every load of the block, issued before any use ----
  NR N[PL + 2];  // node planes c0-1+t
  OutRows O[PL];
#pragma unroll
  for (int t = 0; t < PL + 2; ++t) {
    N[t] = NR{};
    const int q = c0 - 1 + t;
    if (q < 0 || (t >= 2 && q - 1 >= Z1)) continue;  // uniform
    const int sz = lsrc(q, a.Lz, a.Ez);
    if constexpr (DEC) {
      const uint32_t* p = lin + sz * lplane;
      if (live) N[t].own = ld8c(p + lo_own);
      if (need_halo) N[t].halo = ld8c(p + lo_h);
    } else {
      const uint32_t* p = hin + 2 * sz * hplane;
      if (live) N[t].own = ld16c(p + ho_own);
      if (need_halo) N[t].halo = ld16c(p + ho_h);
    }
  }
#pragma unroll
  for (int u = 0; u < PL; ++u) {
    O[u] = OutRows{};
    const int q = c0 + u;
    if (q >= Z1) continue;
    const bool vz1 = q < a.Lcz;
    if constexpr (DEC) {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        if (mok_y[k] && (!par[0] || vz1)) O[u].mv[k] = ld8(mbase[k] + q * mplane[k]);
      }
    } else {
      const uint32_t* p = hin + 2 * q * hplane;
      if (live && vy1) O[u].e1 = ld16(p + ho_own + a.W);
      if (live && vz1) O[u].o0 = ld16(p + hplane + ho_own);
      if (live && vz1 && vy1) O[u].o1 = ld16(p + hplane + ho_own + a.W);
    }
  }

  // ---- per node plane: rows Y-1 (A), Y (B), Y+1 (C), each at cols X .. X+VX, as float32 ----
  float FA[PL + 2][VX + 1], FB[PL + 2][VX + 1], FC[PL + 2][VX + 1];
#pragma unroll
  for (int t = 0; t < PL + 2; ++t) {
    uint32_t n[VX + 1], h[VX + 1];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      n[i] = node<DEC>(N[t].own, i);
      h[i] = node<DEC>(N[t].halo, i);
    }
    const uint32_t nx = shdn(n[0], 1), hxx = shdn(h[0], 1);
    n[VX] = xlast ? n[VX - 1] : nx;  // node Ex mirrors Ex-1 (even pad); no cell there otherwise
    h[VX] = xlast ? h[VX - 1] : hxx;
#pragma unroll
    for (int i = 0; i <= VX; ++i) {
      const uint32_t above = shup(n[i], a.txn), below = shdn(n[i], a.txn);
      FB[t][i] = to_f<T>(n[i]);
      FA[t][i] = to_f<T>(first ? h[i] : above);
      FC[t][i] = to_f<T>(last ? h[i] : below);
    }
  }

  // ---- cell means (float32 chain in feature order) of cell plane c0-1+m: rows Y (Mo) / Y-1
  // (Ma), cols X-1 .. X+VX-1 ----
  uint32_t Mo[PL + 1][VX + 1], Ma[PL + 1][VX + 1];
  auto cell_means = [&](int m) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      float so = 0.0f, sa = 0.0f;
#pragma unroll
      for (int dz = 0; dz < 2; ++dz) {
        so += FB[m + dz][i]; so += FB[m + dz][i + 1]; so += FC[m + dz][i]; so += FC[m + dz][i + 1];
        sa += FA[m + dz][i]; sa += FA[m + dz][i + 1]; sa += FB[m + dz][i]; sa += FB[m + dz][i + 1];
      }
      Mo[m][i + 1] = (uint32_t)from_f<T>(so / 8.0f);
      Ma[m][i + 1] = (uint32_t)from_f<T>(sa / 8.0f);
    }
    Mo[m][0] = shup(Mo[m][VX], 1);
    Ma[m][0] = shup(Ma[m][VX], 1);
  };
  cell_means(0);

  bool vx[VX + 1];
  cells_valid<VX>(vx, X, a.Lcx);

#pragma unroll
  for (int u = 0; u < PL; ++u) {
    const int c = c0 + u;
    if (c >= Z1) break;
    cell_means(u + 1);  // all lanes (shuffles), before the idle ones drop out
    if (!live) continue;
    const bool vz1 = c < a.Lcz, vz0 = c >= 1;
    // M[dz][dy][q]: cell (c-1+dz, Y-1+dy, X-1+q) as float32, 0 outside the grid; ok[..] its validity
    float M[2][2][VX + 1];
    bool ok[2][2][VX + 1];
#pragma unroll
    for (int q = 0; q <= VX; ++q) {
      ok[0][0][q] = vz0 && vy0 && vx[q];
      ok[0][1][q] = vz0 && vy1 && vx[q];
      ok[1][0][q] = vz1 && vy0 && vx[q];
      ok[1][1][q] = vz1 && vy1 && vx[q];
      M[0][0][q] = ok[0][0][q] ? to_f<T>(Ma[u][q]) : 0.0f;
      M[0][1][q] = ok[0][1][q] ? to_f<T>(Mo[u][q]) : 0.0f;
      M[1][0][q] = ok[1][0][q] ? to_f<T>(Ma[u + 1][q]) : 0.0f;
      M[1][1][q] = ok[1][1][q] ? to_f<T>(Mo[u + 1][q]) : 0.0f;
    }
    // contributions in the reference's channel order (kmp_aggregate.h map_contribs)
    auto agg2 = [&](float s0, bool k0, float s1, bool k1) -> uint32_t {
      float s = 0.0f;
      s += s0;
      s += s1;
      if (k0 && k1) s *= 0.5f;
      return (uint32_t)from_f<T>(s);
    };
    auto agg4 = [&](float s0, bool k0, float s1, bool k1, float s2, bool k2, float s3, bool k3) -> uint32_t {
      float s = 0.0f;
      s += s0;
      s += s1;
      s += s2;
      s += s3;
      const int cnt = (int)k0 + (int)k1 + (int)k2 + (int)k3;
      if (cnt == 4) s *= 0.25f;
      else if (cnt == 2) s *= 0.5f;
      return (uint32_t)from_f<T>(s);
    };
    uint32_t pred[7][VX];  // LR, UD, FB, C, Z, Y, X
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const int o = i + 1, w = i;  // column X+i / X+i-1
      pred[0][i] = agg2(M[1][1][o], ok[1][1][o], M[1][1][w], ok[1][1][w]);
      pred[1][i] = agg2(M[1][1][o], ok[1][1][o], M[1][0][o], ok[1][0][o]);
      pred[2][i] = agg2(M[1][1][o], ok[1][1][o], M[0][1][o], ok[0][1][o]);
      pred[3][i] = ok[1][1][o] ? Mo[u + 1][o] : 0u;
      pred[4][i] = agg4(M[1][1][o], ok[1][1][o], M[1][1][w], ok[1][1][w], M[1][0][w], ok[1][0][w], M[1][0][o],
                        ok[1][0][o]);
      pred[5][i] = agg4(M[1][1][o], ok[1][1][o], M[1][1][w], ok[1][1][w], M[0][1][w], ok[0][1][w], M[0][1][o],
                        ok[0][1][o]);
      pred[6][i] = agg4(M[1][1][o], ok[1][1][o], M[1][0][o], ok[1][0][o], M[0][0][o], ok[0][0][o], M[0][1][o],
                        ok[0][1][o]);
    }
    if constexpr (!DEC) {
      const uint4 e0 = N[u + 1].own;
      const OutRows& Oc = O[u];
      uint32_t res[7][VX];
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        res[0][i] = ev16(Oc.o1, i) - pred[0][i];   // LR (1,1,0)
        res[1][i] = odd16(Oc.o0, i) - pred[1][i];  // UD (1,0,1)
        res[2][i] = odd16(Oc.e1, i) - pred[2][i];  // FB (0,1,1)
        res[3][i] = odd16(Oc.o1, i) - pred[3][i];  // C  (1,1,1)
        res[4][i] = ev16(Oc.o0, i) - pred[4][i];   // Z  (1,0,0)
        res[5][i] = ev16(Oc.e1, i) - pred[5][i];   // Y  (0,1,0)
        res[6][i] = odd16(e0, i) - pred[6][i];     // X  (0,0,1)
      }
      st8((uint32_t*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, make_uint2(e0.x, e0.z));
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        if (mok_y[k] && (!par[0] || vz1)) st8((uint32_t*)mbase[k] + c * mplane[k], make_uint2(res[k][0], res[k][1]));
      }
    } else {
      const OutRows& Oc = O[u];
      uint32_t dv[7][VX];
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        dv[k][0] = pred[k][0] + Oc.mv[k].x;
        dv[k][1] = pred[k][1] + Oc.mv[k].y;
      }
      const uint2 lo = N[u + 1].own;
      uint32_t* h0 = hout + 2 * c * hplane + ho_own;
      st16(h0, make_uint4(lo.x, dv[6][0], lo.y, dv[6][1]));
      if (vy1) st16(h0 + a.W, make_uint4(dv[5][0], dv[2][0], dv[5][1], dv[2][1]));
      if (vz1) {
        uint32_t* h1 = h0 + hplane;
        st16(h1, make_uint4(dv[4][0], dv[1][0], dv[4][1], dv[1][1]));
        if (vy1) st16(h1 + a.W, make_uint4(dv[0][0], dv[3][0], dv[0][1], dv[3][1]));
      }
    }
  }
}

}  // namespace w32

constexpr int kW32PL = 2;

template <typename T>
static bool wave3d32_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred,
                              const kmp_region* region, w32::W32& a, dim3& grid, dim3& block) {
  constexpr int VX = 2;
  if (!(std::is_same<T, uint32_t>::value || std::is_same<T, int32_t>::value)) return false;
  if (opt(OPT_DISABLE_WAVE, 0) || opt(OPT_DISABLE_FAST, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_MEAN || pred->padding != 0) return false;
  if (g.n[2] % 2 != 0 || (g.n[2] * (int64_t)sizeof(T)) % 16 != 0) return false;
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || txn < 1 || txn > 32 || (txn & (txn - 1)) != 0) return false;
  const int64_t rows = 64 / txn;  // >= 2: a lane is never both its wave's first and last row
  if (g.E[1] % rows == 1) return false;
  const int64_t waves = ceil_div(g.E[1], rows);
  const int64_t nwv = waves < 4 ? waves : 4;
  const int64_t nyg = ceil_div(waves, nwv);
  int64_t zb = 0, ze = g.E[0];
  if (region) {
    if (region->begin[1] > 0 || region->begin[2] > 0 || region->end[1] < g.E[1] || region->end[2] < g.E[2]) return false;
    zb = region->begin[0] < 0 ? 0 : region->begin[0];
    ze = region->end[0] > g.E[0] ? g.E[0] : region->end[0];
    if (ze <= zb) return false;
  }
  a.D = (int)g.n[0]; a.H = (int)g.n[1]; a.W = (int)g.n[2];
  a.Lz = (int)g.L[0]; a.Ly = (int)g.L[1]; a.Lx = (int)g.L[2];
  a.Ez = (int)g.E[0]; a.Ey = (int)g.E[1]; a.Ex = (int)g.E[2];
  a.Lcz = (int)g.Lc[0]; a.Lcy = (int)g.Lc[1]; a.Lcx = (int)g.Lc[2];
  a.txn = (int)txn; a.rows = (int)rows; a.nwv = (int)nwv; a.nyg = (int)nyg;
  a.zbegin = (int)zb;
  a.zend = (int)ze;
  const int64_t nslab = ceil_div(ze - zb, (int64_t)kW32PL);
  a.nslab = (int)nslab;
  const int64_t nblk = B * nslab * nyg;
  a.xcd_per = (opt(OPT_W3_XCD, 1) && B % 8 == 0) ? (int)(nslab * nyg) : 0;
  grid = dim3((unsigned)nblk);
  block = dim3((unsigned)(64 * nwv));
  return nblk < ((int64_t)1 << 31);
}

template <typename T>
int try_wave3d32_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                        const MapPtrs& maps, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint32_t>::value || std::is_same<T, int32_t>::value) {
    w32::W32 a{};
    dim3 grid, block;
    if (!wave3d32_geometry<T>(g, B, C, pred, region, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    w32::wave3d32_kernel<T, false, kW32PL><<<grid, block, 0, stream>>>(a);
    return check_launch("wave3d32_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_wave3d32_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                        const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint32_t>::value || std::is_same<T, int32_t>::value) {
    w32::W32 a{};
    dim3 grid, block;
    if (!wave3d32_geometry<T>(g, B, C, pred, region, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    w32::wave3d32_kernel<T, true, kW32PL><<<grid, block, 0, stream>>>(a);
    return check_launch("wave3d32_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_W32_INST(T)                                                                                   \
  template int try_wave3d32_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,   \
                                      const MapPtrs&, const kmp_region*, hipStream_t);                    \
  template int try_wave3d32_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,            \
                                      const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_W32_INST(uint8_t)
KMP_W32_INST(uint16_t)
KMP_W32_INST(int32_t)
KMP_W32_INST(uint32_t)

}  // namespace kmp
