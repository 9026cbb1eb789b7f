// kmp_codec_wave3dp.hip -- one-pass volume encode / decode for the mean predictor with p = 1, 2
// (BASELINE config C3 "also report p = 1"; SURVEY.md §8a a7-a11 fused).
//
// The data movement of kmp_codec_wave3d.hip (p = 0) carried over to wider neighbourhoods:
//   * a workgroup owns PL = 2 consecutive output planes of one tile, issues every global load of
//     its planes up front (node rows of the PL + 2p + 2 node planes c0-1-p .. c0+PL+p, then the
//     stream rows of its PL output planes) and computes with no LDS and no barrier;
//   * tile-per-XCD block order, so the z-halo node planes a workgroup shares with its neighbours
//     are L2 hits (default-policy loads), while the once-touched stream rows are non-temporal.
// The (2p+2)^3 neighbourhood mean (features_from_lowres + the test predictor's f32 mean and
// truncating cast, volume/utils.py:199-218, tests/volume/test_encode_decode.py:46-51) is a box
// sum, evaluated separably in the order that keeps the exchange cheapest:
//   z -- in-lane: each lane holds its node row of every node plane;
//   x -- 2p+1 cross-lane shuffles of element values (left p, right p+1), mirrored in-lane at the
//        row ends (symmetric neighbourhood pad over the even reflect pad, volume/utils.py:213-237);
//   y -- over the wave's rows by shuffles of the x sums; the p+1 rows above and below the wave
//        are loaded by the wave's first / last p+1 rows (one halo row per lane, rows >= 2p+2).
// floor(sum / (2p+2)^3) equals the f32 mean + truncation for u8/u16 (the sum is exact in f32 and
// 1/N > half an ulp of the quotient).  The 19-way aggregation and the coder are the p = 0
// kernel's (volume/utils.py:83-155, utils.py:38-55).
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace w3p {

using namespace wv;

struct W3P {
  const void* hi_in;  // encode input
  void* hi_out;       // decode output
  const void* lo_in;  // decode input
  void* lo_out;       // encode output
  MapPtrs maps;
  int32_t D, H, W;
  int32_t Lz, Ly, Lx, Ez, Ey, Ex, Lcz, Lcy, Lcx;
  int32_t nslab, zbegin, zend;
  int32_t txn, rows, nwv, nyg;
  int32_t xcd_per;  // > 0: tile-per-XCD block order (blocks per tile), 0: identity
  int32_t zrun;     // wave3dr_kernel: output planes per workgroup (even)
};

template <bool DEC>
struct NodeRow {
  using V = typename std::conditional<DEC, uint2, uint4>::type;
  V own, halo;
};
struct OutRows {
  uint4 e1, o0, o1;  // encode: plane 2q row 2Y+1, plane 2q+1 rows 2Y, 2Y+1
  uint2 mv[7];       // decode: the 7 residual rows
};

template <typename T, bool DEC>
__device__ __forceinline__ uint32_t node_el(const typename NodeRow<DEC>::V& v, int i) {
  if constexpr (DEC) return el8<T>(v, i);
  else return el16<T>(v, 2 * i);
}

// WPE: the amdgpu_waves_per_eu register budget (1 = the compiler's choice)
template <typename T, bool DEC, int P, int PL, int WPE, bool STC = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) wave3dp_kernel(W3P a) {
  constexpr int VX = 8 / (int)sizeof(T);
  constexpr int NB = 2 * P + 2;     // neighbourhood extent per axis
  constexpr int NP = PL + NB;       // node planes c0-1-P .. c0+PL+P
  constexpr uint32_t NN = NB * NB * NB;
  constexpr int NE = VX + 2 * P + 1;  // x-extended row: nodes X-P .. X+VX+P
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  using NR = NodeRow<DEC>;

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
  if (Y0 >= a.Ey) return;  // a whole idle wave: nothing in this kernel waits on it
  const int Y = Y0 + r;
  const bool live = Y < a.Ey;
  const int c0 = a.zbegin + pb * PL;
  const int Z1 = a.zend;
  const int rows = a.rows;

  // rows this lane loads: its own (mirrored past the volume's end, so that the wave's rows are
  // always the virtual rows Y0 .. Y0+rows-1) and, on the first / last P+1 rows, one halo row
  const int ysrc = live ? Y : lsrc(Y, a.Ly, a.Ey);
  const bool hup = r <= P, hdn = r >= rows - P - 1;
  const int hrow = hup ? Y0 - P - 1 + r : Y0 + rows + (r - (rows - P - 1));
  const int hsrc = lsrc(hrow, a.Ly, a.Ey);
  const bool has_halo = hup || hdn;

  const bool vy1 = Y < a.Lcy;
  const bool vy0 = Y >= 1;
  const bool xfirst = tx == 0, xlast = tx == a.txn - 1;
  const bool xdims = a.Lx != a.Ex;

  const int hplane = a.H * a.W;
  const int lplane = a.Ey * a.Ex;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * (int64_t)a.D * hplane;
  T* hout = DEC ? (T*)a.hi_out + b * (int64_t)a.D * hplane : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ez * lplane : nullptr;
  const int hx = 2 * X;
  const int ho_own = 2 * ysrc * a.W + hx, ho_halo = 2 * hsrc * a.W + hx;
  const int lo_own = ysrc * a.Ex + X, lo_halo = hsrc * a.Ex + X;

  const T* mbase[7];
  int mplane[7];
  bool mok_y[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez, ey = par[1] ? a.Lcy : a.Ey;
    mplane[k] = ey * a.Ex;
    mbase[k] = (const T*)a.maps.p[k] + b * (int64_t)ez * mplane[k] + (live ? Y : 0) * a.Ex + X;
    mok_y[k] = live && (!par[1] || vy1);
  }

  // cell planes c0-1+m, m = 0..mmax, are the ones the block's output planes read
  const int mmax = (Z1 - c0) < PL ? (Z1 - c0) : PL;

  // ---- every load of the block, issued before any use ----
  NR N[NP];  // node planes c0-1-P+t
#pragma unroll
  for (int t = 0; t < NP; ++t) {
    N[t] = NR{};
    if (t > mmax + NB - 1) continue;  // uniform: feeds no computed cell plane
    const int sz = lsrc(c0 - 1 - P + t, a.Lz, a.Ez);
    if constexpr (DEC) {
      const T* p = lin + sz * lplane;
      N[t].own = ld8c(p + lo_own);
      if (has_halo) N[t].halo = ld8c(p + lo_halo);
    } else {
      const T* p = hin + 2 * sz * hplane;
      N[t].own = ld16c(p + ho_own);
      if (has_halo) N[t].halo = ld16c(p + ho_halo);
    }
  }
  OutRows O[PL];
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
      const T* p = hin + 2 * q * hplane;
      if (live && vy1) O[u].e1 = ld16(p + ho_own + a.W);
      if (live && vz1) O[u].o0 = ld16(p + hplane + ho_own);
      if (live && vz1 && vy1) O[u].o1 = ld16(p + hplane + ho_own + a.W);
    }
  }

  // x box sum of one row's z sums: nodes X+i-P .. X+i+P+1 for the lane's VX cells
  auto xbox = [&](const uint32_t (&z)[VX], uint32_t (&out)[VX]) __attribute__((always_inline)) {
    uint32_t e[NE];
#pragma unroll
    for (int k = 0; k < P; ++k) {  // left neighbour's last P elements; mirrored at the row start
      const uint32_t s = shup(z[VX - P + k], 1);
      e[k] = xfirst ? z[P - 1 - k] : s;
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) e[P + i] = z[i];
#pragma unroll
    for (int k = 0; k <= P; ++k) {  // right neighbour's first P+1 elements; mirrored at the row end
      const uint32_t s = shdn(z[k], 1);
      e[P + VX + k] = xlast ? (xdims ? z[VX - 1] : z[VX - 1 - k]) : s;
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      uint32_t acc = 0;
#pragma unroll
      for (int k = 0; k < NB; ++k) acc += e[i + k];
      out[i] = acc;
    }
  };

  // cell means of cell plane c0-1+m for rows Y (Mo) and Y-1 (Ma), cols X-1 .. X+VX-1
  uint32_t Mo[PL + 1][VX + 1], Ma[PL + 1][VX + 1];
  auto cell_means = [&](int m) __attribute__((always_inline)) {
    uint32_t zo[VX], zh[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      uint32_t so = 0, sh = 0;
#pragma unroll
      for (int dz = 0; dz < NB; ++dz) {
        so += node_el<T, DEC>(N[m + dz].own, i);
        sh += node_el<T, DEC>(N[m + dz].halo, i);
      }
      zo[i] = so;
      zh[i] = sh;
    }
    uint32_t xo[VX], xh[VX];
    xbox(zo, xo);
    xbox(zh, xh);
    uint32_t so[VX], su[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) so[i] = su[i] = 0;
#pragma unroll
    for (int d = -P - 1; d <= P + 1; ++d) {
      const int j = r + d;  // virtual row Y0 + j
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        uint32_t v = d == 0 ? xo[i] : (d < 0 ? shup(xo[i], -d * a.txn) : shdn(xo[i], d * a.txn));
        if (d < 0) {
          const uint32_t h = d == -P - 1 ? xh[i] : shdn(xh[i], (d + P + 1) * a.txn);
          v = j < 0 ? h : v;
        } else if (d > 0) {
          const uint32_t h = d == P + 1 ? xh[i] : shup(xh[i], (P + 1 - d) * a.txn);
          v = j >= rows ? h : v;
        }
        if (d >= -P) so[i] += v;
        if (d <= P) su[i] += v;
      }
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      Mo[m][i + 1] = so[i] / NN;
      Ma[m][i + 1] = su[i] / NN;
    }
    Mo[m][0] = shup(Mo[m][VX], 1);
    Ma[m][0] = shup(Ma[m][VX], 1);
  };
  cell_means(0);

  bool vx[VX + 1];
  cells_valid<VX>(vx, X, a.Lcx);
  const uint32_t ny = (uint32_t)vy0 + (uint32_t)vy1;

#pragma unroll
  for (int u = 0; u < PL; ++u) {
    const int c = c0 + u;
    if (c >= Z1) break;
    cell_means(u + 1);  // all lanes (shuffles), before the idle ones drop out
    if (!live) continue;
    const bool vz1 = c < a.Lcz, vz0 = c >= 1;
    uint32_t M[2][2][VX + 1];
#pragma unroll
    for (int q = 0; q <= VX; ++q) {
      M[0][0][q] = (vz0 && vy0 && vx[q]) ? Ma[u][q] : 0u;
      M[0][1][q] = (vz0 && vy1 && vx[q]) ? Mo[u][q] : 0u;
      M[1][0][q] = (vz1 && vy0 && vx[q]) ? Ma[u + 1][q] : 0u;
      M[1][1][q] = (vz1 && vy1 && vx[q]) ? Mo[u + 1][q] : 0u;
    }
    const uint32_t nz = (uint32_t)vz0 + (uint32_t)vz1;
    uint32_t pred[7][VX];  // LR, UD, FB, C, Z, Y, X
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
      pred[0][i] = (M[1][1][i] + M[1][1][i + 1]) >> (nx >> 1);
      pred[1][i] = (M[1][0][i + 1] + M[1][1][i + 1]) >> (ny >> 1);
      pred[2][i] = (M[0][1][i + 1] + M[1][1][i + 1]) >> (nz >> 1);
      pred[3][i] = M[1][1][i + 1];
      pred[4][i] = (M[1][0][i] + M[1][0][i + 1] + M[1][1][i] + M[1][1][i + 1]) >> ((ny * nx) >> 1);
      pred[5][i] = (M[0][1][i] + M[0][1][i + 1] + M[1][1][i] + M[1][1][i + 1]) >> ((nz * nx) >> 1);
      pred[6][i] = (M[0][0][i + 1] + M[0][1][i + 1] + M[1][0][i + 1] + M[1][1][i + 1]) >> ((nz * ny) >> 1);
    }
    const auto& own = N[u + 1 + P].own;  // node plane c
    if constexpr (!DEC) {
      const OutRows& Oc = O[u];
      uint32_t res[7][VX], lov[VX];
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        lov[i] = el16<T>(own, 2 * i);
        res[0][i] = (el16<T>(Oc.o1, 2 * i) - pred[0][i]) & MASK;      // LR (1,1,0)
        res[1][i] = (el16<T>(Oc.o0, 2 * i + 1) - pred[1][i]) & MASK;  // UD (1,0,1)
        res[2][i] = (el16<T>(Oc.e1, 2 * i + 1) - pred[2][i]) & MASK;  // FB (0,1,1)
        res[3][i] = (el16<T>(Oc.o1, 2 * i + 1) - pred[3][i]) & MASK;  // C  (1,1,1)
        res[4][i] = (el16<T>(Oc.o0, 2 * i) - pred[4][i]) & MASK;      // Z  (1,0,0)
        res[5][i] = (el16<T>(Oc.e1, 2 * i) - pred[5][i]) & MASK;      // Y  (0,1,0)
        res[6][i] = (el16<T>(own, 2 * i + 1) - pred[6][i]) & MASK;    // X  (0,0,1)
      }
      stp8<STC>((T*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, pack8<T, VX>(lov));
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        if (mok_y[k] && (!par[0] || vz1)) stp8<STC>((T*)mbase[k] + c * mplane[k], pack8<T, VX>(res[k]));
      }
    } else {
      const OutRows& Oc = O[u];
      uint32_t lov[VX], dv[7][VX];
#pragma unroll
      for (int i = 0; i < VX; ++i) lov[i] = el8<T>(own, i);
#pragma unroll
      for (int k = 0; k < 7; ++k)
#pragma unroll
        for (int i = 0; i < VX; ++i) dv[k][i] = (pred[k][i] + el8<T>(Oc.mv[k], i)) & MASK;
      T* h0 = hout + 2 * c * hplane + ho_own;
      st16(h0, pack16<T, VX>(lov, dv[6]));
      if (vy1) st16(h0 + a.W, pack16<T, VX>(dv[5], dv[2]));
      if (vz1) {
        T* h1 = h0 + hplane;
        st16(h1, pack16<T, VX>(dv[4], dv[1]));
        if (vy1) st16(h1 + a.W, pack16<T, VX>(dv[0], dv[3]));
      }
    }
  }
}

// ---- z-rolling variant: a workgroup owns a run of ZR consecutive output planes of one tile and
// keeps the z box sums of its rows in registers.  Going from cell plane m-1 to m adds node plane
// m+P+1 and subtracts node plane m-1-P (integer sums: exact), so each output plane loads 2 node
// rows per lane (plus the halo rows) instead of 2P+3, and the loads of output plane c+1 are issued
// before plane c is computed.  The x / y sums, the means, the 19-way aggregation and the coder
// are the plane-block kernel's above.
template <bool DEC>
struct RollStep {
  typename NodeRow<DEC>::V add_own, add_halo, cur;  // cur: node plane c's own row
  OutRows o;
};

// the VX node values of a lane's row segment packed into 8 bytes: the decode's lowres row as
// loaded; the encode's highres row keeps its even elements (one byte permute per dword)
template <typename T>
__device__ __forceinline__ uint2 node_bytes(const uint2& v) { return v; }
template <typename T>
__device__ __forceinline__ uint2 node_bytes(const uint4& v) {
  constexpr uint32_t sel = sizeof(T) == 2 ? 0x05040100u : 0x06040200u;
  return make_uint2(__builtin_amdgcn_perm(v.y, v.x, sel), __builtin_amdgcn_perm(v.w, v.z, sel));
}

template <typename T, bool DEC, int P, bool STC = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sizeof(T) == 2 ? 3 : 1)))
wave3dr_kernel(W3P a) {
  constexpr int PD = 1;  // prefetch distance in output planes (2 measured no faster: r2ar)
  constexpr int VX = 8 / (int)sizeof(T);
  constexpr int NB = 2 * P + 2;
  constexpr uint32_t NN = NB * NB * NB;
  constexpr int NE = VX + 2 * P + 1;
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  using V = typename NodeRow<DEC>::V;

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
  if (Y0 >= a.Ey) return;
  const int Y = Y0 + r;
  const bool live = Y < a.Ey;
  const int c0 = a.zbegin + pb * a.zrun;
  const int Z1 = a.zend;
  const int c1 = c0 + a.zrun < Z1 ? c0 + a.zrun : Z1;
  const int rows = a.rows;

  const int ysrc = live ? Y : lsrc(Y, a.Ly, a.Ey);
  const bool hup = r <= P, hdn = r >= rows - P - 1;
  const int hrow = hup ? Y0 - P - 1 + r : Y0 + rows + (r - (rows - P - 1));
  const int hsrc = lsrc(hrow, a.Ly, a.Ey);
  const bool has_halo = hup || hdn;
  const bool vy1 = Y < a.Lcy;
  const bool vy0 = Y >= 1;
  const bool xfirst = tx == 0, xlast = tx == a.txn - 1;
  const bool xdims = a.Lx != a.Ex;

  const int hplane = a.H * a.W;
  const int lplane = a.Ey * a.Ex;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * (int64_t)a.D * hplane;
  T* hout = DEC ? (T*)a.hi_out + b * (int64_t)a.D * hplane : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ez * lplane : nullptr;
  const int hx = 2 * X;
  const int ho_own = 2 * ysrc * a.W + hx, ho_halo = 2 * hsrc * a.W + hx;
  const int lo_own = ysrc * a.Ex + X, lo_halo = hsrc * a.Ex + X;

  const T* mbase[7];
  int mplane[7];
  bool mok_y[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez, ey = par[1] ? a.Lcy : a.Ey;
    mplane[k] = ey * a.Ex;
    mbase[k] = (const T*)a.maps.p[k] + b * (int64_t)ez * mplane[k] + (live ? Y : 0) * a.Ex + X;
    mok_y[k] = live && (!par[1] || vy1);
  }

  auto load_node = [&](int t, V& own, V& halo) __attribute__((always_inline)) {
    const int sz = lsrc(t, a.Lz, a.Ez);
    if constexpr (DEC) {
      const T* p = lin + sz * lplane;
      own = ld8c(p + lo_own);
      halo = has_halo ? ld8c(p + lo_halo) : V{};
    } else {
      const T* p = hin + 2 * sz * hplane;
      own = ld16c(p + ho_own);
      halo = has_halo ? ld16c(p + ho_halo) : V{};
    }
  };
  auto load_out = [&](int q, OutRows& O) __attribute__((always_inline)) {
    O = OutRows{};
    const bool vz1 = q < a.Lcz;
    if constexpr (DEC) {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        if (mok_y[k] && (!par[0] || vz1)) O.mv[k] = ld8(mbase[k] + q * mplane[k]);
      }
    } else {
      const T* p = hin + 2 * q * hplane;
      if (live && vy1) O.e1 = ld16(p + ho_own + a.W);
      if (live && vz1) O.o0 = ld16(p + hplane + ho_own);
      if (live && vz1 && vy1) O.o1 = ld16(p + hplane + ho_own + a.W);
    }
  };
  // step for output plane c: add node plane c+P+1, subtract c-1-P (the z sums move from cell
  // plane c-1 to c), node plane c's own row (the lowres / X map samples), the stream rows
  auto load_step = [&](int c, RollStep<DEC>& S) __attribute__((always_inline)) {
    load_node(c + P + 1, S.add_own, S.add_halo);
    if constexpr (DEC) S.cur = ld8c(lin + c * lplane + lo_own);
    else S.cur = ld16c(hin + 2 * c * hplane + ho_own);
    load_out(c, S.o);
  };

  // The node values a step subtracts (node plane c-1-P, own and halo row) are the ones step
  // c - (2P+2) added: each lane keeps its own in an LDS ring of 2P+2 slots (slot c mod 2P+2, read
  // before the step overwrites it with plane c+P+1's), so a node row is read from memory once per
  // run instead of twice -- no cross-lane traffic, no barrier (a lane reads back its own bytes)
  __shared__ __attribute__((aligned(16))) uint4 zring[NB][256];
  uint4* const zr = &zring[0][threadIdx.x];
  // z sums of cell plane c0-1 (node planes c0-1-P .. c0+P): the prologue's 2P+2 planes
  uint32_t zo[VX], zh[VX];
#pragma unroll
  for (int i = 0; i < VX; ++i) zo[i] = zh[i] = 0;
  RollStep<DEC> S[PD + 1];
  int zslot = c0 % NB;  // c mod NB
  {
    V own[NB], halo[NB];
#pragma unroll
    for (int t = 0; t < NB; ++t) load_node(c0 - 1 - P + t, own[t], halo[t]);
#pragma unroll
    for (int k = 0; k < PD; ++k)
      if (c0 + k < c1) load_step(c0 + k, S[k]);
#pragma unroll
    for (int t = 0; t < NB; ++t) {
      const uint2 no = node_bytes<T>(own[t]), nh = node_bytes<T>(halo[t]);
      // prologue plane t is the one step c0 + t subtracts
      const int sl = zslot + t < NB ? zslot + t : zslot + t - NB;
      zr[sl * 256] = make_uint4(no.x, no.y, nh.x, nh.y);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        zo[i] += el8<T>(no, i);
        zh[i] += el8<T>(nh, i);
      }
    }
  }

  auto xbox = [&](const uint32_t (&z)[VX], uint32_t (&out)[VX]) __attribute__((always_inline)) {
    uint32_t e[NE];
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const uint32_t s = shup(z[VX - P + k], 1);
      e[k] = xfirst ? z[P - 1 - k] : s;
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) e[P + i] = z[i];
#pragma unroll
    for (int k = 0; k <= P; ++k) {
      const uint32_t s = shdn(z[k], 1);
      e[P + VX + k] = xlast ? (xdims ? z[VX - 1] : z[VX - 1 - k]) : s;
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      uint32_t acc = 0;
#pragma unroll
      for (int k = 0; k < NB; ++k) acc += e[i + k];
      out[i] = acc;
    }
  };
  // cell means of the cell plane whose z sums are zo / zh, rows Y (Mo) and Y-1 (Ma)
  auto cell_means = [&](uint32_t (&Mo)[VX + 1], uint32_t (&Ma)[VX + 1]) __attribute__((always_inline)) {
    uint32_t xo[VX], xh[VX];
    xbox(zo, xo);
    xbox(zh, xh);
    uint32_t so[VX], su[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) so[i] = su[i] = 0;
#pragma unroll
    for (int d = -P - 1; d <= P + 1; ++d) {
      const int j = r + d;
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        uint32_t v = d == 0 ? xo[i] : (d < 0 ? shup(xo[i], -d * a.txn) : shdn(xo[i], d * a.txn));
        if (d < 0) {
          const uint32_t h = d == -P - 1 ? xh[i] : shdn(xh[i], (d + P + 1) * a.txn);
          v = j < 0 ? h : v;
        } else if (d > 0) {
          const uint32_t h = d == P + 1 ? xh[i] : shup(xh[i], (P + 1 - d) * a.txn);
          v = j >= rows ? h : v;
        }
        if (d >= -P) so[i] += v;
        if (d <= P) su[i] += v;
      }
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      Mo[i + 1] = so[i] / NN;
      Ma[i + 1] = su[i] / NN;
    }
    Mo[0] = shup(Mo[VX], 1);
    Ma[0] = shup(Ma[VX], 1);
  };
  uint32_t Mo[2][VX + 1], Ma[2][VX + 1];  // [0]: cell plane c-1, [1]: cell plane c
  cell_means(Mo[0], Ma[0]);

  bool vx[VX + 1];
  cells_valid<VX>(vx, X, a.Lcx);
  const uint32_t ny = (uint32_t)vy0 + (uint32_t)vy1;

  // one output plane: Sc holds its loads; plane c+PD's loads go into Sn first
  auto step = [&](int c, RollStep<DEC>& Sc, RollStep<DEC>& Sn) __attribute__((always_inline)) {
    if (c + PD < c1) load_step(c + PD, Sn);  // in flight during planes c .. c+PD-1
    {
      const uint4 sub = zr[zslot * 256];  // node plane c-1-P, added by step c - NB
      const uint2 ao = node_bytes<T>(Sc.add_own), ah = node_bytes<T>(Sc.add_halo);
      zr[zslot * 256] = make_uint4(ao.x, ao.y, ah.x, ah.y);
      zslot = zslot + 1 < NB ? zslot + 1 : 0;
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        zo[i] += el8<T>(ao, i) - el8<T>(make_uint2(sub.x, sub.y), i);
        zh[i] += el8<T>(ah, i) - el8<T>(make_uint2(sub.z, sub.w), i);
      }
    }
    cell_means(Mo[1], Ma[1]);  // all lanes (shuffles)
    if (live) {
      const bool vz1 = c < a.Lcz, vz0 = c >= 1;
      uint32_t M[2][2][VX + 1];
#pragma unroll
      for (int q = 0; q <= VX; ++q) {
        M[0][0][q] = (vz0 && vy0 && vx[q]) ? Ma[0][q] : 0u;
        M[0][1][q] = (vz0 && vy1 && vx[q]) ? Mo[0][q] : 0u;
        M[1][0][q] = (vz1 && vy0 && vx[q]) ? Ma[1][q] : 0u;
        M[1][1][q] = (vz1 && vy1 && vx[q]) ? Mo[1][q] : 0u;
      }
      const uint32_t nz = (uint32_t)vz0 + (uint32_t)vz1;
      uint32_t pred[7][VX];  // LR, UD, FB, C, Z, Y, X
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pred[0][i] = (M[1][1][i] + M[1][1][i + 1]) >> (nx >> 1);
        pred[1][i] = (M[1][0][i + 1] + M[1][1][i + 1]) >> (ny >> 1);
        pred[2][i] = (M[0][1][i + 1] + M[1][1][i + 1]) >> (nz >> 1);
        pred[3][i] = M[1][1][i + 1];
        pred[4][i] = (M[1][0][i] + M[1][0][i + 1] + M[1][1][i] + M[1][1][i + 1]) >> ((ny * nx) >> 1);
        pred[5][i] = (M[0][1][i] + M[0][1][i + 1] + M[1][1][i] + M[1][1][i + 1]) >> ((nz * nx) >> 1);
        pred[6][i] = (M[0][0][i + 1] + M[0][1][i + 1] + M[1][0][i + 1] + M[1][1][i + 1]) >> ((nz * ny) >> 1);
      }
      const OutRows& Oc = Sc.o;
      if constexpr (!DEC) {
        const uint4 own = Sc.cur;
        uint32_t res[7][VX], lov[VX];
#pragma unroll
        for (int i = 0; i < VX; ++i) {
          lov[i] = el16<T>(own, 2 * i);
          res[0][i] = (el16<T>(Oc.o1, 2 * i) - pred[0][i]) & MASK;      // LR (1,1,0)
          res[1][i] = (el16<T>(Oc.o0, 2 * i + 1) - pred[1][i]) & MASK;  // UD (1,0,1)
          res[2][i] = (el16<T>(Oc.e1, 2 * i + 1) - pred[2][i]) & MASK;  // FB (0,1,1)
          res[3][i] = (el16<T>(Oc.o1, 2 * i + 1) - pred[3][i]) & MASK;  // C  (1,1,1)
          res[4][i] = (el16<T>(Oc.o0, 2 * i) - pred[4][i]) & MASK;      // Z  (1,0,0)
          res[5][i] = (el16<T>(Oc.e1, 2 * i) - pred[5][i]) & MASK;      // Y  (0,1,0)
          res[6][i] = (el16<T>(own, 2 * i + 1) - pred[6][i]) & MASK;    // X  (0,0,1)
        }
        stp8<STC>((T*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, pack8<T, VX>(lov));
#pragma unroll
        for (int k = 0; k < 7; ++k) {
          int par[3];
          map_parity(3, k, par);
          if (mok_y[k] && (!par[0] || vz1)) stp8<STC>((T*)mbase[k] + c * mplane[k], pack8<T, VX>(res[k]));
        }
      } else {
        const uint2 own = Sc.cur;
        uint32_t lov[VX], dv[7][VX];
#pragma unroll
        for (int i = 0; i < VX; ++i) lov[i] = el8<T>(own, i);
#pragma unroll
        for (int k = 0; k < 7; ++k)
#pragma unroll
          for (int i = 0; i < VX; ++i) dv[k][i] = (pred[k][i] + el8<T>(Oc.mv[k], i)) & MASK;
        T* h0 = hout + 2 * c * hplane + ho_own;
        st16(h0, pack16<T, VX>(lov, dv[6]));
        if (vy1) st16(h0 + a.W, pack16<T, VX>(dv[5], dv[2]));
        if (vz1) {
          T* h1 = h0 + hplane;
          st16(h1, pack16<T, VX>(dv[4], dv[1]));
          if (vy1) st16(h1 + a.W, pack16<T, VX>(dv[0], dv[3]));
        }
      }
    }
#pragma unroll
    for (int q = 0; q <= VX; ++q) {
      Mo[0][q] = Mo[1][q];
      Ma[0][q] = Ma[1][q];
    }
  };
  // PD+1 planes per iteration so the step buffers are addressed statically (no register indexing)
#pragma unroll 1
  for (int c = c0; c < c1; c += PD + 1) {
#pragma unroll
    for (int k = 0; k <= PD; ++k)
      if (c + k < c1) step(c + k, S[k], S[(k + PD) % (PD + 1)]);
  }
}

}  // namespace w3p

// ------------------------------------------------------------------------------------------
// Host: eligibility + launch geometry
// ------------------------------------------------------------------------------------------
// Output planes per workgroup and register budget, per (p, direction): the measured optimum at C3
// (profiles/round1/w3p_sweep.log; 64^3 u16 tiles): p = 1 PL 2 (decode at 4 waves / SIMD),
// p = 2 encode PL 1, decode PL 2 at 3 waves / SIMD.  8-bit samples (8 cells a lane) spill under
// those decode budgets (100-508 bytes of scratch, decode 2.2x the encode's time): the compiler's
// own budget there, and PL 1 at p = 2 (C3-geometry u8 decode p = 1 159 -> 73 us, p = 2 227 -> 106 us,
// profiles/round6/w3p_u8_r6o.log).  KMP_W3P_PL overrides the planes.
static void w3p_cfg(int P, bool dec, int bytes, int& pl, int& wpe) {
  pl = (P == 2 && (!dec || bytes == 1)) ? 1 : 2;
  wpe = dec && bytes == 2 ? (P == 1 ? 4 : 3) : 1;
  pl = opt(OPT_W3P_PL, pl) == 1 ? 1 : 2;
}

template <typename T>
static bool wave3dp_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred,
                             const kmp_region* region, int pl, w3p::W3P& a, dim3& grid, dim3& block) {
  constexpr int VX = 8 / (int)sizeof(T);
  if (!(std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value)) return false;
  if (opt(OPT_DISABLE_WAVE, 0) || opt(OPT_DISABLE_FAST, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_MEAN || pred->padding < 1 || pred->padding > 2) return false;
  const int P = pred->padding;
  if (g.n[2] % 2 != 0 || (g.n[2] * (int64_t)sizeof(T)) % 16 != 0) return false;
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;  // 32-bit offsets inside a tile
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || txn < 1 || txn > 64 || (txn & (txn - 1)) != 0) return false;
  const int64_t rows = 64 / txn;
  if (rows < 2 * P + 2) return false;  // one halo row per lane
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
  const int64_t nslab = ceil_div(ze - zb, (int64_t)pl);
  a.nslab = (int)nslab;
  const int64_t nblk = B * nslab * nyg;
  a.xcd_per = (opt(OPT_W3_XCD, 1) && B % 8 == 0) ? (int)(nslab * nyg) : 0;
  grid = dim3((unsigned)nblk);
  block = dim3((unsigned)(64 * nwv));
  return nblk < ((int64_t)1 << 31);
}

// z-rolling kernel (wave3dr_kernel): runs of 8 output planes per workgroup for p = 2 with 16-bit
// samples (C3: 151 / 127 -> 124 / 108 us per direction, profiles/round2/ab_wave3dr.log); 0 = the
// plane-block kernel, which stays faster for p = 1 (91 / 91 vs 112 / 106) and serves 8-bit samples
static int w3p_roll(int P, int bytes) { return P == 2 && bytes == 2 ? 8 : 0; }

// the encode's lowres / map stores, chosen on the pipelines that follow an encode at C3
// (tools/pipeline_rows.py, profiles/round3/pipeline_store_policy_r3.log; DESIGN §5 "pipeline"):
// p = 1 non-temporal (encodes back to back 103 -> 91 us, encode -> Rice pack and Rice unpack ->
// decode within 1-4 us either way); p = 2 cached, MALL-allocating (stp8 in kmp_wave.h: back to back
// the same, encode -> Rice pack -13 us, encode -> decode -35 us).  KMP_W3P_ST_ENC=0 / 1 forces one
static bool w3p_stc(bool dec, int P) { return !dec && opt(OPT_W3P_ST_ENC, P == 2 ? 1 : 0); }

template <typename T, bool DEC, bool STC>
static void launch_wave3dr_s(int P, dim3 grid, dim3 block, hipStream_t stream, const w3p::W3P& a) {
  (void)P;  // p = 2 only (w3p_roll)
  w3p::wave3dr_kernel<T, DEC, 2, STC><<<grid, block, 0, stream>>>(a);
}
template <typename T, bool DEC>
static void launch_wave3dr(int P, dim3 grid, dim3 block, hipStream_t stream, const w3p::W3P& a) {
  if (w3p_stc(DEC, P)) launch_wave3dr_s<T, DEC, true>(P, grid, block, stream, a);
  else launch_wave3dr_s<T, DEC, false>(P, grid, block, stream, a);
}

template <typename T, bool DEC, bool STC>
static void launch_wave3dp_s(int P, int pl, int wpe, dim3 grid, dim3 block, hipStream_t stream, const w3p::W3P& a) {
  if (P == 1) {
    if (pl == 1) {
      if (wpe == 4) w3p::wave3dp_kernel<T, DEC, 1, 1, 4, STC><<<grid, block, 0, stream>>>(a);
      else w3p::wave3dp_kernel<T, DEC, 1, 1, 1, STC><<<grid, block, 0, stream>>>(a);
    } else {
      if (wpe == 4) w3p::wave3dp_kernel<T, DEC, 1, 2, 4, STC><<<grid, block, 0, stream>>>(a);
      else w3p::wave3dp_kernel<T, DEC, 1, 2, 1, STC><<<grid, block, 0, stream>>>(a);
    }
  } else {
    if (pl == 1) {
      if (wpe == 3) w3p::wave3dp_kernel<T, DEC, 2, 1, 3, STC><<<grid, block, 0, stream>>>(a);
      else w3p::wave3dp_kernel<T, DEC, 2, 1, 1, STC><<<grid, block, 0, stream>>>(a);
    } else {
      if (wpe == 3) w3p::wave3dp_kernel<T, DEC, 2, 2, 3, STC><<<grid, block, 0, stream>>>(a);
      else w3p::wave3dp_kernel<T, DEC, 2, 2, 1, STC><<<grid, block, 0, stream>>>(a);
    }
  }
}

template <typename T, bool DEC>
static void launch_wave3dp(int P, int pl, int wpe, dim3 grid, dim3 block, hipStream_t stream, const w3p::W3P& a) {
  if (w3p_stc(DEC, P)) launch_wave3dp_s<T, DEC, true>(P, pl, wpe, grid, block, stream, a);
  else launch_wave3dp_s<T, DEC, false>(P, pl, wpe, grid, block, stream, a);
}

template <typename T>
int try_wave3dp_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                       const MapPtrs& maps, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w3p::W3P a{};
    dim3 grid, block;
    int pl, wpe;
    w3p_cfg(pred->padding, false, (int)sizeof(T), pl, wpe);
    const int zr = w3p_roll(pred->padding, (int)sizeof(T));
    if (!wave3dp_geometry<T>(g, B, C, pred, region, zr ? zr : pl, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    if (zr) {
      a.zrun = zr;
      launch_wave3dr<T, false>(pred->padding, grid, block, stream, a);
      return check_launch("wave3dr_encode");
    }
    launch_wave3dp<T, false>(pred->padding, pl, wpe, grid, block, stream, a);
    return check_launch("wave3dp_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_wave3dp_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                       const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w3p::W3P a{};
    dim3 grid, block;
    int pl, wpe;
    w3p_cfg(pred->padding, true, (int)sizeof(T), pl, wpe);
    const int zr = w3p_roll(pred->padding, (int)sizeof(T));
    if (!wave3dp_geometry<T>(g, B, C, pred, region, zr ? zr : pl, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    if (zr) {
      a.zrun = zr;
      launch_wave3dr<T, true>(pred->padding, grid, block, stream, a);
      return check_launch("wave3dr_decode");
    }
    launch_wave3dp<T, true>(pred->padding, pl, wpe, grid, block, stream, a);
    return check_launch("wave3dp_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_W3P_INST(T)                                                                                   \
  template int try_wave3dp_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,    \
                                     const MapPtrs&, const kmp_region*, hipStream_t);                     \
  template int try_wave3dp_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,             \
                                     const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_W3P_INST(uint8_t)
KMP_W3P_INST(uint16_t)
KMP_W3P_INST(int32_t)
KMP_W3P_INST(uint32_t)

}  // namespace kmp
