// kmp_codec_wave3d.hip -- one-pass volume encode / decode for the mean predictor with p == 0
// (the metric path: BASELINE config C3, MeanPredictor(0) + the uint16 coder on 64^3 tiles).
//
// Same arithmetic as kmp_codec_fast3d.hip (which keeps p = 1, 2), different data movement:
//   * A workgroup owns PL = 2 consecutive output planes of one tile and issues EVERY global load
//     of its planes up front (node rows of node planes c0-1 .. c0+PL, the stream rows of its PL
//     output planes), then computes: no z-rolling, no LDS, no barrier.  Short workgroups
//     dispatched in order keep the resident set on one contiguous window of the volume -- the
//     access order that reaches the probe ceiling for this shape (tools/probe_bw.hip
//     codec_shape: 6.0 TB/s at one plane per workgroup vs 4.9 TB/s for 4-plane rolling slabs).
//   * Tile-per-XCD block order: XCD x = blockIdx % 8 codes whole tiles, so the two z-halo node
//     planes a workgroup shares with its neighbours are L2 hits (default-policy loads): HBM
//     traffic measured by PMC equals the algorithmic bytes (profiles/pmc_traffic.json).
//   * Every wavefront is independent: it owns ROWS = 64 / TXN output rows (TXN = Ex / VX lanes
//     per row, VX outputs per lane = 8 bytes of lowres).  Neighbour exchange is cross-lane
//     (ds_bpermute shuffles): node row y+1 from the lane TXN below, node x+VX from the next lane
//     (mirrored on the row's last lane: even reflect pad, volume/utils.py:226-237); the wave's
//     first / last row loads one halo row each.
// Per output plane c a lane forms the cell means of planes c-1 and c (2x2x2 node sums, floor / 8
// == the reference test predictor's f32 mean + truncation, tests/volume/test_encode_decode.py:
// 46-51), the 19-way aggregation onto the 7 maps (volume/utils.py:83-155: sums of 1/2/4 means
// >> log2(count) == its f32 x0.5 / x0.25 + truncation for these ranges) and the mod-2^k coder
// (utils.py:38-55), then writes lowres + 7 maps (8 B per lane each) or the 2x2x2 highres block
// rows (16 B per lane each).
#include <algorithm>
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace w3 {

using namespace wv;

struct W3 {
  const void* hi_in;  // encode input
  void* hi_out;       // decode output
  const void* lo_in;  // decode input
  void* lo_out;       // encode output
  MapPtrs maps;
  int32_t D, H, W;
  int32_t Lz, Ly, Lx, Ez, Ey, Ex, Lcz, Lcy, Lcx;
  int32_t slab, nslab, zbegin, zend;
  int32_t txn, rows, nwv, nyg;
  int32_t xcd_per;  // > 0: XCD-contiguous block order (blocks per XCD), 0: identity
  int32_t nt_nodes; // plane kernel: 1 = non-temporal node-row loads, 0 = default policy (L2-shared halo)
  int64_t nB;       // tiles in the batch (debug-build bounds checks only)
  int32_t nvblk;    // blocks (= workgroups launched)
};

// rows a lane reads for one node plane: its own, and (wave's first / last row) one halo row;
// one-row waves (64 lanes per output row) need both: ``halo`` above, ``dn`` below
template <bool DEC>
struct NodeRows {
  using V = typename std::conditional<DEC, uint2, uint4>::type;
  V own, halo, dn;
};
// encode: the non-node rows of output plane q (plane 2q row 2Y+1, plane 2q+1 rows 2Y, 2Y+1)
// decode: the 7 residual rows of output plane q
template <bool DEC>
struct OutRows {
  uint4 e1, o0, o1;
  uint2 mv[7];
};

// Store policy (STC, stp8 in kmp_wave.h), chosen on the pipelines that follow an encode at C3
// (tools/pipeline_rows.py, profiles/round3/pipeline_store_policy_r3.log; DESIGN §5 "pipeline"):
// the encode's lowres and maps are stored non-temporal.  Cached (MALL-allocating) stores let a
// decode that immediately re-reads the same maps find part of them in the MALL (bench.py's
// encode -> decode loop: 177 -> 171 us per pair), but their dirty lines drain during the next
// encode when encodes run back to back (a producer of chunks: 85 -> 103 us per encode), and encode
// -> Rice pack / Rice unpack -> decode are within 3 us either way.  The decode's highres is
// non-temporal too (cached: +7 us on the next encode).  KMP_W3_ST_ENC=1: cached encode stores.

// WPE: the amdgpu_waves_per_eu register budget (PL = 2 encode: 3 waves / SIMD without spills).
template <typename T, bool DEC, int PL, bool ONE, bool STC>
__device__ __forceinline__ void wave3d_plane_body(const W3& a, int vblk) {
  constexpr int VX = 8 / (int)sizeof(T);
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  using NR = NodeRows<DEC>;
  using OR = OutRows<DEC>;

  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int tx = lane & (a.txn - 1);          // txn: a power of two (host)
  const int r = lane >> __builtin_ctz(a.txn);
  const int X = tx * VX;
  // a.xcd_per > 0: tile-per-XCD order -- XCD x = blockIdx % 8 codes whole tiles, its k-th block
  // is block (k % per_tile) of tile (k / per_tile) * 8 + x, so the z-halo neighbours share an L2
  int blk = vblk;
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
  const int Yc = live ? Y : a.Ey - 1;
  const int c0 = a.zbegin + pb * PL;
  const int Z1 = a.zend;

  const bool first = r == 0;
  const bool last = r == a.rows - 1 || Y == a.Ey - 1;
  const bool vy1 = Y < a.Lcy;
  const bool vy0 = Y >= 1;
  const bool need_up = live && first && Y0 >= 1;
  const bool need_dn = live && last && vy1;
  const int yup = Y0 >= 1 ? Y0 - 1 : 0;
  const int ydn = lsrc(Yc + 1, a.Ly, a.Ey);
  const bool xlast = tx == a.txn - 1;

  const int hplane = a.H * a.W;
  const int lplane = a.Ey * a.Ex;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * (int64_t)a.D * hplane;
  T* hout = DEC ? (T*)a.hi_out + b * (int64_t)a.D * hplane : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ez * lplane : nullptr;
  const int hx = 2 * X;
  // a lane is never both the wave's first and last row (host eligibility), so one halo row each
  const int ho_own = 2 * Yc * a.W + hx, ho_up = 2 * yup * a.W + hx, ho_dn = 2 * ydn * a.W + hx;
  const int lo_own = Yc * a.Ex + X, lo_up = yup * a.Ex + X, lo_dn = ydn * a.Ex + X;

  const T* mbase[7];
  int mplane[7];
  bool mok_y[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez, ey = par[1] ? a.Lcy : a.Ey;
    mplane[k] = ey * a.Ex;
    const int ym = Yc < ey ? Yc : (ey > 0 ? ey - 1 : 0);  // in-bounds row (encode stores are gated by mok_y)
    mbase[k] = (const T*)a.maps.p[k] + b * (int64_t)ez * mplane[k] + ym * a.Ex + X;
    mok_y[k] = live && (!par[1] || vy1);
  }

  // ---- every load of the block, issued before any use.  Encode: all node rows, then the stream
  // rows.  Decode: in the order the planes consume them (node planes c0-1, c0, then per output
  // plane u node plane c0+u+1 and its 7 map rows), so output plane u waits only for its own loads
  // (vmcnt counts in issue order): 91.0 vs 92.0 us at C3, same box, 3 alternating runs ----
  NR N[PL + 2];  // node planes c0-1+t
  OR O[PL];      // output planes c0+u
  if constexpr (!DEC) {
#pragma unroll
    for (int t = 0; t < PL + 2; ++t) {
      const int q = c0 - 1 + t;
      if (q < 0 || (t >= 2 && q - 1 >= Z1)) {  // uniform
        N[t] = NR{};
        continue;
      }
      N[t].halo = N[t].dn = uint4{};
      const T* p = hin + 2 * lsrc(q, a.Lz, a.Ez) * hplane;
      KMP_SPAN((const T*)a.hi_in, p + ho_own, 2 * VX, a.nB * a.D * hplane);
      KMP_SPAN((const T*)a.hi_in, p + (first ? ho_up : ho_dn), 2 * VX, a.nB * a.D * hplane);
      // own node row: unconditional (row Yc is clamped in bounds; a dead lane's value is unused)
      if (a.nt_nodes) N[t].own = ld16(p + ho_own);
      else N[t].own = ld16c(p + ho_own);
      if constexpr (ONE) {
        if (need_up) N[t].halo = ld16c(p + ho_up);
        if (need_dn) N[t].dn = ld16c(p + ho_dn);
      } else {
        if (need_up || need_dn) N[t].halo = ld16c(p + (first ? ho_up : ho_dn));  // this lane's halo row
      }
    }
#pragma unroll
    for (int u = 0; u < PL; ++u) {
      const int q = c0 + u;
      if (q >= Z1) {  // uniform
        O[u] = OR{};
        continue;
      }
      // stream rows: unconditional from clamped addresses (row 2Y+1 / plane 2q+1 past the edge
      // re-read row 2Y / plane 2q; the maps they would feed are not stored there)
      const int r1 = 2 * Yc + 1 < a.H ? a.W : 0, p1 = 2 * q + 1 < a.D ? hplane : 0;
      const T* p = hin + 2 * q * hplane;
      KMP_SPAN((const T*)a.hi_in, p + p1 + ho_own + r1, 2 * VX, a.nB * a.D * hplane);
      O[u].e1 = ld16(p + ho_own + r1);
      O[u].o0 = ld16(p + p1 + ho_own);
      O[u].o1 = ld16(p + p1 + ho_own + r1);
    }
  } else {
    // own node rows and map rows unconditionally from clamped in-bounds addresses (values of rows
    // past the edges are never used), halo rows only where a lane needs one
    auto load_node = [&](int t) __attribute__((always_inline)) {
      const int q = c0 - 1 + t;
      if (q < 0 || (t >= 2 && q - 1 >= Z1)) {  // uniform
        N[t] = NR{};
        return;
      }
      N[t].halo = N[t].dn = uint2{};
      const T* p = lin + lsrc(q, a.Lz, a.Ez) * lplane;
      KMP_SPAN((const T*)a.lo_in, p + lo_own, VX, a.nB * a.Ez * lplane);
      KMP_SPAN((const T*)a.lo_in, p + (first ? lo_up : lo_dn), VX, a.nB * a.Ez * lplane);
      if (a.nt_nodes) N[t].own = ld8(p + lo_own);
      else N[t].own = ld8c(p + lo_own);
      if constexpr (ONE) {
        if (need_up) N[t].halo = ld8c(p + lo_up);
        if (need_dn) N[t].dn = ld8c(p + lo_dn);
      } else {
        if (need_up || need_dn) N[t].halo = ld8c(p + (first ? lo_up : lo_dn));  // this lane's halo row
      }
    };
    auto load_out = [&](int u) __attribute__((always_inline)) {
      const int q = c0 + u;
      if (q >= Z1) {  // uniform
        O[u] = OR{};
        return;
      }
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        const int ez = par[0] ? a.Lcz : a.Ez;
        if (ez > 0 && mplane[k] > 0) {  // uniform
          KMP_SPAN((const T*)a.maps.p[k], mbase[k] + (q < ez ? q : ez - 1) * mplane[k], VX, a.nB * ez * mplane[k]);
          O[u].mv[k] = ld8(mbase[k] + (q < ez ? q : ez - 1) * mplane[k]);
        } else {
          O[u].mv[k] = uint2{};
        }
      }
    };
    load_node(0);
    load_node(1);
#pragma unroll
    for (int u = 0; u < PL; ++u) {
      load_node(u + 2);
      load_out(u);
    }
  }

  // ---- 2x2 node sums per node plane (rows Y and, on the wave's first row, Y-1) ----
  uint32_t S[PL + 2][VX], Su[PL + 2][VX];
#pragma unroll
  for (int t = 0; t < PL + 2; ++t) {
    // own node row, and the halo row (row Y0-1 on the wave's first row, Y+1 on its last row)
    uint32_t n[VX], nh[VX], nd[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      if constexpr (DEC) {
        n[i] = el8<T>(N[t].own, i); nh[i] = el8<T>(N[t].halo, i); nd[i] = el8<T>(N[t].dn, i);
      } else {
        n[i] = el16<T>(N[t].own, 2 * i); nh[i] = el16<T>(N[t].halo, 2 * i); nd[i] = el16<T>(N[t].dn, 2 * i);
      }
    }
    uint32_t nx1 = shdn(n[0], 1), nhx1 = shdn(nh[0], 1), ndx1 = ONE ? shdn(nd[0], 1) : 0u;
    if (xlast) {
      nx1 = n[VX - 1];
      nhx1 = nh[VX - 1];
      ndx1 = nd[VX - 1];
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t h = n[i] + (i + 1 < VX ? n[i + 1] : nx1);
      const uint32_t hh = nh[i] + (i + 1 < VX ? nh[i + 1] : nhx1);
      if constexpr (ONE) {  // every lane is its wave's first and last row
        const uint32_t hd = nd[i] + (i + 1 < VX ? nd[i + 1] : ndx1);
        S[t][i] = h + hd;
      } else {
        const uint32_t below = shdn(h, a.txn);
        S[t][i] = h + (last ? hh : below);
      }
      Su[t][i] = hh + h;
    }
  }

  // ---- cell means of cell plane c0-1+m (m = 0..PL): rows Y / Y-1, cols X-1 .. X+VX-1; computed
  // just before the output plane that first needs them so that at most two sets are live ----
  uint32_t Mo[PL + 1][VX + 1], Ma[PL + 1][VX + 1];
  auto cell_means = [&](int m) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      Mo[m][i + 1] = (S[m][i] + S[m + 1][i]) >> 3;
      const uint32_t mu = (Su[m][i] + Su[m + 1][i]) >> 3;
      const uint32_t above = shup(Mo[m][i + 1], a.txn);
      Ma[m][i + 1] = first ? mu : above;
    }
    Mo[m][0] = shup(Mo[m][VX], 1);
    Ma[m][0] = shup(Ma[m][VX], 1);
  };
  cell_means(0);

  bool vx[VX + 1];
#pragma unroll
  for (int q = 0; q <= VX; ++q) vx[q] = (X - 1 + q) >= 0 && (X - 1 + q) < a.Lcx;
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
    if constexpr (!DEC) {
      const uint4 e0 = N[u + 1].own;
      const OR& Oc = O[u];
      uint32_t res[7][VX], lov[VX];
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        lov[i] = el16<T>(e0, 2 * i);
        res[0][i] = (el16<T>(Oc.o1, 2 * i) - pred[0][i]) & MASK;      // LR (1,1,0)
        res[1][i] = (el16<T>(Oc.o0, 2 * i + 1) - pred[1][i]) & MASK;  // UD (1,0,1)
        res[2][i] = (el16<T>(Oc.e1, 2 * i + 1) - pred[2][i]) & MASK;  // FB (0,1,1)
        res[3][i] = (el16<T>(Oc.o1, 2 * i + 1) - pred[3][i]) & MASK;  // C  (1,1,1)
        res[4][i] = (el16<T>(Oc.o0, 2 * i) - pred[4][i]) & MASK;      // Z  (1,0,0)
        res[5][i] = (el16<T>(Oc.e1, 2 * i) - pred[5][i]) & MASK;      // Y  (0,1,0)
        res[6][i] = (el16<T>(e0, 2 * i + 1) - pred[6][i]) & MASK;     // X  (0,0,1)
      }
      KMP_SPAN((const T*)a.lo_out, (const T*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, VX,
               a.nB * a.Ez * lplane);
      stp8<STC>((T*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, pack8<T, VX>(lov));
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        if (mok_y[k] && (!par[0] || vz1)) {
          KMP_SPAN((const T*)a.maps.p[k], mbase[k] + c * mplane[k], VX,
                   a.nB * (par[0] ? a.Lcz : a.Ez) * mplane[k]);
          stp8<STC>((T*)mbase[k] + c * mplane[k], pack8<T, VX>(res[k]));
        }
      }
    } else {
      const OR& Oc = O[u];
      uint32_t own[VX], dv[7][VX];
#pragma unroll
      for (int i = 0; i < VX; ++i) own[i] = el8<T>(N[u + 1].own, i);
#pragma unroll
      for (int k = 0; k < 7; ++k)
#pragma unroll
        for (int i = 0; i < VX; ++i) dv[k][i] = (pred[k][i] + el8<T>(Oc.mv[k], i)) & MASK;
      T* h0 = hout + 2 * c * hplane + ho_own;
      KMP_SPAN((T*)a.hi_out, h0 + (vz1 ? hplane : 0) + (vy1 ? a.W : 0), 2 * VX, a.nB * a.D * hplane);
      st16(h0, pack16<T, VX>(own, dv[6]));
      if (vy1) st16(h0 + a.W, pack16<T, VX>(dv[5], dv[2]));
      if (vz1) {
        T* h1 = h0 + hplane;
        st16(h1, pack16<T, VX>(dv[4], dv[1]));
        if (vy1) st16(h1 + a.W, pack16<T, VX>(dv[0], dv[3]));
      }
    }
  }
}

// One workgroup per block (the host launches a.nvblk workgroups).  Not a grid-stride loop: kept
// live across iterations, the loop's kernel arguments overflowed the scalar registers (29 / 32 SGPRs
// spilled into VGPR lanes: 98 / 72 v_readlane per encode / decode wave); without it none spill and
// the waves issue 849 -> 731 / 818 -> 713 VALU instructions (round 5)
template <typename T, bool DEC, int PL, int WPE, bool ONE, bool STC = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) wave3d_plane_kernel(W3 a) {
  wave3d_plane_body<T, DEC, PL, ONE, STC>(a, (int)blockIdx.x);
}

}  // namespace w3

// ------------------------------------------------------------------------------------------
// Host: eligibility + launch geometry
// ------------------------------------------------------------------------------------------
template <typename T>
static bool wave3d_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, const kmp_region* region,
                            int pl, w3::W3& a, dim3& grid, dim3& block) {
  constexpr int VX = 8 / (int)sizeof(T);
  if (!(std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value)) return false;
  if (opt(OPT_DISABLE_WAVE, 0) || opt(OPT_DISABLE_FAST, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_MEAN || pred->padding != 0) return false;
  if (g.n[2] % 2 != 0 || (g.n[2] * (int64_t)sizeof(T)) % 16 != 0) return false;
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;  // 32-bit offsets inside a tile
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || txn < 1 || txn > 64 || (txn & (txn - 1)) != 0) return false;
  const int64_t rows = 64 / txn;
  if (rows > 1 && g.E[1] % rows == 1) return false;  // a one-row wave in a multi-row layout
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
  const int64_t zext = ze - zb;
  a.zbegin = (int)zb;
  a.zend = (int)ze;
  const int64_t nslab = ceil_div(zext, (int64_t)pl);  // plane blocks of PL output planes
  a.slab = pl;
  a.nslab = (int)nslab;
  const int64_t nblk = B * nslab * nyg;
  a.xcd_per = (opt(OPT_W3_XCD, 1) && B % 8 == 0) ? (int)(nslab * nyg) : 0;
  a.nt_nodes = 0;
  a.nB = B;
  a.nvblk = (int)nblk;
  grid = dim3((unsigned)nblk);  // one workgroup per block (grid-stride blocks measured slower, round 2)
  block = dim3((unsigned)(64 * nwv));
  return nblk < ((int64_t)1 << 31);
}

template <typename T, bool DEC, bool STC>
static void launch_wave3d_s(int pl, dim3 grid, dim3 block, hipStream_t stream, const w3::W3& a) {
  // PL = 2 at 3 waves / SIMD is the measured optimum at C3 (profiles/round1/kprof_wave3d.log):
  // PL = 1 re-reads twice the z halo per output plane; forcing 4 waves / SIMD spills
  if (a.rows == 1) {  // 64 lanes per output row (wide volumes): both halo rows per lane
    if (pl == 1) w3::wave3d_plane_kernel<T, DEC, 1, 4, true, STC><<<grid, block, 0, stream>>>(a);
    else w3::wave3d_plane_kernel<T, DEC, 2, 3, true, STC><<<grid, block, 0, stream>>>(a);
  } else if (pl == 1) {
    w3::wave3d_plane_kernel<T, DEC, 1, 4, false, STC><<<grid, block, 0, stream>>>(a);
  } else {
    w3::wave3d_plane_kernel<T, DEC, 2, 3, false, STC><<<grid, block, 0, stream>>>(a);
  }
}

template <typename T, bool DEC>
static void launch_wave3d(int pl, dim3 grid, dim3 block, hipStream_t stream, const w3::W3& a) {
  // non-temporal stores in both directions; KMP_W3_ST_ENC=1: the encode's cached (stp8)
  if (!DEC && opt(OPT_W3_ST_ENC, 0)) launch_wave3d_s<T, DEC, true>(pl, grid, block, stream, a);
  else launch_wave3d_s<T, DEC, false>(pl, grid, block, stream, a);
}

template <typename T>
int try_wave3d_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                      const MapPtrs& maps, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w3::W3 a{};
    dim3 grid, block;
    const int pl = opt(OPT_W3_PL, 2) == 1 ? 1 : 2;
    if (!wave3d_geometry<T>(g, B, C, pred, region, pl, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    launch_wave3d<T, false>(pl, grid, block, stream, a);
    return check_launch("wave3d_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_wave3d_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                      const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w3::W3 a{};
    dim3 grid, block;
    const int pl = opt(OPT_W3_PL, 2) == 1 ? 1 : 2;
    if (!wave3d_geometry<T>(g, B, C, pred, region, pl, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    launch_wave3d<T, true>(pl, grid, block, stream, a);
    return check_launch("wave3d_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_W3_INST(T)                                                                                    \
  template int try_wave3d_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,     \
                                    const MapPtrs&, const kmp_region*, hipStream_t);                      \
  template int try_wave3d_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,              \
                                    const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_W3_INST(uint8_t)
KMP_W3_INST(uint16_t)
KMP_W3_INST(int32_t)
KMP_W3_INST(uint32_t)

}  // namespace kmp
