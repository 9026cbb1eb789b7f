// kmp_codec_wave2dp.hip -- one-pass image encode / decode for the mean predictor with p = 1, 2
// (SURVEY.md §8a a7-a12 fused for the 2D path; BASELINE config C2 geometry with p > 0).
//
// The image counterpart of kmp_codec_wave3dp.hip, with the access pattern of
// kmp_codec_wave2d.hip: each wave rolls down a run of output rows of one image in steps of
// rows = 64 / txn rows (wave2dr_kernel below), with the next steps' loads in flight, and computes
// with shuffles only.  The (2p+2)^2 neighbourhood mean (image/utils.py:120-137 +
// tests/image/test_encode_decode.py:46-51) is a separable box sum: x over the lane's elements and
// its neighbours' (2p+1 shuffles, mirrored in-lane at the row ends), y over the wave's rows by
// shuffles of the x sums (the rows above / below a step come from the neighbouring steps), so the
// C2 geometry (16 lanes per row, 4 rows per wave) serves p = 2 too.  floor(sum / (2p+2)^2) ==
// the f32 mean + truncation for u8/u16.  Aggregation onto LR / UD / C and the coder are the p = 0
// kernel's (image/utils.py:58-86, utils.py:38-55).
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace w2p {

using namespace wv;

struct W2P {
  const void* hi_in;
  void* hi_out;
  const void* lo_in;
  void* lo_out;
  MapPtrs maps;
  int32_t H, W;
  int32_t Ly, Lx, Ey, Ex, Lcy, Lcx;
  int32_t txn, rows, nwv, ngrp;
  int32_t xcd_per;
  int32_t ybeg, yend;
  int32_t wbase;  // first wave (of rows rows) the launch covers
  int32_t rrun;   // wave2dr_kernel: output rows per wave (a multiple of rows)
};

// ---- the y-rolling kernel: a wave owns a run of a.rrun consecutive output rows (steps of ``rows``
// rows, full width).  The x box sums of a step's node rows are computed
// once and serve three steps: as the current rows, as the previous step's rows (the p+1 rows
// above come from them by one shuffle instead of a halo load) and as the next step's rows (the
// p+1 rows below).  So a step loads one node row and its output rows per lane, against the
// plane-group kernel's node row + up to two halo rows; the node rows of step s+2 and the output
// rows of step s+1 are in flight while step s computes.
// STEPS > 0: the run is STEPS steps (rrun == STEPS * rows), fully unrolled, so the pipeline's
// register ring is renamed rather than moved (the moves made every step wait for all its loads,
// vmcnt(0), including the next step's just issued), and the output rows load unconditionally from
// clamped rows (needs Lcy >= 1), so the waits stay counted
template <typename T, bool DEC, int P, bool STC = false, int STEPS = 0>
__global__ void __launch_bounds__(256) wave2dr_kernel(W2P a) {
  constexpr int VX = 8 / (int)sizeof(T);
  constexpr int NB = 2 * P + 2;
  constexpr uint32_t NN = NB * NB;
  constexpr int NE = VX + 2 * P + 1;
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  using V = typename std::conditional<DEC, uint2, uint4>::type;
  constexpr bool SWAR = sizeof(T) == 1;
  constexpr int VW = SWAR ? VX / 2 : VX;

  const int lane = threadIdx.x & 63;
  const int wv_ = threadIdx.x >> 6;
  const int tx = lane & (a.txn - 1);
  const int r = lane >> __builtin_ctz(a.txn);
  const int X = tx * VX;
  int blk = (int)blockIdx.x;
  if (a.xcd_per > 0) {
    const int x = blk % 8, k = blk / 8;
    blk = ((k / a.xcd_per) * 8 + x) * a.xcd_per + (k % a.xcd_per);
  }
  const int grp = blk % a.ngrp;
  const int64_t b = blk / a.ngrp;
  const int rows = a.rows;
  const int Ys = a.ybeg + (grp * a.nwv + wv_) * a.rrun;  // first row of this wave's run
  if (Ys >= a.yend) return;  // whole idle wave
  const int Ye = Ys + a.rrun < a.yend ? Ys + a.rrun : a.yend;
  const bool xfirst = tx == 0, xlast = tx == a.txn - 1;
  const bool xdims = a.Lx != a.Ex;
  const int64_t himg = (int64_t)a.H * a.W;
  const int hx = 2 * X;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * himg;
  T* hout = DEC ? (T*)a.hi_out + b * himg : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ey * a.Ex : nullptr;
  // the image's row arrays: a uniform base plus a 32-bit lane offset per access (an image holds
  // < 2^31 samples), not 64-bit products per lane and step
  T* const mlo = (T*)(DEC ? nullptr : a.lo_out) + b * (int64_t)a.Ey * a.Ex;
  T* const mb[3] = {(T*)a.maps.p[0] + b * (int64_t)a.Lcy * a.Ex, (T*)a.maps.p[1] + b * (int64_t)a.Ey * a.Ex,
                    (T*)a.maps.p[2] + b * (int64_t)a.Lcy * a.Ex};

  auto load_node = [&](int y0) __attribute__((always_inline)) {  // node row y0 + r (mirrored past the ends)
    // STEPS > 0: the host guarantees Ly >= rrun + rows, so every row read lies in [-Ly, 2 Ly) and one
    // reflection (lsrc1) equals the general lsrc, without its divisions
    const int y = STEPS > 0 ? lsrc1(y0 + r, a.Ly, a.Ey) : lsrc(y0 + r, a.Ly, a.Ey);
    if constexpr (DEC) return (V)ld8c(lin + (uint32_t)(y * a.Ex + X));
    else return (V)ld16c(hin + (uint32_t)(2 * y * a.W + hx));
  };
  struct Out {
    uint4 o0;
    uint2 mv[3];
  };
  auto load_out = [&](int y0, Out& O) __attribute__((always_inline)) {
    const int Y = y0 + r;
    const bool live = Y < a.Ey && Y < Ye, vy1 = Y < a.Lcy;
    const int Yc = live ? Y : 0;
    if constexpr (STEPS > 0) {  // unconditional: lanes without the row read row 0 (unused)
      const int Yl = live && vy1 ? Y : 0;
      if constexpr (DEC) {
        O.mv[0] = ld8(mb[0] + (uint32_t)(Yl * a.Ex + X));
        O.mv[1] = ld8(mb[1] + (uint32_t)(Yc * a.Ex + X));
        O.mv[2] = ld8(mb[2] + (uint32_t)(Yl * a.Ex + X));
      } else {
        O.o0 = ld16(hin + (uint32_t)((live && vy1 ? 2 * Y + 1 : 0) * a.W + hx));
      }
      return;
    }
    O.o0 = make_uint4(0, 0, 0, 0);
    O.mv[0] = O.mv[1] = O.mv[2] = make_uint2(0, 0);
    if constexpr (DEC) {
      const int64_t m_lr = (b * a.Lcy + Yc) * a.Ex + X, m_ud = (b * a.Ey + Yc) * a.Ex + X;
      if (live && vy1) O.mv[0] = ld8((const T*)a.maps.p[0] + m_lr);
      if (live) O.mv[1] = ld8((const T*)a.maps.p[1] + m_ud);
      if (live && vy1) O.mv[2] = ld8((const T*)a.maps.p[2] + m_lr);
    } else {
      if (live && vy1) O.o0 = ld16(hin + (2 * Y + 1) * a.W + hx);
    }
  };
  auto nodes = [&](const V& v, uint32_t (&n)[VX]) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      if constexpr (DEC) n[i] = el8<T>(v, i);
      else n[i] = el16<T>(v, 2 * i);
    }
  };
  // x box sums of a node row, SWAR-packed for 8-bit samples (sums < 2^16)
  auto xpack = [&](const V& v, uint32_t (&pk)[VW]) __attribute__((always_inline)) {
    uint32_t z[VX], out[VX];
    nodes(v, z);
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
#pragma unroll
    for (int w = 0; w < VW; ++w) pk[w] = SWAR ? (out[2 * w] | out[2 * w + 1] << 16) : out[w];
  };

  // pipeline: x sums of the previous and current steps, node rows of the next step, output rows
  uint32_t pprev[VW], pcur[VW];
  V own = load_node(Ys), vnext = load_node(Ys + rows);
  Out Ocur, Onext;
  load_out(Ys, Ocur);
  xpack(load_node(Ys - rows), pprev);
  xpack(own, pcur);

  auto step = [&](const int Y0, const bool more, const bool more2) __attribute__((always_inline)) {
    const V vnn = more2 ? load_node(Y0 + 2 * rows) : V{};  // step s+2's node rows
    if (more) load_out(Y0 + rows, Onext);
    uint32_t pnext[VW];
    xpack(vnext, pnext);
    // the y box: row r + d for |d| <= p+1, from this step's rows or, past the step's ends, the previous
    // step's last / the next step's first rows.  One rotation by d rows per d (rows * txn = 64 lanes):
    // the SOURCE lane picks what it sends -- for a given d, each source row feeds exactly one target row,
    // which needs either its current row or (wrapped) the previous / next step's -- so a row shift is one
    // ds_bpermute, not two plus a halo pre-shift
    uint32_t so[VW], su[VW];
#pragma unroll
    for (int w = 0; w < VW; ++w) so[w] = su[w] = 0;
#pragma unroll
    for (int d = -P - 1; d <= P + 1; ++d) {
      const int src = ((lane + d * a.txn) & 63) << 2;  // lane L reads lane L + d rows (mod 64)
#pragma unroll
      for (int w = 0; w < VW; ++w) {
        uint32_t v = pcur[w];
        if (d != 0) {
          const uint32_t send = d < 0 ? (r >= rows + d ? pprev[w] : pcur[w]) : (r < d ? pnext[w] : pcur[w]);
          v = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)send);
        }
        if (d >= -P) so[w] += v;
        if (d <= P) su[w] += v;
      }
    }
    uint32_t M1[VX + 1], M0[VX + 1];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t o = SWAR ? (so[i / 2] >> (16 * (i & 1))) & 0xffffu : so[i];
      const uint32_t u = SWAR ? (su[i / 2] >> (16 * (i & 1))) & 0xffffu : su[i];
      M1[i + 1] = o / NN;
      M0[i + 1] = u / NN;
    }
    M1[0] = shup(M1[VX], 1);
    M0[0] = shup(M0[VX], 1);

    const int Y = Y0 + r;
    if (Y < a.Ey && Y < Ye) {
      const bool vy1 = Y < a.Lcy, vy0 = Y >= 1;
      bool vx[VX + 1];
      cells_valid<VX>(vx, X, a.Lcx);
      const uint32_t ny = (uint32_t)vy0 + (uint32_t)vy1;
#pragma unroll
      for (int q = 0; q <= VX; ++q) {
        M1[q] = (vy1 && vx[q]) ? M1[q] : 0u;
        M0[q] = (vy0 && vx[q]) ? M0[q] : 0u;
      }
      uint32_t pred[3][VX];  // LR, UD, C
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pred[0][i] = (M1[i] + M1[i + 1]) >> (nx >> 1);
        pred[1][i] = (M0[i + 1] + M1[i + 1]) >> (ny >> 1);
        pred[2][i] = M1[i + 1];
      }
      uint32_t n[VX];
      nodes(own, n);
      const uint32_t m_row = (uint32_t)(Y * a.Ex + X);  // in the lowres and every map (rows Y < Lcy)
      if constexpr (!DEC) {
        uint32_t res[3][VX];
#pragma unroll
        for (int i = 0; i < VX; ++i) {
          res[0][i] = (el16<T>(Ocur.o0, 2 * i) - pred[0][i]) & MASK;      // LR (1,0)
          res[1][i] = (el16<T>(own, 2 * i + 1) - pred[1][i]) & MASK;      // UD (0,1)
          res[2][i] = (el16<T>(Ocur.o0, 2 * i + 1) - pred[2][i]) & MASK;  // C  (1,1)
        }
        stp8<STC>(mlo + m_row, pack8<T, VX>(n));
        if (vy1) stp8<STC>(mb[0] + m_row, pack8<T, VX>(res[0]));
        stp8<STC>(mb[1] + m_row, pack8<T, VX>(res[1]));
        if (vy1) stp8<STC>(mb[2] + m_row, pack8<T, VX>(res[2]));
      } else {
        uint32_t dv[3][VX];
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int i = 0; i < VX; ++i) dv[k][i] = (pred[k][i] + el8<T>(Ocur.mv[k], i)) & MASK;
        T* h0 = hout + (uint32_t)(2 * Y * a.W + hx);
        st16(h0, pack16<T, VX>(n, dv[1]));
        if (vy1) st16(h0 + a.W, pack16<T, VX>(dv[0], dv[2]));
      }
    }
    // slide the pipeline by one step
#pragma unroll
    for (int w = 0; w < VW; ++w) {
      pprev[w] = pcur[w];
      pcur[w] = pnext[w];
    }
    own = vnext;
    vnext = vnn;
    Ocur = Onext;
  };
  if constexpr (STEPS > 0) {
#pragma unroll
    for (int s = 0; s < STEPS; ++s) step(Ys + s * rows, s + 1 < STEPS, s + 2 <= STEPS);
  } else {
#pragma unroll 1
    for (int Y0 = Ys; Y0 < Ye; Y0 += rows) step(Y0, Y0 + rows < Ye, Y0 + rows < Ye);
  }
}

}  // namespace w2p

// y-rolling kernel (wave2dr_kernel): 32 output rows per wave, rounded up to a multiple of the wave's
// rows (C2 p = 1: 33.5 / 31.4 -> 28.4 / 28.1 us per direction against the row-group kernel it
// replaced, profiles/round2/ab_wave2dr.log); runs of 8 steps take the unrolled form (C2 p = 1
// 28.5 / 26.0 -> 27.0-28.2 / 24.7-25.7 us, p = 2 32.2 / 29.5 -> 31.3-31.7 / 27.8-28.8 us by
// rocprofv3, profiles/round4/ab_wave2dr_unroll_r4w.log)
constexpr int kW2Run = 32;

template <typename T>
static bool wave2dp_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred,
                             const kmp_region* region, int run, w2p::W2P& a, dim3& grid, dim3& block) {
  constexpr int VX = 8 / (int)sizeof(T);
  if (!(std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value)) return false;
  if (opt(OPT_DISABLE_WAVE, 0) || opt(OPT_DISABLE_FAST, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_MEAN || pred->padding < 1 || pred->padding > 2) return false;
  const int P = pred->padding;
  int64_t yb = 0, ye = g.E[1];
  if (region) {  // only row ranges (full width)
    if (region->begin[2] > 0 || region->end[2] < g.E[2]) return false;
    yb = region->begin[1] < 0 ? 0 : region->begin[1];
    ye = region->end[1] > g.E[1] ? g.E[1] : region->end[1];
    if (ye <= yb) return false;
  }
  if (g.n[2] % 2 != 0 || (g.n[2] * (int64_t)sizeof(T)) % 16 != 0) return false;
  if (g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || txn < 1 || txn > 64 || (txn & (txn - 1)) != 0) return false;
  const int64_t rows = 64 / txn;
  if (rows < P + 1) return false;  // an "above" and a "below" halo row per lane at most
  // only the waves covering the region's rows are launched
  int64_t w0 = yb / rows, w1 = ceil_div(ye, rows);
  // runs of ``run`` rows from the region's first row
  run = (int)(ceil_div(run, rows) * rows);
  w0 = 0;
  w1 = ceil_div(ye - yb, (int64_t)run);
  const int64_t waves = w1 - w0;
  const int64_t nwv = waves < 4 ? waves : 4;
  const int64_t ngrp = ceil_div(waves, nwv);
  a.H = (int)g.n[1]; a.W = (int)g.n[2];
  a.Ly = (int)g.L[1]; a.Lx = (int)g.L[2];
  a.Ey = (int)g.E[1]; a.Ex = (int)g.E[2];
  a.Lcy = (int)g.Lc[1]; a.Lcx = (int)g.Lc[2];
  a.txn = (int)txn; a.rows = (int)rows; a.nwv = (int)nwv; a.ngrp = (int)ngrp;
  a.xcd_per = (opt(OPT_W2_XCD, 1) && B % 8 == 0) ? (int)ngrp : 0;
  a.ybeg = (int)yb;
  a.yend = (int)ye;
  a.wbase = (int)w0;
  a.rrun = run;
  const int64_t nblk = B * ngrp;
  grid = dim3((unsigned)nblk);
  block = dim3((unsigned)(64 * nwv));
  return nblk < ((int64_t)1 << 31);
}

template <typename T, bool DEC, bool STC>
static void launch_wave2dp_s(int P, dim3 grid, dim3 block, hipStream_t s, const w2p::W2P& a) {
  if (a.rrun == 8 * a.rows && a.Lcy >= 1 && a.Ly >= a.rrun + a.rows) {  // C2: runs of 32 rows, 4 per step
    if (P == 1) w2p::wave2dr_kernel<T, DEC, 1, STC, 8><<<grid, block, 0, s>>>(a);
    else w2p::wave2dr_kernel<T, DEC, 2, STC, 8><<<grid, block, 0, s>>>(a);
    return;
  }
  if (P == 1) w2p::wave2dr_kernel<T, DEC, 1, STC><<<grid, block, 0, s>>>(a);
  else w2p::wave2dr_kernel<T, DEC, 2, STC><<<grid, block, 0, s>>>(a);
}

// the encode's lowres / map stores: cached (MALL-allocating, stp8 in kmp_wave.h; alternating pairs at
// C2: p = 1 -0.9 us, p = 2 +-0, profiles/round2/ab_wave2dp_store_policy.log) unless
// KMP_W2P_ST_ENC=0 (non-temporal)
template <typename T, bool DEC>
static void launch_wave2dp(int P, dim3 grid, dim3 block, hipStream_t s, const w2p::W2P& a) {
  if (!DEC && opt(OPT_W2P_ST_ENC, 1)) launch_wave2dp_s<T, DEC, true>(P, grid, block, s, a);
  else launch_wave2dp_s<T, DEC, false>(P, grid, block, s, a);
}

template <typename T>
int try_wave2dp_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                       const MapPtrs& maps, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w2p::W2P a{};
    dim3 grid, block;
    if (!wave2dp_geometry<T>(g, B, C, pred, region, kW2Run, a, grid, block))
      return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 3; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    launch_wave2dp<T, false>(pred->padding, grid, block, stream, a);
    return check_launch("wave2dr_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_wave2dp_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                       const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w2p::W2P a{};
    dim3 grid, block;
    if (!wave2dp_geometry<T>(g, B, C, pred, region, kW2Run, a, grid, block))
      return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 3; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    launch_wave2dp<T, true>(pred->padding, grid, block, stream, a);
    return check_launch("wave2dr_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_W2P_INST(T)                                                                                   \
  template int try_wave2dp_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,    \
                                     const MapPtrs&, const kmp_region*, hipStream_t);                     \
  template int try_wave2dp_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,             \
                                     const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_W2P_INST(uint8_t)
KMP_W2P_INST(uint16_t)
KMP_W2P_INST(int32_t)
KMP_W2P_INST(uint32_t)

}  // namespace kmp
