// kmp_codec_wave2d.hip -- one-pass image encode / decode for the mean predictor with p == 0
// (BASELINE config C2: MeanPredictor(0) + the uint8 coder on 1024 images of 256^2).
//
// The 2D counterpart of kmp_codec_wave3d.hip.  A workgroup owns NW * ROWS consecutive output
// rows of one image; each of its waves owns ROWS = 64 / TXN of them (TXN = Ex / VX lanes per
// row, VX outputs per lane = 8 bytes of lowres) and issues all its loads up front: highres rows
// 2Y and 2Y+1 per lane, plus one halo row on the wave's first row (node row Y0-1, for the cell
// row above) and on its last row (node row Y+1, mirrored at the even-padded edge,
// image/utils.py:145-156).  Neighbours come from cross-lane shuffles (node x+VX from the next
// lane, node row y+1 and the cell row above from the lane TXN away); no LDS, no barrier.
// Per output (Y, X..X+VX-1): cell means of rows Y-1 and Y (2x2 node sums, floor / 4 == the
// reference test predictor's f32 mean + truncation, tests/image/test_encode_decode.py:46-51),
// the 5-way aggregation onto LR / UD / C (image/utils.py:58-86: sums of 1/2 means
// >> log2(count) == its f32 x0.5 + truncation), and the mod-2^k coder (utils.py:38-55).
// Image-per-XCD block order keeps the workgroup-edge halo rows in one L2.
#include <algorithm>
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace w2 {

using namespace wv;

struct W2 {
  const void* hi_in;
  void* hi_out;
  const void* lo_in;
  void* lo_out;
  MapPtrs maps;
  int32_t H, W;
  int32_t Ly, Lx, Ey, Ex, Lcy, Lcx;
  int32_t txn, rows, nwv, ngrp;  // lanes per row, rows per wave, waves per workgroup, workgroups per image
  int32_t xcd_per;               // > 0: image-per-XCD block order (workgroups per image)
  int32_t ybeg, yend;            // output rows written (a chunked-driver region; all rows otherwise)
  int32_t nvblk;                 // virtual blocks (B * ngrp), grid-strided over the workgroups
  UDiv ngrp_div;                 // n / ngrp (host-computed multiplier)
  const float* wt;               // LIN: LinearPredictor weights [4, 5] row-major and bias [5]
  const float* bias;
};

template <typename T>
__device__ __forceinline__ uint32_t cast_t(float v) {  // astype(T) for u8/u16: trunc, saturate, NaN -> 0
  return cvt_sat<T>(v);  // saturating v_cvt_u32_f32 + integer min (kmp_wave.h)
}

// LIN: the LinearPredictor with p = 0 instead of the mean (image/utils.py:58-86 on its 5
// per-cell channels): pred[cell, k] = fma chain over the 4 nodes (n = dy*2 + dx) from b[k], cast
// to T; LR = ch0 (x) + ch1 (x-1), UD = ch2 (y) + ch3 (y-1), C = ch4, with the same counts / shifts.
template <typename T, bool DEC, bool ONE, bool LIN, bool STC>
__device__ __forceinline__ void wave2d_body(const W2& a, int vblk) {
  constexpr int VX = 8 / (int)sizeof(T);
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  using V = typename std::conditional<DEC, uint2, uint4>::type;

  const int lane = threadIdx.x & 63;
  const int wv_ = threadIdx.x >> 6;
  const int tx = lane & (a.txn - 1);          // txn: a power of two (host)
  const int r = lane >> __builtin_ctz(a.txn);
  const int X = tx * VX;
  int blk = vblk;
  if (a.xcd_per > 0) {
    const int x = blk % 8, k = blk / 8;
    blk = ((k / a.xcd_per) * 8 + x) * a.xcd_per + (k % a.xcd_per);
  }
  const int grp = blk % a.ngrp;
  const int64_t b = blk / a.ngrp;
  const int Y0 = (grp * a.nwv + wv_) * a.rows;
  if (Y0 >= a.Ey) return;  // whole idle wave
  const int Y = Y0 + r;
  const bool live = Y < a.Ey;
  const int Yc = live ? Y : a.Ey - 1;
  const bool first = r == 0;
  const bool last = r == a.rows - 1 || Y == a.Ey - 1;
  const bool vy1 = Y < a.Lcy;  // cell row Y (== highres row 2Y+1) exists
  const bool vy0 = Y >= 1;
  // one halo row per lane (its wave's first row: Y0-1, last row: Y+1); a one-row wave (ONE, 64
  // lanes per output row) needs both: ``halo`` above and ``hdn`` below
  const bool need_halo = live && (ONE ? (Y0 >= 1) : ((first && Y0 >= 1) || (last && vy1)));
  const bool need_dn = ONE && live && vy1;
  const int yh = (ONE || first) ? (Y0 >= 1 ? Y0 - 1 : 0) : lsrc(Yc + 1, a.Ly, a.Ey);
  const int ydn = lsrc(Yc + 1, a.Ly, a.Ey);
  const bool xlast = tx == a.txn - 1;

  const int64_t himg = (int64_t)a.H * a.W;
  const int hx = 2 * X;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * himg;
  T* hout = DEC ? (T*)a.hi_out + b * himg : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ey * a.Ex : nullptr;
  const int64_t m_lr = (b * a.Lcy + Yc) * a.Ex + X;  // LR and C maps: [B, Lcy, Ex]
  const int64_t m_ud = (b * a.Ey + Yc) * a.Ex + X;   // UD map and lowres: [B, Ey, Ex]

  // ---- every load up front ----
  V own{}, halo{}, hdn{};
  uint4 o0 = make_uint4(0, 0, 0, 0);
  uint2 mv[3] = {make_uint2(0, 0), make_uint2(0, 0), make_uint2(0, 0)};
  if constexpr (DEC) {
    if (live) own = ld8c(lin + Yc * a.Ex + X);
    if (need_halo) halo = ld8c(lin + yh * a.Ex + X);
    if (need_dn) hdn = ld8c(lin + ydn * a.Ex + X);
    if (live && vy1) mv[0] = ld8((const T*)a.maps.p[0] + m_lr);
    if (live) mv[1] = ld8((const T*)a.maps.p[1] + m_ud);
    if (live && vy1) mv[2] = ld8((const T*)a.maps.p[2] + m_lr);
  } else {
    if (live) own = ld16c(hin + 2 * Yc * a.W + hx);  // node row: re-read as a neighbour's halo
    if (need_halo) halo = ld16c(hin + 2 * yh * a.W + hx);
    if (need_dn) hdn = ld16c(hin + 2 * ydn * a.W + hx);
    if (live && vy1) o0 = ld16(hin + (2 * Yc + 1) * a.W + hx);
  }

  // ---- 2x2 node sums: row Y, and on the wave's first row also row Y-1 ----
  uint32_t n[VX], nh[VX], nd[VX];
#pragma unroll
  for (int i = 0; i < VX; ++i) {
    if constexpr (DEC) {
      n[i] = el8<T>(own, i);
      nh[i] = el8<T>(halo, i);
      nd[i] = el8<T>(hdn, i);
    } else {
      n[i] = el16<T>(own, 2 * i);
      nh[i] = el16<T>(halo, 2 * i);
      nd[i] = el16<T>(hdn, 2 * i);
    }
  }
  uint32_t nx1 = shdn(n[0], 1), nhx1 = shdn(nh[0], 1), ndx1 = ONE ? shdn(nd[0], 1) : 0u;
  if (xlast) {  // node X+VX = Ex: the mirrored node Ex-1 (even pad), or no cell at all (odd)
    nx1 = n[VX - 1];
    nhx1 = nh[VX - 1];
    ndx1 = nd[VX - 1];
  }
  uint32_t M1[VX + 1], M0[VX + 1];  // mean: cell rows Y / Y-1, cols X-1 .. X+VX-1
  uint32_t P0[VX + 1], P1[VX + 1], P2[VX + 1], A3[VX + 1], P4[VX + 1];  // LIN channels (q = cell X-1+q)
  if constexpr (!LIN) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t h = n[i] + (i + 1 < VX ? n[i + 1] : nx1);
      const uint32_t hh = nh[i] + (i + 1 < VX ? nh[i + 1] : nhx1);
      if constexpr (ONE) {
        M1[i + 1] = (h + nd[i] + (i + 1 < VX ? nd[i + 1] : ndx1)) >> 2;
        M0[i + 1] = (hh + h) >> 2;
      } else {
        const uint32_t below = shdn(h, a.txn);
        M1[i + 1] = (h + (last ? hh : below)) >> 2;
        const uint32_t above = shup(M1[i + 1], a.txn);
        M0[i + 1] = first ? (hh + h) >> 2 : above;
      }
    }
    M1[0] = shup(M1[VX], 1);
    M0[0] = shup(M0[VX], 1);
  } else {
    // node rows Y (n), Y+1 (nb) and Y-1 (nu: this lane's halo when it is the wave's first row)
    float fn[VX + 1], fb[VX + 1], fu[VX + 1];
    const uint32_t bx1 = shdn(nx1, a.txn);
#pragma unroll
    for (int i = 0; i <= VX; ++i) {
      const uint32_t own_i = i < VX ? n[i] : nx1;
      const uint32_t below_i = i < VX ? shdn(n[i], a.txn) : bx1;
      const uint32_t halo_dn = ONE ? (i < VX ? nd[i] : ndx1) : (i < VX ? nh[i] : nhx1);
      fn[i] = (float)own_i;
      fb[i] = (float)((ONE || last) ? halo_dn : below_i);
      fu[i] = (float)(i < VX ? nh[i] : nhx1);
    }
    auto chan = [&](int k, const float (&r0)[VX + 1], const float (&r1)[VX + 1], uint32_t (&o)[VX + 1]) {
      const float w0 = a.wt[0 * 5 + k], w1 = a.wt[1 * 5 + k], w2 = a.wt[2 * 5 + k], w3 = a.wt[3 * 5 + k];
      const float bk = a.bias[k];
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        float acc = bk;
        acc = __builtin_fmaf(r0[i], w0, acc);
        acc = __builtin_fmaf(r0[i + 1], w1, acc);
        acc = __builtin_fmaf(r1[i], w2, acc);
        acc = __builtin_fmaf(r1[i + 1], w3, acc);
        o[i + 1] = cast_t<T>(acc);
      }
    };
    uint32_t P3[VX + 1], U3[VX + 1];
    chan(0, fn, fb, P0);
    chan(1, fn, fb, P1);
    chan(2, fn, fb, P2);
    chan(3, fn, fb, P3);
    chan(4, fn, fb, P4);
    chan(3, fu, fn, U3);  // cell row Y-1 (used on the wave's first row)
#pragma unroll
    for (int i = 1; i <= VX; ++i) {
      const uint32_t above = shup(P3[i], a.txn);
      A3[i] = (ONE || first) ? U3[i] : above;
    }
    P1[0] = shup(P1[VX], 1);
  }
  if (!live || Y < a.ybeg || Y >= a.yend) return;

  bool vx[VX + 1];
  cells_valid<VX>(vx, X, a.Lcx);
  const uint32_t ny = (uint32_t)vy0 + (uint32_t)vy1;
  uint32_t pred[3][VX];  // LR, UD, C
  if constexpr (!LIN) {
#pragma unroll
    for (int q = 0; q <= VX; ++q) {
      M1[q] = (vy1 && vx[q]) ? M1[q] : 0u;
      M0[q] = (vy0 && vx[q]) ? M0[q] : 0u;
    }
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
      pred[0][i] = (M1[i] + M1[i + 1]) >> (nx >> 1);      // LR: cells (Y, x-1), (Y, x)
      pred[1][i] = (M0[i + 1] + M1[i + 1]) >> (ny >> 1);  // UD: cells (Y-1, x), (Y, x)
      pred[2][i] = M1[i + 1];                             // C
    }
  } else {
    auto m = [&](const uint32_t (&v)[VX + 1], int q, bool yok) { return (yok && vx[q]) ? v[q] : 0u; };
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
      pred[0][i] = (m(P0, i + 1, vy1) + m(P1, i, vy1)) >> (nx >> 1);  // LR: ch0 (x), ch1 (x-1)
      pred[1][i] = (m(P2, i + 1, vy1) + m(A3, i + 1, vy0)) >> (ny >> 1);  // UD: ch2 (y), ch3 (y-1)
      pred[2][i] = m(P4, i + 1, vy1);                                  // C: ch4
    }
  }
  if constexpr (!DEC) {
    uint32_t lov[VX], res[3][VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      lov[i] = el16<T>(own, 2 * i);
      res[0][i] = (el16<T>(o0, 2 * i) - pred[0][i]) & MASK;       // LR (1,0)
      res[1][i] = (el16<T>(own, 2 * i + 1) - pred[1][i]) & MASK;  // UD (0,1)
      res[2][i] = (el16<T>(o0, 2 * i + 1) - pred[2][i]) & MASK;   // C  (1,1)
    }
    stp8<STC>((T*)a.lo_out + m_ud, pack8<T, VX>(lov));
    if (vy1) stp8<STC>((T*)a.maps.p[0] + m_lr, pack8<T, VX>(res[0]));
    stp8<STC>((T*)a.maps.p[1] + m_ud, pack8<T, VX>(res[1]));
    if (vy1) stp8<STC>((T*)a.maps.p[2] + m_lr, pack8<T, VX>(res[2]));
  } else {
    uint32_t dv[3][VX];
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int i = 0; i < VX; ++i) dv[k][i] = (pred[k][i] + el8<T>(mv[k], i)) & MASK;
    T* h0 = hout + 2 * Yc * a.W + hx;
    st16(h0, pack16<T, VX>(n, dv[1]));                    // row 2Y: lowres | UD
    if (vy1) st16(h0 + a.W, pack16<T, VX>(dv[0], dv[2]));  // row 2Y+1: LR | C
  }
}

// A workgroup codes the virtual blocks blockIdx.x, + gridDim.x, ... (grid-stride; a multiple of 8
// workgroups keeps every virtual block on the XCD of the image-per-XCD order): fewer, longer-lived
// workgroups than one per 16 output rows (2 virtual blocks per workgroup)
template <typename T, bool DEC, bool ONE, bool LIN, bool STC = false>
__global__ void __launch_bounds__(256) wave2d_kernel(W2 a) {
  for (int v = (int)blockIdx.x; v < a.nvblk; v += (int)gridDim.x) wave2d_body<T, DEC, ONE, LIN, STC>(a, v);
}

// uint8 decode form of the mean kernel (BASELINE config C2), SWAR: the lane's 8 cells travel as 4 words
// of two 16-bit lanes each, so every node / mean / prediction / residual step is one 32-bit op
// for two cells (node pair sums <= 510, means <= 255: no carry between the halves; residuals add
// 256 per half before subtracting, so no borrow).  Bytes are split / merged with v_perm.  The
// arithmetic is the generic kernel's above, element for element; the SQ counters showed that
// kernel's VALU busy 67 % of its cycles at C2.
__device__ __forceinline__ uint32_t lo_pair(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c010c00u); }
__device__ __forceinline__ uint32_t hi_pair(uint32_t w) { return __builtin_amdgcn_perm(0u, w, 0x0c030c02u); }
__device__ __forceinline__ uint32_t pack_pairs(uint32_t a, uint32_t b) {  // 16-bit-lane bytes -> 4 bytes
  return __builtin_amdgcn_perm(b, a, 0x06040200u);
}
__device__ __forceinline__ uint32_t shift_pairs(uint32_t hi, uint32_t lo) {  // {lo.hi16, hi.lo16}
  return __builtin_amdgcn_alignbit(hi, lo, 16);
}

__device__ __forceinline__ void wave2d_u8_dec_body(const W2& a, int vblk) {
  constexpr int VX = 8;
  constexpr uint32_t B8 = 0x00ff00ffu;

  const int lane = threadIdx.x & 63;
  const int wv_ = threadIdx.x >> 6;
  const int tx = lane & (a.txn - 1);          // txn: a power of two (host)
  const int r = lane >> __builtin_ctz(a.txn);
  const int X = tx * VX;
  // (the u8 decode: 22.0 -> 21.7 us; the encode body keeps % and /, 24.1 vs 24.6 us with this form,
  // profiles/round4/ab_udiv_r4l5.log)
  // virtual block -> (image b, row group grp); image-per-XCD order (xcd_per == ngrp): XCD x = vblk % 8
  // codes whole images, its k-th block is group k % ngrp of image (k / ngrp) * 8 + x
  const bool xcd = a.xcd_per > 0;
  const uint32_t kk = xcd ? (uint32_t)vblk >> 3 : (uint32_t)vblk;
  const uint32_t qq = udiv(kk, a.ngrp_div);
  const int grp = (int)(kk - qq * (uint32_t)a.ngrp);
  const int64_t b = xcd ? (int64_t)qq * 8 + (vblk & 7) : (int64_t)qq;
  const int Y0 = (grp * a.nwv + wv_) * a.rows;
  if (Y0 >= a.Ey) return;  // whole idle wave
  const int Y = Y0 + r;
  const bool live = Y < a.Ey;
  const int Yc = live ? Y : a.Ey - 1;
  const bool first = r == 0;
  const bool last = r == a.rows - 1 || Y == a.Ey - 1;
  const bool vy1 = Y < a.Lcy;
  const bool vy0 = Y >= 1;
  const bool need_halo = live && ((first && Y0 >= 1) || (last && vy1));
  const int yh = first ? (Y0 >= 1 ? Y0 - 1 : 0) : lsrc(Yc + 1, a.Ly, a.Ey);
  const bool xlast = tx == a.txn - 1;

  const int64_t himg = (int64_t)a.H * a.W;
  const int hx = 2 * X;
  uint8_t* hout = (uint8_t*)a.hi_out + b * himg;
  const uint8_t* lin = (const uint8_t*)a.lo_in + b * (int64_t)a.Ey * a.Ex;
  const int64_t m_lr = (b * a.Lcy + Yc) * a.Ex + X;
  const int64_t m_ud = (b * a.Ey + Yc) * a.Ex + X;

  uint2 own{}, halo{};
  uint2 mv[3] = {make_uint2(0, 0), make_uint2(0, 0), make_uint2(0, 0)};
  if (live) own = ld8c(lin + Yc * a.Ex + X);
  if (need_halo) halo = ld8c(lin + yh * a.Ex + X);
  if (live && vy1) mv[0] = ld8((const uint8_t*)a.maps.p[0] + m_lr);
  if (live) mv[1] = ld8((const uint8_t*)a.maps.p[1] + m_ud);
  if (live && vy1) mv[2] = ld8((const uint8_t*)a.maps.p[2] + m_lr);

  // nodes as pairs: N[k] = {n[2k], n[2k+1]}
  uint32_t N[4], NH[4];
  N[0] = lo_pair(own.x); N[1] = hi_pair(own.x); N[2] = lo_pair(own.y); N[3] = hi_pair(own.y);
  NH[0] = lo_pair(halo.x); NH[1] = hi_pair(halo.x); NH[2] = lo_pair(halo.y); NH[3] = hi_pair(halo.y);
  uint32_t nx1 = shdn(N[0], 1), nhx1 = shdn(NH[0], 1);  // node X+8 (low half)
  if (xlast) {  // the mirrored node Ex-1 (even pad), or no cell at all (odd)
    nx1 = N[3] >> 16;
    nhx1 = NH[3] >> 16;
  }
  uint32_t M1[4], M0[4];  // cell means of rows Y / Y-1, cells X+2k, X+2k+1
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t h = N[k] + shift_pairs(k < 3 ? N[k + 1] : nx1, N[k]);
    const uint32_t hh = NH[k] + shift_pairs(k < 3 ? NH[k + 1] : nhx1, NH[k]);
    const uint32_t below = shdn(h, a.txn);
    M1[k] = ((h + (last ? hh : below)) >> 2) & B8;
    const uint32_t above = shup(M1[k], a.txn);
    M0[k] = first ? ((hh + h) >> 2) & B8 : above;
  }
  uint32_t m1l = shup(M1[3], 1) >> 16;  // cell X-1 (the UD prediction needs no left cell)
  if (!live || Y < a.ybeg || Y >= a.yend) return;

  // validity of cells X-1 .. X+7 (vx[q] = cell X-1+q) as per-half masks
  bool vx[VX + 1];
  cells_valid<VX>(vx, X, a.Lcx);
  uint32_t VM[4], BM[4];  // VM: cells X+2k, X+2k+1 valid; BM: both neighbours of the LR pair valid
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    VM[k] = (vx[2 * k + 1] ? 0x0000ffffu : 0u) | (vx[2 * k + 2] ? 0xffff0000u : 0u);
    BM[k] = (vx[2 * k] && vx[2 * k + 1] ? 0x0000ffffu : 0u) | (vx[2 * k + 1] && vx[2 * k + 2] ? 0xffff0000u : 0u);
  }
  m1l = (vy1 && vx[0]) ? m1l : 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    M1[k] = vy1 ? (M1[k] & VM[k]) : 0u;
    M0[k] = vy0 ? (M0[k] & VM[k]) : 0u;
  }
  const bool ud2 = vy0 && vy1;
  uint32_t PL[4], PU[4];  // LR, UD predictions; C is M1
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t left = shift_pairs(M1[k], k == 0 ? m1l << 16 : M1[k - 1]);  // cells X+2k-1, X+2k
    const uint32_t sl = left + M1[k];
    PL[k] = (((sl >> 1) & 0x7fff7fffu) & BM[k]) | (sl & ~BM[k]);
    const uint32_t su = M0[k] + M1[k];
    PU[k] = ud2 ? (su >> 1) & 0x7fff7fffu : su;
  }
  {
    const uint32_t el[4] = {lo_pair(mv[0].x), hi_pair(mv[0].x), lo_pair(mv[0].y), hi_pair(mv[0].y)};
    const uint32_t eu[4] = {lo_pair(mv[1].x), hi_pair(mv[1].x), lo_pair(mv[1].y), hi_pair(mv[1].y)};
    const uint32_t ec[4] = {lo_pair(mv[2].x), hi_pair(mv[2].x), lo_pair(mv[2].y), hi_pair(mv[2].y)};
    uint32_t r0[4], r1[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t dl = (PL[k] + el[k]) & B8, du = (PU[k] + eu[k]) & B8, dc = (M1[k] + ec[k]) & B8;
      r0[k] = N[k] | (du << 8);  // row 2Y:   lowres | UD
      r1[k] = dl | (dc << 8);    // row 2Y+1: LR | C
    }
    uint8_t* h0 = hout + 2 * Yc * a.W + hx;
    st16(h0, make_uint4(r0[0], r0[1], r0[2], r0[3]));
    if (vy1) st16(h0 + a.W, make_uint4(r1[0], r1[1], r1[2], r1[3]));
  }
}

__global__ void __launch_bounds__(256) wave2d_u8_dec_kernel(W2 a) {
  for (int v = (int)blockIdx.x; v < a.nvblk; v += (int)gridDim.x) wave2d_u8_dec_body(a, v);
}

}  // namespace w2

template <typename T>
static bool wave2d_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, const kmp_region* region,
                            w2::W2& a, dim3& grid, dim3& block) {
  constexpr int VX = 8 / (int)sizeof(T);
  if (!(std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value)) return false;
  if (opt(OPT_DISABLE_WAVE, 0) || opt(OPT_DISABLE_FAST, 0)) return false;
  if (C != 1 || pred->padding != 0) return false;
  if (pred->kind != KMP_PRED_MEAN && !(pred->kind == KMP_PRED_LINEAR && pred->weights && pred->bias)) return false;
  if (pred->kind == KMP_PRED_LINEAR && opt(OPT_DISABLE_LINEAR_FUSED, 0)) return false;
  int64_t yb = 0, ye = g.E[1];
  if (region) {  // only row ranges (full width): the fused chunked drivers' merged slabs
    if (region->begin[2] > 0 || region->end[2] < g.E[2]) return false;
    yb = region->begin[1] < 0 ? 0 : region->begin[1];
    ye = region->end[1] > g.E[1] ? g.E[1] : region->end[1];
    if (ye <= yb) return false;
  }
  if (g.n[2] % 2 != 0 || (g.n[2] * (int64_t)sizeof(T)) % 16 != 0) return false;
  if (g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;  // 32-bit offsets inside an image
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || txn < 1 || txn > 64 || (txn & (txn - 1)) != 0) return false;
  const int64_t rows = 64 / txn;
  if (rows > 1 && g.E[1] % rows == 1) return false;  // a one-row wave in a multi-row layout
  const int64_t waves = ceil_div(g.E[1], rows);
  const int64_t nwv = waves < 4 ? waves : 4;
  const int64_t ngrp = ceil_div(waves, nwv);
  a.H = (int)g.n[1]; a.W = (int)g.n[2];
  a.Ly = (int)g.L[1]; a.Lx = (int)g.L[2];
  a.Ey = (int)g.E[1]; a.Ex = (int)g.E[2];
  a.Lcy = (int)g.Lc[1]; a.Lcx = (int)g.Lc[2];
  a.txn = (int)txn; a.rows = (int)rows; a.nwv = (int)nwv; a.ngrp = (int)ngrp;
  a.xcd_per = (opt(OPT_W2_XCD, 1) && B % 8 == 0) ? (int)ngrp : 0;
  a.ngrp_div = make_udiv((uint32_t)ngrp);
  a.ybeg = (int)yb;
  a.yend = (int)ye;
  const int64_t nblk = B * ngrp;
  const int64_t iters = 2;  // 2: +5 % encode, +1.5 % decode at C2 (ab_wave2d_iters.log)
  int64_t nwg = ceil_div(nblk, iters);
  if (a.xcd_per > 0) nwg = ceil_div(nwg, (int64_t)8) * 8;  // keep v % 8 == blockIdx % 8
  a.nvblk = (int)nblk;
  grid = dim3((unsigned)std::min(nwg, nblk));
  block = dim3((unsigned)(64 * nwv));
  return nblk < ((int64_t)1 << 31);
}

template <typename T, bool DEC, bool STC>
static void launch_wave2d_s(bool one, bool lin, dim3 grid, dim3 block, hipStream_t s, const w2::W2& a) {
  if (one) {
    if (lin) w2::wave2d_kernel<T, DEC, true, true, STC><<<grid, block, 0, s>>>(a);
    else w2::wave2d_kernel<T, DEC, true, false, STC><<<grid, block, 0, s>>>(a);
  } else {
    if (lin) w2::wave2d_kernel<T, DEC, false, true, STC><<<grid, block, 0, s>>>(a);
    // SWAR u8 decode: 24.0 vs 24.8 us at C2 on one box; the SWAR encode measured slower (26.2 vs
    // 25.4: bound by its row loads, not VALU) and was removed -- profiles/round1/ab_wave2d_swar.log
    else if (DEC && std::is_same<T, uint8_t>::value && !opt(OPT_DISABLE_SWAR, 0))
      w2::wave2d_u8_dec_kernel<<<grid, block, 0, s>>>(a);
    else w2::wave2d_kernel<T, DEC, false, false, STC><<<grid, block, 0, s>>>(a);
  }
}

// the encode's lowres / map stores cached (stp8, kmp_wave.h) unless KMP_W2_ST_ENC=0
template <typename T, bool DEC>
static void launch_wave2d(bool one, bool lin, dim3 grid, dim3 block, hipStream_t s, const w2::W2& a) {
  if (!DEC && opt(OPT_W2_ST_ENC, 1)) launch_wave2d_s<T, DEC, true>(one, lin, grid, block, s, a);
  else launch_wave2d_s<T, DEC, false>(one, lin, grid, block, s, a);
}

template <typename T>
int try_wave2d_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                      const MapPtrs& maps, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w2::W2 a{};
    dim3 grid, block;
    if (!wave2d_geometry<T>(g, B, C, pred, region, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 3; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    a.wt = pred->weights;
    a.bias = pred->bias;
    launch_wave2d<T, false>(a.rows == 1, pred->kind == KMP_PRED_LINEAR, grid, block, stream, a);
    return check_launch("wave2d_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_wave2d_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                      const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    w2::W2 a{};
    dim3 grid, block;
    if (!wave2d_geometry<T>(g, B, C, pred, region, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 3; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    a.wt = pred->weights;
    a.bias = pred->bias;
    launch_wave2d<T, true>(a.rows == 1, pred->kind == KMP_PRED_LINEAR, grid, block, stream, a);
    return check_launch("wave2d_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_W2_INST(T)                                                                                    \
  template int try_wave2d_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,     \
                                    const MapPtrs&, const kmp_region*, hipStream_t);                      \
  template int try_wave2d_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,              \
                                    const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_W2_INST(uint8_t)
KMP_W2_INST(uint16_t)
KMP_W2_INST(int32_t)
KMP_W2_INST(uint32_t)

}  // namespace kmp
