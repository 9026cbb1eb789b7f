// kmp_codec_linear3dp.hip -- one-pass volume encode / decode for the LinearPredictor with p >= 1
// (SURVEY.md §8a row a9', the north star's "learned-predictor apply"; p = 1 is instantiated).
//
// pred[cell, k] = fma-chain over n = 0..N-1 of feat[cell, n] * W[n, k] from b[k] (N = (2p+2)^3,
// features in the reference's z-major order, features_from_lowres volume/utils.py:199-210), cast
// to T, aggregated onto the 7 maps (volume/utils.py:83-155) and coded (utils.py:38-55) -- the
// arithmetic of kmp_codec_linear3d.hip (p = 0) with a 64-term chain per channel-cell.
//
// A workgroup owns one output plane c of one tile (its waves own 8 rows each, as in the p = 0
// kernel).  The 2p+3 node planes c-1-p .. c+p+1 that the cells of planes c-1 and c read are
// staged in LDS as f32 with the mirrored halo rows / columns of the symmetric neighbourhood pad
// over the even reflect pad (volume/utils.py:213-237) -- every node byte is read from HBM once
// per plane-workgroup, the neighbourhood comes from LDS.  Each lane evaluates the 19
// channel-cells its 4 outputs read (14 channels of its plane-c cells, 5 of its plane-(c-1) cells;
// the channels of row Y-1 come from the lane above, across waves through LDS), in two sweeps over
// the neighbourhood: per node row (dz, dy) one 2 x 16-byte LDS read of the lane's 7 nodes feeds
// every channel of the sweep.  The chain runs on packed f32 VALU FMAs with the weights in scalar
// registers (uniform loads); the per-channel chain order is n ascending, so the f32 values are
// bit-identical to the oracle's fma chain.
//
// Why not the matrix cores: on MI355X the f32 MFMA (v_mfma_f32_16x16x4_f32 / 32x32x2) runs on the
// same f32 datapath as the VALU -- tools/probe_mfma_valu.hip (profiles/round3/probe_mfma_valu.log):
// one instruction stream interleaving f32 MFMAs with packed FMAs takes the SUM of the two streams'
// times (322-331 us = 244-258 + 72-78), the same stream with bf16 MFMAs about the MAX (198 vs 180 +
// 75).  So an f32 MFMA only replaces packed FMAs at about the same rate (27.7 vs 23.3 MAC/clk/SIMD
// in the probe) and cannot overlap the epilogue, while the 19 channels pad to 16-wide tiles and the
// results need a transpose back to the lanes that own the cells.  Three bit-exact matrix-core forms
// were built and measured slower at C3 (profiles/round3/ab_linear3_mfma_rejected.log: a per-plane
// 4-wave kernel 598 / 581 us and a one-wave-per-workgroup kernel 625 / 591 us against this kernel's
// 551-564 / 509-515 us; round 2's z-rolling kernel 573 / 540) and removed.
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace l3p {

using namespace wv;

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct L3P {
  const void* hi_in;
  void* hi_out;
  const void* lo_in;
  void* lo_out;
  MapPtrs maps;
  const float* W;  // [N, 19] row-major
  const float* b;  // [19]
  const float* Wr; // the weights reordered per sweep (linear_reorder_kernel), in the workspace
  int32_t D, H, W_;
  int32_t Lz, Ly, Lx, Ez, Ey, Ex, Lcz, Lcy, Lcx;
  int32_t zbegin, zend;
  int32_t txn, rows, nwv;
  int32_t xcd_per;
  int32_t nr, pitch;  // staged node rows per plane (Ey + 2p + 1), f32 words per staged row
};

constexpr int kXch = 5;  // channels exchanged downwards: 3, 9, 10, 16 (plane c), 17 (plane c-1)
// The two sweeps' channels: plane c-1 cells (5) then plane c cells (14)
constexpr int kNQ = 5, kNC = 14;
__constant__ const int kKQ[kNQ] = {5, 13, 14, 17, 18};
__constant__ const int kKC[kNC] = {0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 15, 16};

// W [N, 19] -> per sweep [node row][kk][dx] (N = NB^3, rows = NB^2): the order the sweeps consume.
__global__ void __launch_bounds__(256) linear_reorder_kernel(const float* __restrict__ W, float* __restrict__ Wr,
                                                            int NB) {
  const int rows = NB * NB, nq = rows * kNQ * NB, total = nq + rows * kNC * NB;
  for (int t = threadIdx.x; t < total; t += blockDim.x) {
    const bool q = t < nq;
    const int u = q ? t : t - nq, nk = q ? kNQ : kNC;
    const int dx = u % NB, kk = (u / NB) % nk, row = u / (NB * nk);
    const int k = q ? kKQ[kk] : kKC[kk];
    Wr[t] = W[(row * NB + dx) * 19 + k];
  }
}

// One sweep: channels KS[0..NK) of the lane's VX = 4 cells (row Y, cols X..X+3) of cell plane
// c-1+PLANE, from the staged planes.  Results cast to T in out[kk][1..4].
// All-zero weights and bias: the channels of a cell plane outside the tile (plane c-1 at c = 0,
// plane c at c >= Lcz) evaluated with these are 0.0 -> 0, what the aggregation's mask gives them
// (FULL kernel: the plane masks disappear from the aggregation)
__constant__ float kZeroW[kNC * 64 + 19];

template <typename T, int P, int PLANE, int NK>
__device__ __forceinline__ void sweep(const float* st, const L3P& a, int Yc, int X, const int (&KS)[NK], int woff,
                                      bool zero, uint32_t (&out)[NK][5]) {
  constexpr int NB = 2 * P + 2;
  constexpr int NF = 4 + 2 * P + 1;  // nodes X-P .. X+3+P+1
  constexpr int NV = (NF + 3) / 4;   // 16-byte LDS reads per node row
  // the sweep's weights in consumption order [node row][kk][dx] (a.Wr, written by
  // linear_reorder_kernel), read through the constant address space: per node row NK x NB
  // contiguous words = a few wide uniform scalar loads into SGPRs
  typedef const __attribute__((address_space(4))) float* CF;
  const CF Wc = zero ? (CF)kZeroW : (CF)(a.Wr + woff);
  const CF Bc = zero ? (CF)kZeroW : (CF)a.b;
  f32x2 acc[NK][2];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    const float bk = Bc[KS[kk]];
    acc[kk][0] = (f32x2){bk, bk};
    acc[kk][1] = (f32x2){bk, bk};
  }
  // one node row per iteration: its NK x 4 weights fit the scalar registers; dx outer so that
  // consecutive FMAs go to different accumulators (each accumulator's chain stays n-ascending)
#pragma unroll 1
  for (int row = 0; row < NB * NB; ++row) {
    const int dz = row / NB, dy = row % NB;
    // 16-byte aligned: X and the pitch are multiples of 4 words
    const float* rowp = (const float*)__builtin_assume_aligned(st + ((PLANE + dz) * a.nr + (Yc + dy)) * a.pitch + X, 16);
    float f[4 * NV];
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float4 q = *(const float4*)(rowp + 4 * v);
      f[4 * v] = q.x; f[4 * v + 1] = q.y; f[4 * v + 2] = q.z; f[4 * v + 3] = q.w;
    }
    float w[NK][NB];
#pragma unroll
    for (int kk = 0; kk < NK; ++kk)
#pragma unroll
      for (int dx = 0; dx < NB; ++dx) w[kk][dx] = Wc[(row * NK + kk) * NB + dx];
#pragma unroll
    for (int dx = 0; dx < NB; ++dx) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const f32x2 w2 = {w[kk][dx], w[kk][dx]};
        acc[kk][0] = __builtin_elementwise_fma((f32x2){f[dx], f[dx + 1]}, w2, acc[kk][0]);
        acc[kk][1] = __builtin_elementwise_fma((f32x2){f[dx + 2], f[dx + 3]}, w2, acc[kk][1]);
      }
    }
  }
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    out[kk][1] = cvt_sat<T>(acc[kk][0].x);
    out[kk][2] = cvt_sat<T>(acc[kk][0].y);
    out[kk][3] = cvt_sat<T>(acc[kk][1].x);
    out[kk][4] = cvt_sat<T>(acc[kk][1].y);
  }
}

// FULL: the tile's cells fill the stored lowres rows and columns (Lcy == Ey, Lcx == Ex: every
// even-sized tile, C3's 64^3 included).  Then the y+1 validity and every x validity but the row's
// first cell are compile-time true and a missing cell plane is zeroed at the source (kZeroW), so
// the aggregation masks only the row-above channels on row 0 and the left cell on lane 0 (the p = 0
// kernel's FULL body, kmp_codec_linear3d.hip)
template <typename T, bool DEC, int P, bool FULL>
__global__ void __launch_bounds__(256) linear3dp_kernel(L3P a) {
  constexpr int VX = 4;  // 4 outputs per lane (u8 and u16: kmp_wave.h's 4-cell segments)
  static_assert(sizeof(T) <= 2, "u8 / u16");
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  constexpr int NPL = 2 * P + 3;  // staged node planes c-1-P .. c+P+1
  using V = typename std::conditional<DEC, MSeg<T>, HSeg<T>>::type;
  // LDS: staged node planes [NPL][nr][pitch] f32, then the exchange rows [wave][kXch][Ex]
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  float* st = (float*)smem;
  const int plane_words = a.nr * a.pitch;
  uint32_t* xrow = smem + NPL * plane_words;

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
  const int nplanes = a.zend - a.zbegin;
  const int c = a.zbegin + blk % nplanes;
  const int64_t b = blk / nplanes;
  const int Y0 = wv_ * a.rows;
  const bool wave_live = Y0 < a.Ey;
  const int Y = Y0 + r;
  const bool live = wave_live && Y < a.Ey;
  const int Yc = live ? Y : a.Ey - 1;
  const bool first = r == 0;
  const bool vy1 = FULL || Y < a.Lcy;  // FULL: Lcy == Ey, and lanes past Ey are not live
  const bool vy0 = Y >= 1;
  const bool vz1 = c < a.Lcz, vz0 = c >= 1;

  const int hplane = a.H * a.W_;
  const int lplane = a.Ey * a.Ex;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * (int64_t)a.D * hplane;
  T* hout = DEC ? (T*)a.hi_out + b * (int64_t)a.D * hplane : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ez * lplane : nullptr;
  const int hx = 2 * X;
  const int ho_own = 2 * Yc * a.W_ + hx;
  const int lo_own = Yc * a.Ex + X;

  const T* mbase[7];
  int mplane[7];
  bool mok_y[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez, ey = par[1] ? a.Lcy : a.Ey;
    mplane[k] = ey * a.Ex;
    mbase[k] = (const T*)a.maps.p[k] + b * (int64_t)ez * mplane[k] + Yc * a.Ex + X;
    mok_y[k] = live && (!par[1] || vy1);
  }

  // ---- all loads up front: the lane's node row of every staged plane, then the stream rows ----
  V own[NPL] = {};
#pragma unroll
  for (int t = 0; t < NPL; ++t) {
    const int sz = lsrc1(c - 1 - P + t, a.Lz, a.Ez);
    if constexpr (DEC) {
      if (live) own[t] = ldMc<T>(lin + sz * lplane + lo_own);
    } else {
      if (live) own[t] = ldHc<T>(hin + 2 * sz * hplane + ho_own);
    }
  }
  HSeg<T> e1{}, o0{}, o1{};
  MSeg<T> mv[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) mv[k] = MSeg<T>{};
  if constexpr (DEC) {
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      int par[3];
      map_parity(3, k, par);
      if (mok_y[k] && (!par[0] || vz1)) mv[k] = ldM<T>(mbase[k] + c * mplane[k]);
    }
  } else {
    const T* p = hin + 2 * c * hplane;
    if (live && vy1) e1 = ldH<T>(p + ho_own + a.W_);
    if (live && vz1) o0 = ldH<T>(p + hplane + ho_own);
    if (live && vz1 && vy1) o1 = ldH<T>(p + hplane + ho_own + a.W_);
  }

  // ---- stage: every lane writes its 4 nodes of each plane, plus the mirrored halo columns /
  // rows it is the source of (symmetric pad over the even reflect pad: lsrc), then one barrier ----
  if (live) {
    constexpr int NHR = 4 * ((VX + 2 * P + 1 + 3) / 4) - VX - P;  // halo columns right of Ex
    const bool xfirst = tx == 0, xlast = tx == a.txn - 1;
#pragma unroll
    for (int t = 0; t < NPL; ++t) {
      float v[VX];
#pragma unroll
      for (int i = 0; i < VX; ++i)
        v[i] = (float)(DEC ? elM<T>(*(const MSeg<T>*)&own[t], i) : elH<T>(*(const HSeg<T>*)&own[t], 2 * i));
      auto put_row = [&](int ry) __attribute__((always_inline)) {
        float* row = st + (t * a.nr + ry) * a.pitch + P + X;
#pragma unroll
        for (int i = 0; i < VX; ++i) row[i] = v[i];
        if (xfirst) {
#pragma unroll
          for (int k = 1; k <= P; ++k) row[-k] = v[k - 1];  // node column -k mirrors column k-1
        }
        if (xlast) {
#pragma unroll
          for (int j = 0; j < NHR; ++j) {
            const int sx = lsrc1(a.Ex + j, a.Lx, a.Ex) - X;
            float u = v[0];
#pragma unroll
            for (int i = 1; i < VX; ++i) u = sx == i ? v[i] : u;
            row[VX + j] = u;
          }
        }
      };
      put_row(Y + P);
#pragma unroll
      for (int h = 0; h < 2 * P + 1; ++h) {  // node rows -P .. -1 and Ey .. Ey+P
        const int rr = h < P ? h - P : a.Ey + (h - P);
        if (lsrc1(rr, a.Ly, a.Ey) == Y) put_row(rr + P);
      }
    }
  }
  __syncthreads();

  // ---- the 19 channel-cells of the lane's outputs ----
  constexpr int KC[kNC] = {0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 15, 16};  // plane c
  constexpr int KQ[kNQ] = {5, 13, 14, 17, 18};                               // plane c-1
  uint32_t PC[14][5], PQ[5][5];
  sweep<T, P, 0, 5>(st, a, Yc, X, KQ, 0, FULL && !vz0, PQ);
  sweep<T, P, 1, 14>(st, a, Yc, X, KC, kNQ * (2 * P + 2) * (2 * P + 2) * (2 * P + 2), FULL && !vz1, PC);
  auto& P0 = PC[0]; auto& P1 = PC[1]; auto& P2 = PC[2]; auto& P3 = PC[3]; auto& P4 = PC[4];
  auto& P6 = PC[5]; auto& P7 = PC[6]; auto& P8 = PC[7]; auto& P9 = PC[8]; auto& P10 = PC[9];
  auto& P11 = PC[10]; auto& P12 = PC[11]; auto& P15 = PC[12]; auto& P16 = PC[13];
  auto& Q5 = PQ[0]; auto& Q13 = PQ[1]; auto& Q14 = PQ[2]; auto& Q17 = PQ[3]; auto& Q18 = PQ[4];

  // channels 3, 9, 10, 16 (plane c) and 17 (plane c-1) of row Y-1: the lane above, or the wave
  // above through LDS
  uint32_t A3[VX + 1], A9[VX + 1], A10[VX + 1], A16[VX + 1], QA17[VX + 1];
  if (wave_live && r == a.rows - 1) {
    uint32_t* row = xrow + (size_t)wv_ * kXch * a.Ex;
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      row[0 * a.Ex + X + i] = P3[i + 1];
      row[1 * a.Ex + X + i] = P9[i + 1];
      row[2 * a.Ex + X + i] = P10[i + 1];
      row[3 * a.Ex + X + i] = P16[i + 1];
      row[4 * a.Ex + X + i] = Q17[i + 1];
    }
  }
#pragma unroll
  for (int i = 1; i <= VX; ++i) {
    A3[i] = shup(P3[i], a.txn);
    A9[i] = shup(P9[i], a.txn);
    A10[i] = shup(P10[i], a.txn);
    A16[i] = shup(P16[i], a.txn);
    QA17[i] = shup(Q17[i], a.txn);
  }
  __syncthreads();
  if (first && wv_ >= 1) {
    const uint32_t* row = xrow + (size_t)(wv_ - 1) * kXch * a.Ex;
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      A3[i + 1] = row[0 * a.Ex + X + i];
      A9[i + 1] = row[1 * a.Ex + X + i];
      A10[i + 1] = row[2 * a.Ex + X + i];
      A16[i + 1] = row[3 * a.Ex + X + i];
      QA17[i + 1] = row[4 * a.Ex + X + i];
    }
  }
  A9[0] = shup(A9[VX], 1);  // cell (Y-1, X-1): the lane to the left
  P1[0] = shup(P1[VX], 1);
  P8[0] = shup(P8[VX], 1);
  P12[0] = shup(P12[VX], 1);
  Q13[0] = shup(Q13[VX], 1);
  if (!live) return;

  bool vx[VX + 1];
#pragma unroll
  for (int q = 0; q <= VX; ++q) vx[q] = (FULL && q >= 1) || ((X - 1 + q) >= 0 && (X - 1 + q) < a.Lcx);
  const uint32_t ny = (uint32_t)vy0 + (uint32_t)vy1;
  const uint32_t nz = (uint32_t)vz0 + (uint32_t)vz1;
  auto m = [&](const uint32_t (&v)[VX + 1], int q, bool zok, bool yok) {
    return ((FULL || zok) && yok && vx[q]) ? v[q] : 0u;  // FULL: a missing z plane's channels are 0 already
  };
  auto put8 = [&](int k, const uint32_t (&res)[VX]) {
    int par[3];
    map_parity(3, k, par);
    if (mok_y[k] && (!par[0] || vz1)) stM<T>((T*)mbase[k] + c * mplane[k], packM<T>(res));
  };
  const int tc = 1 + P;  // staged plane index of node plane c
  const HSeg<T> e0 = DEC ? HSeg<T>{} : *(const HSeg<T>*)&own[tc];
  T* h0 = DEC ? hout + 2 * c * hplane + ho_own : nullptr;
  uint32_t ownv[VX];
#pragma unroll
  for (int i = 0; i < VX; ++i) {
    if constexpr (DEC) ownv[i] = elM<T>(*(const MSeg<T>*)&own[tc], i);
    else ownv[i] = elH<T>(e0, 2 * i);
  }
  auto code = [&](int k, const uint32_t (&pred)[VX], const HSeg<T>& src, int odd, uint32_t (&outv)[VX]) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      if constexpr (DEC) outv[i] = (pred[i] + elM<T>(mv[k], i)) & MASK;
      else outv[i] = (elH<T>(src, 2 * i + odd) - pred[i]) & MASK;
    }
  };

  {  // X map (0,0,1): ch15 (z,y) ch16 (z,y-1) ch17 (z-1,y-1) ch18 (z-1,y); with the lowres
    uint32_t pred[VX], outv[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i)
      pred[i] = (m(P15, i + 1, vz1, vy1) + m(A16, i + 1, vz1, vy0) + m(QA17, i + 1, vz0, vy0) +
                 m(Q18, i + 1, vz0, vy1)) >> ((nz * ny) >> 1);
    code(6, pred, e0, 1, outv);
    if constexpr (DEC) {
      stH<T>(h0, packH<T>(ownv, outv));
    } else {
      stM<T>((T*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, packM<T>(ownv));
      put8(6, outv);
    }
  }
  {  // Y map (0,1,0): ch11 (z,x) ch12 (z,x-1) ch13 (z-1,x-1) ch14 (z-1,x);  FB (0,1,1): ch4, ch5
    uint32_t pY[VX], pF[VX], oY[VX], oF[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
      pY[i] = (m(P11, i + 1, vz1, vy1) + m(P12, i, vz1, vy1) + m(Q13, i, vz0, vy1) + m(Q14, i + 1, vz0, vy1)) >>
              ((nz * nx) >> 1);
      pF[i] = (m(P4, i + 1, vz1, vy1) + m(Q5, i + 1, vz0, vy1)) >> (nz >> 1);
    }
    code(5, pY, e1, 0, oY);
    code(2, pF, e1, 1, oF);
    if constexpr (DEC) {
      if (vy1) stH<T>(h0 + a.W_, packH<T>(oY, oF));
    } else {
      put8(5, oY);
      put8(2, oF);
    }
  }
  {  // Z map (1,0,0): ch7 (y,x) ch8 (y,x-1) ch9 (y-1,x-1) ch10 (y-1,x);  UD (1,0,1): ch2, ch3
    uint32_t pZ[VX], pU[VX], oZ[VX], oU[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
      pZ[i] = (m(P7, i + 1, vz1, vy1) + m(P8, i, vz1, vy1) + m(A9, i, vz1, vy0) + m(A10, i + 1, vz1, vy0)) >>
              ((ny * nx) >> 1);
      pU[i] = (m(P2, i + 1, vz1, vy1) + m(A3, i + 1, vz1, vy0)) >> (ny >> 1);
    }
    code(4, pZ, o0, 0, oZ);
    code(1, pU, o0, 1, oU);
    if constexpr (DEC) {
      if (vz1) stH<T>(h0 + hplane, packH<T>(oZ, oU));
    } else {
      put8(4, oZ);
      put8(1, oU);
    }
  }
  {  // LR map (1,1,0): ch0 (x), ch1 (x-1);  C (1,1,1): ch6
    uint32_t pL[VX], pC[VX], oL[VX], oC[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
      pL[i] = (m(P0, i + 1, vz1, vy1) + m(P1, i, vz1, vy1)) >> (nx >> 1);
      pC[i] = m(P6, i + 1, vz1, vy1);
    }
    code(0, pL, o1, 0, oL);
    code(3, pC, o1, 1, oC);
    if constexpr (DEC) {
      if (vz1 && vy1) stH<T>(h0 + hplane + a.W_, packH<T>(oL, oC));
    } else {
      put8(0, oL);
      put8(3, oC);
    }
  }
}

}  // namespace l3p

// the reordered weights live in the caller's workspace (kmp_*_workspace_bytes covers them: the
// linear predictor's generic workspace is B * cells * 19 samples)
constexpr size_t kL3pWsBytes = 64 * 19 * sizeof(float);

template <typename T>
static bool linear3dp_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred,
                               const kmp_region* region, l3p::L3P& a, dim3& grid, dim3& block, size_t& lds) {
  constexpr int VX = 4;
  if (!std::is_same<T, uint16_t>::value && !std::is_same<T, uint8_t>::value) return false;
  if (opt(OPT_DISABLE_FAST, 0) || opt(OPT_DISABLE_LINEAR_FUSED, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_LINEAR || pred->padding != 1 || !pred->weights || !pred->bias) return false;
  const int P = pred->padding;
  if (g.n[2] % 8 != 0) return false;  // 8-sample highres row segments, aligned
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || txn < 1 || txn > 32 || (txn & (txn - 1)) != 0) return false;
  const int64_t rows = 64 / txn;
  const int64_t waves = ceil_div(g.E[1], rows);
  if (waves > 4) return false;  // the workgroup covers the whole plane (row exchange through LDS)
  // one reflection covers every halo index (lsrc1): L >= P + 2 on each axis
  if (g.L[0] < P + 2 || g.L[1] < P + 2 || g.L[2] < P + 2) return false;
  int64_t zb = 0, ze = g.E[0];
  if (region) {
    if (region->begin[1] > 0 || region->begin[2] > 0 || region->end[1] < g.E[1] || region->end[2] < g.E[2]) return false;
    zb = region->begin[0] < 0 ? 0 : region->begin[0];
    ze = region->end[0] > g.E[0] ? g.E[0] : region->end[0];
    if (ze <= zb) return false;
  }
  a.D = (int)g.n[0]; a.H = (int)g.n[1]; a.W_ = (int)g.n[2];
  a.Lz = (int)g.L[0]; a.Ly = (int)g.L[1]; a.Lx = (int)g.L[2];
  a.Ez = (int)g.E[0]; a.Ey = (int)g.E[1]; a.Ex = (int)g.E[2];
  a.Lcz = (int)g.Lc[0]; a.Lcy = (int)g.Lc[1]; a.Lcx = (int)g.Lc[2];
  a.zbegin = (int)zb; a.zend = (int)ze;
  a.txn = (int)txn; a.rows = (int)rows; a.nwv = (int)waves;
  // staged rows: node rows -P .. Ey+P (every row a lane's neighbourhood reads); columns: node
  // columns -P .. up to the last lane's 16-byte over-read, rounded to 16 bytes
  a.nr = (int)(g.E[1] + 2 * P + 1);
  a.pitch = (int)(g.E[2] - VX + 4 * ((VX + 2 * P + 1 + 3) / 4));  // the last lane's reads end here
  const int npl = 2 * P + 3;
  lds = (size_t)(npl * a.nr * a.pitch + waves * l3p::kXch * g.E[2]) * sizeof(uint32_t);
  if (lds > 64 * 1024) return false;
  const int64_t nblk = B * (ze - zb);
  a.xcd_per = (opt(OPT_W3_XCD, 1) && B % 8 == 0) ? (int)(ze - zb) : 0;
  grid = dim3((unsigned)nblk);
  block = dim3((unsigned)(64 * waves));
  return nblk < ((int64_t)1 << 31);
}

template <typename T>
int try_linear3dp_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                         const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3p::L3P a{};
    dim3 grid, block;
    size_t lds = 0;
    if (!linear3dp_geometry<T>(g, B, C, pred, region, a, grid, block, lds)) return KMP_ERR_UNSUPPORTED;
    constexpr uintptr_t HA = 8 * sizeof(T) - 1, MA = 4 * sizeof(T) - 1;  // segment alignments
    if (((uintptr_t)hi & HA) || ((uintptr_t)lowres & MA)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & MA) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    a.W = pred->weights;
    a.b = pred->bias;
    if (!ws || ws_bytes < kL3pWsBytes) return KMP_ERR_UNSUPPORTED;
    a.Wr = (const float*)ws;
    l3p::linear_reorder_kernel<<<1, 256, 0, stream>>>(pred->weights, (float*)ws, 4);
    if (a.Lcy == a.Ey && a.Lcx == a.Ex) l3p::linear3dp_kernel<T, false, 1, true><<<grid, block, lds, stream>>>(a);
    else l3p::linear3dp_kernel<T, false, 1, false><<<grid, block, lds, stream>>>(a);
    return check_launch("linear3dp_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_linear3dp_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                         const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3p::L3P a{};
    dim3 grid, block;
    size_t lds = 0;
    if (!linear3dp_geometry<T>(g, B, C, pred, region, a, grid, block, lds)) return KMP_ERR_UNSUPPORTED;
    constexpr uintptr_t HA = 8 * sizeof(T) - 1, MA = 4 * sizeof(T) - 1;
    if (((uintptr_t)hi & HA) || ((uintptr_t)lowres & MA)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k) {
      if ((uintptr_t)maps.p[k] & MA) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    a.W = pred->weights;
    a.b = pred->bias;
    if (!ws || ws_bytes < kL3pWsBytes) return KMP_ERR_UNSUPPORTED;
    a.Wr = (const float*)ws;
    l3p::linear_reorder_kernel<<<1, 256, 0, stream>>>(pred->weights, (float*)ws, 4);
    if (a.Lcy == a.Ey && a.Lcx == a.Ex) l3p::linear3dp_kernel<T, true, 1, true><<<grid, block, lds, stream>>>(a);
    else l3p::linear3dp_kernel<T, true, 1, false><<<grid, block, lds, stream>>>(a);
    return check_launch("linear3dp_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_L3P_INST(T)                                                                                   \
  template int try_linear3dp_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,  \
                                       const MapPtrs&, const kmp_region*, void*, size_t, hipStream_t);    \
  template int try_linear3dp_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,           \
                                       const kmp_predictor*, T*, const kmp_region*, void*, size_t, hipStream_t);
KMP_L3P_INST(uint8_t)
KMP_L3P_INST(uint16_t)
KMP_L3P_INST(int32_t)
KMP_L3P_INST(uint32_t)

}  // namespace kmp
