// kmp_codec_linear3d.hip -- one-pass volume encode / decode for the LinearPredictor with p == 0
// (SURVEY.md §8a row a9': the north star's "learned-predictor apply").
//
// pred[cell, k] = fma-chain over n = 0..7 of feat[cell, n] * W[n, k], started from b[k]
// (kmp_linear.hip, oracle.predictors.linear_fma_chain), cast to the sample dtype
// (XLA truncating / saturating astype), then maps_from_predictions (volume/utils.py:83-155) and
// the mod-2^k coder (utils.py:38-55).  Features are the 2x2x2 lowres nodes of the cell in the
// reference's order (n = dz*4 + dy*2 + dx, features_from_lowres volume/utils.py:199-210).
//
// Data movement is the plane-block scheme of kmp_codec_wave3d.hip with PL = 1: a workgroup owns
// one output plane c of one tile, its waves own 8 rows each, all loads are issued up front, and
// x / y+1 neighbours come from cross-lane shuffles.  A lane evaluates only the channels the
// outputs actually read: 14 of cell plane c (ch 0-4, 6-12, 15, 16) and 5 of plane c-1 (ch 5,
// 13, 14, 17, 18) for its 4 cells -- 19 channel-cells per output, no recomputation.  The
// channels row Y+1 needs from row Y (3, 9, 10, 16, 17) go down by shuffle inside a wave and
// through LDS across waves (one barrier).
//
// The 8x19 matvec runs on packed f32 VALU FMAs (v_pk_fma_f32, two cells per instruction): on
// CDNA4 the f32 MFMA rate equals the packed-VALU f32 rate, and keeping the cells in the lanes
// that own them avoids the cell <-> MFMA-fragment transposes.  Every FMA is correctly rounded
// and in the same n order, so the f32 values are bit-identical to kmp_linear.hip's MFMA chain.
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace l3 {

using namespace wv;

typedef float f32x2 __attribute__((ext_vector_type(2)));

struct L3 {
  const void* hi_in;
  void* hi_out;
  const void* lo_in;
  void* lo_out;
  MapPtrs maps;
  const float* W;  // [8, 19] row-major
  const float* b;  // [19]
  int32_t D, H, W_;
  int32_t Lz, Ly, Lx, Ez, Ey, Ex, Lcz, Lcy, Lcx;
  int32_t zbegin, zend;
  int32_t txn, rows, nwv;
  int32_t xcd_per;
  int32_t uld;
  int32_t full;  // Lcy == Ey and Lcx == Ex: the FULL kernel serves the call
};

// astype(T) for u8/u16: trunc, saturate, NaN -> 0.  v_cvt_u32_f32 truncates and saturates to
// [0, 2^32-1] with NaN -> 0, so one integer min finishes it (cvt_sat, kmp_wave.h): 2 VALU per value,
// where fminf(fmaxf()) compiled to med3 + cvt plus a canonicalising v_max on some of them
template <typename T>
__device__ __forceinline__ uint32_t cast_t(float v) {
  return cvt_sat<T>(v);
}

// Node values are kept as f32 pairs laid out for the packed FMAs: for the 4 cells X+4g .. X+4g+3
// of a group, NP[.][g][0] = {node 4g, 4g+2}, [1] = {4g+1, 4g+3}, [2] = {4g+2, 4g+4}.  Cells
// (0, 2) read pairs dx and cells (1, 3) pairs 1 + dx, so every feature operand is an aligned
// register pair (pairing cells 0/1 and 2/3 instead needs node pairs (x+1, x+2) assembled by
// moves in every channel: 214 v_mov per wave, 18 % of a VALU stream the SQ counters show busy
// 75 % of the cycles).  The chain is unchanged: fma over n = dz*4 + dy*2 + dx from the bias.
// The weights: W [8][19] and b are read with uniform loads into scalar registers, the packed
// operand {w, w} built by the FMA's operand selection -- no LDS copy, no barrier before the first
// channel, and 106 / 100 VGPRs instead of 146 with an LDS copy (4-5 waves per SIMD instead of 3): C3
// 168 / 222 -> 143 / 191 us per direction (profiles/round2/ab_linear3d_sgpr.log; the LDS form was
// removed in round 3).
typedef const __attribute__((address_space(4))) float* CFloat;  // uniform loads (scalar registers)

template <typename T, int K, int G>
__device__ __forceinline__ void channel(const f32x2 (&NP)[3][G][3], const f32x2 (&NP1)[3][G][3], int pl, int g,
                                        CFloat Wc, CFloat Bc, uint32_t (&out)[4]) {
  f32x2 w2[8];
  // W [8][19] and b read with uniform (scalar) loads
#pragma unroll
  for (int n = 0; n < 8; ++n) w2[n] = (f32x2){Wc[n * 19 + K], Wc[n * 19 + K]};
  const float bk = Bc[K];
  // the first FMA takes its weight and the bias from ONE 64-bit scalar pair {w0, b} (op_sel picks
  // the halves: one scalar operand, within the constant bus limit), so the bias needs no move into a
  // vector pair: 64 / 71 fewer VALU per linear3y encode / decode wave
  // (16-bit samples; the 8-bit 8-step kernel then no longer fully unrolls, so it keeps the move)
  f32x2 a02 = {bk, bk}, a13 = {bk, bk};
  constexpr int N0 = sizeof(T) == 2 ? 1 : 0;
  if constexpr (N0 == 1) {
    const uint64_t wb = (uint64_t)__builtin_bit_cast(uint32_t, Wc[K]) | ((uint64_t)__builtin_bit_cast(uint32_t, bk) << 32);
    asm("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(a02) : "v"(NP[pl][g][0]), "s"(wb));
    asm("v_pk_fma_f32 %0, %1, %2, %2 op_sel:[0,0,1] op_sel_hi:[1,0,1]" : "=v"(a13) : "v"(NP[pl][g][1]), "s"(wb));
  }
#pragma unroll
  for (int n = N0; n < 8; ++n) {
    const int dz = n >> 2, dy = (n >> 1) & 1, dx = n & 1;
    const f32x2 wv2 = w2[n];
    const f32x2(&R)[3] = dy ? NP1[pl + dz][g] : NP[pl + dz][g];
    a02 = __builtin_elementwise_fma(R[dx], wv2, a02);
    a13 = __builtin_elementwise_fma(R[1 + dx], wv2, a13);
  }
  out[0] = cast_t<T>(a02.x);
  out[1] = cast_t<T>(a13.x);
  out[2] = cast_t<T>(a02.y);
  out[3] = cast_t<T>(a13.y);
}

constexpr int kXch = 5;  // channels exchanged downwards: 3, 9, 10, 16 (plane c), 17 (plane c-1)

// All-zero weights and bias: a channel of a cell plane outside the tile (plane c-1 at c = 0, plane
// c at c >= Lcz) evaluated with these is 0.0 -> 0, which is what the aggregation's mask gives it
__constant__ float kZeroWeights[8 * 19 + 19];

// FULL: the tile's cells fill the stored lowres rows and columns (Lcy == Ey, Lcx == Ex: every
// even-sized tile, e.g. C3's 64^3).  Then the y+1
// validity and every x validity but the row's first cell (X-1 = -1) are compile-time true, and a
// missing cell plane (z) is zeroed at the source by reading its channels' weights from
// kZeroWeights (uniform), so the aggregation masks only the row-above channels on row 0 and the
// left cell on lane 0 of a row: 938 / 927 instead of 1 030 / 1 041 VALU instructions per encode /
// decode wave, and 5 waves per SIMD (WPE = 5: 96 / 92 VGPRs, the encode with a 20-byte spill;
// WPE = 4 measured the same, profiles/round2/ab_linear3d_full.log).  ULD: the decode's unconditional
// loads compiled in (see there)
template <typename T, bool DEC, bool FULL, int WPE, bool ULD = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) linear3d_kernel(L3 a) {
  constexpr int VX = 8 / (int)sizeof(T);
  static_assert(VX == 4 || VX == 8, "u16 / u8");
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  using V = typename std::conditional<DEC, uint2, uint4>::type;
  // LDS: the exchange rows [wave][kXch][Ex]
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* xrow = smem;
  const CFloat Wc = (CFloat)a.W, Bc = (CFloat)a.b;

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
  const bool last = r == a.rows - 1 || Y == a.Ey - 1;
  const bool vy1 = FULL || Y < a.Lcy;  // FULL: Lcy == Ey, and lanes past Ey are not live
  const bool vy0 = Y >= 1;
  const bool need_dn = live && last && vy1;
  const int ydn = lsrc(Yc + 1, a.Ly, a.Ey);
  const bool xlast = tx == a.txn - 1;
  const bool vz1 = c < a.Lcz, vz0 = c >= 1;
  // FULL: the channels of cell plane c (P) and c-1 (Q) from the weights, or from kZeroWeights where
  // that plane is outside the tile (uniform pointers)
  const CFloat Zc = (CFloat)kZeroWeights;
  const CFloat WcP = (FULL && !vz1) ? Zc : Wc, BcP = (FULL && !vz1) ? Zc + 152 : Bc;
  const CFloat WcQ = (FULL && !vz0) ? Zc : Wc, BcQ = (FULL && !vz0) ? Zc + 152 : Bc;

  const int hplane = a.H * a.W_;
  const int lplane = a.Ey * a.Ex;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * (int64_t)a.D * hplane;
  T* hout = DEC ? (T*)a.hi_out + b * (int64_t)a.D * hplane : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ez * lplane : nullptr;
  const int hx = 2 * X;
  const int ho_own = 2 * Yc * a.W_ + hx, ho_dn = 2 * ydn * a.W_ + hx;
  const int lo_own = Yc * a.Ex + X, lo_dn = ydn * a.Ex + X;

  const T* mbase[7];
  int mplane[7];
  bool mok_y[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez, ey = par[1] ? a.Lcy : a.Ey;
    mplane[k] = ey * a.Ex;
    const int ym = Yc < ey ? Yc : (ey > 0 ? ey - 1 : 0);  // in-bounds row (stores are gated by mok_y)
    mbase[k] = (const T*)a.maps.p[k] + b * (int64_t)ez * mplane[k] + ym * a.Ex + X;
    mok_y[k] = live && (!par[1] || vy1);
  }

  // ---- all loads up front: node planes c-1, c, c+1 (own row + the last row's halo row).  The
  // encode loads unconditionally from clamped, in-bounds addresses (rows / planes past the edges
  // read a valid neighbour whose values the masks discard): no zero-initialised registers and no
  // exec-mask branches, 208 -> 190 us at C3 (same box, ab_linear3d_loads.log).  The decode does
  // the same (map planes clamped to the last one that exists): with the weights in scalar registers
  // 190-205 -> 178-187 us (profiles/round2/ab_linear3d_uld.log); the guarded form remains only for
  // tiles without a cell plane / row to clamp to (Lcz or Lcy == 0). ----
  V own[3], dn[3];
  uint4 e1, o0, o1;
  uint2 mv[7];
  if constexpr (DEC) {
   // ULD: the unconditional form at compile time -- with the runtime choice the guarded form's
   // control flow joins the paths and the compiler waits for every load (map rows included) before
   // the first channel
   if (ULD || a.uld) {  // decode with unconditional clamped loads (masks discard the edge values)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int q = c - 1 + t;
      const T* p = lin + lsrc(q < 0 ? 0 : q, a.Lz, a.Ez) * lplane;
      own[t] = ld8c(p + lo_own);
      dn[t] = ld8c(p + lo_dn);
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      int par[3];
      map_parity(3, k, par);
      const int cz = par[0] ? (c < a.Lcz ? c : (a.Lcz > 0 ? a.Lcz - 1 : 0)) : c;
      mv[k] = ld8(mbase[k] + cz * mplane[k]);
    }
   } else {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      own[t] = dn[t] = V{};
      const int q = c - 1 + t;
      if (q < 0) continue;
      const T* p = lin + lsrc(q, a.Lz, a.Ez) * lplane;
      if (live) own[t] = ld8c(p + lo_own);
      if (need_dn) dn[t] = ld8c(p + lo_dn);
    }
#pragma unroll
    for (int k = 0; k < 7; ++k) {
      int par[3];
      map_parity(3, k, par);
      mv[k] = make_uint2(0, 0);
      if (mok_y[k] && (!par[0] || vz1)) mv[k] = ld8(mbase[k] + c * mplane[k]);
    }
   }
  } else {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int q = c - 1 + t;
      const T* p = hin + 2 * lsrc(q < 0 ? 0 : q, a.Lz, a.Ez) * hplane;
      own[t] = ld16c(p + ho_own);
      dn[t] = ld16c(p + ho_dn);
    }
    const int r1 = 2 * Yc + 1 < a.H ? a.W_ : 0;  // row 2Y+1, or row 2Y again
    const int p1 = 2 * c + 1 < a.D ? hplane : 0;  // plane 2c+1, or plane 2c again
    const T* p = hin + 2 * c * hplane;
    e1 = ld16(p + ho_own + r1);
    o0 = ld16(p + p1 + ho_own);
    o1 = ld16(p + p1 + ho_own + r1);
  }

  // ---- node values: own row Y, row Y+1 (shuffle / halo), each with node x+VX ----
  float nY[3][VX + 1], nY1[3][VX + 1];
  constexpr int G = VX / 4;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    uint32_t n[VX], nd[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      if constexpr (DEC) {
        n[i] = el8<T>(own[t], i);
        nd[i] = el8<T>(dn[t], i);
      } else {
        n[i] = el16<T>(own[t], 2 * i);
        nd[i] = el16<T>(dn[t], 2 * i);
      }
    }
    uint32_t nx = shdn(n[0], 1), ndx = shdn(nd[0], 1);
    if (xlast) {  // node Ex: mirror of node Ex-1 (even pad); no cell there otherwise
      nx = n[VX - 1];
      ndx = nd[VX - 1];
    }
    const uint32_t bx = shdn(nx, a.txn);
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t below = shdn(n[i], a.txn);
      nY[t][i] = (float)n[i];
      nY1[t][i] = (float)(last ? nd[i] : below);
    }
    nY[t][VX] = (float)nx;
    nY1[t][VX] = (float)(last ? ndx : bx);
  }
  f32x2 NP[3][G][3], NP1[3][G][3];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        NP[t][g][q] = (f32x2){nY[t][4 * g + q], nY[t][4 * g + q + 2]};
        NP1[t][g][q] = (f32x2){nY1[t][4 * g + q], nY1[t][4 * g + q + 2]};
      }

  // ---- channels: evaluated map group by map group so only a few are live at a time ----
#define KMP_CH(OUT, PLANE, K)                                             \
  _Pragma("unroll") for (int g = 0; g < G; ++g) {                         \
    uint32_t o[4];                                                        \
    channel<T, K, G>(NP, NP1, PLANE, g, PLANE ? WcP : WcQ, PLANE ? BcP : BcQ, o); \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) OUT[4 * g + j + 1] = o[j]; \
  }

  // 1. the channels row Y+1 reads from row Y: 3, 9, 10, 16 (plane c), 17 (plane c-1)
  uint32_t A3[VX + 1], A9[VX + 1], A10[VX + 1], A16[VX + 1], QA17[VX + 1];
  {
    uint32_t P3[VX + 1], P9[VX + 1], P10[VX + 1], P16[VX + 1], Q17[VX + 1];
    KMP_CH(P3, 1, 3) KMP_CH(P9, 1, 9) KMP_CH(P10, 1, 10) KMP_CH(P16, 1, 16) KMP_CH(Q17, 0, 17)
    if (wave_live && r == a.rows - 1) {  // a wave's full last row publishes its cells for the wave below
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

  bool vx[VX + 1];
#pragma unroll
  for (int q = 0; q <= VX; ++q) vx[q] = (FULL && q >= 1) || ((X - 1 + q) >= 0 && (X - 1 + q) < a.Lcx);
  const uint32_t ny = (uint32_t)vy0 + (uint32_t)vy1;
  const uint32_t nz = (uint32_t)vz0 + (uint32_t)vz1;
  auto m = [&](const uint32_t (&v)[VX + 1], int q, bool zok, bool yok) {
    return ((FULL || zok) && yok && vx[q]) ? v[q] : 0u;  // FULL: a missing z plane's channels are 0 already
  };
  auto left = [&](uint32_t (&v)[VX + 1]) { v[0] = shup(v[VX], 1); };  // cell X-1 (all lanes)
  auto put8 = [&](int k, const uint32_t (&res)[VX]) {  // encode: one map row
    int par[3];
    map_parity(3, k, par);
    if (mok_y[k] && (!par[0] || vz1)) st8((T*)mbase[k] + c * mplane[k], pack8<T, VX>(res));
  };
  const uint4 e0 = DEC ? uint4{} : *(const uint4*)&own[1];
  T* h0 = DEC ? hout + 2 * c * hplane + ho_own : nullptr;
  uint32_t ownv[VX];
#pragma unroll
  for (int i = 0; i < VX; ++i) {
    if constexpr (DEC) ownv[i] = el8<T>(*(const uint2*)&own[1], i);
    else ownv[i] = el16<T>(e0, 2 * i);
  }
  // decoded value (DEC) or residual (encode) of map k from its prediction; encode reads the
  // ground truth element ``gt`` of the stream rows
  auto code = [&](int k, const uint32_t (&pred)[VX], const uint4& src, int odd, uint32_t (&outv)[VX]) {
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      if constexpr (DEC) outv[i] = (pred[i] + el8<T>(mv[k], i)) & MASK;
      else outv[i] = (el16<T>(src, 2 * i + odd) - pred[i]) & MASK;
    }
  };

  // 2. X map (0,0,1): ch15 (z,y) ch16 (z,y-1) ch17 (z-1,y-1) ch18 (z-1,y); shares highres row
  //    2Y of plane 2c with the lowres
  {
    uint32_t P15[VX + 1], Q18[VX + 1], pred[VX], outv[VX];
    KMP_CH(P15, 1, 15) KMP_CH(Q18, 0, 18)
    if (!live) return;
#pragma unroll
    for (int i = 0; i < VX; ++i)
      pred[i] = (m(P15, i + 1, vz1, vy1) + m(A16, i + 1, vz1, vy0) + m(QA17, i + 1, vz0, vy0) +
                 m(Q18, i + 1, vz0, vy1)) >> ((nz * ny) >> 1);
    code(6, pred, e0, 1, outv);
    if constexpr (DEC) {
      st16(h0, pack16<T, VX>(ownv, outv));  // plane 2c, row 2Y: lowres | X
    } else {
      st8((T*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, pack8<T, VX>(ownv));
      put8(6, outv);
    }
  }
  // 3. Y map (0,1,0): ch11 (z,x) ch12 (z,x-1) ch13 (z-1,x-1) ch14 (z-1,x);  FB (0,1,1): ch4, ch5
  {
    uint32_t P11[VX + 1], P12[VX + 1], Q13[VX + 1], Q14[VX + 1], P4[VX + 1], Q5[VX + 1];
    uint32_t pY[VX], pF[VX], oY[VX], oF[VX];
    KMP_CH(P11, 1, 11) KMP_CH(P12, 1, 12) KMP_CH(Q13, 0, 13) KMP_CH(Q14, 0, 14) KMP_CH(P4, 1, 4) KMP_CH(Q5, 0, 5)
    left(P12);
    left(Q13);
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
      if (vy1) st16(h0 + a.W_, pack16<T, VX>(oY, oF));  // plane 2c, row 2Y+1: Y | FB
    } else {
      put8(5, oY);
      put8(2, oF);
    }
  }
  // 4. Z map (1,0,0): ch7 (y,x) ch8 (y,x-1) ch9 (y-1,x-1) ch10 (y-1,x);  UD (1,0,1): ch2, ch3
  {
    uint32_t P7[VX + 1], P8[VX + 1], P2[VX + 1];
    uint32_t pZ[VX], pU[VX], oZ[VX], oU[VX];
    KMP_CH(P7, 1, 7) KMP_CH(P8, 1, 8) KMP_CH(P2, 1, 2)
    left(P8);
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
      if (vz1) st16(h0 + hplane, pack16<T, VX>(oZ, oU));  // plane 2c+1, row 2Y: Z | UD
    } else {
      put8(4, oZ);
      put8(1, oU);
    }
  }
  // 5. LR map (1,1,0): ch0 (x), ch1 (x-1);  C (1,1,1): ch6
  {
    uint32_t P0[VX + 1], P1[VX + 1], P6[VX + 1];
    uint32_t pL[VX], pC[VX], oL[VX], oC[VX];
    KMP_CH(P0, 1, 0) KMP_CH(P1, 1, 1) KMP_CH(P6, 1, 6)
    left(P1);
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
      pL[i] = (m(P0, i + 1, vz1, vy1) + m(P1, i, vz1, vy1)) >> (nx >> 1);
      pC[i] = m(P6, i + 1, vz1, vy1);
    }
    code(0, pL, o1, 0, oL);
    code(3, pC, o1, 1, oC);
    if constexpr (DEC) {
      if (vz1 && vy1) st16(h0 + hplane + a.W_, pack16<T, VX>(oL, oC));  // plane 2c+1, row 2Y+1: LR | C
    } else {
      put8(0, oL);
      put8(3, oC);
    }
  }
#undef KMP_CH
}

// ---------------------------------------------------------------------------------------------
// The y-rolling form (FULL tiles whose rows split into whole wave steps, e.g. C3's 64^3): one wave
// owns one output plane and walks it in STEPS steps of ``rows`` lowres rows, the loads of step
// s+1 in flight while step s computes.  The row-below node values come from the lanes one row down
// by ONE rotation (lane L reads lane L + txn mod 64; the step's last row reads the next step's first
// row, which is already loaded), and the row-above channels (3, 9, 10, 16 of plane c, 17 of plane
// c-1) by the opposite rotation (the first row reads the previous step's last row, carried in
// registers): no halo rows, no LDS and no barrier, and 6 loads per lane per step (encode) where the
// plane-block form issues 9.  The arithmetic per cell -- the k-ordered fma chains, casts, masks,
// aggregation and coder -- is the FULL body of linear3d_kernel, so the results are bit-identical.

// the VX node values of a lane's row segment packed into 8 bytes: the decode's lowres row as
// loaded; the encode's highres row keeps its even elements (one byte permute per dword)
template <typename T>
__device__ __forceinline__ uint2 node_words(const uint2& v) { return v; }
template <typename T>
__device__ __forceinline__ uint2 node_words(const uint4& v) {
  constexpr uint32_t sel = sizeof(T) == 2 ? 0x05040100u : 0x06040200u;
  return make_uint2(__builtin_amdgcn_perm(v.y, v.x, sel), __builtin_amdgcn_perm(v.w, v.z, sel));
}

// lane L reads lane addr/4 of ``v``.  Call it as a statement of its own, never inside one arm of
// a per-lane select: the empty volatile asm pins the permute where it is written, with every lane
// active (inside ``r0 ? prev : rot(v)`` it runs with the r0 lanes disabled, and a permute that
// reads a disabled lane returns a stale value)
__device__ __forceinline__ uint32_t rot(uint32_t v, int addr) {
  uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v);
  asm volatile("" : "+v"(r));
  return r;
}

template <typename T, bool DEC, int STEPS, int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) linear3y_kernel(L3 a) {
  constexpr int VX = 8 / (int)sizeof(T);
  static_assert(VX == 4 || VX == 8, "u16 / u8");
  constexpr int G = VX / 4;
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  using V = typename std::conditional<DEC, uint2, uint4>::type;
  const CFloat Wc = (CFloat)a.W, Bc = (CFloat)a.b;

  const int lane = threadIdx.x;
  const int tx = lane & (a.txn - 1);
  const int r = lane >> __builtin_ctz(a.txn);
  const int rows = a.rows;
  const int X = tx * VX;
  int blk = (int)blockIdx.x;
  if (a.xcd_per > 0) {
    const int x = blk % 8, k = blk / 8;
    blk = ((k / a.xcd_per) * 8 + x) * a.xcd_per + (k % a.xcd_per);
  }
  const int nplanes = a.zend - a.zbegin;
  const int c = a.zbegin + blk % nplanes;
  const int64_t b = blk / nplanes;
  const bool xlast = tx == a.txn - 1;
  const bool r0 = r == 0, rlast = r == rows - 1;
  const bool vz1 = c < a.Lcz, vz0 = c >= 1;
  const CFloat Zc = (CFloat)kZeroWeights;
  const CFloat WcP0 = !vz1 ? Zc : Wc, BcP0 = !vz1 ? Zc + 152 : Bc;
  const CFloat WcQ0 = !vz0 ? Zc : Wc, BcQ0 = !vz0 ? Zc + 152 : Bc;
  const int adn = ((lane + a.txn) & 63) << 2, aup = ((lane - a.txn) & 63) << 2;

  const int hplane = a.H * a.W_;
  const int lplane = a.Ey * a.Ex;
  const int hx = 2 * X;
  // Addresses: a uniform (scalar) base per row stream plus ONE 32-bit lane offset per layout, so the
  // loads and stores take the scalar-base form (no 64-bit vector address arithmetic per access)
  // and no per-stream 64-bit pointers occupy vector registers.  Node rows of node planes c-1, c,
  // c+1: a lowres row is one row of the decode's lowres / two rows of the encode's highres.
  constexpr int SZ = (int)sizeof(T);
  const int nstride = DEC ? a.Ex : 2 * a.W_;  // elements per lowres row in the node planes
  const uint32_t lon = (uint32_t)((r * nstride + (DEC ? X : hx)) * SZ);  // node / stream / highres rows
  const uint32_t lonx = (uint32_t)((DEC ? X : hx) * SZ);                 // the same at row 0
  const uint32_t lom = (uint32_t)((r * a.Ex + X) * SZ);                  // lowres / map rows
  const uint32_t loh = (uint32_t)((2 * r * a.W_ + hx) * SZ);             // highres rows (the decode's output)
  const char* un[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int q = c - 1 + t;
    const int zq = lsrc(q < 0 ? 0 : q, a.Lz, a.Ez);
    un[t] = DEC ? (const char*)a.lo_in + (b * a.Ez + zq) * (int64_t)lplane * SZ
                : (const char*)a.hi_in + (b * a.D + 2 * zq) * (int64_t)hplane * SZ;
  }
  // encode: the stream rows (plane 2c row 2Y+1, plane 2c+1 rows 2Y / 2Y+1; plane 2c+1 is plane 2c
  // again where the tile has no such plane); decode: the 7 map rows (a map's missing last cell plane
  // clamped to the one before: the masks discard it)
  const char* us = DEC ? nullptr : (const char*)a.hi_in + (b * a.D + 2 * c) * (int64_t)hplane * SZ;
  const int p1 = (2 * c + 1 < a.D ? hplane : 0) * SZ;
  char* um[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez;
    const int cz = par[0] ? (c < a.Lcz ? c : a.Lcz - 1) : c;
    um[k] = (char*)a.maps.p[k] + (b * ez + cz) * (int64_t)lplane * SZ;  // FULL: every map is Ey x Ex
  }
  char* ulo = DEC ? nullptr : (char*)a.lo_out + (b * a.Ez + c) * (int64_t)lplane * SZ;
  char* uho = DEC ? (char*)a.hi_out + (b * a.D + 2 * c) * (int64_t)hplane * SZ : nullptr;
  const int nstep = rows * nstride * SZ, mstep = rows * a.Ex * SZ, hstep = rows * 2 * a.W_ * SZ;

  // node rows: a ring of three steps -- the current one, the next (its first row is the current
  // last row's row below) and the one after, in flight; stream / map rows: the next step's in flight
  V cur[3], nxt[3], nx2[3];
  uint4 cs[3], ns[3];  // encode stream rows e1, o0, o1
  uint2 cm[7], nm[7];  // decode map rows
  auto load_nodes = [&](int s, V (&o)[3]) {
    // the step past the last reads the mirrored row Ey - 1 (only row 0's values are used)
    const bool past = s >= STEPS;
    const int so = past ? (a.Ey - 1) * nstride * SZ : s * nstep;
    const uint32_t lo = past ? lonx : lon;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      if constexpr (DEC) o[t] = ld8c(un[t] + so + lo);
      else o[t] = ld16c(un[t] + so + lo);
    }
  };
  auto load_rest = [&](int s, uint4 (&os)[3], uint2 (&om)[7]) {
    if constexpr (DEC) {
#pragma unroll
      for (int k = 0; k < 7; ++k) om[k] = ld8(um[k] + s * mstep + lom);
    } else {
      const char* p = us + s * hstep;
      const int rw = a.W_ * SZ;
      os[0] = ld16(p + rw + lon);
      os[1] = ld16(p + p1 + lon);
      os[2] = ld16(p + p1 + rw + lon);
    }
  };
  load_nodes(0, cur);
  load_rest(0, cs, cm);
  load_nodes(1, nxt);

  // The channels 3, 9, 10, 16 (plane c) and 17 (plane c-1) that row Y+1 reads from row Y go
  // through an LDS ring of rows + 1 row slots (row Y in slot Y mod (rows + 1)): a step writes its
  // rows' channels, then reads the slots of the rows above -- the previous step's last row is in a
  // slot the current step does not overwrite.  Slot rows (row -1) starts zeroed: row 0 has no row
  // above.  One wave per workgroup: its own LDS accesses are ordered, so no barrier.
  extern __shared__ __attribute__((aligned(16))) uint32_t xring[];  // [rows + 1][txn][kXch][VX]
  const int xslot = a.txn * kXch * VX;  // words per row slot
  if (r0) {
#pragma unroll
    for (int q = 0; q < kXch; ++q)
#pragma unroll
      for (int i = 0; i < VX; ++i) xring[rows * xslot + (tx * kXch + q) * VX + i] = 0;
  }
  int wslot = r;  // Y mod (rows + 1): rows advance by rows == -1 (mod rows + 1) per step

#pragma unroll
  for (int s = 0; s < STEPS; ++s) {
    // unconditional (clamped: the last steps re-read rows already loaded), so every iteration
    // issues the same loads and the waits stay counted (vmcnt(N)) instead of draining (vmcnt(0))
    load_nodes(s + 2 <= STEPS ? s + 2 : STEPS, nx2);
    load_rest(s + 1 < STEPS ? s + 1 : STEPS - 1, ns, nm);
    // the weights are re-read (scalar loads, cache hits) in every step rather than hoisted out of
    // the loop: 171 values do not fit the scalar register file
    CFloat WcP = WcP0, BcP = BcP0, WcQ = WcQ0, BcQ = BcQ0;
    asm volatile("" : "+s"(WcP), "+s"(BcP), "+s"(WcQ), "+s"(BcQ));
    const int Y = s * rows + r;
    const bool vy0 = Y >= 1;

    // ---- node values: own row Y, row Y+1 (one rotation: the step's last row reads the next's first) ----
    f32x2 NP[3][G][3], NP1[3][G][3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const uint2 nw = node_words<T>(cur[t]);
      const uint2 nn = node_words<T>(nxt[t]);
      const uint2 dw = make_uint2(rot(r0 ? nn.x : nw.x, adn), rot(r0 ? nn.y : nw.y, adn));
      float nY[VX + 1], nY1[VX + 1];
      uint32_t n[VX], nd[VX];
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        n[i] = el8<T>(nw, i);
        nd[i] = el8<T>(dw, i);
        nY[i] = (float)n[i];
        nY1[i] = (float)nd[i];
      }
      uint32_t nx = shdn(n[0], 1), ndx = shdn(nd[0], 1);
      if (xlast) {  // node Ex: mirror of node Ex-1 (even pad)
        nx = n[VX - 1];
        ndx = nd[VX - 1];
      }
      nY[VX] = (float)nx;
      nY1[VX] = (float)ndx;
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
          NP[t][g][q] = (f32x2){nY[4 * g + q], nY[4 * g + q + 2]};
          NP1[t][g][q] = (f32x2){nY1[4 * g + q], nY1[4 * g + q + 2]};
        }
    }

#define KMP_CH(OUT, PLANE, K)                                                     \
  _Pragma("unroll") for (int g = 0; g < G; ++g) {                                 \
    uint32_t o[4];                                                                \
    channel<T, K, G>(NP, NP1, PLANE, g, PLANE ? WcP : WcQ, PLANE ? BcP : BcQ, o); \
    _Pragma("unroll") for (int j = 0; j < 4; ++j) OUT[4 * g + j + 1] = o[j];      \
  }
    // 1. the channels row Y+1 reads from row Y; row Y reads row Y-1's by the opposite rotation (row
    // 0 of step 0 reads the zero-initialised carry: no masks on the row-above channels)
    uint32_t A3[VX + 1], A9[VX + 1], A10[VX + 1], A16[VX + 1], QA17[VX + 1];
    {
      uint32_t P3[VX + 1], P9[VX + 1], P10[VX + 1], P16[VX + 1], Q17[VX + 1];
      KMP_CH(P3, 1, 3) KMP_CH(P9, 1, 9) KMP_CH(P10, 1, 10) KMP_CH(P16, 1, 16) KMP_CH(Q17, 0, 17)
      {
        uint32_t* w = xring + (wslot * xslot + tx * kXch * VX);
#pragma unroll
        for (int i = 0; i < VX; ++i) {
          w[0 * VX + i] = P3[i + 1];
          w[1 * VX + i] = P9[i + 1];
          w[2 * VX + i] = P10[i + 1];
          w[3 * VX + i] = P16[i + 1];
          w[4 * VX + i] = Q17[i + 1];
        }
      }
      const int rslot = wslot == 0 ? rows : wslot - 1;  // row Y - 1
      const uint32_t* rd = xring + (rslot * xslot + tx * kXch * VX);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        A3[i + 1] = rd[0 * VX + i];
        A9[i + 1] = rd[1 * VX + i];
        A10[i + 1] = rd[2 * VX + i];
        A16[i + 1] = rd[3 * VX + i];
        QA17[i + 1] = rd[4 * VX + i];
      }
    }
    A9[0] = shup(A9[VX], 1);  // cell (Y-1, X-1): the lane to the left

    bool vx[VX + 1];
#pragma unroll
    for (int q = 0; q <= VX; ++q) vx[q] = q >= 1 || X >= 1;
    const uint32_t ny = (uint32_t)vy0 + 1u;
    const uint32_t nz = (uint32_t)vz0 + (uint32_t)vz1;
    auto m = [&](const uint32_t (&v)[VX + 1], int q, bool yok) { return (yok && vx[q]) ? v[q] : 0u; };
    auto left = [&](uint32_t (&v)[VX + 1]) { v[0] = shup(v[VX], 1); };
    auto put8 = [&](int k, const uint32_t (&res)[VX]) {
      int par[3];
      map_parity(3, k, par);
      if (!par[0] || vz1) st8(um[k] + s * mstep + lom, pack8<T, VX>(res));
    };
    const uint4 e0 = DEC ? uint4{} : *(const uint4*)&cur[1];
    const uint4 e1 = cs[0], o0 = cs[1], o1 = cs[2];
    char* h0 = DEC ? uho + s * hstep : nullptr;  // + loh: plane 2c, row 2Y
    uint32_t ownv[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      if constexpr (DEC) ownv[i] = el8<T>(*(const uint2*)&cur[1], i);
      else ownv[i] = el16<T>(e0, 2 * i);
    }
    auto code = [&](int k, const uint32_t (&pred)[VX], const uint4& src, int odd, uint32_t (&outv)[VX]) {
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        if constexpr (DEC) outv[i] = (pred[i] + el8<T>(cm[k], i)) & MASK;
        else outv[i] = (el16<T>(src, 2 * i + odd) - pred[i]) & MASK;
      }
    };

    // 2. X map (0,0,1): ch15 (z,y) ch16 (z,y-1) ch17 (z-1,y-1) ch18 (z-1,y)
    {
      uint32_t P15[VX + 1], Q18[VX + 1], pred[VX], outv[VX];
      KMP_CH(P15, 1, 15) KMP_CH(Q18, 0, 18)
#pragma unroll
      for (int i = 0; i < VX; ++i)
        pred[i] = (m(P15, i + 1, true) + m(A16, i + 1, true) + m(QA17, i + 1, true) + m(Q18, i + 1, true)) >>
                  ((nz * ny) >> 1);
      code(6, pred, e0, 1, outv);
      if constexpr (DEC) {
        st16(h0 + loh, pack16<T, VX>(ownv, outv));  // plane 2c, row 2Y: lowres | X
      } else {
        st8(ulo + s * mstep + lom, pack8<T, VX>(ownv));
        put8(6, outv);
      }
    }
    // 3. Z map (1,0,0): ch7 (y,x) ch8 (y,x-1) ch9 (y-1,x-1) ch10 (y-1,x);  UD (1,0,1): ch2, ch3
    {
      uint32_t P7[VX + 1], P8[VX + 1], P2[VX + 1];
      uint32_t pZ[VX], pU[VX], oZ[VX], oU[VX];
      KMP_CH(P7, 1, 7) KMP_CH(P8, 1, 8) KMP_CH(P2, 1, 2)
      left(P8);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pZ[i] = (m(P7, i + 1, true) + m(P8, i, true) + m(A9, i, true) + m(A10, i + 1, true)) >> ((ny * nx) >> 1);
        pU[i] = (P2[i + 1] + m(A3, i + 1, true)) >> (ny >> 1);
      }
      code(4, pZ, o0, 0, oZ);
      code(1, pU, o0, 1, oU);
      if constexpr (DEC) {
        if (vz1) st16(h0 + hplane * SZ + loh, pack16<T, VX>(oZ, oU));  // plane 2c+1, row 2Y: Z | UD
      } else {
        put8(4, oZ);
        put8(1, oU);
      }
    }
    // 4. Y map (0,1,0): ch11 (z,x) ch12 (z,x-1) ch13 (z-1,x-1) ch14 (z-1,x);  FB (0,1,1): ch4, ch5
    {
      uint32_t P11[VX + 1], P12[VX + 1], Q13[VX + 1], Q14[VX + 1], P4[VX + 1], Q5[VX + 1];
      uint32_t pY[VX], pF[VX], oY[VX], oF[VX];
      KMP_CH(P11, 1, 11) KMP_CH(P12, 1, 12) KMP_CH(Q13, 0, 13) KMP_CH(Q14, 0, 14) KMP_CH(P4, 1, 4) KMP_CH(Q5, 0, 5)
      left(P12);
      left(Q13);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pY[i] = (m(P11, i + 1, true) + m(P12, i, true) + m(Q13, i, true) + m(Q14, i + 1, true)) >> ((nz * nx) >> 1);
        pF[i] = (P4[i + 1] + Q5[i + 1]) >> (nz >> 1);
      }
      code(5, pY, e1, 0, oY);
      code(2, pF, e1, 1, oF);
      if constexpr (DEC) {
        st16(h0 + a.W_ * SZ + loh, pack16<T, VX>(oY, oF));  // plane 2c, row 2Y+1: Y | FB
      } else {
        put8(5, oY);
        put8(2, oF);
      }
    }
    // 5. LR map (1,1,0): ch0 (x), ch1 (x-1);  C (1,1,1): ch6
    {
      uint32_t P0[VX + 1], P1[VX + 1], P6[VX + 1];
      uint32_t pL[VX], pC[VX], oL[VX], oC[VX];
      KMP_CH(P0, 1, 0) KMP_CH(P1, 1, 1) KMP_CH(P6, 1, 6)
      left(P1);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pL[i] = (P0[i + 1] + m(P1, i, true)) >> (nx >> 1);
        pC[i] = P6[i + 1];
      }
      code(0, pL, o1, 0, oL);
      code(3, pC, o1, 1, oC);
      if constexpr (DEC) {
        if (vz1) st16(h0 + (hplane + a.W_) * SZ + loh, pack16<T, VX>(oL, oC));  // plane 2c+1, row 2Y+1: LR | C
      } else {
        put8(0, oL);
        put8(3, oC);
      }
    }
#undef KMP_CH
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      cur[t] = nxt[t];
      nxt[t] = nx2[t];
    }
    wslot = wslot == 0 ? rows : wslot - 1;
#pragma unroll
    for (int q = 0; q < 3; ++q) cs[q] = ns[q];
#pragma unroll
    for (int k = 0; k < 7; ++k) cm[k] = nm[k];
  }
}

}  // namespace l3

// the y-rolling kernel serves FULL tiles whose rows split into 1, 2, 4 or 8 whole wave steps
// (KMP_L3Y=0: the plane-block kernel, for A/B)
// waves per SIMD: 16-bit samples 127 / 123 VGPRs (encode / decode, 4 steps fully unrolled; 8 steps
// at 3 waves), 8-bit ~200 (2 waves)
#define L3Y_WPE (sizeof(T) == 2 ? L3Y_W16 : 2)
#ifndef L3Y_W16
#define L3Y_W16 4
#endif
static int l3y_steps(const l3::L3& a) {
  if (!a.full || a.Lcz < 1 || !opt(OPT_L3Y, 1)) return 0;
  if (a.Ey % a.rows != 0) return 0;
  const int steps = a.Ey / a.rows;
  return (steps == 1 || steps == 2 || steps == 4 || steps == 8) ? steps : 0;
}

template <typename T>
static bool linear3d_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred,
                              const kmp_region* region, l3::L3& a, dim3& grid, dim3& block, size_t& lds) {
  constexpr int VX = 8 / (int)sizeof(T);
  if (!(std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value)) return false;
  if (opt(OPT_DISABLE_FAST, 0) || opt(OPT_DISABLE_LINEAR_FUSED, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_LINEAR || pred->padding != 0) return false;
  if (g.n[2] % 2 != 0 || (g.n[2] * (int64_t)sizeof(T)) % 16 != 0) return false;
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || txn < 1 || txn > 32 || (txn & (txn - 1)) != 0) return false;
  const int64_t rows = 64 / txn;
  const int64_t waves = ceil_div(g.E[1], rows);
  const bool tall = waves > 4;  // the plane-block workgroup covers the whole plane (row exchange through LDS)
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
  const int64_t nblk = B * (ze - zb);
  a.xcd_per = (opt(OPT_W3_XCD, 1) && B % 8 == 0) ? (int)(ze - zb) : 0;
  a.full = g.Lc[1] == g.E[1] && g.Lc[2] == g.E[2];
  lds = (size_t)(waves * l3::kXch * g.E[2]) * sizeof(uint32_t);
  grid = dim3((unsigned)nblk);
  block = dim3((unsigned)(64 * waves));
  if (tall && !l3y_steps(a)) return false;  // only the y-rolling kernel serves it
  return nblk < ((int64_t)1 << 31);
}

template <typename T>
int try_linear3d_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                        const MapPtrs& maps, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3::L3 a{};
    dim3 grid, block;
    size_t lds = 0;
    if (!linear3d_geometry<T>(g, B, C, pred, region, a, grid, block, lds)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    a.W = pred->weights;
    a.b = pred->bias;
    if (const int steps = l3y_steps(a)) {
      const dim3 g1(grid.x), b1(64);  // one wave per output plane
      const size_t xl = (size_t)(a.rows + 1) * a.txn * l3::kXch * (8 / sizeof(T)) * 4;  // the row ring
      if (steps == 1) l3::linear3y_kernel<T, false, 1, L3Y_WPE><<<g1, b1, xl, stream>>>(a);
      else if (steps == 2) l3::linear3y_kernel<T, false, 2, L3Y_WPE><<<g1, b1, xl, stream>>>(a);
      else if (steps == 4) l3::linear3y_kernel<T, false, 4, L3Y_WPE><<<g1, b1, xl, stream>>>(a);
      else l3::linear3y_kernel<T, false, 8, (sizeof(T) == 2 ? 3 : 2)><<<g1, b1, xl, stream>>>(a);
      return check_launch("linear3y_encode");
    }
    if (a.full) l3::linear3d_kernel<T, false, true, 5><<<grid, block, lds, stream>>>(a);
    else l3::linear3d_kernel<T, false, false, 1><<<grid, block, lds, stream>>>(a);
    return check_launch("linear3d_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_linear3d_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                        const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3::L3 a{};
    dim3 grid, block;
    size_t lds = 0;
    if (!linear3d_geometry<T>(g, B, C, pred, region, a, grid, block, lds)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    a.W = pred->weights;
    a.b = pred->bias;
    a.uld = a.Lcz > 0 && a.Lcy > 0;  // clamped map planes / rows exist
    if (const int steps = l3y_steps(a)) {
      const dim3 g1(grid.x), b1(64);  // one wave per output plane
      const size_t xl = (size_t)(a.rows + 1) * a.txn * l3::kXch * (8 / sizeof(T)) * 4;  // the row ring
      if (steps == 1) l3::linear3y_kernel<T, true, 1, L3Y_WPE><<<g1, b1, xl, stream>>>(a);
      else if (steps == 2) l3::linear3y_kernel<T, true, 2, L3Y_WPE><<<g1, b1, xl, stream>>>(a);
      else if (steps == 4) l3::linear3y_kernel<T, true, 4, L3Y_WPE><<<g1, b1, xl, stream>>>(a);
      else l3::linear3y_kernel<T, true, 8, (sizeof(T) == 2 ? 3 : 2)><<<g1, b1, xl, stream>>>(a);
      return check_launch("linear3y_decode");
    }
    if (a.full && a.uld) l3::linear3d_kernel<T, true, true, 5, true><<<grid, block, lds, stream>>>(a);
    else if (a.full) l3::linear3d_kernel<T, true, true, 5><<<grid, block, lds, stream>>>(a);
    else l3::linear3d_kernel<T, true, false, 1><<<grid, block, lds, stream>>>(a);
    return check_launch("linear3d_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_L3_INST(T)                                                                                    \
  template int try_linear3d_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,   \
                                      const MapPtrs&, const kmp_region*, hipStream_t);                    \
  template int try_linear3d_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,            \
                                      const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_L3_INST(uint8_t)
KMP_L3_INST(uint16_t)
KMP_L3_INST(int32_t)
KMP_L3_INST(uint32_t)

}  // namespace kmp
