// kmp_codec_linear3r.hip -- one-pass volume encode / decode for the LinearPredictor with p == 1 on
// the matrix cores, rolling along z (SURVEY.md §8a row a9': the north star's "learned-predictor
// apply / MFMA only for the small dense predictor matmul").
//
// Arithmetic: that of kmp_codec_linear3dp.hip -- pred[cell, k] = the fma chain over the 64
// features n = dz*16 + dy*4 + dx (features_from_lowres order, volume/utils.py:199-210) from b[k],
// cast to u16, aggregated onto the 7 maps (volume/utils.py:83-155), coded (utils.py:48-55).
//
// Work decomposition: a workgroup owns a run of output planes [z0, z1) of one tile and walks it
// cell plane by cell plane.  Node planes live in a 5-slot LDS ring as f32 with the mirrored halo
// rows / columns of the symmetric neighbourhood pad over the even reflect pad; each step stages ONE
// new node plane (k + 3), prefetched into registers a step ahead, so HBM / L2 latency overlaps the
// matrix work.  Per cell plane k every one of the 19 channels is computed once:
//   * 16 on the matrix cores: v_mfma_f32_16x16x4_f32 tiles, M = 16 cells of one row, N = the 16
//     channel columns KM (the 14 channels plane-k outputs read + channels 5 and 13 the next output
//     plane reads), K = the 4 node columns dx of one node row (dz, dy), 16 steps = 64 features.
//     An f32 MFMA is bit-for-bit the k-ordered fmaf chain from its C input
//     (cdna_hip_programming.md §3): seeded with the bias, stepped in n order, every value equals
//     the oracle's chain (oracle.predictors.linear_fma_chain);
//   * 3 (14, 17, 18) on packed-FMA VALU, the same chain, interleaved with the MFMAs of each step.
// The MFMA results return to the lane-owns-4-cells layout of the epilogue through a per-wave LDS
// tile; channels 5, 13, 14, 17, 18 of plane k stay in registers for output plane k + 1 (which
// reads plane k as its "c - 1"), so no channel is evaluated twice.
//
// Measured at C3 (profiles/round2/ab_linear3r.log, sq_linear3r.txt): bit-exact, 573 / 540 us per
// direction against 549-565 / 504-507 for the per-plane packed-FMA kernel, so it is selected only
// with KMP_L3R=1.  The matrix pipe is 38 % busy: at 256 VGPRs (2 waves per SIMD) 43 % of the wave
// cycles are issue stalls -- the B operands come from LDS one read per MFMA, and the epilogue's
// ~1 300 VALU instructions per step do not overlap the other wave's MFMAs enough.
#include <algorithm>
#include <cstdlib>

#include "kmp_wave.h"

namespace kmp {
namespace l3r {

using namespace wv;

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

struct L3R {
  const void* hi_in;
  void* hi_out;
  const void* lo_in;
  void* lo_out;
  MapPtrs maps;
  const float* W;   // [64, 19] row-major
  const float* b;   // [19]
  const float* Wv;  // the VALU channels' weights [node row 16][kk 3][dx 4] (reorder_kernel)
  int32_t D, H, W_;
  int32_t Lz, Ly, Lx, Ez, Ey, Ex, Lcz, Lcy, Lcx;
  int32_t zbegin, zend, zper, nrange;  // output planes [zbegin, zend) in runs of zper per workgroup
  int32_t txn, rows, nwv;
  int32_t xcd_per;
  int32_t nr, pitch;  // staged node rows per plane (Ey + 3), f32 words per staged row
};

constexpr int kP = 1;      // neighbourhood padding
constexpr int kNB = 4;     // 2p + 2 nodes per axis
constexpr int kNS = 5;     // LDS ring slots (4 node planes read per step + 1 being staged)
constexpr int kXch = 5;    // channels exchanged downwards: 3, 9, 10, 16, 17 of plane k
constexpr int kNV = 3;     // VALU channels
__constant__ const int kKV[kNV] = {14, 17, 18};
// MFMA columns: plane-k outputs read KC = {0-4, 6-12, 15, 16}; the next output plane reads 5 and 13
__constant__ const int kKM[16] = {0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 15, 16, 5, 13};

__global__ void __launch_bounds__(256) reorder_kernel(const float* __restrict__ W, float* __restrict__ Wv) {
  for (int t = threadIdx.x; t < 16 * kNV * kNB; t += blockDim.x) {
    const int dx = t % kNB, kk = (t / kNB) % kNV, row = t / (kNB * kNV);
    Wv[t] = W[(row * kNB + dx) * 19 + kKV[kk]];
  }
}

#ifndef KMP_L3R_WPE
#define KMP_L3R_WPE 2
#endif
template <bool DEC, int GPR>  // GPR: 16-cell groups per row (Ex / 16); the wave's 16 groups = 16 / GPR rows
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(KMP_L3R_WPE))) linear3r_kernel(L3R a) {
  using T = uint16_t;
  constexpr int VX = 4;
  constexpr uint32_t MASK = 0xffffu;
  using V = typename std::conditional<DEC, uint2, uint4>::type;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  float* st = (float*)smem;
  const int plane_words = a.nr * a.pitch;
  uint32_t* xrow = smem + kNS * plane_words;
  const int tstride = a.rows * a.Ex + 8;  // the pad staggers the channels' rows over the banks
  uint16_t* tile = (uint16_t*)(xrow + a.nwv * kXch * a.Ex) + (size_t)(threadIdx.x >> 6) * 16 * tstride;

  const int lane = threadIdx.x & 63;
  const int wv_ = threadIdx.x >> 6;
  const int tx = lane % a.txn;
  const int r = lane / a.txn;
  const int X = tx * VX;
  int blk = (int)blockIdx.x;
  if (a.xcd_per > 0) {
    const int x = blk % 8, k = blk / 8;
    blk = ((k / a.xcd_per) * 8 + x) * a.xcd_per + (k % a.xcd_per);
  }
  const int rng = blk % a.nrange;
  const int64_t b = blk / a.nrange;
  const int z0 = a.zbegin + rng * a.zper;
  const int z1 = min(z0 + a.zper, a.zend);
  const int Y0 = wv_ * a.rows;
  const bool wave_live = Y0 < a.Ey;
  const int Y = Y0 + r;
  const bool live = wave_live && Y < a.Ey;
  const int Yc = live ? Y : a.Ey - 1;
  const bool first = r == 0;
  const bool vy1 = Y < a.Lcy;
  const bool vy0 = Y >= 1;

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

  // matrix operands: B[dx][column] = W[4s + dx][KM[column]] for step s, the bias seeding the
  // accumulator column of this lane
  const int mj = lane & 15, mq = lane >> 4;
  const float bias_col = a.b[kKM[mj]];

  auto slot = [](int qn) __attribute__((always_inline)) {
    const int m = qn % kNS;
    return m < 0 ? m + kNS : m;
  };
  // the lane's own row of node plane qn (mirrored into range), from HBM
  auto load_node = [&](int qn) __attribute__((always_inline)) {
    V v{};
    const int sz = lsrc1(qn, a.Lz, a.Ez);
    if constexpr (DEC) {
      if (live) v = ld8c(lin + sz * lplane + lo_own);
    } else {
      if (live) v = ld16c(hin + 2 * sz * hplane + ho_own);
    }
    return v;
  };
  // node plane qn into its ring slot: the lane's 4 nodes, plus the mirrored halo columns / rows
  // it is the source of (symmetric pad over the even reflect pad: lsrc)
  auto stage = [&](int qn, const V& own) __attribute__((always_inline)) {
    if (!live) return;
    constexpr int NHR = 4 * ((VX + 2 * kP + 1 + 3) / 4) - VX - kP;  // halo columns right of Ex
    const bool xfirst = tx == 0, xlast = tx == a.txn - 1;
    float v[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i)
      v[i] = (float)(DEC ? el8<T>(*(const uint2*)&own, i) : el16<T>(*(const uint4*)&own, 2 * i));
    float* base = st + slot(qn) * plane_words;
    auto put_row = [&](int ry) __attribute__((always_inline)) {
      float* row = base + ry * a.pitch + kP + X;
#pragma unroll
      for (int i = 0; i < VX; ++i) row[i] = v[i];
      if (xfirst) row[-1] = v[0];  // node column -1 mirrors column 0
      if (xlast) {
#pragma unroll
        for (int jj = 0; jj < NHR; ++jj) {
          const int sx = lsrc1(a.Ex + jj, a.Lx, a.Ex) - X;
          float u = v[0];
#pragma unroll
          for (int i = 1; i < VX; ++i) u = sx == i ? v[i] : u;
          row[VX + jj] = u;
        }
      }
    };
    put_row(Y + kP);
#pragma unroll
    for (int h = 0; h < 2 * kP + 1; ++h) {  // node rows -1 and Ey, Ey+1
      const int rr = h < kP ? h - kP : a.Ey + (h - kP);
      if (lsrc1(rr, a.Ly, a.Ey) == Y) put_row(rr + kP);
    }
  };
  // the rows output plane c reads besides the staged nodes: encode -- highres rows 2Y (its odd
  // samples are the X map) and 2Y+1 of plane 2c, rows 2Y / 2Y+1 of plane 2c+1; decode -- the 7
  // residual rows
  struct OutsEnc {
    uint4 e0, e1, o0, o1;
  };
  struct OutsDec {
    uint2 mv[7];
  };
  using Outs = typename std::conditional<DEC, OutsDec, OutsEnc>::type;
  auto load_out = [&](int c) __attribute__((always_inline)) {
    Outs o;
    const bool vz1 = c < a.Lcz;
    if constexpr (DEC) {
#pragma unroll
      for (int k = 0; k < 7; ++k) o.mv[k] = make_uint2(0, 0);
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        if (mok_y[k] && (!par[0] || vz1)) o.mv[k] = ld8(mbase[k] + c * mplane[k]);
      }
    } else {
      const T* p = hin + 2 * c * hplane;
      o.e0 = o.e1 = o.o0 = o.o1 = make_uint4(0, 0, 0, 0);
      if (live) o.e0 = ld16(p + ho_own);
      if (live && vy1) o.e1 = ld16(p + ho_own + a.W_);
      if (live && vz1) o.o0 = ld16(p + hplane + ho_own);
      if (live && vz1 && vy1) o.o1 = ld16(p + hplane + ho_own + a.W_);
    }
    return o;
  };

  // ---- prologue: node planes kb-1 .. kb+2 staged, output plane z0's rows in flight ----
  const int kb = z0 - 1;  // first cell plane computed: the "c - 1" of output plane z0
  {
    V pre[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) pre[t] = load_node(kb - 1 + t);
#pragma unroll
    for (int t = 0; t < 4; ++t) stage(kb - 1 + t, pre[t]);
  }
  __syncthreads();

  // channels of cell plane k - 1 the output plane k reads: 5, 13 (and 13 of cell x-1), 14, 18,
  // and 17 of the row above
  uint32_t Q5[VX + 1] = {}, Q13[VX + 1] = {}, Q14[VX + 1] = {}, Q18[VX + 1] = {}, QA17[VX + 1] = {};

#pragma unroll 1
  for (int k = kb; k < z1; ++k) {
    const bool more = k + 1 < z1;
    V nxt{};
    if (more) nxt = load_node(k + 3);  // staged at the end of this step
    Outs cur;  // output plane k's rows, consumed after the sweeps
    if (k >= z0) cur = load_out(k);

    uint32_t PC[16][VX + 1];   // MFMA columns KM of cell plane k (cells X .. X+3 at [1..4])
    uint32_t PV[kNV][VX + 1];  // VALU channels 14, 17, 18
    if (k >= 0) {  // uniform; cell plane -1 does not exist (output plane 0 masks it)
      f32x4 acc[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) acc[u] = (f32x4){bias_col, bias_col, bias_col, bias_col};
      const __attribute__((address_space(4))) float* Wc = (const __attribute__((address_space(4))) float*)a.Wv;
      f32x2 av[kNV][2];
#pragma unroll
      for (int kk = 0; kk < kNV; ++kk) {
        const float bk = a.b[kKV[kk]];
        av[kk][0] = (f32x2){bk, bk};
        av[kk][1] = (f32x2){bk, bk};
      }
      // staged word of group u's B operand: row min(Y0 + u / GPR, Ey - 1), column 16 (u % GPR) + j + dx
      const int colj = mj + mq;
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int dz = s >> 2, dy = s & 3;
        const float* pl = st + slot(k - 1 + dz) * plane_words + dy * a.pitch + colj;
        const float wbs = a.W[(4 * s + mq) * 19 + kKM[mj]];  // B operand: one L1-resident load per step
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int yc = min(Y0 + u / GPR, a.Ey - 1);  // rows past the plane compute a clamped row (never read)
          acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(pl[yc * a.pitch + (u % GPR) * 16], wbs, acc[u], 0, 0, 0);
        }
        const float* rowp = (const float*)__builtin_assume_aligned(
            st + slot(k - 1 + dz) * plane_words + (Yc + dy) * a.pitch + X, 16);
        const float4 f0 = *(const float4*)rowp, f1 = *(const float4*)(rowp + 4);
        const float f[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
#pragma unroll
        for (int dx = 0; dx < kNB; ++dx) {
#pragma unroll
          for (int kk = 0; kk < kNV; ++kk) {
            const float w = Wc[(s * kNV + kk) * kNB + dx];
            const f32x2 w2 = {w, w};
            av[kk][0] = __builtin_elementwise_fma((f32x2){f[dx], f[dx + 1]}, w2, av[kk][0]);
            av[kk][1] = __builtin_elementwise_fma((f32x2){f[dx + 2], f[dx + 3]}, w2, av[kk][1]);
          }
        }
      }
#pragma unroll
      for (int kk = 0; kk < kNV; ++kk) {
        PV[kk][1] = cvt_sat<T>(av[kk][0].x);
        PV[kk][2] = cvt_sat<T>(av[kk][0].y);
        PV[kk][3] = cvt_sat<T>(av[kk][1].x);
        PV[kk][4] = cvt_sat<T>(av[kk][1].y);
      }
      // accumulator column mj holds cells 4 mq .. 4 mq + 3 of its group: one 8-byte tile store
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int ry = u / GPR, cx = (u % GPR) * 16 + 4 * mq;
        const uint32_t c0 = cvt_sat_mfma<T>(acc[u][0]), c1 = cvt_sat_mfma<T>(acc[u][1]);
        const uint32_t c2 = cvt_sat_mfma<T>(acc[u][2]), c3 = cvt_sat_mfma<T>(acc[u][3]);
        *(uint2*)(tile + mj * tstride + ry * a.Ex + cx) = make_uint2(c0 | (c1 << 16), c2 | (c3 << 16));
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the wave reads back its own tile
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#pragma unroll
      for (int kk = 0; kk < 16; ++kk) {
        const uint2 v = *(const uint2*)(tile + kk * tstride + r * a.Ex + X);
        PC[kk][1] = v.x & 0xffffu;
        PC[kk][2] = v.x >> 16;
        PC[kk][3] = v.y & 0xffffu;
        PC[kk][4] = v.y >> 16;
      }
    } else {
#pragma unroll
      for (int kk = 0; kk < 16; ++kk)
#pragma unroll
        for (int i = 1; i <= VX; ++i) PC[kk][i] = 0u;
#pragma unroll
      for (int kk = 0; kk < kNV; ++kk)
#pragma unroll
        for (int i = 1; i <= VX; ++i) PV[kk][i] = 0u;
    }
    auto& P0 = PC[0]; auto& P1 = PC[1]; auto& P2 = PC[2]; auto& P3 = PC[3]; auto& P4 = PC[4];
    auto& P6 = PC[5]; auto& P7 = PC[6]; auto& P8 = PC[7]; auto& P9 = PC[8]; auto& P10 = PC[9];
    auto& P11 = PC[10]; auto& P12 = PC[11]; auto& P15 = PC[12]; auto& P16 = PC[13];
    auto& P5 = PC[14]; auto& P13 = PC[15];
    auto& P14 = PV[0]; auto& P17 = PV[1]; auto& P18 = PV[2];

    // channels 3, 9, 10, 16, 17 of row Y-1: the lane above, or the wave above through LDS
    uint32_t A3[VX + 1], A9[VX + 1], A10[VX + 1], A16[VX + 1], A17[VX + 1];
    if (wave_live && r == a.rows - 1) {
      uint32_t* row = xrow + (size_t)wv_ * kXch * a.Ex;
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        row[0 * a.Ex + X + i] = P3[i + 1];
        row[1 * a.Ex + X + i] = P9[i + 1];
        row[2 * a.Ex + X + i] = P10[i + 1];
        row[3 * a.Ex + X + i] = P16[i + 1];
        row[4 * a.Ex + X + i] = P17[i + 1];
      }
    }
#pragma unroll
    for (int i = 1; i <= VX; ++i) {
      A3[i] = shup(P3[i], a.txn);
      A9[i] = shup(P9[i], a.txn);
      A10[i] = shup(P10[i], a.txn);
      A16[i] = shup(P16[i], a.txn);
      A17[i] = shup(P17[i], a.txn);
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
        A17[i + 1] = row[4 * a.Ex + X + i];
      }
    }
    A9[0] = shup(A9[VX], 1);  // cell (Y-1, X-1): the lane to the left
    P1[0] = shup(P1[VX], 1);
    P8[0] = shup(P8[VX], 1);
    P12[0] = shup(P12[VX], 1);
    P13[0] = shup(P13[VX], 1);

    // ---- output plane c = k (cells of planes c and c-1) ----
    const int c = k;
    if (c >= z0 && live) {
      const bool vz1 = c < a.Lcz, vz0 = c >= 1;
      bool vx[VX + 1];
#pragma unroll
      for (int qq = 0; qq <= VX; ++qq) vx[qq] = (X - 1 + qq) >= 0 && (X - 1 + qq) < a.Lcx;
      const uint32_t ny = (uint32_t)vy0 + (uint32_t)vy1;
      const uint32_t nz = (uint32_t)vz0 + (uint32_t)vz1;
      auto m = [&](const uint32_t (&v)[VX + 1], int qq, bool zok, bool yok) {
        return (zok && yok && vx[qq]) ? v[qq] : 0u;
      };
      auto put8 = [&](int kmap, const uint32_t (&res)[VX]) {
        int par[3];
        map_parity(3, kmap, par);
        if (mok_y[kmap] && (!par[0] || vz1)) st8((T*)mbase[kmap] + c * mplane[kmap], pack8<T, VX>(res));
      };
      // the lowres row: node plane c from its ring slot (f32 of a u16 is exact)
      uint32_t ownv[VX];
      {
        const float* own = st + slot(c) * plane_words + (Yc + kP) * a.pitch + kP + X;
#pragma unroll
        for (int i = 0; i < VX; ++i) ownv[i] = (uint32_t)own[i];
      }
      T* h0 = DEC ? hout + 2 * c * hplane + ho_own : nullptr;
      // decoded value (DEC) or residual of map kmap; the encode reads the ground truth from stream
      // row w (0: e0 = row 2Y of plane 2c, 1: e1 = its row 2Y+1, 2: o0, 3: o1 = plane 2c+1)
      auto code = [&](int kmap, const uint32_t (&pred)[VX], int w, int odd, uint32_t (&outv)[VX]) {
#pragma unroll
        for (int i = 0; i < VX; ++i) {
          if constexpr (DEC) {
            outv[i] = (pred[i] + el8<T>(cur.mv[kmap], i)) & MASK;
          } else {
            const uint4 src = w == 0 ? cur.e0 : (w == 1 ? cur.e1 : (w == 2 ? cur.o0 : cur.o1));
            outv[i] = (el16<T>(src, 2 * i + odd) - pred[i]) & MASK;
          }
        }
      };
      {  // X map (0,0,1): ch15 (z,y) ch16 (z,y-1) ch17 (z-1,y-1) ch18 (z-1,y); with the lowres
        uint32_t pred[VX], outv[VX];
#pragma unroll
        for (int i = 0; i < VX; ++i)
          pred[i] = (m(P15, i + 1, vz1, vy1) + m(A16, i + 1, vz1, vy0) + m(QA17, i + 1, vz0, vy0) +
                     m(Q18, i + 1, vz0, vy1)) >> ((nz * ny) >> 1);
        code(6, pred, 0, 1, outv);
        if constexpr (DEC) {
          st16(h0, pack16<T, VX>(ownv, outv));
        } else {
          st8((T*)a.lo_out + b * (int64_t)a.Ez * lplane + c * lplane + lo_own, pack8<T, VX>(ownv));
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
        code(5, pY, 1, 0, oY);
        code(2, pF, 1, 1, oF);
        if constexpr (DEC) {
          if (vy1) st16(h0 + a.W_, pack16<T, VX>(oY, oF));
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
        code(4, pZ, 2, 0, oZ);
        code(1, pU, 2, 1, oU);
        if constexpr (DEC) {
          if (vz1) st16(h0 + hplane, pack16<T, VX>(oZ, oU));
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
        code(0, pL, 3, 0, oL);
        code(3, pC, 3, 1, oC);
        if constexpr (DEC) {
          if (vz1 && vy1) st16(h0 + hplane + a.W_, pack16<T, VX>(oL, oC));
        } else {
          put8(0, oL);
          put8(3, oC);
        }
      }
    }
    // plane k's channels become output plane k+1's "c - 1" channels
#pragma unroll
    for (int i = 0; i <= VX; ++i) {
      Q5[i] = P5[i];
      Q13[i] = P13[i];
      Q14[i] = P14[i];
      Q18[i] = P18[i];
      QA17[i] = A17[i];
    }
    if (!more) break;  // uniform
    stage(k + 3, nxt);  // slot of plane k - 2: no longer read (step k read planes k-1 .. k+2)
    __syncthreads();
  }
}

}  // namespace l3r

constexpr size_t kL3rWsBytes = 16 * l3r::kNV * l3r::kNB * sizeof(float);

static int l3r_env(const char* name, int dflt) {
  const char* v = std::getenv(name);
  return v ? std::atoi(v) : dflt;
}

static bool linear3r_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, const kmp_region* region,
                              l3r::L3R& a, dim3& grid, dim3& block, size_t& lds) {
  constexpr int VX = 4;
  if (l3r_env("KMP_DISABLE_FAST", 0) || l3r_env("KMP_DISABLE_LINEAR_FUSED", 0) || !l3r_env("KMP_L3R", 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_LINEAR || pred->padding != 1 || !pred->weights || !pred->bias) return false;
  if (g.n[2] % 2 != 0 || (g.n[2] * 2) % 16 != 0) return false;
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;
  const int64_t txn = g.E[2] / VX;
  if (txn * VX != g.E[2] || g.E[2] % 16 != 0 || txn > 32 || (txn & (txn - 1)) != 0) return false;  // Ex 16..128
  const int64_t rows = 64 / txn;
  const int64_t waves = ceil_div(g.E[1], rows);
  if (waves > 4) return false;  // the workgroup covers the whole plane (row exchange through LDS)
  if (g.L[0] < 3 || g.L[1] < 3 || g.L[2] < 3) return false;  // lsrc1: one reflection covers every halo index
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
  const int64_t zext = ze - zb;
  const int64_t zper = std::max<int64_t>(1, std::min<int64_t>(zext, l3r_env("KMP_L3R_ZPER", 32)));
  a.zper = (int)zper;
  a.nrange = (int)ceil_div(zext, zper);
  a.txn = (int)txn; a.rows = (int)rows; a.nwv = (int)waves;
  a.nr = (int)(g.E[1] + 2 * l3r::kP + 1);
  a.pitch = (int)(g.E[2] - VX + 4 * ((VX + 2 * l3r::kP + 1 + 3) / 4));
  lds = ((size_t)l3r::kNS * a.nr * a.pitch + (size_t)waves * l3r::kXch * g.E[2]) * sizeof(uint32_t) +
        (size_t)waves * 16 * (rows * g.E[2] + 8) * sizeof(uint16_t);
  if (lds > 64 * 1024) return false;
  const int64_t nblk = B * a.nrange;
  a.xcd_per = (l3r_env("KMP_W3_XCD", 1) && B % 8 == 0) ? a.nrange : 0;
  grid = dim3((unsigned)nblk);
  block = dim3((unsigned)(64 * waves));
  return nblk < ((int64_t)1 << 31);
}

template <typename T>
int try_linear3r_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                        const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value) {
    l3r::L3R a{};
    dim3 grid, block;
    size_t lds = 0;
    if (!linear3r_geometry(g, B, C, pred, region, a, grid, block, lds)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    if (!ws || ws_bytes < kL3rWsBytes) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    a.W = pred->weights;
    a.b = pred->bias;
    a.Wv = (const float*)ws;
    l3r::reorder_kernel<<<1, 256, 0, stream>>>(pred->weights, (float*)ws);
    switch (a.Ex / 16) {
      case 1: l3r::linear3r_kernel<false, 1><<<grid, block, lds, stream>>>(a); break;
      case 2: l3r::linear3r_kernel<false, 2><<<grid, block, lds, stream>>>(a); break;
      case 4: l3r::linear3r_kernel<false, 4><<<grid, block, lds, stream>>>(a); break;
      default: l3r::linear3r_kernel<false, 8><<<grid, block, lds, stream>>>(a); break;
    }
    return check_launch("linear3r_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_linear3r_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                        const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                        hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value) {
    l3r::L3R a{};
    dim3 grid, block;
    size_t lds = 0;
    if (!linear3r_geometry(g, B, C, pred, region, a, grid, block, lds)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    if (!ws || ws_bytes < kL3rWsBytes) return KMP_ERR_UNSUPPORTED;
    a.hi_out = hi;
    a.lo_in = lowres;
    a.W = pred->weights;
    a.b = pred->bias;
    a.Wv = (const float*)ws;
    l3r::reorder_kernel<<<1, 256, 0, stream>>>(pred->weights, (float*)ws);
    switch (a.Ex / 16) {
      case 1: l3r::linear3r_kernel<true, 1><<<grid, block, lds, stream>>>(a); break;
      case 2: l3r::linear3r_kernel<true, 2><<<grid, block, lds, stream>>>(a); break;
      case 4: l3r::linear3r_kernel<true, 4><<<grid, block, lds, stream>>>(a); break;
      default: l3r::linear3r_kernel<true, 8><<<grid, block, lds, stream>>>(a); break;
    }
    return check_launch("linear3r_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_L3R_INST(T)                                                                                   \
  template int try_linear3r_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,   \
                                      const MapPtrs&, const kmp_region*, void*, size_t, hipStream_t);     \
  template int try_linear3r_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,            \
                                      const kmp_predictor*, T*, const kmp_region*, void*, size_t, hipStream_t);
KMP_L3R_INST(uint8_t)
KMP_L3R_INST(uint16_t)
KMP_L3R_INST(int32_t)
KMP_L3R_INST(uint32_t)

}  // namespace kmp
