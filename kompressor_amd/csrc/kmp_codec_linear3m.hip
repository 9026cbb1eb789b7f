// kmp_codec_linear3m.hip -- one-pass volume encode / decode for the LinearPredictor on the matrix
// cores (KMP_PRED_LINEAR_MFMA, padding 0; SURVEY.md §8a row a9': the north star's "learned-predictor
// apply ... MFMA only for the small dense predictor matmul").
//
// The data movement, row stepping and the aggregation / coder of kmp_codec_linear3d.hip's y-rolling
// kernel (one wave per output plane c, steps of ``rows`` lowres rows, the next steps' loads in flight);
// what changes is how the 19 channels of each cell are evaluated.  In the f32 form that is 152 packed
// FMAs per cell on the vector unit, which bounds that kernel (a memory-only variant runs at the HBM
// floor).  Here they run as bf16 MFMAs (kmp_bf16x2.h), which issue to the matrix pipe:
//   1. the lane's node rows of node planes c-1, c, c+1 go to an LDS node table as feature dwords
//      (bf16 hi byte | bf16 lo byte), rows Y mod (rows + 1) -- the step's rows plus the next step's
//      first row;
//   2. per 16-cell tile (16 per step for 16-bit samples) two v_mfma_f32_16x16x32_bf16: cell plane c
//      (node planes c, c+1: the 14 channels output plane c reads there) and cell plane c-1 (node
//      planes c-1, c: channels 5, 13, 14, 17, 18), the A fragment of a lane = its cell's 4 nodes of
//      one z-plane (two LDS reads), the B fragments (the weights' bf16 terms) and the bias per lane
//      built once; an MFMA writes each lane 4 consecutive cells of one channel -- cast to the sample
//      dtype and stored to an LDS channel table [channel][row][x];
//   3. the aggregation reads the table back in the lane-owns-VX-cells layout of linear3d (the row
//      above: the table's previous row, or for a step's first row the previous step's last row,
//      kept in a small LDS row), then the maps / coder / stores are linear3d's.
// One wave per workgroup: its LDS accesses are ordered, no barrier.  Bit-identical to kmp_linear.hip's
// linear_bf16x2_kernel (the callable / generic path of the same predictor kind).
#include <cstdlib>

#include "kmp_bf16x2.h"
#include "kmp_wave.h"

namespace kmp {
namespace l3m {

using namespace wv;

struct M3 {
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
  int32_t xcd_per;
};

// columns of the two tiles: cell plane c (P) and c-1 (Q); -1 = unused column
__constant__ int8_t kPch[16] = {0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 15, 16, -1, -1};
__constant__ int8_t kQch[16] = {5, 13, 14, 17, 18, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
constexpr int kXch = 5;                           // channels the next row reads: 3, 9, 10, 16, 17
__constant__ int8_t kXlist[kXch] = {3, 9, 10, 16, 17};

template <typename T>
__device__ __forceinline__ uint2 node_words8(const uint2& v) { return v; }
template <typename T>
__device__ __forceinline__ uint2 node_words8(const uint4& v) {  // the even elements of a highres row
  constexpr uint32_t sel = sizeof(T) == 2 ? 0x05040100u : 0x06040200u;
  return make_uint2(__builtin_amdgcn_perm(v.y, v.x, sel), __builtin_amdgcn_perm(v.w, v.z, sel));
}

template <typename T, bool DEC, int EX, int STEPS>
__global__ void __launch_bounds__(64) linear3m_kernel(M3 a) {
  constexpr int VX = 8 / (int)sizeof(T);
  static_assert(VX == 4 || VX == 8, "u16 / u8");
  constexpr int TXN = EX / VX;       // lanes per row
  constexpr int ROWS = 64 / TXN;     // rows per step
  constexpr int TPR = EX / 16;       // 16-cell tiles per row
  constexpr int NTILE = ROWS * TPR;  // tiles per step (4 VX)
  constexpr int RS = ROWS + 1;       // node table row slots
  constexpr int NS = EX + 4;         // node table row stride (dwords; EX + 1 nodes, 16-byte rows)
  constexpr int SZ = (int)sizeof(T);
  // LDS strides padded against bank conflicts (64 banks of 4 bytes): a node plane is 16 banks past
  // the previous one, so an A-fragment read (lane groups g = 0 / 1 on adjacent planes, 16 cells
  // each) touches disjoint banks; a channel is 8 banks past the previous one, so an MFMA's
  // channel-table write (16 channels x 4 cell groups, 8 / 4 bytes each) is conflict-free -- with the
  // unpadded 512-byte channel stride all 16 channels of a write hit one bank
  constexpr int PS = RS * NS + ((16 - (RS * NS) % 64) + 64) % 64;  // node plane stride (dwords)
  constexpr int CSB = ROWS * EX * SZ + ((32 - (ROWS * EX * SZ) % 256) + 256) % 256;  // channel stride (bytes)
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  static_assert(TXN >= 1 && TXN <= 32 && EX % 16 == 0, "geometry");
  using V = typename std::conditional<DEC, uint2, uint4>::type;

  // LDS: node table [3][RS][NS] dwords | channel table [19][ROWS][EX] T | previous last row [5][EX] T
  // (plane / channel strides padded, below)
  __shared__ __attribute__((aligned(16))) uint32_t nt[3 * PS];
  __shared__ __attribute__((aligned(16))) T ct[19 * CSB / SZ];
  __shared__ __attribute__((aligned(16))) T xr[kXch * EX];

  const int lane = threadIdx.x;
  const int tx = lane % TXN;
  const int r = lane / TXN;
  const int X = tx * VX;
  const int m = lane & 15, g = lane >> 4;  // MFMA roles: column / cell m, lane group g
  int blk = (int)blockIdx.x;
  if (a.xcd_per > 0) {
    const int x = blk % 8, k = blk / 8;
    blk = ((k / a.xcd_per) * 8 + x) * a.xcd_per + (k % a.xcd_per);
  }
  const int nplanes = a.zend - a.zbegin;
  const int c = a.zbegin + blk % nplanes;
  const int64_t b = blk / nplanes;
  const bool xlast = tx == TXN - 1;
  const bool r0 = r == 0, rlast = r == ROWS - 1;
  const bool vz1 = c < a.Lcz, vz0 = c >= 1;

  // ---- the weights' fragments and the bias, per lane (channel of column m); a cell plane outside
  // the tile gets zero weights and bias: its channels are 0, as the aggregation's masks want ----
  const int chP = kPch[m], chQ = kQch[m];
  const bool okP = chP >= 0 && vz1, okQ = chQ >= 0 && vz0;
  const bx::u32x4 bP = bx::b_fragment(a.W + (chP >= 0 ? chP : 0), 19, 8, 3, 0, 0, g, okP);
  const bx::u32x4 bQ = bx::b_fragment(a.W + (chQ >= 0 ? chQ : 0), 19, 8, 3, 0, 0, g, okQ);
  const float biasP = okP ? a.b[chP] : 0.0f, biasQ = okQ ? a.b[chQ] : 0.0f;

  const int hplane = a.H * a.W_;
  const int lplane = a.Ey * EX;
  const int hx = 2 * X;
  const int nstride = DEC ? EX : 2 * a.W_;
  const uint32_t lon = (uint32_t)((r * nstride + (DEC ? X : hx)) * SZ);
  const uint32_t lonx = (uint32_t)((DEC ? X : hx) * SZ);
  const uint32_t lom = (uint32_t)((r * EX + X) * SZ);
  const uint32_t loh = (uint32_t)((2 * r * a.W_ + hx) * SZ);
  const char* un[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const int q = c - 1 + t;
    const int zq = lsrc(q < 0 ? 0 : q, a.Lz, a.Ez);
    un[t] = DEC ? (const char*)a.lo_in + (b * a.Ez + zq) * (int64_t)lplane * SZ
                : (const char*)a.hi_in + (b * a.D + 2 * zq) * (int64_t)hplane * SZ;
  }
  const char* us = DEC ? nullptr : (const char*)a.hi_in + (b * a.D + 2 * c) * (int64_t)hplane * SZ;
  const int p1 = (2 * c + 1 < a.D ? hplane : 0) * SZ;
  char* um[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez;
    const int cz = par[0] ? (c < a.Lcz ? c : a.Lcz - 1) : c;
    um[k] = (char*)a.maps.p[k] + (b * ez + cz) * (int64_t)lplane * SZ;
  }
  char* ulo = DEC ? nullptr : (char*)a.lo_out + (b * a.Ez + c) * (int64_t)lplane * SZ;
  char* uho = DEC ? (char*)a.hi_out + (b * a.D + 2 * c) * (int64_t)hplane * SZ : nullptr;
  const int nstep = ROWS * nstride * SZ, mstep = ROWS * EX * SZ, hstep = ROWS * 2 * a.W_ * SZ;

  V cur[3], nxt[3], nx2[3];
  uint4 cs[3], ns[3];
  uint2 cm[7], nm[7];
  auto load_nodes = [&](int s, V (&o)[3]) {
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

  // the previous step's last row of the exchanged channels: zero before step 0 (no row above)
  if (r0) {
#pragma unroll
    for (int j = 0; j < kXch; ++j) *(uint2*)&xr[j * EX + X] = make_uint2(0, 0);
  }
  // node table writes: the lane's VX nodes of row ``slot`` in each plane (+ the mirrored node EX)
  auto stage = [&](const V (&rowv)[3], int slot) {
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const uint2 nw = node_words8<T>(rowv[t]);
      uint32_t d[VX];
#pragma unroll
      for (int i = 0; i < VX; ++i) d[i] = bx::feature_dword(el8<T>(nw, i));
      uint32_t* dst = nt + t * PS + slot * NS + X;
#pragma unroll
      for (int i = 0; i < VX; i += 4) *(uint4*)(dst + i) = make_uint4(d[i], d[i + 1], d[i + 2], d[i + 3]);
      if (xlast) dst[VX] = d[VX - 1];  // node EX: mirror of node EX - 1 (even pad)
    }
  };

#pragma unroll
  for (int s = 0; s < STEPS; ++s) {
    load_nodes(s + 2 <= STEPS ? s + 2 : STEPS, nx2);
    load_rest(s + 1 < STEPS ? s + 1 : STEPS - 1, ns, nm);
    const int Y = s * ROWS + r;
    const bool vy0 = Y >= 1;
    // slot of row s * ROWS + j: (j - s) mod RS, a compile-time constant in the unrolled loop
    const int sb = ((RS - s % RS) % RS);

    // 1. node table: this step's rows, and the next step's first row (written by the row-0 lanes)
    stage(cur, (sb + r) % RS);
    if (r0) stage(nxt, (sb + ROWS) % RS);

    // 2. the channels: two MFMAs per 16-cell tile, cast, channel table -- in batches of TB tiles
    // (all A reads of a batch, then its MFMAs, then its casts and stores), so the LDS latency and
    // the MFMA latency overlap across tiles instead of chaining tile by tile
    constexpr int TB = 4;
    static_assert(NTILE % TB == 0, "tile batches");
#pragma unroll
    for (int i0 = 0; i0 < NTILE; i0 += TB) {
      bx::u32x4 aP[TB], aQ[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        const int i = i0 + u;
        const int ri = i / TPR, x0 = 16 * (i % TPR);
        const int sl0 = (sb + ri) % RS, sl1 = (sb + ri + 1) % RS;
        const int x = x0 + m;
        const int dz = g & 1;
        const uint32_t* pP = nt + (1 + dz) * PS + x;  // cell plane c: node planes c, c+1
        const uint32_t* pQ = nt + dz * PS + x;        // cell plane c-1: node planes c-1, c
        aP[u] = (bx::u32x4){pP[sl0 * NS], pP[sl0 * NS + 1], pP[sl1 * NS], pP[sl1 * NS + 1]};
        aQ[u] = (bx::u32x4){pQ[sl0 * NS], pQ[sl0 * NS + 1], pQ[sl1 * NS], pQ[sl1 * NS + 1]};
      }
      bx::f32x4 dP[TB], dQ[TB];
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        dP[u] = bx::mfma(aP[u], bP, (bx::f32x4){biasP, biasP, biasP, biasP});
        dQ[u] = bx::mfma(aQ[u], bQ, (bx::f32x4){biasQ, biasQ, biasQ, biasQ});
      }
#pragma unroll
      for (int u = 0; u < TB; ++u) {
        const int i = i0 + u;
        const int ri = i / TPR, x0 = 16 * (i % TPR);
        // lane (g, m): cells x0 + 4g .. + 3 of channel chP / chQ, cast (XLA astype: truncate, NaN
        // and negatives 0, saturate; bx::cast_pack4) and packed
        const int cx = x0 + 4 * g;
        auto put = [&](int ch, const bx::f32x4& d) {
          const uint2 v = bx::cast_pack4<T>(d, (float)std::numeric_limits<T>::max());
          T* dst = ct + ch * (CSB / SZ) + ri * EX + cx;
          if constexpr (sizeof(T) == 2) *(uint2*)dst = v;
          else *(uint32_t*)dst = v.x;
        };
        if (chP >= 0) put(chP, dP[u]);
        if (chQ >= 0) put(chQ, dQ[u]);
      }
    }

    // 3. back in the lane-owns-VX-cells layout: channel k of cells X .. X + VX - 1 at index 1 .. VX
    auto rd = [&](int k, uint32_t (&v)[VX + 1]) {
      const uint2 w = *(const uint2*)&ct[k * (CSB / SZ) + r * EX + X];
#pragma unroll
      for (int i = 0; i < VX; ++i) v[i + 1] = el8<T>(w, i);
    };
    uint32_t A3[VX + 1], A9[VX + 1], A10[VX + 1], A16[VX + 1], QA17[VX + 1];
    {
      uint32_t* const A[kXch] = {A3, A9, A10, A16, QA17};
#pragma unroll
      for (int j = 0; j < kXch; ++j) {
        const int k = j == 0 ? 3 : j == 1 ? 9 : j == 2 ? 10 : j == 3 ? 16 : 17;
        const T* src = r0 ? &xr[j * EX + X] : &ct[k * (CSB / SZ) + (r - 1) * EX + X];  // the row above
        const uint2 w = *(const uint2*)src;
#pragma unroll
        for (int i = 0; i < VX; ++i) A[j][i + 1] = el8<T>(w, i);
      }
      if (rlast) {  // this step's last row, for the next step's first row
#pragma unroll
        for (int j = 0; j < kXch; ++j) {
          const int k = j == 0 ? 3 : j == 1 ? 9 : j == 2 ? 10 : j == 3 ? 16 : 17;
          *(uint2*)&xr[j * EX + X] = *(const uint2*)&ct[k * (CSB / SZ) + r * EX + X];
        }
      }
    }
    A9[0] = shup(A9[VX], 1);

    bool vx[VX + 1];
#pragma unroll
    for (int q = 0; q <= VX; ++q) vx[q] = q >= 1 || X >= 1;
    const uint32_t ny = (uint32_t)vy0 + 1u;
    const uint32_t nz = (uint32_t)vz0 + (uint32_t)vz1;
    auto mk = [&](const uint32_t (&v)[VX + 1], int q) { return vx[q] ? v[q] : 0u; };
    auto left = [&](uint32_t (&v)[VX + 1]) { v[0] = shup(v[VX], 1); };
    auto put8 = [&](int k, const uint32_t (&res)[VX]) {
      int par[3];
      map_parity(3, k, par);
      if (!par[0] || vz1) st8(um[k] + s * mstep + lom, pack8<T, VX>(res));
    };
    const uint4 e0 = DEC ? uint4{} : *(const uint4*)&cur[1];
    const uint4 e1 = cs[0], o0 = cs[1], o1 = cs[2];
    char* h0 = DEC ? uho + s * hstep : nullptr;
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

    // X map (0,0,1): ch15 (z,y) ch16 (z,y-1) ch17 (z-1,y-1) ch18 (z-1,y)
    {
      uint32_t P15[VX + 1], Q18[VX + 1], pred[VX], outv[VX];
      rd(15, P15);
      rd(18, Q18);
#pragma unroll
      for (int i = 0; i < VX; ++i) pred[i] = (P15[i + 1] + A16[i + 1] + QA17[i + 1] + Q18[i + 1]) >> ((nz * ny) >> 1);
      code(6, pred, e0, 1, outv);
      if constexpr (DEC) {
        st16(h0 + loh, pack16<T, VX>(ownv, outv));
      } else {
        st8(ulo + s * mstep + lom, pack8<T, VX>(ownv));
        put8(6, outv);
      }
    }
    // Z map (1,0,0): ch7 (y,x) ch8 (y,x-1) ch9 (y-1,x-1) ch10 (y-1,x);  UD (1,0,1): ch2, ch3
    {
      uint32_t P7[VX + 1], P8[VX + 1], P2[VX + 1];
      uint32_t pZ[VX], pU[VX], oZ[VX], oU[VX];
      rd(7, P7);
      rd(8, P8);
      rd(2, P2);
      left(P8);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pZ[i] = (P7[i + 1] + mk(P8, i) + mk(A9, i) + A10[i + 1]) >> ((ny * nx) >> 1);
        pU[i] = (P2[i + 1] + A3[i + 1]) >> (ny >> 1);
      }
      code(4, pZ, o0, 0, oZ);
      code(1, pU, o0, 1, oU);
      if constexpr (DEC) {
        if (vz1) st16(h0 + hplane * SZ + loh, pack16<T, VX>(oZ, oU));
      } else {
        put8(4, oZ);
        put8(1, oU);
      }
    }
    // Y map (0,1,0): ch11 (z,x) ch12 (z,x-1) ch13 (z-1,x-1) ch14 (z-1,x);  FB (0,1,1): ch4, ch5
    {
      uint32_t P11[VX + 1], P12[VX + 1], Q13[VX + 1], Q14[VX + 1], P4[VX + 1], Q5[VX + 1];
      uint32_t pY[VX], pF[VX], oY[VX], oF[VX];
      rd(11, P11);
      rd(12, P12);
      rd(13, Q13);
      rd(14, Q14);
      rd(4, P4);
      rd(5, Q5);
      left(P12);
      left(Q13);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pY[i] = (P11[i + 1] + mk(P12, i) + mk(Q13, i) + Q14[i + 1]) >> ((nz * nx) >> 1);
        pF[i] = (P4[i + 1] + Q5[i + 1]) >> (nz >> 1);
      }
      code(5, pY, e1, 0, oY);
      code(2, pF, e1, 1, oF);
      if constexpr (DEC) {
        st16(h0 + a.W_ * SZ + loh, pack16<T, VX>(oY, oF));
      } else {
        put8(5, oY);
        put8(2, oF);
      }
    }
    // LR map (1,1,0): ch0 (x), ch1 (x-1);  C (1,1,1): ch6
    {
      uint32_t P0[VX + 1], P1[VX + 1], P6[VX + 1];
      uint32_t pL[VX], pC[VX], oL[VX], oC[VX];
      rd(0, P0);
      rd(1, P1);
      rd(6, P6);
      left(P1);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pL[i] = (P0[i + 1] + mk(P1, i)) >> (nx >> 1);
        pC[i] = P6[i + 1];
      }
      code(0, pL, o1, 0, oL);
      code(3, pC, o1, 1, oC);
      if constexpr (DEC) {
        if (vz1) st16(h0 + (hplane + a.W_) * SZ + loh, pack16<T, VX>(oL, oC));
      } else {
        put8(0, oL);
        put8(3, oC);
      }
    }
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      cur[t] = nxt[t];
      nxt[t] = nx2[t];
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) cs[q] = ns[q];
#pragma unroll
    for (int k = 0; k < 7; ++k) cm[k] = nm[k];
  }
}

}  // namespace l3m

// FULL tiles (even y / x: Lcy == Ey, Lcx == Ex) with Ex in {16, 32} whose rows split into 1, 2 or 4
// wave steps; anything else is served by the generic path with kmp_linear.hip's kernel of the same
// predictor kind (bit-identical arithmetic)
template <typename T>
static bool linear3m_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, const kmp_region* region,
                              l3m::M3& a, int& steps, dim3& grid) {
  constexpr int VX = 8 / (int)sizeof(T);
  if (!(std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value)) return false;
  if (opt(OPT_DISABLE_FAST, 0) || opt(OPT_DISABLE_LINEAR_FUSED, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_LINEAR_MFMA || pred->padding != 0 || !pred->weights || !pred->bias) return false;
  if (g.Lc[1] != g.E[1] || g.Lc[2] != g.E[2] || g.Lc[0] < 1) return false;
  const int64_t ex = g.E[2];
  if (ex != 16 && ex != 32) return false;
  if ((g.n[2] * (int64_t)sizeof(T)) % 16 != 0) return false;
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;
  const int64_t rows = 64 / (ex / VX);
  if (g.E[1] % rows != 0) return false;
  steps = (int)(g.E[1] / rows);
  if (steps != 1 && steps != 2 && steps != 4) return false;
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
  const int64_t nblk = B * (ze - zb);
  a.xcd_per = (opt(OPT_W3_XCD, 1) && B % 8 == 0) ? (int)(ze - zb) : 0;
  grid = dim3((unsigned)nblk);
  return nblk < ((int64_t)1 << 31);
}

template <typename T, bool DEC>
static void launch_linear3m(int ex, int steps, dim3 grid, hipStream_t stream, const l3m::M3& a) {
  const dim3 block(64);  // one wave per output plane
#define KMP_L3M(EX, ST) l3m::linear3m_kernel<T, DEC, EX, ST><<<grid, block, 0, stream>>>(a)
  if (ex == 16) {
    if (steps == 1) KMP_L3M(16, 1);
    else if (steps == 2) KMP_L3M(16, 2);
    else KMP_L3M(16, 4);
  } else {
    if (steps == 1) KMP_L3M(32, 1);
    else if (steps == 2) KMP_L3M(32, 2);
    else KMP_L3M(32, 4);
  }
#undef KMP_L3M
}

template <typename T>
int try_linear3m_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                        const MapPtrs& maps, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3m::M3 a{};
    int steps = 0;
    dim3 grid;
    if (!linear3m_geometry<T>(g, B, C, pred, region, a, steps, grid)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    a.W = pred->weights;
    a.b = pred->bias;
    launch_linear3m<T, false>(a.Ex, steps, grid, stream, a);
    return check_launch("linear3m_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_linear3m_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                        const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3m::M3 a{};
    int steps = 0;
    dim3 grid;
    if (!linear3m_geometry<T>(g, B, C, pred, region, a, steps, grid)) return KMP_ERR_UNSUPPORTED;
    if (((uintptr_t)hi & 15) || ((uintptr_t)lowres & 7)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k) {
      if ((uintptr_t)maps.p[k] & 7) return KMP_ERR_UNSUPPORTED;
      a.maps.p[k] = (void*)maps.p[k];
    }
    a.hi_out = hi;
    a.lo_in = lowres;
    a.W = pred->weights;
    a.b = pred->bias;
    launch_linear3m<T, true>(a.Ex, steps, grid, stream, a);
    return check_launch("linear3m_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_L3M_INST(T)                                                                                   \
  template int try_linear3m_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,   \
                                      const MapPtrs&, const kmp_region*, hipStream_t);                    \
  template int try_linear3m_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,            \
                                      const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_L3M_INST(uint8_t)
KMP_L3M_INST(uint16_t)
KMP_L3M_INST(int32_t)
KMP_L3M_INST(uint32_t)

}  // namespace kmp
