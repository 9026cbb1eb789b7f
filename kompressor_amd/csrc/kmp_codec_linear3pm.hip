// kmp_codec_linear3pm.hip -- one-pass volume encode / decode for the LinearPredictor with padding 1
// on the matrix cores (KMP_PRED_LINEAR_MFMA; SURVEY.md §8a row a9', the north star's
// "learned-predictor apply").
//
// pred[cell, k] = b[k] + sum_n f_n W[n, k] over the (2p+2)^3 = 64 features of the cell's node
// neighbourhood (features_from_lowres, volume/utils.py:199-210), in the bf16x2 arithmetic of
// kmp_bf16x2.h: 8 chunks of 8 features, one v_mfma_f32_16x16x32_bf16 each, accumulated from the
// bias in chunk_at order -- the same MFMAs on the same fragments as kmp_linear.hip's linear_bf16x2_kernel, so the
// predictions are bit-identical to the callable / generic path of this predictor kind.  In the f32
// form (kmp_codec_linear3dp.hip) these are 1216 FMAs per cell on the vector unit, which bound that
// kernel at 510-560 us per C3 volume; as bf16 MFMAs they go to the matrix pipe (16 x 16 cells x
// channels per MFMA, 16 cycles).
//
// A workgroup owns a run of output planes of one tile (all 32 at C3) and rolls along z; its waves own
// ROWS lowres rows each (the lane layout, loads and aggregation of kmp_codec_linear3dp.hip).  Per
// output plane c, two phases between barriers:
//   1. each lane fetches its cells' channels of plane c-1 from the channel table into registers
//      (the row above too: the wave above's last row, or zeros on row 0); node plane c+2's rows,
//      loaded a step earlier, are staged in LDS as feature dwords (bf16 hi byte | bf16 lo byte)
//      with the mirrored halo rows / columns of the symmetric neighbourhood pad over the even
//      reflect pad (volume/utils.py:213-237) into a 5-slot ring; node plane c+3 and plane c's
//      streams are loaded for the next step -- so each node plane is read from HBM and staged once
//      per run;
//   2. the channel phase of plane c and, between its MFMA groups, the maps and coder of plane c-1
//      from the fetched registers (linear3dp's aggregation; four parts after tile rows 3, 7, 11,
//      15), so one wave issues vector work in the cycles its own MFMAs leave free.  Per 16-cell
//      tile (16 consecutive x of one row) two column tiles: cell plane c (node planes c-1 .. c+2,
//      its 14 channels) and cell plane c-1 (node planes c-2 .. c+1, channels 5, 13, 14, 17, 18),
//      8 MFMAs each.  Chunk q = 2 dz + h covers node rows dy = 2h, 2h+1 of plane dz: the A fragment
//      of lane (g, m) is its cell's 4 consecutive nodes x-1 .. x+2 of node row 2h + (g & 1) -- so
//      the plane-c tile's chunk (dz, h) and the plane-(c-1) tile's chunk (dz+1, h) read the same
//      fragment, and row Y's h = 1 fragment is row Y+2's h = 0 one: the wave walks its rows by
//      parity and reads 5 fragments per row instead of 16, the next row's while this row's odd
//      chunks run.  The weights' B fragments (built once per call, fragments_kernel) stay in
//      registers for the whole run.  Each MFMA leaves a lane one channel of 4 cells, cast to u16
//      (clamped first, kmp_bf16x2.h) and written to the wave's channel table [slot][row][x].
// 75 KB of LDS a workgroup (ring 34 KB, channel tables 42 KB), 2 workgroups per CU (<= 256 VGPRs).
// LDS pitches and the table's slot order are chosen so the fragment reads (ds_read2_b32: banks
// (a/4) mod 32 per half wave) and the channel-table writes (ds_write_b64, every column of the tile,
// the unused ones into dummy slots: no exec-mask branches) are conflict-free.
// Round 5: 296 / 289 -> 262-270 / 256-266 us per direction at C3 (rocprofv3, alternating;
// profiles/round5/): fragment bases in 10 LDS pointers per plane with immediate offsets (VALU per
// wave and plane 819 -> 601), the coder overlapped with the channel phase, the row-above masked
// instead of branched, conflict-free table slots (LDS bank-conflict cycles 6.8 M -> 2.6 M).
#include <cstdlib>

#include "kmp_bf16x2.h"
#include "kmp_wave.h"

namespace kmp {
namespace l3q {

using namespace wv;

struct PM {
  const bx::u32x4* frag;  // [3][8][64] B fragments (column tiles C, Q, zero), then [3][64] biases
  const void* hi_in;
  void* hi_out;
  const void* lo_in;
  void* lo_out;
  MapPtrs maps;
  const float* W;  // [64, 19] row-major
  const float* b;  // [19]
  int32_t D, H, W_;
  int32_t Lz, Ly, Lx, Ez, Ey, Ex, Lcz, Lcy, Lcx;
  int32_t zbegin, zend;
  int32_t nsplit, zper;  // runs of output planes per tile, planes per run
  int32_t xcd_per;
};

// a 32-bit LDS pointer (kept as one through inline-asm barriers, unlike a generic pointer)
typedef const uint32_t __attribute__((address_space(3)))* lds_cptr;

constexpr int P = 1;         // padding
constexpr int NPL = 2 * P + 2;  // staged node planes: cell plane c's neighbourhood c-P .. c+1+P
// column tiles of one cell plane: the 14 channels its own output plane reads (C) and the 5 the next
// output plane reads as its z-1 channels (Q); -1 = unused column
__constant__ int8_t kCch[16] = {0, 1, 2, 3, 4, 6, 7, 8, 9, 10, 11, 12, 15, 16, -1, -1};
__constant__ int8_t kQch[16] = {5, 13, 14, 17, 18, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};
// the channel table's slot of channel k: column m of the C tile is slot m, column m of the Q tile
// slot 14 + 5 q + m (q: the parity of the Q channels' cell plane -- they live one output plane
// longer than the C channels), so the lanes of one ds_write_b64 lane group (one column each) land
// on distinct bank pairs (a slot moves the bank by 2: CS / 2 = 2 mod 32) -- the channel numbers
// themselves collide (0 and 16)
constexpr int kSlots = 24;
#ifndef KMP_L3PM_DY0
#define KMP_L3PM_DY0 3
#endif
#ifndef KMP_L3PM_PD
#define KMP_L3PM_PD 2
#endif
__host__ __device__ constexpr int slot_of(int k, int q) {
  constexpr int8_t s[19] = {0, 1, 2, 3, 4, 14, 5, 6, 7, 8, 9, 10, 11, 15, 16, 12, 13, 17, 18};
  return s[k] + (s[k] >= 14 ? 5 * q : 0);
}

// (the 4-cell segments of either sample dtype: kmp_wave.h's HSeg / MSeg helpers; the channel table
// holds u16 either way, u8 predictions saturating at 255 before they are stored)
// an MFMA result's 4 cells cast to T (XLA astype) as the table's packed u16; ``late``: the u16
// form without the hazard pad (see kmp_bf16x2.h), for a caller with >= 8 MFMAs in between
template <typename T, bool LATE> __device__ __forceinline__ uint2 cast_cells(const bx::f32x4& v) {
  if constexpr (sizeof(T) == 2) return LATE ? bx::cast_pack4_u16_late(v) : bx::cast_pack4_u16(v);
  else return LATE ? bx::cast_pack4_u8_late(v) : bx::cast_pack4_u8(v);
}

// The weights' B fragments of both column tiles (kmp_bf16x2.h's b_fragment) and the per-column
// biases, built once per call into the workspace instead of in every wave: one workgroup per
// (tile, step), a lane one fragment (a single wave building all 24 serialised their weight loads:
// 22 us per call, as long as a tenth of the codec kernel)
constexpr int kFragBlocks = 3 * 8;
__global__ void __launch_bounds__(64) fragments_kernel(const float* __restrict__ W, const float* __restrict__ bias,
                                                       bx::u32x4* __restrict__ frag) {
  const int lane = threadIdx.x, m = lane & 15, g = lane >> 4;
  const int t = blockIdx.x / 8, q = blockIdx.x % 8;  // C, Q, and a zero tile (a cell plane outside the tile)
  const int ch = t == 0 ? kCch[m] : t == 1 ? kQch[m] : -1;
  frag[(t * 8 + q) * 64 + lane] = bx::b_fragment(W + (ch >= 0 ? ch : 0), 19, 64, 3, 1, q, g, ch >= 0);
  if (q == 0) ((float*)(frag + 3 * 8 * 64))[t * 64 + lane] = ch >= 0 ? bias[ch] : 0.0f;
}
constexpr size_t kFragBytes = 3 * 8 * 64 * sizeof(bx::u32x4) + 3 * 64 * sizeof(float);
// + the dummy store slots (8 u16 per lane) after the fragments
constexpr size_t kWsBytes = kFragBytes + 64 * 8 * sizeof(uint16_t);

template <typename T, bool DEC, int EX, int EY>
__global__ void __launch_bounds__(64 * (EY / (256 / EX))) __attribute__((amdgpu_waves_per_eu(2, 2))) linear3pm_kernel(PM a) {
  typedef uint16_t CT_T;              // channel table entries
  constexpr int VX = 4;               // cells per lane
  constexpr int TXN = EX / VX;        // lanes per row
  constexpr int ROWS = 64 / TXN;      // rows per wave
  constexpr int NW = EY / ROWS;       // waves
  constexpr int TPR = EX / 16;        // 16-cell tiles per row
  constexpr int NR = EY + 2 * P + 1;  // staged node rows -P .. EY+P
  constexpr int NHR = 4 * ((VX + 2 * P + 1 + 3) / 4) - VX - P;  // halo columns right of EX
  // staged row: node columns -P .. EX-1+NHR (dwords), the pitch padded to 16 banks past a multiple
  // of 32 (ds_read2_b32 banks are (a/4) mod 32 per half wave): an A-fragment read's lane groups
  // g = 0 / 1 (adjacent node rows) then take disjoint banks
  constexpr int PITCH0 = EX + P + NHR;
  constexpr int PITCH = PITCH0 + ((16 - PITCH0 % 32) + 32) % 32;
  // a wave's channel table (u16) [slot][row][x], the slot stride padded 2 banks past a multiple
  // of 32 so that an MFMA's 16 columns (one ds_write_b64 lane group) write 32 banks, then DMY u16
  // where the MFMA columns that carry no channel write (no exec-mask branch around the table
  // stores): a column's dummy address takes the bank pair of a slot its tile does not use
  constexpr int CS = ROWS * EX + 4;
  constexpr int DPAD = (64 - (kSlots * CS) % 64) % 64;  // dummy base: bank offset 0, like slot 0
  constexpr int DMY = DPAD + 4 * 15 + 4 * 3 + (ROWS - 1) * EX + EX / 2 + 4;
  constexpr int CT = kSlots * CS + DMY;
  static_assert(CS % 64 == 4, "bank layout");
  constexpr uint32_t MASK = sizeof(T) == 2 ? 0xffffu : 0xffu;
  static_assert(EX % 16 == 0 && ROWS % 2 == 0 && NW * ROWS == EY && NW <= 4, "geometry");
  using V = typename std::conditional<DEC, MSeg<T>, HSeg<T>>::type;

  __shared__ __attribute__((aligned(16))) uint32_t st[NPL * NR * PITCH];  // ring of 4 node planes
  __shared__ __attribute__((aligned(16))) CT_T ct[NW * CT];

  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int tx = lane % TXN;
  const int r = lane / TXN;
  const int X = tx * VX;
  const int m = lane & 15, g = lane >> 4;  // MFMA roles
  int blk = (int)blockIdx.x;
  if (a.xcd_per > 0) {
    const int x = blk % 8, k = blk / 8;
    blk = ((k / a.xcd_per) * 8 + x) * a.xcd_per + (k % a.xcd_per);
  }
  // the workgroup's tile and its run of output planes [cb, ce)
  const int64_t b = blk / a.nsplit;
  const int cb = a.zbegin + (blk % a.nsplit) * a.zper;
  const int ce = min(cb + a.zper, a.zend);
  const int Y0 = w * ROWS;
  const int Y = Y0 + r;

  const int hplane = a.H * a.W_;
  const int lplane = EY * EX;
  const T* hin = DEC ? nullptr : (const T*)a.hi_in + b * (int64_t)a.D * hplane;
  T* hout = DEC ? (T*)a.hi_out + b * (int64_t)a.D * hplane : nullptr;
  const T* lin = DEC ? (const T*)a.lo_in + b * (int64_t)a.Ez * lplane : nullptr;
  T* lout = DEC ? nullptr : (T*)a.lo_out + b * (int64_t)a.Ez * lplane;
  const int hx = 2 * X;
  const int ho_own = 2 * Y * a.W_ + hx;
  const int lo_own = Y * EX + X;
  T* mbase[7];
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    int par[3];
    map_parity(3, k, par);
    const int ez = par[0] ? a.Lcz : a.Ez;
    // a uniform base per map (scalar registers) and the lane's 32-bit offset lo_own: no 64-bit
    // pointer per map in vector registers
    mbase[k] = (T*)a.maps.p[k] + b * (int64_t)ez * lplane;  // FULL: Lcy == Ey
  }

  // the lane's node row of node plane q (any q within one reflection of the axis)
  auto node_row = [&](int q) -> V {
    const int sz = lsrc1(q, a.Lz, a.Ez);
    if constexpr (DEC) return ldMc<T>(lin + sz * lplane + lo_own);
    else return ldHc<T>(hin + 2 * sz * hplane + ho_own);
  };
  // the rows an output plane's coder reads besides its nodes: the maps (decode) / the highres
  // rows of the odd positions (encode)
  struct Streams {
    MSeg<T> mv[7];
    HSeg<T> e1, o0, o1;
  };
  auto load_streams = [&](int c, Streams& sv) {
    // unconditional: a plane past an odd-sized z axis (c >= Lcz) re-reads the one before, its
    // values unused (the outputs go to the dummy slot)
    const bool vz1 = c < a.Lcz;
    if constexpr (DEC) {
#pragma unroll
      for (int k = 0; k < 7; ++k) {
        int par[3];
        map_parity(3, k, par);
        sv.mv[k] = ldM<T>(mbase[k] + (((!par[0] || vz1) ? c : c - 1) * lplane + lo_own));
      }
    } else {
      const T* p = hin + 2 * c * hplane;
      const int o = vz1 ? hplane : 0;
      sv.e1 = ldH<T>(p + ho_own + a.W_);
      sv.o0 = ldH<T>(p + o + ho_own);
      sv.o1 = ldH<T>(p + o + ho_own + a.W_);
    }
  };

  const int chC = kCch[m], chQ = kQch[m];
  CT_T* const ctw = ct + w * CT;
  // the lane's column of the channel table (its C / Q channel, 4 cells from x0 + 4g), or its dummy slot
  // dummy addresses mimic the bank pair of a slot (mod 16) the tile's real columns do not take:
  // C: slots 14, 15; Q of parity 0 (slots 14 .. 18, banks of slots 14, 15, 0, 1, 2): slots 3 .. 13;
  // Q of parity 1 (slots 19 .. 23, banks of slots 3 .. 7): slots 8 .. 15, 0 .. 2
  CT_T* const dmy = ctw + kSlots * CS + DPAD + 4 * g;
  CT_T* const ctC = m < 14 ? ctw + m * CS + 4 * g : dmy + 4 * m;
  CT_T* const ctQ0 = m < 5 ? ctw + (14 + m) * CS + 4 * g : dmy + 4 * (m - 2);
  CT_T* const ctQ1 = m < 5 ? ctw + (19 + m) * CS + 4 * g : dmy + 4 * ((m + 3) & 15);
  // the lane's A-fragment origin: ring slot 0, node row Y0 + (g & 1), node column m
  const lds_cptr fl = (lds_cptr)st + Y0 * PITCH + m;

  // ---- staging: the node row of node plane q as feature dwords into ring slot q mod 5, plus
  // the mirrored halo columns / rows this lane is the source of (lsrc1) ----
  auto stage = [&](const V& own, int q) {
    const int slot = (q + 2 * NPL) % NPL;  // q >= -2
    const bool xfirst = tx == 0, xlast = tx == TXN - 1;
    uint32_t v[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i)
      v[i] = bx::feature_dword(DEC ? elM<T>(*(const MSeg<T>*)&own, i) : elH<T>(*(const HSeg<T>*)&own, 2 * i));
    auto put_row = [&](int ry) __attribute__((always_inline)) {
      uint32_t* row = st + (slot * NR + ry) * PITCH + P + X;
#pragma unroll
      for (int i = 0; i < VX; ++i) row[i] = v[i];
      if (xfirst) {
#pragma unroll
        for (int k = 1; k <= P; ++k) row[-k] = v[k - 1];  // node column -k mirrors column k-1
      }
      if (xlast) {
#pragma unroll
        for (int j = 0; j < NHR; ++j) {
          const int sx = lsrc1(EX + j, a.Lx, EX) - X;
          uint32_t u = v[0];
#pragma unroll
          for (int i = 1; i < VX; ++i) u = sx == i ? v[i] : u;
          row[VX + j] = u;
        }
      }
    };
    put_row(Y + P);
#pragma unroll
    for (int h = 0; h < 2 * P + 1; ++h) {  // node rows -P .. -1 and EY .. EY+P
      const int rr = h < P ? h - P : EY + (h - P);
      if (lsrc1(rr, a.Ly, EY) == Y) put_row(rr + P);
    }
  };

  // ---- the channels of cell plane c on the matrix cores, into the wave's channel table: its C
  // channels (skipped with withC = false) and its Q channels (into the slots of parity c & 1).  A
  // cell plane outside the tile (c < 0 or c >= Lcz) has channels 0, what the aggregation's masks
  // want: its computed channels are overwritten with zeros ----
  // hook(tr) runs after tile row tr (0 .. 2 ROWS - 1): the caller's vector work placed between the
  // MFMA groups in program order
  auto channels = [&](int c, bool withC, const bx::u32x4 (&bC)[8], const bx::u32x4 (&bQ)[8], float biasC,
                      float biasQ, auto&& hook) {
    CT_T* const ctQ = (c & 1) ? ctQ1 : ctQ0;
    constexpr int NJ = ROWS + 3;
    // A fragment: node plane c - 1 + t (ring slot (c - 1 + t) mod 4), staged rows Y0 + ry + (g & 1),
    // cells x0 + m: one base per slot and half of the wave's rows, the rest immediate offsets
    // A fragment of plane pair e: this lane's plane c - 1 + 2 e + (g & 1) (ring slot mod 4), staged
    // row Y0 + ry, cells x0 + m: one base per pair and half of the wave's rows, the rest immediate
    // offsets
    lds_cptr fb[2][2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      fb[e][0] = fl + ((c - 1 + 2 * e + (g & 1) + 2 * NPL) % NPL) * (NR * PITCH);
      fb[e][1] = fb[e][0] + 5 * PITCH;
      // opaque to the optimiser: otherwise it folds fb[e][1] back into fb[e][0] + a constant past
      // ds_read2_b32's 8-bit offsets and pays a v_add_u32 per fragment half
      asm volatile("" : "+v"(fb[e][0]));
      asm volatile("" : "+v"(fb[e][1]));
    }
    auto frag = [&](int e, int ry, int x0) {
      const lds_cptr p = fb[e][ry >= 5] + (ry >= 5 ? ry - 5 : ry) * PITCH + x0;
      return (bx::u32x4){p[0], p[1], p[2], p[3]};
    };
    // per x tile, the node rows j = 0 .. ROWS+2 of the wave's rows (node row Y0-1+j): the two
    // fragments of node row j (plane pairs 0, 1) feed accumulation steps 2 (j - r) + e of the cell
    // rows r = j-3 .. j (C and Q tiles alike), so each fragment is read once and used by up to 4
    // rows x 2 tiles; row r starts at j = r (from the bias) and is cast and stored after j = r + 3.
    // The x tiles' node rows run as one sequence of TPR * NJ steps whose fragments are read KMP_L3PM_PD
    // steps ahead (a ring of KMP_L3PM_PD + 1 fragment pairs), across the x-tile boundary too: the
    // steps at the ends of a tile run few MFMAs (1 to 3 rows), too few to cover an LDS read.
    constexpr int NS = TPR * NJ, PD = KMP_L3PM_PD, NF = PD + 1;
    bx::u32x4 F[NF][2];
#pragma unroll
    for (int q = 0; q < PD; ++q) {
      F[q][0] = frag(0, q % NJ, 16 * (q / NJ));
      F[q][1] = frag(1, q % NJ, 16 * (q / NJ));
    }
    bx::f32x4 aC[4], aQ[4];  // cell row r in slot r & 3
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      {
        const int xt = st / NJ, j = st % NJ, cur = st % NF;
        if (st + PD < NS) {
          F[(st + PD) % NF][0] = frag(0, (st + PD) % NJ, 16 * ((st + PD) / NJ));
          F[(st + PD) % NF][1] = frag(1, (st + PD) % NJ, 16 * ((st + PD) / NJ));
        }
        if (j < ROWS) {
          aC[j & 3] = (bx::f32x4){biasC, biasC, biasC, biasC};
          aQ[j & 3] = (bx::f32x4){biasQ, biasQ, biasQ, biasQ};
        }
        // cell row r = j - dy (its steps 2 dy + e in order), the row that completes here (dy = 3)
        // first: the other rows' MFMAs then cover its results' latency before the cast reads them
#pragma unroll
        for (int dy = KMP_L3PM_DY0; KMP_L3PM_DY0 ? dy >= 0 : dy < 4; dy += KMP_L3PM_DY0 ? -1 : 1) {
          const int rr = j - dy;
          if (rr < 0 || rr >= ROWS) continue;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            if (withC) aC[rr & 3] = bx::mfma(F[cur][e], bC[2 * dy + e], aC[rr & 3]);
            aQ[rr & 3] = bx::mfma(F[cur][e], bQ[2 * dy + e], aQ[rr & 3]);
          }
        }
        if (j >= 3) {  // cell row j - 3 is complete
          const int row = j - 3;
          // MFMAs issued after the row's last one: those of rows j - 2 .. j
          int after = 0;
#pragma unroll
          for (int rr = j - 2; rr <= j; ++rr) after += (rr < ROWS) ? (withC ? 4 : 2) : 0;
          if (KMP_L3PM_DY0 && after >= 8) {
            __builtin_amdgcn_sched_barrier(0);
            if (withC) *(uint2*)(ctC + row * EX + 16 * xt) = cast_cells<T, true>(aC[row & 3]);
            *(uint2*)(ctQ + row * EX + 16 * xt) = cast_cells<T, true>(aQ[row & 3]);
          } else {
            if (withC) *(uint2*)(ctC + row * EX + 16 * xt) = cast_cells<T, false>(aC[row & 3]);
            *(uint2*)(ctQ + row * EX + 16 * xt) = cast_cells<T, false>(aQ[row & 3]);
          }
        }
        hook(st);
      }
    }
    if (c < 0 || c >= a.Lcz) {  // (uniform; the tile's first / last plane) overwritten with zeros
#pragma unroll
      for (int xt = 0; xt < TPR; ++xt)
#pragma unroll
        for (int row = 0; row < ROWS; ++row) {
          if (withC) *(uint2*)(ctC + row * EX + 16 * xt) = make_uint2(0, 0);
          *(uint2*)(ctQ + row * EX + 16 * xt) = make_uint2(0, 0);
        }
    }
  };

  const CT_T* const upt = (r > 0 ? ctw + (r - 1) * EX : w > 0 ? ctw - CT + (ROWS - 1) * EX : ctw) + X;
  const uint32_t upm = Y > 0 ? 0xffffffffu : 0u;
  // the channels the coder of one output plane reads: the lane's 4 cells of all 19 channels (slot
  // order) and the 5 row-above channels (3, 9, 10, 16, 17; this wave's row r - 1, the wave above's
  // last row, or zeros by a mask on row 0), as packed u16.  Fetched right after the barrier that
  // completes the plane's table, so the next plane's channel phase may overwrite the table while
  // this plane is coded from registers.
  struct Chan {
    uint2 v[19];
    uint2 up[5];
  };
  // (q: the parity of the output plane before the one being coded -- its Q slots hold the z-1 channels)
  auto fetch = [&](Chan& ch, int q) {
#pragma unroll
    for (int k = 0; k < 19; ++k) ch.v[k] = *(const uint2*)(ctw + slot_of(k, q) * CS + r * EX + X);
    constexpr int kUp[5] = {3, 9, 10, 16, 17};
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      uint2 u = *(const uint2*)(upt + slot_of(kUp[j], q) * CS);
      ch.up[j] = make_uint2(u.x & upm, u.y & upm);
    }
  };
  // where the stores of outputs that do not exist go (a plane past an odd-sized axis): a scratch
  // slot per lane in the workspace, so the store needs no branch
  T* const dummy = (T*)((char*)a.frag + kFragBytes) + 8 * lane;

  constexpr int kAggParts = 7;
  // ---- the maps / coder of output plane c from its channels (linear3dp's aggregation): channel k
  // of the lane's cells X .. X+3 at index 1 .. 4 ----
  // part 0: the lowres and X map; 1: Z; 2: UD; 3: Y; 4: FB; 5: LR; 6: C (the decode's Z, Y, LR
  // values wait in ``keep`` for the map stored in the same highres row)
  auto aggregate = [&](int c, const V& own, const Streams& sv, const Chan& ch, int part, uint32_t (&keep)[VX]) {
    const bool vz1 = c < a.Lcz, vz0 = c >= 1;
    auto rd = [&](int k, uint32_t (&v)[VX + 1]) {
#pragma unroll
      for (int i = 0; i < VX; ++i) v[i + 1] = el8<CT_T>(ch.v[k], i);
    };
    auto rd_up = [&](int j, uint32_t (&v)[VX + 1]) {
#pragma unroll
      for (int i = 0; i < VX; ++i) v[i + 1] = el8<CT_T>(ch.up[j], i);
    };
    uint32_t A3[VX + 1], A9[VX + 1], A10[VX + 1], A16[VX + 1], QA17[VX + 1];
    rd_up(0, A3);
    rd_up(1, A9);
    rd_up(2, A10);
    rd_up(3, A16);
    rd_up(4, QA17);
    A9[0] = shup(A9[VX], 1);

    const bool vy0 = Y >= 1;
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
      stM<T>((!par[0] || vz1) ? mbase[k] + (c * lplane + lo_own) : dummy, packM<T>(res));
    };
    const HSeg<T> e0 = DEC ? HSeg<T>{} : *(const HSeg<T>*)&own;
    T* h0 = DEC ? hout + 2 * c * hplane + ho_own : nullptr;
    uint32_t ownv[VX];
#pragma unroll
    for (int i = 0; i < VX; ++i) {
      if constexpr (DEC) ownv[i] = elM<T>(*(const MSeg<T>*)&own, i);
      else ownv[i] = elH<T>(e0, 2 * i);
    }
    auto code = [&](int k, const uint32_t (&pred)[VX], const HSeg<T>& src, int odd, uint32_t (&outv)[VX]) {
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        if constexpr (DEC) outv[i] = (pred[i] + elM<T>(sv.mv[k], i)) & MASK;
        else outv[i] = (elH<T>(src, 2 * i + odd) - pred[i]) & MASK;
      }
    };

    // X map (0,0,1): ch15 (z,y) ch16 (z,y-1) ch17 (z-1,y-1) ch18 (z-1,y); with the lowres
    if (part == 0) {
      uint32_t P15[VX + 1], Q18[VX + 1], pred[VX], outv[VX];
      rd(15, P15);
      rd(18, Q18);
#pragma unroll
      for (int i = 0; i < VX; ++i) pred[i] = (P15[i + 1] + A16[i + 1] + QA17[i + 1] + Q18[i + 1]) >> ((nz * ny) >> 1);
      code(6, pred, e0, 1, outv);
      if constexpr (DEC) {
        stH<T>(h0, packH<T>(ownv, outv));
      } else {
        stM<T>(lout + c * lplane + lo_own, packM<T>(ownv));
        put8(6, outv);
      }
    }
    // Z map (1,0,0): ch7 (y,x) ch8 (y,x-1) ch9 (y-1,x-1) ch10 (y-1,x);  UD (1,0,1): ch2, ch3
    if (part == 1) {
      uint32_t P7[VX + 1], P8[VX + 1], pZ[VX];
      rd(7, P7);
      rd(8, P8);
      left(P8);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pZ[i] = (P7[i + 1] + mk(P8, i) + mk(A9, i) + A10[i + 1]) >> ((ny * nx) >> 1);
      }
      code(4, pZ, sv.o0, 0, keep);
      if constexpr (!DEC) put8(4, keep);
    }
    if (part == 2) {
      uint32_t P2[VX + 1], pU[VX], oU[VX];
      rd(2, P2);
#pragma unroll
      for (int i = 0; i < VX; ++i) pU[i] = (P2[i + 1] + A3[i + 1]) >> (ny >> 1);
      code(1, pU, sv.o0, 1, oU);
      if constexpr (DEC) stH<T>(vz1 ? h0 + hplane : dummy, packH<T>(keep, oU));
      else put8(1, oU);
    }
    // Y map (0,1,0): ch11 (z,x) ch12 (z,x-1) ch13 (z-1,x-1) ch14 (z-1,x);  FB (0,1,1): ch4, ch5
    if (part == 3) {
      uint32_t P11[VX + 1], P12[VX + 1], Q13[VX + 1], Q14[VX + 1], pY[VX];
      rd(11, P11);
      rd(12, P12);
      rd(13, Q13);
      rd(14, Q14);
      left(P12);
      left(Q13);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pY[i] = (P11[i + 1] + mk(P12, i) + mk(Q13, i) + Q14[i + 1]) >> ((nz * nx) >> 1);
      }
      code(5, pY, sv.e1, 0, keep);
      if constexpr (!DEC) put8(5, keep);
    }
    if (part == 4) {
      uint32_t P4[VX + 1], Q5[VX + 1], pF[VX], oF[VX];
      rd(4, P4);
      rd(5, Q5);
#pragma unroll
      for (int i = 0; i < VX; ++i) pF[i] = (P4[i + 1] + Q5[i + 1]) >> (nz >> 1);
      code(2, pF, sv.e1, 1, oF);
      if constexpr (DEC) stH<T>(h0 + a.W_, packH<T>(keep, oF));
      else put8(2, oF);
    }
    // LR map (1,1,0): ch0 (x), ch1 (x-1);  C (1,1,1): ch6
    if (part == 5) {
      uint32_t P0[VX + 1], P1[VX + 1], pL[VX];
      rd(0, P0);
      rd(1, P1);
      left(P1);
#pragma unroll
      for (int i = 0; i < VX; ++i) {
        const uint32_t nx = (uint32_t)vx[i] + (uint32_t)vx[i + 1];
        pL[i] = (P0[i + 1] + mk(P1, i)) >> (nx >> 1);
      }
      code(0, pL, sv.o1, 0, keep);
      if constexpr (!DEC) put8(0, keep);
    }
    if (part == 6) {
      uint32_t P6[VX + 1], pC[VX], oC[VX];
      rd(6, P6);
#pragma unroll
      for (int i = 0; i < VX; ++i) pC[i] = P6[i + 1];
      code(3, pC, sv.o1, 1, oC);
      if constexpr (DEC) stH<T>(vz1 ? h0 + hplane + a.W_ : dummy, packH<T>(keep, oC));
      else put8(3, oC);
    }
  };

  // ---- the run, one barrier pair per output plane c:
  //   [fetch plane c-1's channels | stage node plane c+2 | load node plane c+3 and plane c's streams]
  //   barrier
  //   [channels of plane c (matrix cores, into the table) || maps + coder of plane c-1 (registers)]
  //   barrier
  // The second phase holds both the MFMA work and the vector work, independent of each other, so
  // one wave issues vector instructions between its own MFMAs.  Node planes c-1 .. c+3 stay in
  // registers (R0 .. R4) until their coder step; each node plane is loaded and staged once per run.
  bx::u32x4 bC[8], bQ[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    bC[q] = a.frag[q * 64 + lane];
    bQ[q] = a.frag[(8 + q) * 64 + lane];
  }
  const float* fb = (const float*)(a.frag + 3 * 8 * 64);
  const float biasC = fb[lane], biasQ = fb[64 + lane];
  V R0 = node_row(cb - 1), R1 = node_row(cb), R2 = node_row(cb + 1), R3 = node_row(cb + 2);
  // the Q channels of cell plane cb - 1 (the first output plane's z-1 channels; zeros at cb = 0),
  // from node planes cb - 2 .. cb + 1
  stage(node_row(cb - 2), cb - 2);
  stage(R0, cb - 1);
  stage(R1, cb);
  stage(R2, cb + 1);
  __syncthreads();
  channels(cb - 1, false, bC, bQ, biasC, biasQ, [](int) {});
  __syncthreads();
  Streams Sp, Sc;
  Chan ch;
  uint32_t keep[VX];
  // plane cb: no coder work yet
  stage(R3, cb + 2);
  V R4 = node_row(cb + 3 < ce + 2 ? cb + 3 : cb + 2);
  load_streams(cb, Sc);
  __syncthreads();
  channels(cb, true, bC, bQ, biasC, biasQ, [](int) {});
  __syncthreads();
  for (int c = cb + 1; c < ce; ++c) {
    R0 = R1;
    R1 = R2;
    R2 = R3;
    R3 = R4;
    Sp = Sc;
    fetch(ch, c & 1);  // plane c-1's channels, the Q channels of cell plane c-2
    stage(R3, c + 2);
    R4 = node_row(c + 1 < ce ? c + 3 : c + 2);  // the last step re-reads a plane (unused)
    load_streams(c, Sc);
    __syncthreads();
    // the coder's vector work in kAggParts parts between the MFMA groups (an MFMA leaves 8 of its
    // 16 cycles free for issue), not after the last one
    constexpr int NSTEP = TPR * (ROWS + 3);
    channels(c, true, bC, bQ, biasC, biasQ, [&](int st_) {
      if ((st_ + 1) * kAggParts / NSTEP != st_ * kAggParts / NSTEP)
        aggregate(c - 1, R0, Sp, ch, (st_ + 1) * kAggParts / NSTEP - 1, keep);
    });
    __syncthreads();
  }
  fetch(ch, ce & 1);
#pragma unroll
  for (int part = 0; part < kAggParts; ++part) aggregate(ce - 1, R1, Sc, ch, part, keep);
}

}  // namespace l3q

// u8 / u16 FULL tiles (Lcy == Ey, Lcx == Ex) with Ex, Ey in {16, 32}; anything else is served by the
// generic path with kmp_linear.hip's kernel of the same predictor kind (bit-identical arithmetic)
template <typename T>
static bool linear3pm_geometry(const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred,
                               const kmp_region* region, l3q::PM& a, dim3& grid, dim3& block) {
  constexpr int P = l3q::P;
  if (!std::is_same<T, uint16_t>::value && !std::is_same<T, uint8_t>::value) return false;
  if (opt(OPT_DISABLE_FAST, 0) || opt(OPT_DISABLE_LINEAR_FUSED, 0)) return false;
  if (C != 1 || pred->kind != KMP_PRED_LINEAR_MFMA || pred->padding != P || !pred->weights || !pred->bias) return false;
  if (g.E[2] != 16 && g.E[2] != 32) return false;
  if (g.E[1] != 16 && g.E[1] != 32) return false;
  if (g.Lc[1] != g.E[1] || g.Lc[2] != g.E[2] || g.Lc[0] < 1) return false;
  if (g.n[2] % 8 != 0) return false;  // 8-sample highres row segments, aligned
  if (g.n[0] * g.n[1] * g.n[2] >= ((int64_t)1 << 31)) return false;
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
  // each workgroup codes a run of output planes of one tile (node planes staged once per run):
  // runs of >= 4 planes, enough of them for 2 workgroups per CU (the LDS holds 2)
  const int64_t nz = ze - zb;
  int64_t nsplit = std::min<int64_t>(ceil_div(512, B), ceil_div(nz, 4));
  if (nsplit < 1) nsplit = 1;
  a.zper = (int)ceil_div(nz, nsplit);
  a.nsplit = (int)ceil_div(nz, a.zper);
  const int64_t nblk = B * a.nsplit;
  a.xcd_per = (opt(OPT_W3_XCD, 1) && B % 8 == 0) ? a.nsplit : 0;
  const int rows = 64 / (a.Ex / 4);
  grid = dim3((unsigned)nblk);
  block = dim3((unsigned)(64 * (a.Ey / rows)));
  return nblk < ((int64_t)1 << 31);
}

template <typename T, bool DEC>
static void launch_linear3pm(const l3q::PM& a, dim3 grid, dim3 block, hipStream_t stream) {
#define KMP_L3Q(EX, EY) l3q::linear3pm_kernel<T, DEC, EX, EY><<<grid, block, 0, stream>>>(a)
  if (a.Ex == 32) {
    if (a.Ey == 32) KMP_L3Q(32, 32);
    else KMP_L3Q(32, 16);
  } else {
    if (a.Ey == 32) KMP_L3Q(16, 32);
    else KMP_L3Q(16, 16);
  }
#undef KMP_L3Q
}

template <typename T>
int try_linear3pm_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                         const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3q::PM a{};
    dim3 grid, block;
    if (!linear3pm_geometry<T>(g, B, C, pred, region, a, grid, block)) return KMP_ERR_UNSUPPORTED;
    constexpr uintptr_t HA = 8 * sizeof(T) - 1, MA = 4 * sizeof(T) - 1;  // segment alignments
    if (((uintptr_t)hi & HA) || ((uintptr_t)lowres & MA)) return KMP_ERR_UNSUPPORTED;
    for (int k = 0; k < 7; ++k)
      if ((uintptr_t)maps.p[k] & MA) return KMP_ERR_UNSUPPORTED;
    a.hi_in = hi;
    a.lo_out = lowres;
    a.maps = maps;
    a.W = pred->weights;
    a.b = pred->bias;
    if (!ws || ws_bytes < l3q::kWsBytes || ((uintptr_t)ws & 15)) return KMP_ERR_UNSUPPORTED;
    a.frag = (const bx::u32x4*)ws;
    l3q::fragments_kernel<<<l3q::kFragBlocks, 64, 0, stream>>>(pred->weights, pred->bias, (bx::u32x4*)ws);
    launch_linear3pm<T, false>(a, grid, block, stream);
    return check_launch("linear3pm_encode");
  }
  return KMP_ERR_UNSUPPORTED;
}

template <typename T>
int try_linear3pm_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                         const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream) {
  if constexpr (std::is_same<T, uint16_t>::value || std::is_same<T, uint8_t>::value) {
    l3q::PM a{};
    dim3 grid, block;
    if (!linear3pm_geometry<T>(g, B, C, pred, region, a, grid, block)) return KMP_ERR_UNSUPPORTED;
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
    if (!ws || ws_bytes < l3q::kWsBytes || ((uintptr_t)ws & 15)) return KMP_ERR_UNSUPPORTED;
    a.frag = (const bx::u32x4*)ws;
    l3q::fragments_kernel<<<l3q::kFragBlocks, 64, 0, stream>>>(pred->weights, pred->bias, (bx::u32x4*)ws);
    launch_linear3pm<T, true>(a, grid, block, stream);
    return check_launch("linear3pm_decode");
  }
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_L3Q_INST(T)                                                                                   \
  template int try_linear3pm_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,  \
                                       const MapPtrs&, const kmp_region*, void*, size_t, hipStream_t);    \
  template int try_linear3pm_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,           \
                                       const kmp_predictor*, T*, const kmp_region*, void*, size_t, hipStream_t);
KMP_L3Q_INST(uint8_t)
KMP_L3Q_INST(uint16_t)
KMP_L3Q_INST(int32_t)
KMP_L3Q_INST(uint32_t)

}  // namespace kmp
