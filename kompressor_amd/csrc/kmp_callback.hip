// kmp_callback.hip -- the reference's step sequence around an OPAQUE predictions_fn, fused on
// either side of the callback when the coder is a built-in one (utils.py:38-55 for the sample
// dtype).  A user's predictor (a network, any callable) keeps its exact contract -- it is called
// once with the reference's padded lowres window and returns the 7 (2D: 3) untrimmed prediction
// maps -- while the reference's other steps collapse into two launches per direction:
//
//   encode (volume/encode_decode.py:30-56):
//     kmp_window_from_highres      pad_neighborhood(lowres_from_highres(pad_highres(h)), p)
//     predictions_fn(window)       (caller)
//     kmp_encode_with_predictions  trim(lowres), trim_maps([encode_fn(p, g) for p, g in
//                                  zip(preds, maps_from_highres(pad_highres(h)))])
//   decode (volume/encode_decode.py:59-85):
//     kmp_window_from_lowres       pad_neighborhood(pad_lowres(lowres, dims), p)
//     predictions_fn(window)       (caller)
//     kmp_decode_with_predictions  trim(highres_from_lowres_and_maps(pad_lowres(lowres),
//                                  [decode_fn(p, e) for p, e in zip(preds, pad_maps(maps))]))
//
// Every element the trims keep lies inside the unpadded arrays (an output block o < E reads
// highres 2o + parity < n), so the coder kernels need no mirroring at all: the pads only ever
// produce entries the trims drop.  The window is a gather through the composed mirror maps
// (even reflect pad, then the symmetric neighbourhood pad).
#include <cstdlib>

#include "kmp_codec.h"

namespace kmp {
namespace cb {

constexpr int kThreads = 256;

static inline unsigned grid_for(int64_t n) {
  int64_t g = ceil_div(n, kThreads);
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

// window[b, j, c] = src[b, mult * sym(sym(j - p, L), E), c] per spatial axis (mult 2: highres,
// 1: trimmed lowres); W = L + 2p, unused leading axis has extent 1.
template <typename T>
__global__ void __launch_bounds__(kThreads) window_kernel(const T* __restrict__ src, int64_t B, Geo g, int64_t S0,
                                                        int64_t S1, int64_t S2, int mult, int nsp, int p, int64_t C,
                                                        int64_t W0, int64_t W1, int64_t W2, T* __restrict__ out,
                                                        int64_t total) {
  const int pz = nsp == 3 ? p : 0;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t b, jz, jy, jx, c;
    unflat5(t, W0, W1, W2, C, b, jz, jy, jx, c);
    const int64_t z = mult * sym_index(sym_index(jz - pz, g.L[0]), g.E[0]);
    const int64_t y = mult * sym_index(sym_index(jy - p, g.L[1]), g.E[1]);
    const int64_t x = mult * sym_index(sym_index(jx - p, g.L[2]), g.E[2]);
    out[t] = src[(((b * S0 + z) * S1 + y) * S2 + x) * C + c];
  }
}

// Row form (C == 1, < 2^30 elements): item = 16 B of one window row; the row's source row is
// resolved once, interior chunks are one 16-byte copy (lowres source) or two 16-byte loads whose
// even elements are kept (highres source), edge chunks mirror per element.
__device__ __forceinline__ int32_t sym32(int32_t i, int32_t n) {
  if (i >= 0 && i < n) return i;
  if (i >= -n && i < 2 * n) return i < 0 ? -1 - i : 2 * n - 1 - i;
  int32_t m = i % (2 * n);
  if (m < 0) m += 2 * n;
  return m < n ? m : 2 * n - 1 - m;
}

template <typename T>
__global__ void __launch_bounds__(kThreads) rows_window_kernel(const T* __restrict__ src, int32_t S0, int32_t S1,
                                                             int32_t S2, Geo g, int mult, int pz, int p, int32_t W0,
                                                             int32_t W1, int32_t W2, T* __restrict__ out, int32_t nch,
                                                             int32_t items) {
  constexpr int V = Vec16<T>::V;
  const int32_t L0 = (int32_t)g.L[0], L1 = (int32_t)g.L[1], L2 = (int32_t)g.L[2];
  const int32_t E0 = (int32_t)g.E[0], E1 = (int32_t)g.E[1], E2 = (int32_t)g.E[2];
  for (int32_t t = blockIdx.x * kThreads + threadIdx.x; t < items; t += gridDim.x * kThreads) {
    const RowItem q = row_item((uint32_t)t, W0, W1, nch);
    const int32_t z = mult * sym32(sym32(q.z - pz, L0), E0), y = mult * sym32(sym32(q.y - p, L1), E1);
    const T* row = src + ((q.b * S0 + z) * S1 + y) * S2;
    T* dst = out + ((q.b * W0 + q.z) * W1 + q.y) * W2;
    const int32_t x0 = q.j * V, xs = x0 - p;
    const bool inner = x0 + V <= W2 && xs >= 0 && xs + V <= E2;
    if (inner && mult == 1) {
      Vec16<T> v;
      v.load(row + xs);
      v.store(dst + x0);
    } else if (inner && 2 * xs + 2 * V <= S2) {
      Vec16<T> a, b, o;
      a.load(row + 2 * xs);
      b.load(row + 2 * xs + V);
#pragma unroll
      for (int i = 0; i < V / 2; ++i) {
        o.e[i] = a.e[2 * i];
        o.e[V / 2 + i] = b.e[2 * i];
      }
      o.store(dst + x0);
    } else {
      for (int32_t x = x0; x < x0 + V && x < W2; ++x) dst[x] = row[mult * sym32(sym32(x - p, L2), E2)];
    }
  }
}

// Untrimmed (prediction) and trimmed (coded) extents of map k.
__device__ __forceinline__ void map_ext(const Geo& g, int nsp, int k, int64_t (&u)[3], int64_t (&e)[3]) {
  int par[3];
  map_parity(nsp, k, par);
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) { u[a] = e[a] = 1; continue; }
    u[a] = par[a] ? g.Lc[a] : g.L[a];
    e[a] = par[a] ? g.Lc[a] : g.E[a];
  }
}

// Per-map extents, precomputed on the host: untrimmed (prediction) u and trimmed (coded) e.
struct MapExt {
  int32_t u[7][3], e[7][3];
  int32_t par[7][3];
  int32_t mn[3];  // the smallest trimmed extent per axis over the lowres and the maps
};

static MapExt map_exts(const Geo& g, int nsp) {
  MapExt m{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    int par[3];
    map_parity(nsp, k, par);
    for (int a = 0; a < 3; ++a) {
      m.par[k][a] = par[a];
      if (a < 3 - nsp) { m.u[k][a] = m.e[k][a] = 1; continue; }
      m.u[k][a] = (int32_t)(par[a] ? g.Lc[a] : g.L[a]);
      m.e[k][a] = (int32_t)(par[a] ? g.Lc[a] : g.E[a]);
    }
  }
  for (int a = 0; a < 3; ++a) {
    m.mn[a] = a < 3 - nsp ? 1 : (int32_t)g.E[a];
    for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) m.mn[a] = std::min(m.mn[a], m.e[k][a]);
  }
  return m;
}

// 32-bit index versions (every array below 2^31 elements), C == 1: one output block per thread,
// x fastest, the 2^d highres block addressed from one base.
template <typename T, int CODER, bool DEC, int NM, typename P = T>
__global__ void __launch_bounds__(kThreads) code_preds_kernel32(const T* __restrict__ src, CMapPtrs maps_in,
                                                              MapPtrs maps_out, CMapPtrs preds, T* __restrict__ dst,
                                                              MapExt me, int32_t n0, int32_t n1, int32_t n2,
                                                              int32_t E0, int32_t E1, int32_t E2, int32_t total) {
  using TO = typename coder_out<CODER>::type;
  for (int32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    uint32_t q = (uint32_t)t;
    const int32_t ox = q % (uint32_t)E2; q /= (uint32_t)E2;
    const int32_t oy = q % (uint32_t)E1; q /= (uint32_t)E1;
    const int32_t oz = q % (uint32_t)E0;
    const int32_t b = q / (uint32_t)E0;
    const int32_t hbase = ((b * n0 + 2 * oz) * n1 + 2 * oy) * n2 + 2 * ox;
    if constexpr (DEC) dst[hbase] = src[t];
    else dst[t] = src[hbase];
#pragma unroll
    for (int k = 0; k < NM; ++k) {
      const int32_t* e = me.e[k];
      if (oz >= e[0] || oy >= e[1] || ox >= e[2]) continue;
      const int32_t* u = me.u[k];
      const int32_t* par = me.par[k];
      const int32_t hidx = hbase + (par[0] * n1 + par[1]) * n2 + par[2];
      const P pred = ((const P*)preds.p[k])[((b * u[0] + oz) * u[1] + oy) * u[2] + ox];
      const int32_t midx = ((b * e[0] + oz) * e[1] + oy) * e[2] + ox;
      if constexpr (DEC) {
        const TO enc = ((const TO*)maps_in.p[k])[midx];
        dst[hidx] = (T)code_decode<CODER>(to_i32(pred), to_i32(enc));
      } else {
        ((TO*)maps_out.p[k])[midx] = code_encode<CODER>(to_i32(pred), to_i32(src[hidx]));
      }
    }
  }
}

// Row form of the coder pass (C == 1, 32-bit sizes): item = V = 16 / sizeof(T) consecutive
// outputs x0 .. x0+V-1 of output row (oz, oy).  For each highres row parity (pz, py) the 2V
// highres samples are two 16-byte accesses whose even / odd elements are the classes (pz, py, 0)
// and (pz, py, 1) -- the lowres or a map -- and each class's prediction, residual / decoded row
// is one 16-byte access (unaligned: rows of odd length).  Partial chunks go per element.
__host__ __device__ constexpr int class_index(int nsp, int pz, int py, int px) {  // map k, -1 = lowres
  return (pz == 0 && py == 0 && px == 0) ? -1
         : nsp == 3 ? (pz ? (py ? (px ? 3 : 0) : (px ? 1 : 4)) : (py ? (px ? 2 : 5) : 6))
                    : (py ? (px ? 2 : 0) : 1);
}

// One item's prediction row: V = 16 / sizeof(T) values of the prediction dtype P (the sample
// dtype: one 16-byte access; float32: sizeof(P) / sizeof(T) of them), as int32 the way the
// reference's coder reads its operand (jnp.int32: floats truncate, saturating)
template <typename T, typename P>
__device__ __forceinline__ void load_pred_row(const P* p, int32_t nv, int32_t (&out)[Vec16<T>::V]) {
  constexpr int V = Vec16<T>::V, VP = Vec16<P>::V;
  static_assert(V % VP == 0, "whole 16-byte prediction chunks");
  if (nv == V) {
#pragma unroll
    for (int c = 0; c < V / VP; ++c) {
      Vec16<P> v;
      v.load(p + c * VP);
#pragma unroll
      for (int i = 0; i < VP; ++i) out[c * VP + i] = to_i32(v.e[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < V; ++i) out[i] = i < nv ? to_i32(p[i]) : 0;
  }
}

template <typename T, int CODER, bool DEC, int NSP, typename P = T>
__global__ void __launch_bounds__(kThreads) rows_code_preds_kernel(const T* __restrict__ src, CMapPtrs maps_in,
                                                                 MapPtrs maps_out, CMapPtrs preds, T* __restrict__ dst,
                                                                 MapExt me, int32_t n0, int32_t n1, int32_t n2,
                                                                 int32_t E0, int32_t E1, int32_t E2, int32_t nch,
                                                                 int32_t items) {
  using TO = typename coder_out<CODER>::type;
  static_assert(sizeof(TO) == sizeof(T), "same-width coder");
  constexpr int V = Vec16<T>::V;
  constexpr int NPZ = NSP == 3 ? 2 : 1, NK = NSP == 3 ? 7 : 3, VP = Vec16<P>::V;
  for (int32_t t = blockIdx.x * kThreads + threadIdx.x; t < items; t += gridDim.x * kThreads) {
    const RowItem q = row_item((uint32_t)t, E0, E1, nch);
    const int32_t oz = q.z, oy = q.y, x0 = q.j * V;
    // interior item (every class row full and inside, the usual case): all loads of the item
    // (2 x 2^(d-1) highres vectors, every class's prediction row and, decoding, its coded row)
    // issued before any compute -- one memory latency per item instead of one per class row.
    // Measured per call at 512 C3 tiles, the three forms alternating on one box
    // (profiles/round3/ab_callback_coder_r3s20.log): sample-dtype predictions, encode 249-250 ->
    // 239-243 us; float32 predictions, decode 382-387 -> 376-382 us.  The other two directions are
    // slower this way (u16 decode 251 -> 262 us: 81 VGPRs, 6 waves per SIMD instead of 8; float32
    // encode 373 -> 379 us), so they keep the per-class-row path below
    constexpr bool kFast = DEC ? sizeof(P) > sizeof(T) : sizeof(P) == sizeof(T);
    if (kFast && oz < me.mn[0] && oy < me.mn[1] && x0 + V <= me.mn[2] && 2 * x0 + 2 * V <= n2) {
      Vec16<P> pv[NK][V / VP];
#pragma unroll
      for (int k = 0; k < NK; ++k) {
        const P* pp = (const P*)preds.p[k] + ((q.b * me.u[k][0] + oz) * me.u[k][1] + oy) * me.u[k][2] + x0;
#pragma unroll
        for (int c = 0; c < V / VP; ++c) pv[k][c].load(pp + c * VP);
      }
      auto cls_off = [&](int k) { return ((q.b * me.e[k][0] + oz) * me.e[k][1] + oy) * me.e[k][2] + x0; };
      const int32_t lo_off = ((q.b * E0 + oz) * E1 + oy) * E2 + x0;
      if constexpr (!DEC) {
        Vec16<T> h[NPZ][2][2];
#pragma unroll
        for (int pz = 0; pz < NPZ; ++pz)
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            const int32_t hoff = ((q.b * n0 + 2 * oz + pz) * n1 + 2 * oy + py) * n2 + 2 * x0;
            h[pz][py][0].load(src + hoff);
            h[pz][py][1].load(src + hoff + V);
          }
#pragma unroll
        for (int pz = 0; pz < NPZ; ++pz)
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            Vec16<T> ev, od;
#pragma unroll
            for (int i = 0; i < V / 2; ++i) {
              ev.e[i] = h[pz][py][0].e[2 * i]; od.e[i] = h[pz][py][0].e[2 * i + 1];
              ev.e[V / 2 + i] = h[pz][py][1].e[2 * i]; od.e[V / 2 + i] = h[pz][py][1].e[2 * i + 1];
            }
            const int k0 = class_index(NSP, pz, py, 0), k1 = class_index(NSP, pz, py, 1);
            auto code_row = [&](int k, const Vec16<T>& gt) {
              Vec16<T> res;
#pragma unroll
              for (int i = 0; i < V; ++i) res.e[i] = (T)code_encode<CODER>(to_i32(pv[k][i / VP].e[i % VP]), to_i32(gt.e[i]));
              res.store((T*)maps_out.p[k] + cls_off(k));
            };
            if (k0 < 0) ev.store(dst + lo_off);
            else code_row(k0, ev);
            code_row(k1, od);
          }
      } else {
        Vec16<T> lov, en[NK];
        lov.load(src + lo_off);
#pragma unroll
        for (int k = 0; k < NK; ++k) en[k].load((const T*)maps_in.p[k] + cls_off(k));
#pragma unroll
        for (int pz = 0; pz < NPZ; ++pz)
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            const int k0 = class_index(NSP, pz, py, 0), k1 = class_index(NSP, pz, py, 1);
            const int k0c = k0 < 0 ? 0 : k0;
            Vec16<T> ev, od, a, b2;
#pragma unroll
            for (int i = 0; i < V; ++i) {
              ev.e[i] = k0 < 0 ? lov.e[i]
                               : (T)code_decode<CODER>(to_i32(pv[k0c][i / VP].e[i % VP]), to_i32((TO)en[k0c].e[i]));
              od.e[i] = (T)code_decode<CODER>(to_i32(pv[k1][i / VP].e[i % VP]), to_i32((TO)en[k1].e[i]));
            }
#pragma unroll
            for (int i = 0; i < V / 2; ++i) {
              a.e[2 * i] = ev.e[i]; a.e[2 * i + 1] = od.e[i];
              b2.e[2 * i] = ev.e[V / 2 + i]; b2.e[2 * i + 1] = od.e[V / 2 + i];
            }
            const int32_t hoff = ((q.b * n0 + 2 * oz + pz) * n1 + 2 * oy + py) * n2 + 2 * x0;
            a.store(dst + hoff);
            b2.store(dst + hoff + V);
          }
      }
      continue;
    }
    // the sample-dtype decode's interior items: the loads of one highres plane parity (up to 4
    // class rows and their prediction rows) issued together -- twice the loads in flight of the
    // per-class-row path at its register budget (the all-loads-first form needs 81 VGPRs)
    if constexpr (DEC && std::is_same<P, T>::value) {
      if (oz < me.mn[0] && oy < me.mn[1] && x0 + V <= me.mn[2] && 2 * x0 + 2 * V <= n2) {
        auto cls_off = [&](int k) { return ((q.b * me.e[k][0] + oz) * me.e[k][1] + oy) * me.e[k][2] + x0; };
        auto pred_off = [&](int k) { return ((q.b * me.u[k][0] + oz) * me.u[k][1] + oy) * me.u[k][2] + x0; };
        const int32_t lo_off = ((q.b * E0 + oz) * E1 + oy) * E2 + x0;
#pragma unroll
        for (int pz = 0; pz < NPZ; ++pz) {
          Vec16<T> en[2][2], pr[2][2];
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            const int k0 = class_index(NSP, pz, py, 0), k1 = class_index(NSP, pz, py, 1);
            if (k0 < 0) {
              en[py][0].load(src + lo_off);
            } else {
              en[py][0].load((const T*)maps_in.p[k0] + cls_off(k0));
              pr[py][0].load((const T*)preds.p[k0] + pred_off(k0));
            }
            en[py][1].load((const T*)maps_in.p[k1] + cls_off(k1));
            pr[py][1].load((const T*)preds.p[k1] + pred_off(k1));
          }
#pragma unroll
          for (int py = 0; py < 2; ++py) {
            const int k0 = class_index(NSP, pz, py, 0);
            Vec16<T> a, b2;
#pragma unroll
            for (int i = 0; i < V / 2; ++i) {
              auto dec0 = [&](int e) {
                return k0 < 0 ? en[py][0].e[e]
                              : (T)code_decode<CODER>(to_i32(pr[py][0].e[e]), to_i32((TO)en[py][0].e[e]));
              };
              auto dec1 = [&](int e) { return (T)code_decode<CODER>(to_i32(pr[py][1].e[e]), to_i32((TO)en[py][1].e[e])); };
              a.e[2 * i] = dec0(i); a.e[2 * i + 1] = dec1(i);
              b2.e[2 * i] = dec0(V / 2 + i); b2.e[2 * i + 1] = dec1(V / 2 + i);
            }
            const int32_t hoff = ((q.b * n0 + 2 * oz + pz) * n1 + 2 * oy + py) * n2 + 2 * x0;
            a.store(dst + hoff);
            b2.store(dst + hoff + V);
          }
        }
        continue;
      }
    }
#pragma unroll
    for (int pz = 0; pz < (NSP == 3 ? 2 : 1); ++pz)
#pragma unroll
      for (int py = 0; py < 2; ++py) {
        const int k0 = class_index(NSP, pz, py, 0), k1 = class_index(NSP, pz, py, 1);
        const int32_t ez = NSP == 3 ? (pz ? me.e[k1][0] : E0) : 1, ey = py ? me.e[k1][1] : E1;
        if (oz >= ez || oy >= ey) continue;
        const int32_t e2_0 = k0 < 0 ? E2 : me.e[k0][2], e2_1 = me.e[k1][2];
        const int32_t nx0 = min(V, e2_0 - x0), nx1 = min(V, e2_1 - x0);  // valid even / odd outputs
        const int32_t hoff = ((q.b * n0 + 2 * oz + pz) * n1 + 2 * oy + py) * n2 + 2 * x0;
        // class rows: (lowres | map k0) and map k1, their prediction rows
        auto cls_off = [&](int k) { return ((q.b * me.e[k][0] + oz) * me.e[k][1] + oy) * me.e[k][2] + x0; };
        auto pred_off = [&](int k) { return ((q.b * me.u[k][0] + oz) * me.u[k][1] + oy) * me.u[k][2] + x0; };
        auto load_row = [&](const T* p, int32_t nv, Vec16<T>& v) {
          if (nv == V) {
            v.load(p);
          } else {
#pragma unroll
            for (int i = 0; i < V; ++i) v.e[i] = i < nv ? p[i] : T(0);
          }
        };
        auto store_row = [&](T* p, int32_t nv, const Vec16<T>& v) {
          if (nv == V) {
            v.store(p);
          } else {
#pragma unroll
            for (int i = 0; i < V; ++i)
              if (i < nv) p[i] = v.e[i];
          }
        };
        const int32_t lo_off = ((q.b * E0 + oz) * E1 + oy) * E2 + x0;
        if constexpr (!DEC) {
          Vec16<T> ev, od;
          if (2 * x0 + 2 * V <= n2) {
            Vec16<T> a, b2;
            a.load(src + hoff);
            b2.load(src + hoff + V);
#pragma unroll
            for (int i = 0; i < V / 2; ++i) {
              ev.e[i] = a.e[2 * i]; od.e[i] = a.e[2 * i + 1];
              ev.e[V / 2 + i] = b2.e[2 * i]; od.e[V / 2 + i] = b2.e[2 * i + 1];
            }
          } else {
#pragma unroll
            for (int i = 0; i < V; ++i) {
              ev.e[i] = 2 * (x0 + i) < n2 ? src[hoff + 2 * i] : T(0);
              od.e[i] = 2 * (x0 + i) + 1 < n2 ? src[hoff + 2 * i + 1] : T(0);
            }
          }
          auto code_row = [&](int k, int32_t nv, const Vec16<T>& gt) {
            Vec16<T> res;
            int32_t pr[V];
            load_pred_row<T, P>((const P*)preds.p[k] + pred_off(k), nv, pr);
#pragma unroll
            for (int i = 0; i < V; ++i) res.e[i] = (T)code_encode<CODER>(pr[i], to_i32(gt.e[i]));
            store_row((T*)maps_out.p[k] + cls_off(k), nv, res);
          };
          if (nx0 > 0) {
            if (k0 < 0) store_row(dst + lo_off, nx0, ev);
            else code_row(k0, nx0, ev);
          }
          if (nx1 > 0) code_row(k1, nx1, od);
        } else {
          auto decode_row = [&](int k, int32_t nv, Vec16<T>& outv) {
            Vec16<T> en;
            int32_t pr[V];
            load_pred_row<T, P>((const P*)preds.p[k] + pred_off(k), nv, pr);
            load_row((const T*)maps_in.p[k] + cls_off(k), nv, en);
#pragma unroll
            for (int i = 0; i < V; ++i) outv.e[i] = (T)code_decode<CODER>(pr[i], to_i32((TO)en.e[i]));
          };
          Vec16<T> ev, od;
          if (nx0 > 0) {
            if (k0 < 0) load_row(src + lo_off, nx0, ev);
            else decode_row(k0, nx0, ev);
          }
          if (nx1 > 0) decode_row(k1, nx1, od);
          if (nx0 == V && nx1 == V && 2 * x0 + 2 * V <= n2) {
            Vec16<T> a, b2;
#pragma unroll
            for (int i = 0; i < V / 2; ++i) {
              a.e[2 * i] = ev.e[i]; a.e[2 * i + 1] = od.e[i];
              b2.e[2 * i] = ev.e[V / 2 + i]; b2.e[2 * i + 1] = od.e[V / 2 + i];
            }
            a.store(dst + hoff);
            b2.store(dst + hoff + V);
          } else {
#pragma unroll
            for (int i = 0; i < V; ++i) {
              if (i < nx0) dst[hoff + 2 * i] = ev.e[i];
              if (i < nx1) dst[hoff + 2 * i + 1] = od.e[i];
            }
          }
        }
      }
  }
}

template <typename T, int CODER, typename P = T>
__global__ void __launch_bounds__(kThreads) encode_preds_kernel(const T* __restrict__ hi, Geo g, int nsp, int64_t C,
                                                              CMapPtrs preds, T* __restrict__ lowres, MapPtrs maps,
                                                              int64_t total) {
  using TO = typename coder_out<CODER>::type;
  const int nmaps = nsp == 3 ? 7 : 3;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t b, oz, oy, ox, c;
    unflat5(t, g.E[0], g.E[1], g.E[2], C, b, oz, oy, ox, c);
    auto hv = [&](int pz, int py, int px) -> T {
      return hi[(((b * g.n[0] + 2 * oz + pz) * g.n[1] + 2 * oy + py) * g.n[2] + 2 * ox + px) * C + c];
    };
    lowres[t] = hv(0, 0, 0);
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      int64_t u[3], e[3];
      map_ext(g, nsp, k, u, e);
      if (oz >= e[0] || oy >= e[1] || ox >= e[2]) continue;
      const P pred = ((const P*)preds.p[k])[(((b * u[0] + oz) * u[1] + oy) * u[2] + ox) * C + c];
      ((TO*)maps.p[k])[(((b * e[0] + oz) * e[1] + oy) * e[2] + ox) * C + c] =
          code_encode<CODER>(to_i32(pred), to_i32(hv(par[0], par[1], par[2])));
    }
  }
}

template <typename T, int CODER, typename P = T>
__global__ void __launch_bounds__(kThreads) decode_preds_kernel(const T* __restrict__ lowres, CMapPtrs maps, Geo g,
                                                              int nsp, int64_t C, CMapPtrs preds, T* __restrict__ hi,
                                                              int64_t total) {
  using TO = typename coder_out<CODER>::type;
  const int nmaps = nsp == 3 ? 7 : 3;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t b, oz, oy, ox, c;
    unflat5(t, g.E[0], g.E[1], g.E[2], C, b, oz, oy, ox, c);
    auto hout = [&](int pz, int py, int px) -> T& {
      return hi[(((b * g.n[0] + 2 * oz + pz) * g.n[1] + 2 * oy + py) * g.n[2] + 2 * ox + px) * C + c];
    };
    hout(0, 0, 0) = lowres[t];
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      int64_t u[3], e[3];
      map_ext(g, nsp, k, u, e);
      if (oz >= e[0] || oy >= e[1] || ox >= e[2]) continue;
      const P pred = ((const P*)preds.p[k])[(((b * u[0] + oz) * u[1] + oy) * u[2] + ox) * C + c];
      const TO enc = ((const TO*)maps.p[k])[(((b * e[0] + oz) * e[1] + oy) * e[2] + ox) * C + c];
      hout(par[0], par[1], par[2]) = (T)code_decode<CODER>(to_i32(pred), to_i32(enc));
    }
  }
}

template <typename F>
static int dispatch_coder(int dtype, int coder, F&& f) {  // the built-in coder of each sample dtype
  if (dtype == KMP_U8 && coder == KMP_CODER_U8) return f(uint8_t{}, std::integral_constant<int, KMP_CODER_U8>{});
  if (dtype == KMP_U16 && coder == KMP_CODER_U16) return f(uint16_t{}, std::integral_constant<int, KMP_CODER_U16>{});
  if (dtype == KMP_I32 && coder == KMP_CODER_RAW) return f(int32_t{}, std::integral_constant<int, KMP_CODER_RAW>{});
  if (dtype == KMP_U32 && coder == KMP_CODER_U32) return f(uint32_t{}, std::integral_constant<int, KMP_CODER_U32>{});
  return fail(KMP_ERR_UNSUPPORTED, "callback coder kernels support (uint8, U8), (uint16, U16), (int32, RAW), "
                                   "(uint32, U32); got dtype " + std::to_string(dtype) + " coder " + std::to_string(coder));
}

// the prediction maps' dtype: the sample dtype itself, or float32 (a network's output)
template <typename T, typename F>
static int dispatch_pred(int dtype, int pred_dtype, F&& f) {
  if (pred_dtype == dtype) return f(T{});
  if (pred_dtype == KMP_F32) return f(float{});
  return fail(KMP_ERR_UNSUPPORTED, "prediction maps must have the sample dtype or float32; got dtype " +
                                       std::to_string(pred_dtype));
}

static int window_launch(int nsp, int dtype, const void* src, int mult, const int64_t* S, int64_t B, int64_t C,
                         const Geo& g, int p, void* out, hipStream_t stream) {
  int64_t W[3], total = B * C;
  for (int a = 0; a < 3; ++a) {
    W[a] = a < 3 - nsp ? 1 : g.L[a] + 2 * p;
    total *= W[a];
  }
  if (total == 0) return KMP_OK;
  return dispatch_any_dtype(dtype, [&](auto tag) {
    using T = decltype(tag);
    const int64_t src_n = B * S[0] * S[1] * S[2] * C;
    if (C == 1 && total < ((int64_t)1 << 30) && src_n < ((int64_t)1 << 30) && !opt(OPT_DISABLE_ROWS, 0)) {
      const int64_t nch = ceil_div(W[2], Vec16<T>::V), items = B * W[0] * W[1] * nch;
      rows_window_kernel<T><<<grid_for(items), kThreads, 0, stream>>>(
          (const T*)src, (int32_t)S[0], (int32_t)S[1], (int32_t)S[2], g, mult, nsp == 3 ? p : 0, p, (int32_t)W[0],
          (int32_t)W[1], (int32_t)W[2], (T*)out, (int32_t)nch, (int32_t)items);
      return check_launch("window");
    }
    window_kernel<T><<<grid_for(total), kThreads, 0, stream>>>((const T*)src, B, g, S[0], S[1], S[2], mult, nsp, p, C,
                                                               W[0], W[1], W[2], (T*)out, total);
    return check_launch("window");
  });
}

}  // namespace cb
}  // namespace kmp

using namespace kmp;

extern "C" {

int kmp_window_from_highres(int32_t nsp, int32_t dtype, const void* highres, int64_t B, const int64_t shape[3],
                            int64_t C, int32_t padding, void* window_out, kmp_stream_t stream) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(highres && window_out && shape && padding >= 0 && B >= 0 && C >= 1, "bad argument");
  for (int a = 0; a < nsp; ++a) KMP_REQUIRE(shape[a] >= 2, "spatial dims must be >= 2");
  const Geo g = make_geo_from_highres(nsp, shape);
  int64_t S[3];
  for (int a = 0; a < 3; ++a) S[a] = g.n[a];
  return cb::window_launch(nsp, dtype, highres, 2, S, B, C, g, padding, window_out, (hipStream_t)stream);
}

int kmp_window_from_lowres(int32_t nsp, int32_t dtype, const void* lowres, int64_t B, const int64_t shape[3],
                           int64_t C, const int32_t dims[3], int32_t padding, void* window_out, kmp_stream_t stream) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(lowres && window_out && shape && dims && padding >= 0 && B >= 0 && C >= 1, "bad argument");
  for (int a = 0; a < nsp; ++a) {
    KMP_REQUIRE(dims[a] == 0 || dims[a] == 1, "dims must be 0 or 1");
    KMP_REQUIRE(shape[a] >= 1 && shape[a] + dims[a] >= 2, "lowres too small");
  }
  const Geo g = make_geo_from_lowres(nsp, shape, dims);
  int64_t S[3];
  for (int a = 0; a < 3; ++a) S[a] = g.E[a];
  return cb::window_launch(nsp, dtype, lowres, 1, S, B, C, g, padding, window_out, (hipStream_t)stream);
}

int kmp_encode_with_predictions(int32_t nsp, int32_t dtype, int32_t coder, const void* highres, int64_t B,
                                const int64_t shape[3], int64_t C, const void* const preds[7], void* lowres_out,
                                void* const maps_out[7], kmp_stream_t stream) {
  return kmp_encode_with_predictions_typed(nsp, dtype, coder, dtype, highres, B, shape, C, preds, lowres_out, maps_out,
                                           stream);
}

int kmp_encode_with_predictions_typed(int32_t nsp, int32_t dtype, int32_t coder, int32_t pred_dtype,
                                      const void* highres, int64_t B, const int64_t shape[3], int64_t C,
                                      const void* const preds[7], void* lowres_out, void* const maps_out[7],
                                      kmp_stream_t stream) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(highres && shape && preds && lowres_out && maps_out && B >= 0 && C >= 1, "bad argument");
  for (int a = 0; a < nsp; ++a) KMP_REQUIRE(shape[a] >= 2, "spatial dims must be >= 2");
  const Geo g = make_geo_from_highres(nsp, shape);
  CMapPtrs pp{};
  MapPtrs mp{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(preds[k] && maps_out[k], "null map pointer");
    pp.p[k] = preds[k];
    mp.p[k] = maps_out[k];
  }
  const int64_t total = B * g.E[0] * g.E[1] * g.E[2] * C;
  if (total == 0) return KMP_OK;
  const bool small = C == 1 && B * g.n[0] * g.n[1] * g.n[2] < ((int64_t)1 << 31) &&
                     B * g.L[0] * g.L[1] * g.L[2] < ((int64_t)1 << 31);
  return cb::dispatch_coder(dtype, coder, [&](auto tag, auto coder_c) {
   using T = decltype(tag);
   constexpr int CODER = decltype(coder_c)::value;
   return cb::dispatch_pred<T>(dtype, pred_dtype, [&](auto ptag) {
    using P = decltype(ptag);
    if (small && !opt(OPT_DISABLE_ROWS, 0)) {
      const cb::MapExt me = cb::map_exts(g, nsp);
      const int64_t nch = ceil_div(g.E[2], Vec16<T>::V), items = B * g.E[0] * g.E[1] * nch;
      auto k = nsp == 3 ? cb::rows_code_preds_kernel<T, CODER, false, 3, P> : cb::rows_code_preds_kernel<T, CODER, false, 2, P>;
      k<<<cb::grid_for(items), cb::kThreads, 0, (hipStream_t)stream>>>(
          (const T*)highres, CMapPtrs{}, mp, pp, (T*)lowres_out, me, (int32_t)g.n[0], (int32_t)g.n[1],
          (int32_t)g.n[2], (int32_t)g.E[0], (int32_t)g.E[1], (int32_t)g.E[2], (int32_t)nch, (int32_t)items);
    } else if (small) {
      const cb::MapExt me = cb::map_exts(g, nsp);
      auto k = nsp == 3 ? cb::code_preds_kernel32<T, CODER, false, 7, P> : cb::code_preds_kernel32<T, CODER, false, 3, P>;
      k<<<cb::grid_for(total), cb::kThreads, 0, (hipStream_t)stream>>>(
          (const T*)highres, CMapPtrs{}, mp, pp, (T*)lowres_out, me, (int32_t)g.n[0], (int32_t)g.n[1],
          (int32_t)g.n[2], (int32_t)g.E[0], (int32_t)g.E[1], (int32_t)g.E[2], (int32_t)total);
    } else {
      cb::encode_preds_kernel<T, CODER, P><<<cb::grid_for(total), cb::kThreads, 0, (hipStream_t)stream>>>(
          (const T*)highres, g, nsp, C, pp, (T*)lowres_out, mp, total);
    }
    return check_launch("encode_with_predictions");
   });
  });
}

int kmp_decode_with_predictions(int32_t nsp, int32_t dtype, int32_t coder, const void* lowres,
                                const void* const maps[7], int64_t B, const int64_t shape[3], int64_t C,
                                const int32_t dims[3], const void* const preds[7], void* highres_out,
                                kmp_stream_t stream) {
  return kmp_decode_with_predictions_typed(nsp, dtype, coder, dtype, lowres, maps, B, shape, C, dims, preds,
                                           highres_out, stream);
}

int kmp_decode_with_predictions_typed(int32_t nsp, int32_t dtype, int32_t coder, int32_t pred_dtype,
                                      const void* lowres, const void* const maps[7], int64_t B, const int64_t shape[3],
                                      int64_t C, const int32_t dims[3], const void* const preds[7], void* highres_out,
                                      kmp_stream_t stream) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(lowres && maps && shape && dims && preds && highres_out && B >= 0 && C >= 1, "bad argument");
  for (int a = 0; a < nsp; ++a) {
    KMP_REQUIRE(dims[a] == 0 || dims[a] == 1, "dims must be 0 or 1");
    KMP_REQUIRE(shape[a] >= 1 && shape[a] + dims[a] >= 2, "lowres too small");
  }
  const Geo g = make_geo_from_lowres(nsp, shape, dims);
  CMapPtrs pp{}, mp{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(preds[k] && maps[k], "null map pointer");
    pp.p[k] = preds[k];
    mp.p[k] = maps[k];
  }
  const int64_t total = B * g.E[0] * g.E[1] * g.E[2] * C;
  if (total == 0) return KMP_OK;
  const bool small = C == 1 && B * g.n[0] * g.n[1] * g.n[2] < ((int64_t)1 << 31) &&
                     B * g.L[0] * g.L[1] * g.L[2] < ((int64_t)1 << 31);
  return cb::dispatch_coder(dtype, coder, [&](auto tag, auto coder_c) {
   using T = decltype(tag);
   constexpr int CODER = decltype(coder_c)::value;
   return cb::dispatch_pred<T>(dtype, pred_dtype, [&](auto ptag) {
    using P = decltype(ptag);
    if (small && !opt(OPT_DISABLE_ROWS, 0)) {
      const cb::MapExt me = cb::map_exts(g, nsp);
      const int64_t nch = ceil_div(g.E[2], Vec16<T>::V), items = B * g.E[0] * g.E[1] * nch;
      auto k = nsp == 3 ? cb::rows_code_preds_kernel<T, CODER, true, 3, P> : cb::rows_code_preds_kernel<T, CODER, true, 2, P>;
      k<<<cb::grid_for(items), cb::kThreads, 0, (hipStream_t)stream>>>(
          (const T*)lowres, mp, MapPtrs{}, pp, (T*)highres_out, me, (int32_t)g.n[0], (int32_t)g.n[1],
          (int32_t)g.n[2], (int32_t)g.E[0], (int32_t)g.E[1], (int32_t)g.E[2], (int32_t)nch, (int32_t)items);
    } else if (small) {
      const cb::MapExt me = cb::map_exts(g, nsp);
      auto k = nsp == 3 ? cb::code_preds_kernel32<T, CODER, true, 7, P> : cb::code_preds_kernel32<T, CODER, true, 3, P>;
      k<<<cb::grid_for(total), cb::kThreads, 0, (hipStream_t)stream>>>(
          (const T*)lowres, mp, MapPtrs{}, pp, (T*)highres_out, me, (int32_t)g.n[0], (int32_t)g.n[1],
          (int32_t)g.n[2], (int32_t)g.E[0], (int32_t)g.E[1], (int32_t)g.E[2], (int32_t)total);
    } else {
      cb::decode_preds_kernel<T, CODER, P><<<cb::grid_for(total), cb::kThreads, 0, (hipStream_t)stream>>>(
          (const T*)lowres, mp, g, nsp, C, pp, (T*)highres_out, total);
    }
    return check_launch("decode_with_predictions");
   });
  });
}

}  // extern "C"
