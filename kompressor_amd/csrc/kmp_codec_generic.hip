// kmp_codec_generic.hip -- the fused encode/decode for ANY shape, channel count, padding and
// integer dtype: two launches per direction.
//
//   1. predictor apply: one value per cell (MEAN) or K per cell (LINEAR) into a workspace
//      [B, Lc..., K, C] -- the reference's features_from_lowres + mean/astype
//      (tests/volume/test_encode_decode.py:46-51) without materialising the features;
//   2. residual pass: per output block position o, read the 2^d highres block at 2o, aggregate
//      the cell predictions exactly as maps_from_predictions does (kmp_aggregate.h), apply the
//      coder and write lowres + every map in its trimmed shape (encode), or the inverse
//      (decode: interleave into highres, highres_from_lowres_and_maps + trim).
//
// Lowres node j of the padded volume along an axis is source sample 2*sym(j, E) (encode: even
// reflect pad volume/utils.py:226-237) or sym(j, E) of the trimmed lowres (decode: symmetric
// pad_lowres volume/utils.py:240-244); the neighbourhood padding adds sym(., L)
// (pad_neighborhood volume/utils.py:213-218).  Costs ~1.25x the HBM bytes of the one-pass
// fast kernels (kmp_codec_fast3d.hip); used whenever those are not eligible.
#include "kmp_codec.h"

namespace kmp {

constexpr int kGThreads = 256;

static inline unsigned ggrid(int64_t n) {
  int64_t g = ceil_div(n, kGThreads);
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

struct Src {
  int64_t S[3];  // source extents (highres n for encode, trimmed lowres E for decode)
  int32_t mult;  // 2 (encode: lowres node j <- highres 2j) or 1 (decode)
};

template <typename T>
__device__ __forceinline__ T lowres_node(const T* __restrict__ src, const Src& s, const Geo& g, int64_t b, int64_t c,
                                         int64_t C, int64_t jz, int64_t jy, int64_t jx) {
  const int64_t z = s.mult * sym_index(sym_index(jz, g.L[0]), g.E[0]);
  const int64_t y = s.mult * sym_index(sym_index(jy, g.L[1]), g.E[1]);
  const int64_t x = s.mult * sym_index(sym_index(jx, g.L[2]), g.E[2]);
  return src[(((b * s.S[0] + z) * s.S[1] + y) * s.S[2] + x) * C + c];
}

// Cell mean, float32 sum in feature order (z-major, y, x) / N, XLA cast (the reference test
// predictor).  Exact (order-independent) for uint8 with p <= 4 and uint16 with p <= 2.
struct Frame {
  int64_t begin[3], ext[3];
};

// ``cf`` is the box of cells to compute (a region launch needs cells [begin-1, end) only);
// results land at their global position in ``cells`` [B, Lc..., C].
template <typename T>
__global__ void __launch_bounds__(kGThreads) cell_mean_kernel(const T* __restrict__ src, Src s, Geo g, int nsp,
                                                            int64_t B, int64_t C, int p, Frame cf,
                                                            T* __restrict__ cells, int64_t total) {
  const int k = 2 * p + 2;
  const int kz = nsp == 3 ? k : 1;
  const float inv_n = (float)(kz * k * k);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t b, cz, cy, cx, c;
    unflat5(t, cf.ext[0], cf.ext[1], cf.ext[2], C, b, cz, cy, cx, c);
    cz += cf.begin[0];
    cy += cf.begin[1];
    cx += cf.begin[2];
    const int pz = nsp == 3 ? p : 0;
    float sum = 0.0f;
    for (int dz = 0; dz < kz; ++dz)
      for (int dy = 0; dy < k; ++dy)
        for (int dx = 0; dx < k; ++dx)
          sum += (float)lowres_node(src, s, g, b, c, C, cz - pz + dz, cy - p + dy, cx - p + dx);
    cells[(((b * g.Lc[0] + cz) * g.Lc[1] + cy) * g.Lc[2] + cx) * C + c] = cast_f32<T>(sum / inv_n);
  }
}

template <typename T, int CODER, bool PERCH>
__global__ void __launch_bounds__(kGThreads) encode_generic_kernel(const T* __restrict__ hi, Geo g, int nsp, int64_t B,
                                                                 int64_t C, const T* __restrict__ cells, int K,
                                                                 T* __restrict__ lowres, MapPtrs maps, Frame f,
                                                                 int64_t total) {
  using TO = typename coder_out<CODER>::type;
  const int nmaps = nsp == 3 ? 7 : 3;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t b, oz, oy, ox, c;
    unflat5(t, f.ext[0], f.ext[1], f.ext[2], C, b, oz, oy, ox, c);
    oz += f.begin[0];
    oy += f.begin[1];
    ox += f.begin[2];
    auto hv = [&](int pz, int py, int px) -> T {
      return hi[(((b * g.n[0] + 2 * oz + pz) * g.n[1] + 2 * oy + py) * g.n[2] + 2 * ox + px) * C + c];
    };
    if (oz < g.E[0] && oy < g.E[1] && ox < g.E[2])
      lowres[(((b * g.E[0] + oz) * g.E[1] + oy) * g.E[2] + ox) * C + c] = hv(0, 0, 0);
    auto get = [&](int64_t z, int64_t y, int64_t x, int ch) -> T {
      return cells[((((b * g.Lc[0] + z) * g.Lc[1] + y) * g.Lc[2] + x) * K + (PERCH ? ch : 0)) * C + c];
    };
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      const int64_t e0 = par[0] ? g.Lc[0] : g.E[0], e1 = par[1] ? g.Lc[1] : g.E[1], e2 = par[2] ? g.Lc[2] : g.E[2];
      if (oz >= e0 || oy >= e1 || ox >= e2) continue;
      const T pred = aggregate_map<T>(nsp, k, oz, oy, ox, g.Lc[0], g.Lc[1], g.Lc[2], get);
      const T gt = hv(par[0], par[1], par[2]);
      ((TO*)maps.p[k])[(((b * e0 + oz) * e1 + oy) * e2 + ox) * C + c] = code_encode<CODER>(to_i32(pred), to_i32(gt));
    }
  }
}

template <typename T, int CODER, bool PERCH>
__global__ void __launch_bounds__(kGThreads) decode_generic_kernel(const T* __restrict__ lowres, CMapPtrs maps, Geo g,
                                                                 int nsp, int64_t B, int64_t C,
                                                                 const T* __restrict__ cells, int K,
                                                                 T* __restrict__ hi, Frame f, int64_t total) {
  using TO = typename coder_out<CODER>::type;
  const int nmaps = nsp == 3 ? 7 : 3;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    int64_t b, oz, oy, ox, c;
    unflat5(t, f.ext[0], f.ext[1], f.ext[2], C, b, oz, oy, ox, c);
    oz += f.begin[0];
    oy += f.begin[1];
    ox += f.begin[2];
    auto hout = [&](int pz, int py, int px) -> T& {
      return hi[(((b * g.n[0] + 2 * oz + pz) * g.n[1] + 2 * oy + py) * g.n[2] + 2 * ox + px) * C + c];
    };
    if (oz < g.E[0] && oy < g.E[1] && ox < g.E[2])
      hout(0, 0, 0) = lowres[(((b * g.E[0] + oz) * g.E[1] + oy) * g.E[2] + ox) * C + c];
    auto get = [&](int64_t z, int64_t y, int64_t x, int ch) -> T {
      return cells[((((b * g.Lc[0] + z) * g.Lc[1] + y) * g.Lc[2] + x) * K + (PERCH ? ch : 0)) * C + c];
    };
    for (int k = 0; k < nmaps; ++k) {
      int par[3];
      map_parity(nsp, k, par);
      const int64_t e0 = par[0] ? g.Lc[0] : g.E[0], e1 = par[1] ? g.Lc[1] : g.E[1], e2 = par[2] ? g.Lc[2] : g.E[2];
      if (oz >= e0 || oy >= e1 || ox >= e2) continue;
      const T pred = aggregate_map<T>(nsp, k, oz, oy, ox, g.Lc[0], g.Lc[1], g.Lc[2], get);
      const TO enc = ((const TO*)maps.p[k])[(((b * e0 + oz) * e1 + oy) * e2 + ox) * C + c];
      hout(par[0], par[1], par[2]) = (T)code_decode<CODER>(to_i32(pred), to_i32(enc));
    }
  }
}

// ------------------------------------------------------------------------------------------
// Host side of the generic path
// ------------------------------------------------------------------------------------------
int64_t generic_workspace_bytes(int dtype, int nsp, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred) {
  const bool lin = pred && (pred->kind == KMP_PRED_LINEAR || pred->kind == KMP_PRED_LINEAR_MFMA);
  const int K = lin ? (nsp == 3 ? 19 : 5) : 1;
  int64_t need = B * g.Lc[0] * g.Lc[1] * g.Lc[2] * K * C * dtype_size(dtype);
  if (lin && B > 0) {  // the fused LinearPredictor kernels keep a reordered copy of W [N, K] there
    const int64_t nb = 2 * pred->padding + 2, N = nsp == 3 ? nb * nb * nb : nb * nb;
    int64_t wbytes = N * K * (int64_t)sizeof(float);
    // the matrix-core kernels' B fragments (3 column tiles x 8 chunks x 64 lanes x 16 B) + biases
    // + linear3pm's dummy store slots (64 lanes x 16 B)
    constexpr int64_t kMfmaWs = 3 * 8 * 64 * 16 + 3 * 64 * 4 + 64 * 16;
    if (pred->kind == KMP_PRED_LINEAR_MFMA) wbytes = wbytes > kMfmaWs ? wbytes : kMfmaWs;
    need = need > wbytes ? need : wbytes;
  }
  return need;
}

static Frame make_frame(int nsp, const Geo& g, const kmp_region* region) {
  Frame f{};
  for (int a = 0; a < 3; ++a) {
    int64_t lo = 0, hi = g.E[a];
    if (region && a >= 3 - nsp) {
      lo = region->begin[a] < 0 ? 0 : region->begin[a];
      hi = region->end[a] > g.E[a] ? g.E[a] : region->end[a];
    }
    f.begin[a] = lo;
    f.ext[a] = hi > lo ? hi - lo : 0;
  }
  return f;
}

// Cells a frame of outputs depends on: [begin-1, end) clipped to [0, Lc).
static Frame cell_frame(const Geo& g, const Frame& f) {
  Frame cf{};
  for (int a = 0; a < 3; ++a) {
    int64_t lo = f.begin[a] - 1, hi = f.begin[a] + f.ext[a];
    lo = lo < 0 ? 0 : lo;
    hi = hi > g.Lc[a] ? g.Lc[a] : hi;
    cf.begin[a] = lo;
    cf.ext[a] = (f.ext[a] > 0 && hi > lo) ? hi - lo : 0;
  }
  return cf;
}

template <typename T>
static int run_predictor(const T* src, const Src& s, const Geo& g, int nsp, int64_t B, int64_t C,
                         const kmp_predictor* pred, const Frame& f, T* cells, hipStream_t stream) {
  const Frame cf = cell_frame(g, f);
  const int64_t ncell = B * cf.ext[0] * cf.ext[1] * cf.ext[2] * C;
  if (ncell == 0) return KMP_OK;
  if (pred->kind == KMP_PRED_MEAN) {
    cell_mean_kernel<T><<<ggrid(ncell), kGThreads, 0, stream>>>(src, s, g, nsp, B, C, pred->padding, cf, cells, ncell);
    return check_launch("cell_mean");
  }
  const int64_t cbeg[3] = {cf.begin[0], cf.begin[1], cf.begin[2]}, cext[3] = {cf.ext[0], cf.ext[1], cf.ext[2]};
  return linear_cells<T>(src, s.S, s.mult, g, nsp, B, C, pred, cbeg, cext, cells, stream);
}

template <typename T, int CODER>
static int encode_generic_t(const T* hi, const Geo& g, int nsp, int64_t B, int64_t C, const kmp_predictor* pred,
                            T* lowres, const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  const int64_t need = generic_workspace_bytes(dtype_code<T>(), nsp, g, B, C, pred);
  if ((int64_t)ws_bytes < need || (!ws && need > 0))
    return fail(KMP_ERR_ARG, "encode: workspace too small (" + std::to_string(ws_bytes) + " < " + std::to_string(need) + ")");
  Src s{{g.n[0], g.n[1], g.n[2]}, 2};
  T* cells = (T*)ws;
  Frame f = make_frame(nsp, g, region);
  if (int st = run_predictor<T>(hi, s, g, nsp, B, C, pred, f, cells, stream)) return st;
  const int64_t total = B * f.ext[0] * f.ext[1] * f.ext[2] * C;
  if (total == 0) return KMP_OK;
  if (pred->kind == KMP_PRED_MEAN)
    encode_generic_kernel<T, CODER, false><<<ggrid(total), kGThreads, 0, stream>>>(hi, g, nsp, B, C, cells, 1, lowres,
                                                                                  maps, f, total);
  else
    encode_generic_kernel<T, CODER, true><<<ggrid(total), kGThreads, 0, stream>>>(
        hi, g, nsp, B, C, cells, nsp == 3 ? 19 : 5, lowres, maps, f, total);
  return check_launch("encode_generic");
}

template <typename T, int CODER>
static int decode_generic_t(const T* lowres, const CMapPtrs& maps, const Geo& g, int nsp, int64_t B, int64_t C,
                            const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                            hipStream_t stream) {
  const int64_t need = generic_workspace_bytes(dtype_code<T>(), nsp, g, B, C, pred);
  if ((int64_t)ws_bytes < need || (!ws && need > 0))
    return fail(KMP_ERR_ARG, "decode: workspace too small (" + std::to_string(ws_bytes) + " < " + std::to_string(need) + ")");
  Src s{{g.E[0], g.E[1], g.E[2]}, 1};
  T* cells = (T*)ws;
  Frame f = make_frame(nsp, g, region);
  if (int st = run_predictor<T>(lowres, s, g, nsp, B, C, pred, f, cells, stream)) return st;
  const int64_t total = B * f.ext[0] * f.ext[1] * f.ext[2] * C;
  if (total == 0) return KMP_OK;
  if (pred->kind == KMP_PRED_MEAN)
    decode_generic_kernel<T, CODER, false><<<ggrid(total), kGThreads, 0, stream>>>(lowres, maps, g, nsp, B, C, cells, 1,
                                                                                  hi, f, total);
  else
    decode_generic_kernel<T, CODER, true><<<ggrid(total), kGThreads, 0, stream>>>(
        lowres, maps, g, nsp, B, C, cells, nsp == 3 ? 19 : 5, hi, f, total);
  return check_launch("decode_generic");
}

// Natural coder per dtype: (u8, U8), (u16, U16), (i32, RAW), (u32, U32).
template <typename F>
static int dispatch_natural(int dtype, int coder, F&& f) {
  if (dtype == KMP_U8 && coder == KMP_CODER_U8) return f(uint8_t{}, std::integral_constant<int, KMP_CODER_U8>{});
  if (dtype == KMP_U16 && coder == KMP_CODER_U16) return f(uint16_t{}, std::integral_constant<int, KMP_CODER_U16>{});
  if (dtype == KMP_I32 && coder == KMP_CODER_RAW) return f(int32_t{}, std::integral_constant<int, KMP_CODER_RAW>{});
  if (dtype == KMP_U32 && coder == KMP_CODER_U32) return f(uint32_t{}, std::integral_constant<int, KMP_CODER_U32>{});
  return fail(KMP_ERR_UNSUPPORTED, "fused codec supports (uint8, U8), (uint16, U16), (int32, RAW), (uint32, U32); got dtype " +
                                       std::to_string(dtype) + " coder " + std::to_string(coder));
}

static int check_predictor(const kmp_predictor* pred, int dtype) {
  KMP_REQUIRE(pred, "null predictor");
  KMP_REQUIRE(pred->padding >= 0, "negative padding");
  KMP_REQUIRE(pred->kind == KMP_PRED_MEAN || pred->kind == KMP_PRED_LINEAR || pred->kind == KMP_PRED_LINEAR_MFMA,
              "unknown predictor kind");
  if (pred->kind != KMP_PRED_MEAN) KMP_REQUIRE(pred->weights && pred->bias, "linear predictor needs weights and bias");
  if (pred->kind == KMP_PRED_LINEAR_MFMA)
    KMP_REQUIRE(dtype == KMP_U8 || dtype == KMP_U16, "the matrix-core LinearPredictor takes uint8 / uint16 samples");
  return KMP_OK;
}

int codec_encode(int nsp, int dtype, const void* highres, int64_t B, const int64_t* shape, int64_t C,
                 const kmp_predictor* pred, int coder, void* lowres_out, void* const* maps_out, int32_t* dims_out,
                 const kmp_region* region, void* ws, size_t ws_bytes, hipStream_t stream) {
  KMP_REQUIRE(B >= 0 && C >= 1, "bad batch or channel count");
  for (int a = 0; a < nsp; ++a) KMP_REQUIRE(shape[a] >= 2, "spatial dims must be >= 2 (>= 3 after even padding)");
  if (int st = check_predictor(pred, dtype)) return st;
  Geo g = make_geo_from_highres(nsp, shape);
  if (dims_out)
    for (int a = 0; a < nsp; ++a) dims_out[a] = g.dims[a + 3 - nsp];
  KMP_REQUIRE(highres && lowres_out && maps_out, "null pointer");
  MapPtrs maps{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(maps_out[k], "null map pointer");
    maps.p[k] = maps_out[k];
  }
  if (B == 0) return KMP_OK;
  return dispatch_natural(dtype, coder, [&](auto tag, auto coder_c) {
    using T = decltype(tag);
    constexpr int CODER = decltype(coder_c)::value;
    int st = try_fast_encode<T>(nsp, (const T*)highres, g, B, C, pred, (T*)lowres_out, maps, region, ws, ws_bytes,
                                stream);
    if (st != KMP_ERR_UNSUPPORTED) return st;
    return encode_generic_t<T, CODER>((const T*)highres, g, nsp, B, C, pred, (T*)lowres_out, maps, region, ws,
                                      ws_bytes, stream);
  });
}

int codec_decode(int nsp, int dtype, const void* lowres, const void* const* maps_in, int64_t B, const int64_t* E,
                 int64_t C, const int32_t* dims, const kmp_predictor* pred, int coder, void* highres_out,
                 const kmp_region* region, void* ws, size_t ws_bytes, hipStream_t stream) {
  KMP_REQUIRE(B >= 0 && C >= 1 && dims, "bad batch/channel count or dims");
  for (int a = 0; a < nsp; ++a) {
    KMP_REQUIRE(dims[a] == 0 || dims[a] == 1, "dims must be 0 or 1");
    KMP_REQUIRE(E[a] >= 1 && E[a] + dims[a] >= 2, "lowres too small");
  }
  if (int st = check_predictor(pred, dtype)) return st;
  Geo g = make_geo_from_lowres(nsp, E, dims);
  KMP_REQUIRE(lowres && maps_in && highres_out, "null pointer");
  CMapPtrs maps{};
  for (int k = 0; k < (nsp == 3 ? 7 : 3); ++k) {
    KMP_REQUIRE(maps_in[k], "null map pointer");
    maps.p[k] = maps_in[k];
  }
  if (B == 0) return KMP_OK;
  return dispatch_natural(dtype, coder, [&](auto tag, auto coder_c) {
    using T = decltype(tag);
    constexpr int CODER = decltype(coder_c)::value;
    int st = try_fast_decode<T>(nsp, (const T*)lowres, maps, g, B, C, pred, (T*)highres_out, region, ws, ws_bytes,
                                stream);
    if (st != KMP_ERR_UNSUPPORTED) return st;
    return decode_generic_t<T, CODER>((const T*)lowres, maps, g, nsp, B, C, pred, (T*)highres_out, region, ws,
                                      ws_bytes, stream);
  });
}

}  // namespace kmp

using namespace kmp;

extern "C" {

int kmp_volume_encode(int32_t dtype, const void* highres, int64_t B, int64_t D, int64_t H, int64_t W, int64_t C,
                      const kmp_predictor* predictor, int32_t coder, void* lowres_out, void* const maps_out[7],
                      int32_t dims_out[3], const kmp_region* region, void* workspace, size_t workspace_bytes,
                      kmp_stream_t stream) {
  const int64_t shape[3] = {D, H, W};
  return codec_encode(3, dtype, highres, B, shape, C, predictor, coder, lowres_out, maps_out, dims_out, region,
                      workspace, workspace_bytes, (hipStream_t)stream);
}

int kmp_volume_decode(int32_t dtype, const void* lowres, const void* const maps[7], int64_t B, int64_t Ed, int64_t Eh,
                      int64_t Ew, int64_t C, const int32_t dims[3], const kmp_predictor* predictor, int32_t coder,
                      void* highres_out, const kmp_region* region, void* workspace, size_t workspace_bytes,
                      kmp_stream_t stream) {
  const int64_t E[3] = {Ed, Eh, Ew};
  return codec_decode(3, dtype, lowres, maps, B, E, C, dims, predictor, coder, highres_out, region, workspace,
                      workspace_bytes, (hipStream_t)stream);
}

int64_t kmp_volume_workspace_bytes(int32_t dtype, int64_t B, int64_t D, int64_t H, int64_t W, int64_t C,
                                   const kmp_predictor* predictor) {
  const int64_t shape[3] = {D, H, W};
  Geo g = make_geo_from_highres(3, shape);
  return generic_workspace_bytes(dtype, 3, g, B, C, predictor);
}

int kmp_image_encode(int32_t dtype, const void* highres, int64_t B, int64_t H, int64_t W, int64_t C,
                     const kmp_predictor* predictor, int32_t coder, void* lowres_out, void* const maps_out[3],
                     int32_t dims_out[2], const kmp_region* region, void* workspace, size_t workspace_bytes,
                     kmp_stream_t stream) {
  const int64_t shape[2] = {H, W};
  return codec_encode(2, dtype, highres, B, shape, C, predictor, coder, lowres_out, maps_out, dims_out, region,
                      workspace, workspace_bytes, (hipStream_t)stream);
}

int kmp_image_decode(int32_t dtype, const void* lowres, const void* const maps[3], int64_t B, int64_t Eh, int64_t Ew,
                     int64_t C, const int32_t dims[2], const kmp_predictor* predictor, int32_t coder,
                     void* highres_out, const kmp_region* region, void* workspace, size_t workspace_bytes,
                     kmp_stream_t stream) {
  const int64_t E[2] = {Eh, Ew};
  return codec_decode(2, dtype, lowres, maps, B, E, C, dims, predictor, coder, highres_out, region, workspace,
                      workspace_bytes, (hipStream_t)stream);
}

int64_t kmp_image_workspace_bytes(int32_t dtype, int64_t B, int64_t H, int64_t W, int64_t C,
                                  const kmp_predictor* predictor) {
  const int64_t shape[2] = {H, W};
  Geo g = make_geo_from_highres(2, shape);
  return generic_workspace_bytes(dtype, 2, g, B, C, predictor);
}

}  // extern "C"
