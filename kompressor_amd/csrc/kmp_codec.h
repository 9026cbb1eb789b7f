// kmp_codec.h -- internal interfaces between the fused-codec translation units.
#pragma once

#include "kmp_aggregate.h"

namespace kmp {

template <typename T> constexpr int dtype_code();
template <> constexpr int dtype_code<uint8_t>() { return KMP_U8; }
template <> constexpr int dtype_code<uint16_t>() { return KMP_U16; }
template <> constexpr int dtype_code<int32_t>() { return KMP_I32; }
template <> constexpr int dtype_code<uint32_t>() { return KMP_U32; }
template <> constexpr int dtype_code<float>() { return KMP_F32; }

int64_t generic_workspace_bytes(int dtype, int nsp, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred);

// Linear predictor over a box of cells: writes cells[b, c..., k, C] (K = 19 / 5) in T
// (kmp_linear.hip).  ``src`` is highres (mult 2) or trimmed lowres (mult 1), extents S.
template <typename T>
int linear_cells(const T* src, const int64_t* S, int mult, const Geo& g, int nsp, int64_t B, int64_t C,
                 const kmp_predictor* pred, const int64_t* cbegin, const int64_t* cext, T* cells, hipStream_t stream);

// One-pass kernels (kmp_codec_fast3d.hip / kmp_codec_fast2d.hip).  Return KMP_ERR_UNSUPPORTED
// (without touching anything) when the request is not eligible, so the caller falls back.
template <typename T>
int try_fast2d_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                      const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_fast2d_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                      const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_linear3pm_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                         const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream);
template <typename T>
int try_linear3pm_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                         const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream);
template <typename T>
int try_linear3m_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                        const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_linear3m_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                        const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_linear3d_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                        const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_linear3d_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                        const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave2d_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                      const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave2d_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                      const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave3d_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                      const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave3d_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                      const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave3dp_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                       const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave3dp_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                       const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave2dp_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                       const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave2dp_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                       const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_linear3dp_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                         const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream);
template <typename T>
int try_linear3dp_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                         const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                         hipStream_t stream);
template <typename T>
int try_wave3d32_encode(const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                        const MapPtrs& maps, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_wave3d32_decode(const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                        const kmp_predictor* pred, T* hi, const kmp_region* region, hipStream_t stream);
template <typename T>
int try_fast_encode(int nsp, const T* hi, const Geo& g, int64_t B, int64_t C, const kmp_predictor* pred, T* lowres,
                    const MapPtrs& maps, const kmp_region* region, void* ws, size_t ws_bytes, hipStream_t stream);
template <typename T>
int try_fast_decode(int nsp, const T* lowres, const CMapPtrs& maps, const Geo& g, int64_t B, int64_t C,
                    const kmp_predictor* pred, T* hi, const kmp_region* region, void* ws, size_t ws_bytes,
                    hipStream_t stream);

}  // namespace kmp
