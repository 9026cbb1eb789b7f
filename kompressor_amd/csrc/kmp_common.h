// kmp_common.h -- shared device/host helpers for libkompressor_hip (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cmath>
#include <limits>
#include <string>
#include <type_traits>

#include "../../include/kompressor_hip.h"

namespace kmp {

// ------------------------------------------------------------------------------------------
// Error plumbing: every C entry point returns a kmp_status and leaves a thread-local message.
// ------------------------------------------------------------------------------------------
void set_error(const std::string& msg);
int fail(int status, const std::string& msg);
int check_launch(const char* what);

// Device-side bounds checks of the debug build (``KMP_DEBUG=1 python kompressor_amd/_build.py``
// -> libkompressor_hip_debug.so, loaded when KMP_DEBUG=1): a failed check prints the kernel's
// file:line and the offending access, then traps so the fault is localised to one access instead
// of surfacing as a memory fault somewhere later.  Compiled out of the release library.
#ifdef KMP_DEBUG
#define KMP_DCHECK(cond, ...)                                                               \
  do {                                                                                     \
    if (!(cond)) {                                                                         \
      printf("KMP_DCHECK failed %s:%d: %s -- ", __FILE__, __LINE__, #cond);               \
      printf(__VA_ARGS__);                                                                 \
      printf("\n");                                                                        \
      __builtin_trap();                                                                    \
    }                                                                                      \
  } while (0)
#else
#define KMP_DCHECK(cond, ...) do { } while (0)
#endif

// [p, p + cnt) inside the array [base, base + n) (elements); a no-op in the release build
template <typename T>
__device__ __forceinline__ void dcheck_span(const T* base, const T* p, int64_t cnt, int64_t n, int line) {
  KMP_DCHECK(p >= base && p + cnt <= base + n, "line %d: access [%lld, %lld) of an array of %lld elements", line,
             (long long)(p - base), (long long)(p - base + cnt), (long long)n);
}
#define KMP_SPAN(base, p, cnt, n) ::kmp::dcheck_span((base), (p), (int64_t)(cnt), (int64_t)(n), __LINE__)

// ------------------------------------------------------------------------------------------
// Dispatch options (kmp_set_option): one table per process, seeded from the
// environment once at load (kmp_options.hip); a launch reads it with one relaxed atomic load.
// ------------------------------------------------------------------------------------------
enum Opt {
  OPT_DISABLE_WAVE, OPT_DISABLE_FAST, OPT_DISABLE_LINEAR_FUSED, OPT_DISABLE_ROWS, OPT_DISABLE_SWAR,
  OPT_W3_PL, OPT_W3P_PL, OPT_W3_XCD, OPT_W2_XCD, OPT_W3_ST_ENC, OPT_W3P_ST_ENC, OPT_W2_ST_ENC,
  OPT_W2P_ST_ENC, OPT_L3Y, OPT_LINEAR_F32_MFMA, OPT_COUNT
};
// the option's value, or ``dflt`` while it is unset
int opt(Opt id, int dflt);

#define KMP_REQUIRE(cond, msg)                                         \
  do {                                                                 \
    if (!(cond)) return ::kmp::fail(KMP_ERR_ARG, std::string(__func__) + ": " + (msg)); \
  } while (0)

// ------------------------------------------------------------------------------------------
// dtype traits
// ------------------------------------------------------------------------------------------
template <int DT> struct dtype_of;
template <> struct dtype_of<KMP_U8> { using type = uint8_t; };
template <> struct dtype_of<KMP_U16> { using type = uint16_t; };
template <> struct dtype_of<KMP_I32> { using type = int32_t; };
template <> struct dtype_of<KMP_F32> { using type = float; };
template <> struct dtype_of<KMP_U32> { using type = uint32_t; };

inline int dtype_size(int dt) {
  switch (dt) {
    case KMP_U8: return 1;
    case KMP_U16: return 2;
    case KMP_I32: case KMP_F32: case KMP_U32: return 4;
    default: return 0;
  }
}

// Dispatch a runtime dtype to a templated callable: f(T{}) with T the element type.
template <typename F>
int dispatch_int_dtype(int dt, F&& f) {  // integer sample dtypes (highres / lowres / maps)
  switch (dt) {
    case KMP_U8: return f(uint8_t{});
    case KMP_U16: return f(uint16_t{});
    case KMP_I32: return f(int32_t{});
    case KMP_U32: return f(uint32_t{});
    default: return fail(KMP_ERR_ARG, "unsupported sample dtype " + std::to_string(dt));
  }
}
template <typename F>
int dispatch_any_dtype(int dt, F&& f) {
  if (dt == KMP_F32) return f(float{});
  return dispatch_int_dtype(dt, f);
}

// ------------------------------------------------------------------------------------------
// Reference arithmetic restated on device
// ------------------------------------------------------------------------------------------

// ``astype(T)`` of a float32 as XLA does it: identity for float;
// truncation toward zero for integers, saturating at the range, NaN -> 0.
template <typename T>
__host__ __device__ __forceinline__ T cast_f32(float v) {
  if constexpr (std::is_same<T, float>::value) {
    return v;
  } else {
    constexpr double lo = (double)std::numeric_limits<T>::min();
    constexpr double hi = (double)std::numeric_limits<T>::max();
    double t = (double)v;
    if (!(t == t)) return T(0);
    t = t < 0 ? ceil(t) : floor(t);
    if (t <= lo) return std::numeric_limits<T>::min();
    if (t >= hi) return std::numeric_limits<T>::max();
    return T(t);
  }
}

// ``jnp.int32(x)`` on an operand: integers wrap into int32, floats truncate (saturating).
template <typename T>
__host__ __device__ __forceinline__ int32_t to_i32(T v) {
  if constexpr (std::is_same<T, float>::value) return cast_f32<int32_t>(v);
  else return (int32_t)v;
}

// Coders: utils.py:28-55.  Every coder is "wrapping int32 add/sub, narrowed to the coder's
// width": ((a + 2^k) % 2^k) of an int32 equals its low k bits for a floor-mod.
template <int CODER> struct coder_out;
template <> struct coder_out<KMP_CODER_RAW> { using type = int32_t; };
template <> struct coder_out<KMP_CODER_U8> { using type = uint8_t; };
template <> struct coder_out<KMP_CODER_U16> { using type = uint16_t; };
template <> struct coder_out<KMP_CODER_U32> { using type = uint32_t; };

template <int CODER>
__host__ __device__ __forceinline__ typename coder_out<CODER>::type code_encode(int32_t pred, int32_t gt) {
  return (typename coder_out<CODER>::type)(uint32_t)((uint32_t)gt - (uint32_t)pred);
}
template <int CODER>
__host__ __device__ __forceinline__ typename coder_out<CODER>::type code_decode(int32_t pred, int32_t enc) {
  return (typename coder_out<CODER>::type)(uint32_t)((uint32_t)pred + (uint32_t)enc);
}

// numpy/jnp mode='symmetric' source index for any integer i (periodic mirror, period 2n).
__host__ __device__ __forceinline__ int64_t sym_index(int64_t i, int64_t n) {
  if (i >= 0 && i < n) return i;  // interior: no (emulated 64-bit) modulo
  if (i >= -n && i < 2 * n) return i < 0 ? -1 - i : 2 * n - 1 - i;  // one reflection
  int64_t m = i % (2 * n);
  if (m < 0) m += 2 * n;
  return m < n ? m : 2 * n - 1 - m;
}

// ------------------------------------------------------------------------------------------
// Geometry of the reference's single pyramid level (volume/utils.py:226-237, 263-276)
// ------------------------------------------------------------------------------------------
struct Geo {
  int64_t n[3];    // highres extent per spatial axis (unpadded); unused axes = 1
  int64_t L[3];    // lowres nodes of the padded highres
  int64_t E[3];    // stored (trimmed) node extent = L - dims
  int64_t Lc[3];   // cells = L - 1
  int32_t dims[3]; // even padding
};

inline Geo make_geo_from_highres(int nsp, const int64_t* sp) {
  Geo g{};
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) { g.n[a] = 1; g.L[a] = 1; g.E[a] = 1; g.Lc[a] = 1; g.dims[a] = 0; continue; }
    int64_t n = sp[a - (3 - nsp)];
    g.n[a] = n;
    g.dims[a] = (int32_t)((n + 1) % 2);
    g.L[a] = (n + g.dims[a] + 1) / 2;
    g.E[a] = g.L[a] - g.dims[a];
    g.Lc[a] = g.L[a] - 1;
  }
  return g;
}

inline Geo make_geo_from_lowres(int nsp, const int64_t* E, const int32_t* dims) {
  Geo g{};
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) { g.n[a] = 1; g.L[a] = 1; g.E[a] = 1; g.Lc[a] = 1; g.dims[a] = 0; continue; }
    int i = a - (3 - nsp);
    g.E[a] = E[i];
    g.dims[a] = dims[i];
    g.L[a] = E[i] + dims[i];
    g.Lc[a] = g.L[a] - 1;
    g.n[a] = 2 * g.L[a] - 1 - dims[i];
  }
  return g;
}

// Map tables.  Class 0 is the lowres (all-even) class; classes 1..7 (1..3 in 2D) are the maps
// in the reference's order.  Parities are (z, y, x); in 2D z is a dummy axis.
// volume/utils.py:161-169 : LR(1,1,0) UD(1,0,1) FB(0,1,1) C(1,1,1) Z(1,0,0) Y(0,1,0) X(0,0,1)
// image/utils.py:92-94    : LR(y1,x0) UD(y0,x1) C(y1,x1)
__host__ __device__ __forceinline__ void map_parity(int nsp, int k, int par[3]) {
  if (nsp == 3) {
    const int t[7][3] = {{1, 1, 0}, {1, 0, 1}, {0, 1, 1}, {1, 1, 1}, {1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    par[0] = t[k][0]; par[1] = t[k][1]; par[2] = t[k][2];
  } else {
    const int t[3][2] = {{1, 0}, {0, 1}, {1, 1}};
    par[0] = 0; par[1] = t[k][0]; par[2] = t[k][1];
  }
}

// Extent of map k (0-based, excluding lowres) along axis a in its trimmed (stored) form.
inline int64_t map_extent(const Geo& g, int nsp, int k, int a) {
  int par[3];
  map_parity(nsp, k, par);
  if (a < 3 - nsp) return 1;
  return par[a] ? g.Lc[a] : g.E[a];
}

constexpr int kMaxMaps = 7;

struct MapPtrs {  // passed by value to kernels
  void* p[kMaxMaps];
};
struct CMapPtrs {
  const void* p[kMaxMaps];
};

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// n / d for a wave-uniform 0 <= n < 2^31 and a launch-constant d >= 1 as q = mulhi(n, m) >> s (s < 0:
// d == 1, q = n), m = floor(2^(31+l) / d) + 1 with l = ceil(log2 d): exact on 31-bit n (error m d - 2^(31+l)
// is in (0, d] and n d < 2^(31+l)).  Computed on the host, so the kernel divides with two scalar
// instructions instead of a VALU reciprocal sequence with quarter-rate multiplies.
struct UDiv {
  uint32_t m;
  int32_t s;
};
inline UDiv make_udiv(uint32_t d) {
  if (d <= 1) return UDiv{0u, -1};
  int l = 0;
  while ((1ull << l) < d) ++l;
  return UDiv{(uint32_t)(((uint64_t)1 << (31 + l)) / d + 1), l - 1};
}
__device__ __forceinline__ uint32_t udiv(uint32_t n, UDiv f) {
  return f.s < 0 ? n : __umulhi(n, f.m) >> f.s;
}

// 16-byte vectors: aligned, and any-alignment (gfx950 serves unaligned dwordx4 global accesses;
// rows of odd length are only element-aligned)
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

// V = 16 / sizeof(T) consecutive elements moved as one 16-byte access
template <typename T>
struct Vec16 {
  static constexpr int V = 16 / (int)sizeof(T);
  T e[V];
  __device__ __forceinline__ void load(const T* p) {
    const u32x4u v = *(const u32x4u*)p;
    __builtin_memcpy(e, &v, 16);
  }
  __device__ __forceinline__ void store(T* p) const {
    u32x4u v;
    __builtin_memcpy(&v, e, 16);
    *(u32x4u*)p = v;
  }
};

// row-kernel work item: chunk j of row (b, z, y)
struct RowItem {
  int32_t b, z, y, j;
};
// item t over [B, nz, ny, nch] (all extents >= 1)
__device__ __forceinline__ RowItem row_item(uint32_t t, uint32_t nz, uint32_t ny, uint32_t nch) {
  RowItem r;
  r.j = (int32_t)(t % nch); t /= nch;
  r.y = (int32_t)(t % ny); t /= ny;
  r.z = (int32_t)(t % nz);
  r.b = (int32_t)(t / nz);
  return r;
}


// Flat index t over [B, e0, e1, e2, C] (C fastest).  The grid-stride kernels decompose one index
// per element: 64-bit division is a long emulated sequence on gfx950, so indices below 2^32 (every
// array axis and, in practice, every flat index fits) take 32-bit divisions; C == 1 skips one.
__device__ __forceinline__ void unflat5(int64_t t, int64_t e0, int64_t e1, int64_t e2, int64_t C, int64_t& b,
                                        int64_t& i0, int64_t& i1, int64_t& i2, int64_t& c) {
  if ((uint64_t)t < 0x100000000ull) {
    uint32_t u = (uint32_t)t;
    const uint32_t uC = (uint32_t)C, u2 = (uint32_t)e2, u1 = (uint32_t)e1, u0 = (uint32_t)e0;
    if (uC == 1) {
      c = 0;
    } else {
      c = u % uC;
      u /= uC;
    }
    i2 = u % u2; u /= u2;
    i1 = u % u1; u /= u1;
    i0 = u % u0;
    b = u / u0;
  } else {
    c = t % C; t /= C;
    i2 = t % e2; t /= e2;
    i1 = t % e1; t /= e1;
    i0 = t % e0;
    b = t / e0;
  }
}

}  // namespace kmp
