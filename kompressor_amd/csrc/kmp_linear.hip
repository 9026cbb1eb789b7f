// kmp_linear.hip -- LinearPredictor apply (placeholder until the MFMA kernel lands).
#include "kmp_codec.h"

namespace kmp {

template <typename T>
int linear_cells(const T*, const int64_t*, int, const Geo&, int, int64_t, int64_t, const kmp_predictor*,
                 const int64_t*, const int64_t*, T*, hipStream_t) {
  return fail(KMP_ERR_UNSUPPORTED, "linear predictor not built yet");
}

#define KMP_INSTL(T)                                                                                             \
  template int linear_cells<T>(const T*, const int64_t*, int, const Geo&, int, int64_t, int64_t,               \
                               const kmp_predictor*, const int64_t*, const int64_t*, T*, hipStream_t);
KMP_INSTL(uint8_t)
KMP_INSTL(uint16_t)
KMP_INSTL(int32_t)
KMP_INSTL(uint32_t)

}  // namespace kmp

extern "C" int kmp_linear_predict(int32_t, int32_t, const void*, int64_t, const int64_t*, int64_t, int32_t,
                                  const float*, const float*, void*, float*, kmp_stream_t) {
  return kmp::fail(KMP_ERR_UNSUPPORTED, "linear predictor not built yet");
}
