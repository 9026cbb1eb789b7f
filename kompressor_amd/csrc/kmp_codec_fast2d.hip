// kmp_codec_fast2d.hip -- one-pass fused encode / decode for images (placeholder: not yet
// specialised; every request falls back to the generic two-pass path).
#include "kmp_codec.h"

namespace kmp {

template <typename T>
int try_fast2d_encode(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*, const MapPtrs&,
                      const kmp_region*, hipStream_t) {
  return KMP_ERR_UNSUPPORTED;
}
template <typename T>
int try_fast2d_decode(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,
                      const kmp_region*, hipStream_t) {
  return KMP_ERR_UNSUPPORTED;
}

#define KMP_INST2(T)                                                                                             \
  template int try_fast2d_encode<T>(const T*, const Geo&, int64_t, int64_t, const kmp_predictor*, T*,          \
                                    const MapPtrs&, const kmp_region*, hipStream_t);                           \
  template int try_fast2d_decode<T>(const T*, const CMapPtrs&, const Geo&, int64_t, int64_t,                   \
                                    const kmp_predictor*, T*, const kmp_region*, hipStream_t);
KMP_INST2(uint8_t)
KMP_INST2(uint16_t)
KMP_INST2(int32_t)
KMP_INST2(uint32_t)

}  // namespace kmp
