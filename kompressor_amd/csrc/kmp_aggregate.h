// kmp_aggregate.h -- the reference's maps_from_predictions arithmetic for ONE output element.
//
// volume/utils.py:83-155 (image/utils.py:58-86) build each map by float32 scatter-adds of the
// per-cell predictions (in channel order, starting from zero), multiply interior entries by
// 0.5 (two-way lattices) or by 0.25 / 0.5 (four-way lattices: interior / one-sided edge), then
// truncate to the prediction dtype.  Restated per output element: sum the contributions of the
// cells that exist, in the reference's channel order, scale by 1/count (count in {1, 2, 4};
// the 0.5 / 0.25 multiplies are exactly those), cast.  The C map is the raw channel-6 (2D:
// channel-4) value with no float round trip (volume/utils.py:117).
#pragma once

#include "kmp_common.h"

namespace kmp {

// One contribution: a cell offset (subtracted from the output coordinate) and a channel.
struct Contrib {
  int8_t dz, dy, dx, ch;
};

// Contribution lists per map, reference channel order.  Offsets are "cell = o - d".
// 3D: LR ch0 (cell x), ch1 (cell x-1); UD ch2, ch3; FB ch4, ch5; C ch6;
//     Z ch7 (y,x) ch8 (y,x-1) ch9 (y-1,x-1) ch10 (y-1,x); Y ch11..14 over (z,x); X ch15..18 over (z,y).
// 2D: LR ch0, ch1 (x); UD ch2, ch3 (y); C ch4.
__host__ __device__ __forceinline__ int map_contribs(int nsp, int k, Contrib c[4]) {
  if (nsp == 3) {
    switch (k) {
      case 0: c[0] = {0, 0, 0, 0}; c[1] = {0, 0, 1, 1}; return 2;
      case 1: c[0] = {0, 0, 0, 2}; c[1] = {0, 1, 0, 3}; return 2;
      case 2: c[0] = {0, 0, 0, 4}; c[1] = {1, 0, 0, 5}; return 2;
      case 3: c[0] = {0, 0, 0, 6}; return 1;
      case 4: c[0] = {0, 0, 0, 7}; c[1] = {0, 0, 1, 8}; c[2] = {0, 1, 1, 9}; c[3] = {0, 1, 0, 10}; return 4;
      case 5: c[0] = {0, 0, 0, 11}; c[1] = {0, 0, 1, 12}; c[2] = {1, 0, 1, 13}; c[3] = {1, 0, 0, 14}; return 4;
      default: c[0] = {0, 0, 0, 15}; c[1] = {0, 1, 0, 16}; c[2] = {1, 1, 0, 17}; c[3] = {1, 0, 0, 18}; return 4;
    }
  } else {
    switch (k) {
      case 0: c[0] = {0, 0, 0, 0}; c[1] = {0, 0, 1, 1}; return 2;
      case 1: c[0] = {0, 0, 0, 2}; c[1] = {0, 1, 0, 3}; return 2;
      default: c[0] = {0, 0, 0, 4}; return 1;
    }
  }
}

__host__ __device__ __forceinline__ int center_map(int nsp) { return nsp == 3 ? 3 : 2; }

// get(cz, cy, cx, ch) -> T, called only for existing cells (0 <= c < Lc on every axis).
template <typename T, typename Get>
__device__ __forceinline__ T aggregate_map(int nsp, int k, int64_t oz, int64_t oy, int64_t ox,
                                           int64_t Lcz, int64_t Lcy, int64_t Lcx, Get&& get) {
  Contrib c[4];
  const int nc = map_contribs(nsp, k, c);
  if (k == center_map(nsp)) return get(oz, oy, ox, (int)c[0].ch);
  float s = 0.0f;
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i >= nc) break;
    const int64_t z = oz - c[i].dz, y = oy - c[i].dy, x = ox - c[i].dx;
    if (z >= 0 && z < Lcz && y >= 0 && y < Lcy && x >= 0 && x < Lcx) {
      s += (float)get(z, y, x, (int)c[i].ch);
      ++cnt;
    }
  }
  if (cnt == 4) s *= 0.25f;
  else if (cnt == 2) s *= 0.5f;
  return cast_f32<T>(s);
}

}  // namespace kmp
