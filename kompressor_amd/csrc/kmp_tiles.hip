// kmp_tiles.hip -- split a volume (image) into a batch of independent tiles and reassemble it.
//
// The metric workload (BASELINE config C3/C4) is one 512^3 volume cut into
// 64^3 sub-volumes that become the batch axis of encode/decode (every primitive of the
// reference is [:, ...]-parallel, volume/utils.py:80,161-169).  Tile t = (tz, ty, tx) in z-major
// order holds volume[tz*Tz : (tz+1)*Tz, ty*Ty : .., tx*Tx : .., :].
//
// HBM-bound permutation: one thread moves 16 bytes of one tile row (a row of Tx*C elements
// is contiguous on both sides), so both the read and the write are full 16-B-per-lane
// streams when Tx*C*sizeof(T) is a multiple of 16; other shapes take the element kernel.
#include "kmp_common.h"

namespace kmp {

constexpr int kTileThreads = 256;
typedef uint32_t tile_u32x4 __attribute__((ext_vector_type(4)));

struct TileGeo {
  int64_t n[3];   // volume extents (z, y, x)
  int64_t t[3];   // tile extents
  int64_t nt[3];  // tiles per axis
  int64_t rowb;   // bytes per tile row (Tx * C * sizeof(T))
};

// direction 0: volume -> tiles, 1: tiles -> volume.  ``V`` = bytes moved per thread (16 or 1).
template <int V>
__global__ void __launch_bounds__(kTileThreads) tiles_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                            TileGeo g, int direction, int64_t total) {
  const int64_t per_row = g.rowb / V;
  for (int64_t i = blockIdx.x * (int64_t)kTileThreads + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kTileThreads) {
    int64_t r = i / per_row;
    const int64_t v = i - r * per_row;
    // r = ((tile * Tz) + z) * Ty + y over the tile batch
    const int64_t y = r % g.t[1];
    r /= g.t[1];
    const int64_t z = r % g.t[0];
    int64_t tile = r / g.t[0];
    const int64_t tx = tile % g.nt[2];
    tile /= g.nt[2];
    const int64_t ty = tile % g.nt[1];
    const int64_t tz = tile / g.nt[1];
    const int64_t tile_off = (r * g.t[1] + y) * g.rowb + v * V;  // r == tile index * Tz + z
    const int64_t vol_off =
        (((tz * g.t[0] + z) * g.n[1] + ty * g.t[1] + y) * (g.n[2] / g.t[2]) + tx) * g.rowb + v * V;
    const int64_t so = direction == 0 ? vol_off : tile_off;
    const int64_t dof = direction == 0 ? tile_off : vol_off;
    if constexpr (V == 16) {
      *(tile_u32x4*)(dst + dof) = __builtin_nontemporal_load((const tile_u32x4*)(src + so));
    } else {
      dst[dof] = src[so];
    }
  }
}

}  // namespace kmp

using namespace kmp;

extern "C" int kmp_tiles(int32_t nsp, int32_t dtype, int32_t direction, const void* src, const int64_t shape[3],
                         int64_t C, const int64_t tile[3], void* dst, kmp_stream_t stream) {
  KMP_REQUIRE(nsp == 2 || nsp == 3, "nsp must be 2 or 3");
  KMP_REQUIRE(direction == 0 || direction == 1, "direction must be 0 (split) or 1 (assemble)");
  KMP_REQUIRE(src && dst && shape && tile, "null pointer");
  KMP_REQUIRE(C >= 1, "channels must be >= 1");
  const int es = dtype_size(dtype);
  KMP_REQUIRE(es > 0, "unsupported dtype");
  TileGeo g{};
  int64_t total_rows = 1;
  for (int a = 0; a < 3; ++a) {
    if (a < 3 - nsp) {
      g.n[a] = g.t[a] = g.nt[a] = 1;
      continue;
    }
    const int i = a - (3 - nsp);
    KMP_REQUIRE(shape[i] > 0 && tile[i] > 0 && shape[i] % tile[i] == 0,
                "every spatial extent must be a positive multiple of the tile extent");
    g.n[a] = shape[i];
    g.t[a] = tile[i];
    g.nt[a] = shape[i] / tile[i];
  }
  g.rowb = g.t[2] * C * es;
  total_rows = g.n[0] * g.n[1] * g.nt[2];  // tile rows in the whole volume
  const bool vec = g.rowb % 16 == 0 && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 15) == 0;
  const int V = vec ? 16 : 1;
  const int64_t total = total_rows * (g.rowb / V);
  int64_t grid = (total + kTileThreads - 1) / kTileThreads;
  if (grid > 65536) grid = 65536;
  if (vec)
    tiles_kernel<16><<<(unsigned)grid, kTileThreads, 0, (hipStream_t)stream>>>((const uint8_t*)src, (uint8_t*)dst, g,
                                                                               direction, total);
  else
    tiles_kernel<1><<<(unsigned)grid, kTileThreads, 0, (hipStream_t)stream>>>((const uint8_t*)src, (uint8_t*)dst, g,
                                                                              direction, total);
  return check_launch("tiles");
}
