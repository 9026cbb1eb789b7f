// capi_example.cpp -- the C-ABI used from a plain C++ host, no Python, no torch: what a caller
// that is not the Python package (another runtime, an FFI binding) does with
// libkompressor_hip.so.  Encodes and decodes a batch of 64^3 uint16 tiles with the mean
// predictor, checks the round trip and one map value against a host restatement, and times
// the fused launches.
//   built by python kompressor_amd/_build.py:  tools/capi_example
//   run:  ./tools/capi_example [tiles]   -> prints "capi ok ..." and exits 0
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../include/kompressor_hip.h"

#define CHECK_HIP(x)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) {                                                              \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
      return 2;                                                                          \
    }                                                                                    \
  } while (0)
#define CHECK_KMP(x)                                                                     \
  do {                                                                                   \
    int s_ = (x);                                                                        \
    if (s_ != KMP_OK) {                                                                  \
      std::fprintf(stderr, "%s: status %d: %s\n", #x, s_, kmp_last_error());            \
      return 3;                                                                          \
    }                                                                                    \
  } while (0)

int main(int argc, char** argv) {
  const int64_t B = argc > 1 ? std::atoll(argv[1]) : 16, D = 64, H = 64, W = 64, C = 1;
  const int64_t n = B * D * H * W;
  const int64_t E = 32;                     // stored lowres / map extent per axis for 64 (even)
  const int64_t nmap = B * E * E * E;       // every map of an even 64^3 tile is 32^3
  std::vector<uint16_t> host(n);
  uint32_t s = 12345u;
  for (int64_t i = 0; i < n; ++i) {         // xorshift noise
    s ^= s << 13; s ^= s >> 17; s ^= s << 5;
    host[i] = (uint16_t)s;
  }
  uint16_t *hi, *rec, *lo, *maps[7];
  CHECK_HIP(hipMalloc(&hi, n * 2));
  CHECK_HIP(hipMalloc(&rec, n * 2));
  CHECK_HIP(hipMalloc(&lo, nmap * 2));
  for (auto& m : maps) CHECK_HIP(hipMalloc(&m, nmap * 2));
  CHECK_HIP(hipMemcpy(hi, host.data(), n * 2, hipMemcpyHostToDevice));

  kmp_predictor pred{};
  pred.kind = KMP_PRED_MEAN;
  pred.padding = 0;
  hipStream_t stream;
  CHECK_HIP(hipStreamCreate(&stream));
  int32_t dims[3];
  void* mo[7];
  const void* mi[7];
  for (int k = 0; k < 7; ++k) {
    mo[k] = maps[k];
    mi[k] = maps[k];
  }
  const int64_t ws = kmp_volume_workspace_bytes(KMP_U16, B, D, H, W, C, &pred);
  void* wsp = nullptr;
  if (ws > 0) CHECK_HIP(hipMalloc(&wsp, ws));

  CHECK_KMP(kmp_volume_encode(KMP_U16, hi, B, D, H, W, C, &pred, KMP_CODER_U16, lo, mo, dims, nullptr, wsp,
                              (size_t)ws, (kmp_stream_t)stream));
  CHECK_KMP(kmp_volume_decode(KMP_U16, lo, mi, B, E, E, E, C, dims, &pred, KMP_CODER_U16, rec, nullptr, wsp,
                              (size_t)ws, (kmp_stream_t)stream));
  CHECK_HIP(hipStreamSynchronize(stream));
  std::vector<uint16_t> back(n), cmap(nmap);
  CHECK_HIP(hipMemcpy(back.data(), rec, n * 2, hipMemcpyDeviceToHost));
  CHECK_HIP(hipMemcpy(cmap.data(), maps[3], nmap * 2, hipMemcpyDeviceToHost));
  if (std::memcmp(back.data(), host.data(), n * 2) != 0 || dims[0] != 1 || dims[1] != 1 || dims[2] != 1) {
    std::fprintf(stderr, "round trip failed (dims %d %d %d)\n", dims[0], dims[1], dims[2]);
    return 4;
  }
  // C map (volume/utils.py:117) at cell (0, 0, 0) of tile 0: highres (1,1,1) minus the floor
  // mean of the 2x2x2 lowres nodes (0|2, 0|2, 0|2), mod 2^16 (utils.py:48-50)
  uint32_t sum = 0;
  for (int z = 0; z < 2; ++z)
    for (int y = 0; y < 2; ++y)
      for (int x = 0; x < 2; ++x) sum += host[((2 * z) * H + 2 * y) * W + 2 * x];
  const uint16_t want = (uint16_t)(host[(1 * H + 1) * W + 1] - (uint16_t)(sum / 8));
  if (cmap[0] != want) {
    std::fprintf(stderr, "C map value %u, expected %u\n", cmap[0], want);
    return 5;
  }

  hipEvent_t e0, e1;
  CHECK_HIP(hipEventCreate(&e0));
  CHECK_HIP(hipEventCreate(&e1));
  const int reps = 20;
  CHECK_HIP(hipEventRecord(e0, stream));
  for (int r = 0; r < reps; ++r) {
    CHECK_KMP(kmp_volume_encode(KMP_U16, hi, B, D, H, W, C, &pred, KMP_CODER_U16, lo, mo, dims, nullptr, wsp,
                                (size_t)ws, (kmp_stream_t)stream));
    CHECK_KMP(kmp_volume_decode(KMP_U16, lo, mi, B, E, E, E, C, dims, &pred, KMP_CODER_U16, rec, nullptr, wsp,
                                (size_t)ws, (kmp_stream_t)stream));
  }
  CHECK_HIP(hipEventRecord(e1, stream));
  CHECK_HIP(hipEventSynchronize(e1));
  float ms = 0;
  CHECK_HIP(hipEventElapsedTime(&ms, e0, e1));
  std::printf("capi ok: %lld tiles of 64^3 uint16, %s, encode+decode %.1f GB/s of raw volume\n", (long long)B,
              kmp_version(), (double)n * 2 * reps / (ms * 1e-3) / 1e9);
  return 0;
}
