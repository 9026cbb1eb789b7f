// kmp_options.hip -- the process-wide dispatch options (include/kompressor_hip.h: kmp_set_option).
//
// Each option starts from the environment variable of the same name, read ONCE when the library
// is loaded (a static initialiser); after that only kmp_set_option / kmp_clear_option change it.
// Launches read the table (kmp::opt: one relaxed atomic load) and never call getenv.
#include <atomic>
#include <climits>
#include <cstdlib>
#include <cstring>

#include "kmp_common.h"

namespace kmp {
namespace {

constexpr int kUnset = INT_MIN;

const char* const kNames[OPT_COUNT] = {
    "KMP_DISABLE_WAVE", "KMP_DISABLE_FAST", "KMP_DISABLE_LINEAR_FUSED", "KMP_DISABLE_ROWS", "KMP_DISABLE_SWAR",
    "KMP_W3_PL",        "KMP_W3P_PL",       "KMP_W3_XCD",               "KMP_W2_XCD",       "KMP_W3_ST_ENC",
    "KMP_W3P_ST_ENC",   "KMP_W2_ST_ENC",    "KMP_W2P_ST_ENC",           "KMP_L3Y",
    "KMP_LINEAR_F32_MFMA",
};

struct Table {
  std::atomic<int> v[OPT_COUNT];
  Table() {
    for (int i = 0; i < OPT_COUNT; ++i) {
      const char* e = std::getenv(kNames[i]);
      v[i].store(e && *e ? std::atoi(e) : kUnset, std::memory_order_relaxed);
    }
  }
};

Table& table() {
  static Table t;  // built at load (the initialiser below), thread-safe either way
  return t;
}
const Table& g_init = table();

int find(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < OPT_COUNT; ++i)
    if (!std::strcmp(name, kNames[i])) return i;
  return -1;
}

}  // namespace

int opt(Opt id, int dflt) {
  const int v = table().v[id].load(std::memory_order_relaxed);
  return v == kUnset ? dflt : v;
}

}  // namespace kmp

extern "C" {

int kmp_set_option(const char* name, int value) {
  const int i = kmp::find(name);
  if (i < 0) return kmp::fail(KMP_ERR_ARG, std::string("kmp_set_option: unknown option ") + (name ? name : "(null)"));
  if (value == kmp::kUnset) return kmp::fail(KMP_ERR_ARG, "kmp_set_option: value out of range");
  kmp::table().v[i].store(value, std::memory_order_relaxed);
  return KMP_OK;
}

int kmp_clear_option(const char* name) {
  const int i = kmp::find(name);
  if (i < 0) return kmp::fail(KMP_ERR_ARG, std::string("kmp_clear_option: unknown option ") + (name ? name : "(null)"));
  kmp::table().v[i].store(kmp::kUnset, std::memory_order_relaxed);
  return KMP_OK;
}

int kmp_get_option(const char* name, int* value) {
  const int i = kmp::find(name);
  if (i < 0) return kmp::fail(KMP_ERR_ARG, std::string("kmp_get_option: unknown option ") + (name ? name : "(null)"));
  const int v = kmp::table().v[i].load(std::memory_order_relaxed);
  if (v == kmp::kUnset) return 0;
  if (value) *value = v;
  return 1;
}

}  // extern "C"
