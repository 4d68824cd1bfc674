// Host runtime of libhonk_hip.so: error state, device queries, kernel timing.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <mutex>
#include <vector>

#include "common.h"

namespace honk {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* get_error() { return g_err; }

int cu_count() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cache[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// ---- timing window -----------------------------------------------------------
struct TimingRec {
  hipEvent_t a, b;
  double flop;
};
static std::mutex g_tmu;
static bool g_timing = false;
static std::vector<TimingRec> g_recs;
static std::vector<hipEvent_t> g_free;

static hipEvent_t take_event() {
  if (!g_free.empty()) {
    hipEvent_t e = g_free.back();
    g_free.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

TimedLaunch::TimedLaunch(hipStream_t s, double flop) {
  std::lock_guard<std::mutex> g(g_tmu);
  if (!g_timing) return;
  start = take_event();
  stop = take_event();
  if (!start || !stop) return;
  on = true;
  (void)hipEventRecord(start, s);
  g_recs.push_back({start, stop, flop});
}

void TimedLaunch::done(hipStream_t s) {
  if (on) (void)hipEventRecord(stop, s);
}

}  // namespace honk

using namespace honk;

extern "C" {

const char* honk_last_error(void) { return get_error(); }
const char* honk_version(void) { return "honk_hip 0.1 gfx950 fp32"; }

int honk_timing_enable(int32_t enable) {
  std::lock_guard<std::mutex> g(g_tmu);
  for (auto& r : g_recs) {
    (void)hipEventSynchronize(r.b);
    g_free.push_back(r.a);
    g_free.push_back(r.b);
  }
  g_recs.clear();
  g_timing = enable != 0;
  return HONK_OK;
}

int honk_timing_read(double* total_ms, int64_t* launches, double* flop) {
  std::lock_guard<std::mutex> g(g_tmu);
  double ms = 0.0, fl = 0.0;
  for (auto& r : g_recs) {
    float t = 0.f;
    HONK_HIP_CHECK(hipEventSynchronize(r.b));
    HONK_HIP_CHECK(hipEventElapsedTime(&t, r.a, r.b));
    ms += t;
    fl += r.flop;
  }
  if (total_ms) *total_ms = ms;
  if (launches) *launches = (int64_t)g_recs.size();
  if (flop) *flop = fl;
  return HONK_OK;
}

}  // extern "C"
