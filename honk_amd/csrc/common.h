// Shared host/device helpers for libhonk_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/honk_hip.h"

namespace honk {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// thread-local last error; set by fail(), read through honk_last_error()
void set_error(const char* fmt, ...);
const char* get_error();

inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  set_error("%s", buf);
  return code;
}

#define HONK_HIP_CHECK(expr)                                                           \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      return ::honk::fail(HONK_ERR_HIP, "%s failed: %s (%s:%d)", #expr,                \
                          hipGetErrorString(_e), __FILE__, __LINE__);                  \
  } while (0)

#define HONK_LAUNCH_CHECK(name)                                                        \
  do {                                                                                 \
    hipError_t _e = hipGetLastError();                                                 \
    if (_e != hipSuccess)                                                              \
      return ::honk::fail(HONK_ERR_HIP, "launch of %s failed: %s", name,               \
                          hipGetErrorString(_e));                                      \
  } while (0)

// ReLU with torch.relu's NaN behaviour: x <= 0 (either zero included) -> +0,
// otherwise x -- a NaN of either sign stays a NaN.  IEEE 754-2019 maximum(x, +0)
// (gfx950's v_maximum3_f32: one VALU; -0 < +0 and a NaN operand gives a NaN) -- fmaxf
// (maxNum) and an integer max on the bits would turn a NaN, resp. a -NaN, into 0, and a
// compare + select costs two VALU.
__device__ __forceinline__ float relu_keepnan(float x) { return __builtin_elementwise_maximum(x, 0.f); }

// sum over the 16 lanes of a row (lane group) by DPP: quad_perm [1,0,3,2], [2,3,0,1],
// row_half_mirror, row_mirror -- after each step the lanes of the combined span hold
// the same value (IEEE addition is commutative), so every lane of the row returns the
// row's sum; VALU only (a __shfl_xor tree goes through the LDS crossbar)
__device__ __forceinline__ float sum16_dpp(float t) {
  // (mov_dpp with bound_ctrl: every source lane of these patterns exists, and the
  // combiner then folds each step into one v_add_f32 with a DPP operand -- update_dpp's
  // explicit old value kept a separate v_mov_b32_dpp and a temporary per step, which
  // spilled the row-band kernel's last layer: 102 vs 65 us per res8 launch)
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0xB1, 0xF, 0xF, true));
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0x4E, 0xF, 0xF, true));
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0x141, 0xF, 0xF, true));
  t += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0x140, 0xF, 0xF, true));
  return t;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// number of CUs of the current device (cached per device)
int cu_count();

// kernel timing window (honk_timing_*): wraps one launch with hipEvents
struct TimedLaunch {
  hipEvent_t start = nullptr, stop = nullptr;
  bool on = false;
  TimedLaunch(hipStream_t s, double flop);
  void done(hipStream_t s);
};

}  // namespace honk
