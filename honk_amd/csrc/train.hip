// Training-step helpers for the data-parallel train() path (C5).
//
// honk_sgd_step_f32: one fused pass of torch.optim.SGD over a FLAT parameter
// bucket (utils/train.py:99 -- lr, momentum, weight_decay, nesterov; dampening
// 0), applied after the bucket's gradients were all-reduced (RCCL) and scaled:
//     g  = grad * grad_scale + weight_decay * p
//     buf = momentum * buf + g          (buf starts at 0 == torch's clone on step 1)
//     d  = nesterov ? g + momentum * buf : buf         (momentum == 0: d = g)
//     p  = p - lr * d
// One launch per step, 16 B per lane, HBM-bound (3 reads + 2 writes per param).
#include "common.h"

namespace honk {
namespace train {

__global__ __launch_bounds__(256) void sgd_kernel(float* __restrict__ p, const float* __restrict__ grad,
                                                  float* __restrict__ buf, int64_t n, float lr, float momentum,
                                                  float wd, float gscale, int nesterov) {
#pragma clang fp contract(off)  // round like torch.optim.SGD: separate mul and add
  const int64_t i4 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i4 >= n) return;
  if (i4 + 4 <= n && ((((uintptr_t)p) | ((uintptr_t)grad) | ((uintptr_t)buf)) & 15) == 0) {
    f32x4 pv = *(f32x4*)(p + i4);
    const f32x4 gv = *(const f32x4*)(grad + i4);
    f32x4 bv = momentum != 0.f ? *(f32x4*)(buf + i4) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float g = gv[k] * gscale;
      if (wd != 0.f) g = g + wd * pv[k];
      float d = g;
      if (momentum != 0.f) {
        bv[k] = momentum * bv[k] + g;
        d = nesterov ? g + momentum * bv[k] : bv[k];
      }
      pv[k] = pv[k] - lr * d;
    }
    *(f32x4*)(p + i4) = pv;
    if (momentum != 0.f) *(f32x4*)(buf + i4) = bv;
    return;
  }
  for (int64_t i = i4; i < n && i < i4 + 4; ++i) {
    float g = grad[i] * gscale;
    if (wd != 0.f) g = g + wd * p[i];
    float d = g;
    if (momentum != 0.f) {
      const float b = momentum * buf[i] + g;
      buf[i] = b;
      d = nesterov ? g + momentum * b : b;
    }
    p[i] = p[i] - lr * d;
  }
}

}  // namespace train
}  // namespace honk

using namespace honk;

extern "C" int honk_sgd_step_f32(float* params, const float* grads, float* momentum_buf, int64_t n, float lr,
                                 float momentum, float weight_decay, float grad_scale, int32_t nesterov,
                                 void* stream) {
  if (n < 0) return fail(HONK_ERR_ARG, "negative size");
  if (n == 0) return HONK_OK;
  if (!params || !grads || (momentum != 0.f && !momentum_buf)) return fail(HONK_ERR_ARG, "null pointer argument");
  const int64_t threads = cdiv(n, 4);
  hipLaunchKernelGGL(train::sgd_kernel, dim3((unsigned)cdiv(threads, 256)), dim3(256), 0, (hipStream_t)stream,
                     params, grads, momentum_buf, n, lr, momentum, weight_decay, grad_scale, nesterov);
  HONK_LAUNCH_CHECK("sgd_kernel");
  return HONK_OK;
}
