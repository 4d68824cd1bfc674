// The training step's head on gfx950: the spatial mean of SpeechResModel
// (/root/reference/utils/model.py:119-120, x.view(B, C, -1) then torch.mean(x, 2)),
// and the loss nn.CrossEntropyLoss() (mean reduction) of the training loop
// (/root/reference/utils/train.py:99, :129-131), with their backward passes.  The
// Linear layers run on the cnn implicit-GEMM conv kernels as 1x1 convolutions
// (honk_amd/head_train.py).  Every reduction is in a fixed order (deterministic).
#include "common.h"

namespace honk {
namespace head {

// z[r] = (sum_i x[r][i]) / hw: one wave per row, lanes stride the row (float4 when
// hw % 4 == 0), a fixed xor-shuffle tree across the wave
__global__ __launch_bounds__(256) void mean_kernel(const float* __restrict__ x, float* __restrict__ z, int64_t rows,
                                                   int hw) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + r * hw;
  float s = 0.f;
  if ((hw & 3) == 0) {
    for (int i = 4 * lane; i < hw; i += 256) {
      const float4 v = *(const float4*)(xr + i);
      s += (v.x + v.y) + (v.z + v.w);
    }
  } else {
    for (int i = lane; i < hw; i += 64) s += xr[i];
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) z[r] = s / (float)hw;
}

// gx[r][i] = gz[r] / hw (torch.mean's backward: the gradient expanded, divided by hw)
__global__ __launch_bounds__(256) void mean_bwd_kernel(const float* __restrict__ gz, float* __restrict__ gx,
                                                       int64_t total, int hw) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((hw & 3) == 0) {
    const int64_t i4 = 4 * i;
    if (i4 >= total) return;
    const float g = gz[i4 / hw] / (float)hw;
    *(float4*)(gx + i4) = float4{g, g, g, g};
    return;
  }
  if (i >= total) return;
  gx[i] = gz[i / hw] / (float)hw;
}

constexpr int CE_THREADS = 1024;

// log-sum-exp of row z[0..n) (max-shifted, as log_softmax)
__device__ __forceinline__ float row_lse(const float* z, int n, float& mx) {
  mx = z[0];
  for (int j = 1; j < n; ++j) mx = fmaxf(mx, z[j]);
  float s = 0.f;
  for (int j = 0; j < n; ++j) s += expf(z[j] - mx);
  return mx + logf(s);
}

// loss = mean_b (lse(z_b) - z_b[y_b]); one workgroup, rows strided over its threads,
// per-thread double sums combined by a fixed LDS tree.  A label outside [0, n) makes
// the loss NaN (torch raises: head_train.py checks the labels before the launch).
__global__ __launch_bounds__(CE_THREADS) void ce_fwd_kernel(const float* __restrict__ z,
                                                           const int64_t* __restrict__ y, float* __restrict__ loss,
                                                           int64_t batch, int n) {
  __shared__ double red[CE_THREADS];
  double acc = 0.0;
  for (int64_t b = threadIdx.x; b < batch; b += CE_THREADS) {
    const float* zb = z + b * n;
    float mx;
    const float lse = row_lse(zb, n, mx);
    const int64_t t = y[b];
    acc += (t >= 0 && t < n) ? (double)(lse - zb[t]) : (double)NAN;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = CE_THREADS / 2; w >= 1; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = (float)(red[0] / (double)batch);
}

// dz[b][j] = (softmax(z_b)[j] - [j == y_b]) * g / batch, g = *gloss (the upstream
// gradient of the mean loss, a device scalar); a row whose label is outside [0, n)
// gets NaN, as its loss term (head_train.py checks labels before either kernel)
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ y,
                                                     const float* __restrict__ gloss, float* __restrict__ dz,
                                                     int64_t batch, int n) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  const float* zb = z + b * n;
  float mx;
  const float lse = row_lse(zb, n, mx);
  const float scale = *gloss / (float)batch;
  const int64_t t = y[b];
  const bool ok = t >= 0 && t < n;
  for (int j = 0; j < n; ++j) dz[b * n + j] = ok ? (expf(zb[j] - lse) - (j == t ? 1.f : 0.f)) * scale : NAN;
}

}  // namespace head
}  // namespace honk

using namespace honk;

extern "C" int honk_spatial_mean_f32(const float* x, float* z, int64_t rows, int32_t hw, void* stream) {
  if (!x || !z) return fail(HONK_ERR_ARG, "null pointer argument");
  if (rows < 0 || hw < 1) return fail(HONK_ERR_ARG, "spatial mean: rows=%lld hw=%d", (long long)rows, hw);
  if (rows == 0) return HONK_OK;
  if (cdiv(rows, 4) > 0x7fffffff) return fail(HONK_ERR_ARG, "spatial mean: too many rows");
  hipLaunchKernelGGL(head::mean_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, (hipStream_t)stream, x, z, rows,
                     hw);
  HONK_LAUNCH_CHECK("mean_kernel");
  return HONK_OK;
}

extern "C" int honk_spatial_mean_bwd_f32(const float* gz, float* gx, int64_t rows, int32_t hw, void* stream) {
  if (!gz || !gx) return fail(HONK_ERR_ARG, "null pointer argument");
  if (rows < 0 || hw < 1) return fail(HONK_ERR_ARG, "spatial mean bwd: rows=%lld hw=%d", (long long)rows, hw);
  if (rows == 0) return HONK_OK;
  const int64_t total = rows * hw;
  const int64_t threads = (hw & 3) == 0 ? total / 4 : total;
  if (cdiv(threads, 256) > 0x7fffffff) return fail(HONK_ERR_ARG, "spatial mean bwd: too large");
  hipLaunchKernelGGL(head::mean_bwd_kernel, dim3((unsigned)cdiv(threads, 256)), dim3(256), 0, (hipStream_t)stream, gz,
                     gx, total, hw);
  HONK_LAUNCH_CHECK("mean_bwd_kernel");
  return HONK_OK;
}

extern "C" int honk_cross_entropy_f32(const float* logits, const int64_t* labels, float* loss, int64_t batch,
                                      int32_t n, void* stream) {
  if (!logits || !labels || !loss) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 1 || n < 1) return fail(HONK_ERR_ARG, "cross entropy: batch=%lld n=%d", (long long)batch, n);
  hipLaunchKernelGGL(head::ce_fwd_kernel, dim3(1), dim3(head::CE_THREADS), 0, (hipStream_t)stream, logits, labels,
                     loss, batch, n);
  HONK_LAUNCH_CHECK("ce_fwd_kernel");
  return HONK_OK;
}

extern "C" int honk_cross_entropy_bwd_f32(const float* logits, const int64_t* labels, const float* grad_loss,
                                          float* dlogits, int64_t batch, int32_t n, void* stream) {
  if (!logits || !labels || !grad_loss || !dlogits) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 1 || n < 1) return fail(HONK_ERR_ARG, "cross entropy bwd: batch=%lld n=%d", (long long)batch, n);
  if (cdiv(batch, 256) > 0x7fffffff) return fail(HONK_ERR_ARG, "cross entropy bwd: batch too large");
  hipLaunchKernelGGL(head::ce_bwd_kernel, dim3((unsigned)cdiv(batch, 256)), dim3(256), 0, (hipStream_t)stream, logits,
                     labels, grad_loss, dlogits, batch, n);
  HONK_LAUNCH_CHECK("ce_bwd_kernel");
  return HONK_OK;
}
