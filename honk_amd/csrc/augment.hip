// Training-set audio augmentation on the device: the per-clip transform of
// SpeechDataset.load_audio (/root/reference/utils/model.py:282-306) --
//   time shift (_timeshift_audio, :264-270): out[i] = data[i + shift] inside the
//     clip, 0 outside (shift < 0 delays, shift > 0 advances);
//   background noise (:302-304): out = clip(amp * noise[off + i] + out, -1, 1) in
//     float32 (NumPy's float32 array arithmetic: the product rounded, then the sum);
//   silence (:290-293): the clip is zeros and the noise is always mixed.
// The random draws (which noise file and offset, the shift, whether and how loud
// the noise is, the 0.7 cache reuse) stay on the host, in the reference's order and
// on its `random` stream (honk_amd/augment.py); this kernel applies them to a whole
// batch of [B][len] PCM in one pass (HBM-bound: one read of the clip and the noise
// slice, one write).
#include "common.h"

namespace honk {
namespace aug {

__global__ __launch_bounds__(256) void augment_kernel(const float* __restrict__ audio, const float* __restrict__ noise,
                                                      const int32_t* __restrict__ shift,
                                                      const int64_t* __restrict__ noise_off,
                                                      const float* __restrict__ amp, const int32_t* __restrict__ flags,
                                                      float* __restrict__ out, int len, int64_t noise_len) {
  const int64_t b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= len) return;
  const int fl = flags[b];
  float v = 0.f;
  if (!(fl & HONK_AUG_SILENCE)) {
    const int j = i + shift[b];
    v = (j >= 0 && j < len) ? audio[b * len + j] : 0.f;
  }
  if (fl & HONK_AUG_NOISE) {
#pragma clang fp contract(off)  // NumPy rounds the product, then the sum: no fma
    const int64_t k = noise_off[b] + i;
    const float nz = (k >= 0 && k < noise_len) ? noise[k] : 0.f;
    const float s = amp[b] * nz + v;
    v = fminf(fmaxf(s, -1.f), 1.f);
    if (s != s) v = s;  // np.clip keeps NaN
  }
  out[b * len + i] = v;
}

}  // namespace aug
}  // namespace honk

using namespace honk;

extern "C" int honk_augment_f32(const float* audio, const float* noise, const int32_t* shift,
                                const int64_t* noise_off, const float* amp, const int32_t* flags, float* out,
                                int64_t batch, int32_t len, int64_t noise_len, void* stream) {
  if (!audio || !shift || !noise_off || !amp || !flags || !out) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 0 || len < 1 || noise_len < 0 || (noise_len > 0 && !noise))
    return fail(HONK_ERR_ARG, "augment: batch=%lld len=%d noise_len=%lld", (long long)batch, len,
                (long long)noise_len);
  if (batch > 65535) return fail(HONK_ERR_ARG, "augment: batch %lld > 65535 per call", (long long)batch);
  if (batch == 0) return HONK_OK;
  hipLaunchKernelGGL(aug::augment_kernel, dim3((unsigned)cdiv(len, 256), (unsigned)batch), dim3(256), 0,
                     (hipStream_t)stream, audio, noise, shift, noise_off, amp, flags, out, len, noise_len);
  HONK_LAUNCH_CHECK("augment_kernel");
  return HONK_OK;
}
