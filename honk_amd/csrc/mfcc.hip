// MFCC front-end on the GPU: AudioPreprocessor.compute_mfccs
// (/root/reference/utils/manage_audio.py:30-42, librosa 0.6 semantics), batched.
//
//   pcm [B][S] f32 (int16/32768) -> reflect-pad n_fft/2 -> frames (hop) ->
//   periodic Hann window -> |rDFT|^2 (n_fft/2+1 bins) -> mel filterbank ->
//   log of the positive entries -> DCT basis -> out [B][frames][n_dct] f32
//
// One workgroup per (clip, FPB frames): the padded samples of its frames are
// staged in LDS; each thread computes the power of some (frame, bin) pairs by a
// direct DFT with a twiddle table in LDS (n_fft = 480 is not a power of two;
// 23 MMAC/clip is far below the conv net behind it); mel + log + DCT follow in
// the same workgroup from LDS.  The mel and DCT matrices come from the host
// (honk_amd/audio.py builds them exactly as librosa 0.6 does).
#include "common.h"

namespace honk {
namespace mfcc {

constexpr int FPB = 4;  // frames per workgroup

struct Args {
  const float* pcm;     // [B][S]
  const float* window;  // [n_fft]
  const float* melw;    // [n_mels][n_bins]
  const float* dct;     // [n_dct][n_mels]
  float* out;           // [B][frames][n_dct]
  int S, n_fft, hop, n_bins, n_mels, n_dct, frames;
};

__device__ __forceinline__ int reflect(int i, int n) {
  // numpy 'reflect' padding (no edge repeat), valid for |overhang| < n
  if (i < 0) return -i;
  if (i >= n) return 2 * n - 2 - i;
  return i;
}

__global__ __launch_bounds__(256) void mfcc_kernel(Args a) {
  extern __shared__ float sm[];
  const int b = blockIdx.y;
  const int f0 = blockIdx.x * FPB;
  const int nf = min(FPB, a.frames - f0);
  const int pad = a.n_fft / 2;
  const int span = (FPB - 1) * a.hop + a.n_fft;
  float* xs = sm;                          // [span] windowless samples
  float* tw_c = xs + span;                 // [n_fft] cos(2 pi t / n_fft)
  float* tw_s = tw_c + a.n_fft;            // [n_fft] sin
  float* pw = tw_s + a.n_fft;              // [FPB][n_bins] power
  float* lm = pw + FPB * a.n_bins;         // [FPB][n_mels] log-mel
  const float* x = a.pcm + (int64_t)b * a.S;
  for (int i = threadIdx.x; i < span; i += blockDim.x) {
    const int gi = f0 * a.hop + i - pad;
    xs[i] = (f0 * a.hop + i < a.S + 2 * pad) ? x[reflect(gi, a.S)] : 0.f;
  }
  for (int t = threadIdx.x; t < a.n_fft; t += blockDim.x) {
    float s, c;
    sincosf(6.283185307179586f * (float)t / (float)a.n_fft, &s, &c);
    tw_c[t] = c;
    tw_s[t] = s;
  }
  __syncthreads();
  // power spectrum: X_k = sum_n w[n] x[n] e^{-2 pi i k n / N}
  for (int q = threadIdx.x; q < nf * a.n_bins; q += blockDim.x) {
    const int f = q / a.n_bins, k = q - f * a.n_bins;
    const float* xf = xs + f * a.hop;
    float re = 0.f, im = 0.f;
    int idx = 0;
    for (int n = 0; n < a.n_fft; ++n) {
      const float v = xf[n] * a.window[n];
      re = fmaf(v, tw_c[idx], re);
      im = fmaf(v, tw_s[idx], im);
      idx += k;
      if (idx >= a.n_fft) idx -= a.n_fft;
    }
    pw[f * a.n_bins + k] = re * re + im * im;
  }
  __syncthreads();
  // mel filterbank + log of positive entries (manage_audio.py:31-39)
  for (int q = threadIdx.x; q < nf * a.n_mels; q += blockDim.x) {
    const int f = q / a.n_mels, m = q - f * a.n_mels;
    const float* w = a.melw + (int64_t)m * a.n_bins;
    float s = 0.f;
    for (int k = 0; k < a.n_bins; ++k) s = fmaf(w[k], pw[f * a.n_bins + k], s);
    lm[f * a.n_mels + m] = s > 0.f ? logf(s) : s;
  }
  __syncthreads();
  // DCT (manage_audio.py:40): out[frame][i] = sum_m dct[i][m] * logmel[m]
  for (int q = threadIdx.x; q < nf * a.n_dct; q += blockDim.x) {
    const int f = q / a.n_dct, i = q - f * a.n_dct;
    const float* d = a.dct + (int64_t)i * a.n_mels;
    float s = 0.f;
    for (int m = 0; m < a.n_mels; ++m) s = fmaf(d[m], lm[f * a.n_mels + m], s);
    a.out[((int64_t)b * a.frames + f0 + f) * a.n_dct + i] = s;
  }
}

}  // namespace mfcc
}  // namespace honk

using namespace honk;

extern "C" int honk_mfcc_f32(const float* pcm, int64_t batch, int32_t samples, const float* window,
                             int32_t n_fft, int32_t hop, const float* mel_weights, int32_t n_mels,
                             const float* dct, int32_t n_dct, float* out, void* stream) {
  if (batch < 0 || samples < 1 || n_fft < 2 || hop < 1 || n_mels < 1 || n_dct < 1)
    return fail(HONK_ERR_ARG, "bad mfcc arguments");
  if (batch == 0) return HONK_OK;
  if (!pcm || !window || !mel_weights || !dct || !out) return fail(HONK_ERR_ARG, "null pointer argument");
  if (n_fft / 2 >= samples) return fail(HONK_ERR_ARG, "reflect padding needs samples > n_fft/2");
  if (batch > 65535) return fail(HONK_ERR_ARG, "batch > 65535 per call");
  mfcc::Args a;
  a.pcm = pcm; a.window = window; a.melw = mel_weights; a.dct = dct; a.out = out;
  a.S = samples; a.n_fft = n_fft; a.hop = hop; a.n_bins = n_fft / 2 + 1; a.n_mels = n_mels; a.n_dct = n_dct;
  a.frames = 1 + samples / hop;  // centre padding: 1 + (S + 2*(n_fft/2) - n_fft) / hop for even n_fft
  const int span = (mfcc::FPB - 1) * hop + n_fft;
  const size_t lds = sizeof(float) * ((size_t)span + 2 * n_fft + mfcc::FPB * (a.n_bins + n_mels));
  if (lds > 64 * 1024) return fail(HONK_ERR_UNSUPPORTED, "mfcc: n_fft too large for the LDS plan");
  dim3 grid((unsigned)cdiv(a.frames, mfcc::FPB), (unsigned)batch);
  hipLaunchKernelGGL(mfcc::mfcc_kernel, grid, dim3(256), lds, (hipStream_t)stream, a);
  HONK_LAUNCH_CHECK("mfcc_kernel");
  return HONK_OK;
}
