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


// ---------------------------------------------------------------------------- //
// MFMA path (the default when the shape allows it): the power spectrum of a
// clip's frames as one GEMM on v_mfma_f32_16x16x4_f32,
//     D[c][f] = sum_k T[c][k] * S[k][f],   S[k][f] = xpad[f*hop + k],
//     T[2b][k] = w[k] cos(2 pi b k / N),  T[2b+1][k] = -w[k] sin(2 pi b k / N),
// one workgroup per clip.  The padded signal lives in LDS (S fragments are 16-B
// reads of 4 consecutive samples); T fragments are built on the fly from a
// twiddle table + the window in LDS (index (b*k) mod N stepped incrementally),
// shared by all frame tiles of a column tile.  The accumulator layout gives each
// lane the (re, im) pairs of 2 bins of one frame, so |X|^2 needs no shuffles;
// power goes straight into the mel bins (LDS float atomics over each bin's
// nonzero mel range), then log and the DCT run from LDS.
constexpr int MF_WAVES = 4;
constexpr int MF_MT = 7;  // frame tiles of 16 (frames <= 112)

struct MfmaArgs {
  Args a;
  int ntiles;  // column tiles of 16 (2 * n_bins columns, padded)
  int xp;      // floats of the padded signal image
};

__global__ __launch_bounds__(64 * MF_WAVES) void mfcc_mfma_kernel(MfmaArgs ma) {
  const Args& a = ma.a;
  extern __shared__ __attribute__((aligned(16))) float smf[];
  const int N = a.n_fft, F = a.frames, NB = a.n_bins, NM = a.n_mels;
  float* xpad = smf;                  // [xp]
  float* win = xpad + ma.xp;          // [N]
  float* tw = win + N;                // [2N] cos | sin
  float* melw = tw + 2 * N;           // [NM][NB]
  float* melacc = melw + NM * NB;     // [MF_MT*16][NM]
  int* brange = (int*)(melacc + MF_MT * 16 * NM);  // [NB] first | last << 16
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int b = blockIdx.x;
  const int pad = N / 2;
  const float* x = a.pcm + (int64_t)b * a.S;
  for (int i = tid; i < ma.xp; i += blockDim.x)
    xpad[i] = (i < a.S + 2 * pad) ? x[reflect(i - pad, a.S)] : 0.f;
  for (int t = tid; t < N; t += blockDim.x) {
    float sn, cs;
    sincosf(6.283185307179586f * (float)t / (float)N, &sn, &cs);
    win[t] = a.window[t];
    tw[t] = cs;
    tw[N + t] = -sn;
  }
  for (int i = tid; i < NM * NB; i += blockDim.x) melw[i] = a.melw[i];
  for (int i = tid; i < MF_MT * 16 * NM; i += blockDim.x) melacc[i] = 0.f;
  __syncthreads();
  for (int bb = tid; bb < NB; bb += blockDim.x) {
    int lo = NM, hi = -1;
    for (int m = 0; m < NM; ++m)
      if (melw[m * NB + bb] != 0.f) { lo = min(lo, m); hi = max(hi, m); }
    brange[bb] = (hi < lo) ? 0x7fff : (lo | (hi << 16));
  }
  __syncthreads();

  const int nkb = N / 16;
  for (int t = wave; t < ma.ntiles; t += MF_WAVES) {
    // this lane's T row: column c = 16 t + i16 -> bin c/2, cos (even) / -sin (odd)
    const int c = 16 * t + i16;
    const int bin = c >> 1;
    const float* twp = tw + ((c & 1) ? N : 0);
    const int bstep = (int)(((int64_t)bin * 16) % N);
    const int bj = bin % N;
    int idx = (int)(((int64_t)bin * (4 * g)) % N);  // (bin * k) mod N at k = 16 kb + 4 g
    f32x4 acc[MF_MT];
#pragma unroll
    for (int m = 0; m < MF_MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kb = 0; kb < nkb; ++kb) {
      const int k0 = 16 * kb + 4 * g;
      float tv[4];
      int ij = idx;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        tv[j] = twp[ij] * win[k0 + j];
        ij += bj;
        if (ij >= N) ij -= N;
      }
      idx += bstep;
      if (idx >= N) idx -= N;
#pragma unroll
      for (int m = 0; m < MF_MT; ++m) {
        const f32x4 sv = *(const f32x4*)(xpad + (16 * m + i16) * a.hop + k0);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(tv[j], sv[j], acc[m], 0, 0, 0);
      }
    }
    // lane holds D[c = 16 t + 4 g + r][f = 16 m + i16]: bins 8 t + 2 g + {0, 1}
#pragma unroll
    for (int m = 0; m < MF_MT; ++m) {
      const int f = 16 * m + i16;
      if (f >= F) continue;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int bb = 8 * t + 2 * g + q;
        if (bb >= NB) continue;
        const float p = acc[m][2 * q] * acc[m][2 * q] + acc[m][2 * q + 1] * acc[m][2 * q + 1];
        const int r = brange[bb];
        for (int mm = r & 0xffff; mm <= (r >> 16); ++mm) atomicAdd(&melacc[f * NM + mm], melw[mm * NB + bb] * p);
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < F * NM; i += blockDim.x) {
    const float v = melacc[i];
    melacc[i] = v > 0.f ? logf(v) : v;
  }
  __syncthreads();
  for (int q = tid; q < F * a.n_dct; q += blockDim.x) {
    const int f = q / a.n_dct, i = q - f * a.n_dct;
    const float* d = a.dct + (int64_t)i * NM;
    float acc = 0.f;
    for (int m = 0; m < NM; ++m) acc = fmaf(d[m], melacc[f * NM + m], acc);
    a.out[((int64_t)b * F + f) * a.n_dct + i] = acc;
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
  // MFMA path: frames <= 112, n_fft and hop multiples of 16 / 4, its LDS plan fits
  {
    mfcc::MfmaArgs ma;
    ma.a = a;
    ma.ntiles = (int)cdiv(2 * a.n_bins, 16);
    ma.xp = (mfcc::MF_MT * 16 - 1) * hop + n_fft;
    const size_t lds = sizeof(float) * ((size_t)ma.xp + 3 * n_fft + (size_t)n_mels * a.n_bins +
                                        mfcc::MF_MT * 16 * n_mels) + sizeof(int) * a.n_bins;
    if (a.frames <= mfcc::MF_MT * 16 && n_fft % 16 == 0 && hop % 4 == 0 && lds <= 160 * 1024 &&
        !getenv("HONK_MFCC_VALU")) {
      if (lds > 64 * 1024) HONK_HIP_CHECK(hipFuncSetAttribute((const void*)mfcc::mfcc_mfma_kernel,
                                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(mfcc::mfcc_mfma_kernel, dim3((unsigned)batch), dim3(64 * mfcc::MF_WAVES), lds,
                         (hipStream_t)stream, ma);
      HONK_LAUNCH_CHECK("mfcc_mfma_kernel");
      return HONK_OK;
    }
  }
  const int span = (mfcc::FPB - 1) * hop + n_fft;
  const size_t lds = sizeof(float) * ((size_t)span + 2 * n_fft + mfcc::FPB * (a.n_bins + n_mels));
  if (lds > 64 * 1024) return fail(HONK_ERR_UNSUPPORTED, "mfcc: n_fft too large for the LDS plan");
  dim3 grid((unsigned)cdiv(a.frames, mfcc::FPB), (unsigned)batch);
  hipLaunchKernelGGL(mfcc::mfcc_kernel, grid, dim3(256), lds, (hipStream_t)stream, a);
  HONK_LAUNCH_CHECK("mfcc_kernel");
  return HONK_OK;
}
