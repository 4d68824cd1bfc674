// SpeechModel forward (cnn-trad-pool2, cnn-one-*, cnn-tpool*, cnn-tstride*) for
// gfx950, fp32.  Reference: /root/reference/utils/model.py:123-205.
//
//   conv1 (+bias, ReLU) -> maxpool1 -> [conv2 (+bias, ReLU) -> maxpool2]
//   -> flatten (c,h,w) -> [lin] -> [dnn1 (+ReLU unless tf_variant)] -> [dnn2]
//   -> output                                  (dropout = identity in eval)
//
// Every conv and every Linear is one implicit GEMM on fp32 MFMA
// (v_mfma_f32_16x16x4_f32), computed transposed so stores are coalesced:
//     D[n][m] = bias[n] + sum_k W[n][k] * X[k][m]
// n = out channel, m = (clip, oh, ow) output pixel, k = (ci, kh, kw) -- the
// OIHW weight tensor IS the [N][K] operand, X is gathered on the fly from the
// NCHW input (valid convolution, stride (sh, sw)).  A Linear is the same GEMM
// with H = W = KH = KW = 1.  Activations stay NCHW so flatten is free.
#include "common.h"

namespace honk {
namespace cnn {

constexpr int BM = 64;   // output pixels per block
constexpr int BN = 64;   // output channels per block
constexpr int BK = 16;   // reduction slice per LDS stage
constexpr int PAD = 4;   // LDS row padding (floats)

struct GemmArgs {
  const float* in;   // NCHW [B][Cin][H][W]
  const float* w;    // [N][K]
  const float* bias; // [N] or nullptr
  float* out;        // NCHW [B][N][OH][OW]
  int64_t M;         // B * OH * OW
  int N, K;
  int Cin, H, W, KH, KW, SH, SW, OH, OW;
  int relu;
};

// 256 threads = 4 waves in a 2 (n) x 2 (m) grid; each wave owns a 32x32 output
// tile = 2x2 MFMA 16x16 tiles.  LDS: Ws[k][n], Xs[k][m], double-buffered via
// registers (global loads for slice t+1 are issued before the MFMAs of slice t).
__global__ __launch_bounds__(256) void conv_gemm_kernel(GemmArgs a) {
  __shared__ float Ws[2][BK][BN + PAD];
  __shared__ float Xs[2][BK][BM + PAD];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wn = wave >> 1, wm = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int OHW = a.OH * a.OW;
  const int KHW = a.KH * a.KW;
  const int64_t CinHW = (int64_t)a.Cin * a.H * a.W;

  // X loads: this thread always stages pixel column mm = tid % 64, rows kk = tid/64 + 4r
  const int mm = tid & 63;
  const int kq = tid >> 6;
  const int64_t mg = m0 + mm;
  const bool mvalid = mg < a.M;
  int64_t xbase = 0;
  if (mvalid) {
    const int64_t b = mg / OHW;
    const int pix = (int)(mg - b * OHW);
    const int oh = pix / a.OW, ow = pix - oh * a.OW;
    xbase = b * CinHW + (int64_t)(oh * a.SH) * a.W + ow * a.SW;
  }
  // W loads: thread stages rows nn = tid/16 + 16r, column kk = tid % 16
  const int wk = tid & 15;
  const int wr = tid >> 4;

  float xr[4], wv[4];
  auto load_slice = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int k = k0 + kq + 4 * r;
      float v = 0.f;
      if (mvalid && k < a.K) {
        const int ci = k / KHW;
        const int rem = k - ci * KHW;
        const int kh = rem / a.KW, kw = rem - kh * a.KW;
        v = a.in[xbase + (int64_t)ci * a.H * a.W + kh * a.W + kw];
      }
      xr[r] = v;
      const int n = n0 + wr + 16 * r;
      const int kk = k0 + wk;
      wv[r] = (n < a.N && kk < a.K) ? a.w[(int64_t)n * a.K + kk] : 0.f;
    }
  };
  auto store_slice = [&](int buf) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      Xs[buf][kq + 4 * r][mm] = xr[r];
      Ws[buf][wk][wr + 16 * r] = wv[r];
    }
  };

  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nslices = (a.K + BK - 1) / BK;
  load_slice(0);
  store_slice(0);
  __syncthreads();
  for (int t = 0; t < nslices; ++t) {
    const int buf = t & 1;
    if (t + 1 < nslices) load_slice((t + 1) * BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kk = ks * 4 + (lane >> 4);
      float av[2], bv[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) av[i] = Ws[buf][kk][wn * 32 + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) bv[j] = Xs[buf][kk][wm * 32 + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < nslices) store_slice(buf ^ 1);
    __syncthreads();
  }

  // epilogue: D[n][m]; lane holds rows n = (lane>>4)*4 + r, column m = lane & 15
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t m = m0 + wm * 32 + j * 16 + (lane & 15);
    if (m >= a.M) continue;
    const int64_t b = m / OHW;
    const int pix = (int)(m - b * OHW);
    float* ob = a.out + b * (int64_t)a.N * OHW + pix;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + i * 16 + (lane >> 4) * 4 + r;
        if (n < a.N) {
          float v = acc[i][j][r] + (a.bias ? a.bias[n] : 0.f);
          if (a.relu) v = fmaxf(v, 0.f);
          ob[(int64_t)n * OHW] = v;
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void maxpool_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                      int64_t planes, int H, int W, int KH, int KW) {
  const int PH = H / KH, PW = W / KW;
  const int64_t total = planes * PH * PW;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int pw = (int)(i % PW);
  const int64_t t = i / PW;
  const int ph = (int)(t % PH);
  const int64_t pl = t / PH;
  const float* p = in + pl * H * W + (int64_t)(ph * KH) * W + pw * KW;
  float m = p[0];
  for (int a = 0; a < KH; ++a)
    for (int b = 0; b < KW; ++b) {
      const float v = p[a * W + b];
      m = (v > m || v != v) ? v : m;  // NaN propagates like torch
    }
  out[i] = m;
}

static int launch_gemm(const GemmArgs& a, hipStream_t st) {
  if (a.M <= 0 || a.N <= 0) return HONK_OK;
  const int64_t gm = cdiv(a.M, BM);
  if (gm > 0x7fffffff) return fail(HONK_ERR_ARG, "GEMM too large (M=%lld)", (long long)a.M);
  dim3 grid((unsigned)gm, (unsigned)cdiv(a.N, BN));
  TimedLaunch tl(st, 2.0 * (double)a.M * a.N * a.K);
  hipLaunchKernelGGL(conv_gemm_kernel, grid, dim3(256), 0, st, a);
  tl.done(st);
  HONK_LAUNCH_CHECK("conv_gemm_kernel");
  return HONK_OK;
}

static int conv(const float* in, const float* w, const float* bias, float* out, int64_t batch, int cin,
                int h, int wd, int cout, int kh, int kw, int sh, int sw, int relu, hipStream_t st) {
  if (kh > h || kw > wd || sh < 1 || sw < 1 || cin < 1 || cout < 1)
    return fail(HONK_ERR_ARG, "bad conv geometry (cin=%d %dx%d k=%dx%d s=%dx%d)", cin, h, wd, kh, kw, sh, sw);
  GemmArgs a;
  a.in = in; a.w = w; a.bias = bias; a.out = out;
  a.Cin = cin; a.H = h; a.W = wd; a.KH = kh; a.KW = kw; a.SH = sh; a.SW = sw;
  a.OH = (h - kh) / sh + 1;
  a.OW = (wd - kw) / sw + 1;
  a.M = batch * a.OH * a.OW;
  a.N = cout;
  a.K = cin * kh * kw;
  a.relu = relu;
  return launch_gemm(a, st);
}

static int linear(const float* x, const float* w, const float* b, float* y, int64_t m, int k, int n,
                  int relu, hipStream_t st) {
  return conv(x, w, b, y, m, k, 1, 1, n, 1, 1, 1, 1, relu, st);
}

static int maxpool(const float* in, float* out, int64_t planes, int h, int w, int kh, int kw, hipStream_t st) {
  if (kh < 1 || kw < 1 || kh > h || kw > w) return fail(HONK_ERR_ARG, "bad pool %dx%d on %dx%d", kh, kw, h, w);
  const int64_t total = planes * (h / kh) * (w / kw);
  if (total == 0) return HONK_OK;
  hipLaunchKernelGGL(maxpool_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, in, out, planes, h, w,
                     kh, kw);
  HONK_LAUNCH_CHECK("maxpool_kernel");
  return HONK_OK;
}

struct Shapes {
  int oh1, ow1, ph1, pw1, oh2, ow2, ph2, pw2;
  int64_t a1, p1, a2, p2;  // floats per clip of conv1 / pool1 / conv2 / pool2 outputs
  int flat;
  int64_t vec;  // floats per clip of the largest vector stage
};

static int shapes(const honk_cnn_desc* d, Shapes* s) {
  if (!d) return fail(HONK_ERR_ARG, "null descriptor");
  if (d->height < 1 || d->width < 1 || d->n_labels < 1 || d->c1_out < 1 || d->c1_kh < 1 || d->c1_kw < 1 ||
      d->c1_sh < 1 || d->c1_sw < 1 || d->p1_h < 1 || d->p1_w < 1 || d->c1_kh > d->height || d->c1_kw > d->width)
    return fail(HONK_ERR_ARG, "bad cnn descriptor");
  s->oh1 = (d->height - d->c1_kh) / d->c1_sh + 1;
  s->ow1 = (d->width - d->c1_kw) / d->c1_sw + 1;
  s->ph1 = s->oh1 / d->p1_h;
  s->pw1 = s->ow1 / d->p1_w;
  if (s->ph1 < 1 || s->pw1 < 1) return fail(HONK_ERR_ARG, "pool1 larger than conv1 output");
  s->a1 = (int64_t)d->c1_out * s->oh1 * s->ow1;
  s->p1 = (int64_t)d->c1_out * s->ph1 * s->pw1;
  s->flat = (int)s->p1;
  s->a2 = s->p2 = 0;
  if (d->has_conv2) {
    if (d->c2_out < 1 || d->c2_kh < 1 || d->c2_kw < 1 || d->c2_sh < 1 || d->c2_sw < 1 || d->p2_h < 1 ||
        d->p2_w < 1 || d->c2_kh > s->ph1 || d->c2_kw > s->pw1)
      return fail(HONK_ERR_ARG, "bad conv2 descriptor");
    s->oh2 = (s->ph1 - d->c2_kh) / d->c2_sh + 1;
    s->ow2 = (s->pw1 - d->c2_kw) / d->c2_sw + 1;
    s->ph2 = s->oh2 / d->p2_h;
    s->pw2 = s->ow2 / d->p2_w;
    if (s->ph2 < 1 || s->pw2 < 1) return fail(HONK_ERR_ARG, "pool2 larger than conv2 output");
    s->a2 = (int64_t)d->c2_out * s->oh2 * s->ow2;
    s->p2 = (int64_t)d->c2_out * s->ph2 * s->pw2;
    s->flat = (int)s->p2;
  }
  int64_t v = 32;
  if (d->dnn1 > v) v = d->dnn1;
  if (d->dnn2 > v) v = d->dnn2;
  s->vec = v;
  return HONK_OK;
}

// ping-pong buffers A/B hold the per-stage activations of a chunk of clips
static int64_t per_clip_floats(const Shapes& s) {
  int64_t m = s.a1;
  if (s.p1 > m) m = s.p1;
  if (s.a2 > m) m = s.a2;
  if (s.p2 > m) m = s.p2;
  if (s.vec > m) m = s.vec;
  return m;
}

static int64_t chunk_clips(const Shapes& s, int64_t batch) {
  int64_t ch = (int64_t)((size_t)2 << 30) / (per_clip_floats(s) * 4);  // ~2 GiB per buffer
  if (const char* e = getenv("HONK_CNN_CHUNK")) ch = atoll(e);
  if (ch < 1) ch = 1;
  return batch < ch ? batch : ch;
}

}  // namespace cnn
}  // namespace honk

using namespace honk;
using namespace honk::cnn;

extern "C" {

int honk_conv2d_f32(const float* in, const float* w, const float* bias, float* out, int64_t batch, int32_t cin,
                    int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw, int32_t sh, int32_t sw,
                    int32_t relu, void* stream) {
  if (!in || !w || !out) return fail(HONK_ERR_ARG, "null pointer argument");
  return conv(in, w, bias, out, batch, cin, h, w_, cout, kh, kw, sh, sw, relu, (hipStream_t)stream);
}

int honk_maxpool2d_f32(const float* in, float* out, int64_t batch, int32_t c, int32_t h, int32_t w, int32_t kh,
                       int32_t kw, void* stream) {
  if (!in || !out) return fail(HONK_ERR_ARG, "null pointer argument");
  return maxpool(in, out, batch * c, h, w, kh, kw, (hipStream_t)stream);
}

int honk_linear_f32(const float* x, const float* w, const float* b, float* y, int64_t m, int32_t k, int32_t n,
                    int32_t relu, void* stream) {
  if (!x || !w || !y) return fail(HONK_ERR_ARG, "null pointer argument");
  if (k < 1 || n < 1 || m < 0) return fail(HONK_ERR_ARG, "bad linear shape");
  return linear(x, w, b, y, m, k, n, relu, (hipStream_t)stream);
}

size_t honk_cnn_workspace_bytes(const honk_cnn_desc* d, int64_t batch) {
  Shapes s;
  if (shapes(d, &s) != HONK_OK || batch < 1) return 0;
  return (size_t)2 * chunk_clips(s, batch) * per_clip_floats(s) * sizeof(float);
}

int honk_cnn_forward(const honk_cnn_desc* d, const float* const* t, const float* x, float* logits, int64_t batch,
                     void* workspace, size_t ws_bytes, void* stream) {
  Shapes s;
  int rc = shapes(d, &s);
  if (rc) return rc;
  if (batch < 0) return fail(HONK_ERR_ARG, "negative batch");
  if (batch == 0) return HONK_OK;
  if (!t || !x || !logits || !workspace) return fail(HONK_ERR_ARG, "null pointer argument");
  if (!t[0] || !t[1] || !t[10] || !t[11]) return fail(HONK_ERR_ARG, "conv1/output tensors are required");
  if (d->has_conv2 && (!t[2] || !t[3])) return fail(HONK_ERR_ARG, "conv2 tensors missing");
  if (d->has_lin && (!t[4] || !t[5])) return fail(HONK_ERR_ARG, "lin tensors missing");
  if (d->dnn1 && (!t[6] || !t[7])) return fail(HONK_ERR_ARG, "dnn1 tensors missing");
  if (d->dnn2 && (!t[8] || !t[9])) return fail(HONK_ERR_ARG, "dnn2 tensors missing");
  if (d->dnn2 && !d->dnn1) return fail(HONK_ERR_ARG, "dnn2 without dnn1");
  const size_t need = honk_cnn_workspace_bytes(d, batch);
  if (ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int64_t chunk = chunk_clips(s, batch);
  float* A = (float*)workspace;
  float* B = A + chunk * per_clip_floats(s);

  for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
    const int64_t n = (batch - c0 < chunk) ? batch - c0 : chunk;
    const float* xin = x + c0 * d->height * d->width;
    // conv1 + ReLU (model.py:187) -> A ; pool1 (:189) -> B (skip when 1x1)
    rc = conv(xin, t[0], t[1], A, n, 1, d->height, d->width, d->c1_out, d->c1_kh, d->c1_kw, d->c1_sh, d->c1_sw, 1,
              st);
    if (rc) return rc;
    const float* cur = A;
    float* other = B;
    if (d->p1_h * d->p1_w > 1) {
      rc = maxpool(A, B, n * d->c1_out, s.oh1, s.ow1, d->p1_h, d->p1_w, st);
      if (rc) return rc;
      cur = B;
      other = A;
    }
    if (d->has_conv2) {  // model.py:190-193
      rc = conv(cur, t[2], t[3], other, n, d->c1_out, s.ph1, s.pw1, d->c2_out, d->c2_kh, d->c2_kw, d->c2_sh,
                d->c2_sw, 1, st);
      if (rc) return rc;
      const float* c2 = other;
      float* o2 = (float*)cur;
      if (d->p2_h * d->p2_w > 1) {
        rc = maxpool(c2, o2, n * d->c2_out, s.oh2, s.ow2, d->p2_h, d->p2_w, st);
        if (rc) return rc;
        cur = o2;
        other = (float*)c2;
      } else {
        cur = c2;
        other = o2;
      }
    }
    int width = s.flat;  // flatten is free: NCHW (model.py:194)
    if (d->has_lin) {    // :195-196
      rc = linear(cur, t[4], t[5], other, n, width, 32, 0, st);
      if (rc) return rc;
      width = 32;
      float* tmp = other; other = (float*)cur; cur = tmp;
    }
    if (d->dnn1) {       // :197-201
      rc = linear(cur, t[6], t[7], other, n, width, d->dnn1, d->dnn1_relu, st);
      if (rc) return rc;
      width = d->dnn1;
      float* tmp = other; other = (float*)cur; cur = tmp;
    }
    if (d->dnn2) {       // :202-204
      rc = linear(cur, t[8], t[9], other, n, width, d->dnn2, 0, st);
      if (rc) return rc;
      width = d->dnn2;
      float* tmp = other; other = (float*)cur; cur = tmp;
    }
    rc = linear(cur, t[10], t[11], logits + c0 * d->n_labels, n, width, d->n_labels, 0, st);  // :205
    if (rc) return rc;
  }
  return HONK_OK;
}

}  // extern "C"
