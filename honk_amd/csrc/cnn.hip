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

constexpr int BM = 128;  // output pixels per block
constexpr int BN = 64;   // output channels per block
constexpr int BK = 32;   // reduction slice per LDS stage
constexpr int PADM = 4;  // LDS row padding (floats)
constexpr int KTAB = 4096;  // max K with an LDS k->offset table (else computed)

struct GemmArgs {
  const float* in;   // NCHW [B][Cin][H][W]
  const float* w;    // [N][K]
  const float* bias; // [N] or nullptr
  float* out;        // NCHW [B][N][OH][OW], or [B][N][OH/2][OW/2] when pool2 fused
  int64_t M;         // GEMM rows: B*OH*OW, or B*PH*PW*4 (pool2: 4 window members per pooled pixel)
  int N, K;
  int Cin, H, W, KH, KW, SH, SW, OH, OW;
  int PH, PW;        // pooled output dims (pool2 fused)
  int relu;
};

// D[n][m] = act(bias[n] + sum_k W[n][k] * X[k][m]) on v_mfma_f32_16x16x4_f32.
// 256 threads = 4 waves; wave w owns pixels [32w, 32w+32) of the block's 128
// (2 m-tiles) and all 64 out channels (4 n-tiles) -> 8 accumulators.  X is
// gathered from NCHW through a per-block k->offset table in LDS (no integer
// division in the K loop); W rows are read 16 B at a time.  Slices are staged
// LDS <- registers with the next slice's global loads in flight during the MFMAs.
// POOL2: rows are ordered (clip, ph, pw, 2x2 member) so the four members of a
// max-pool window sit in 4 adjacent lanes: the epilogue max-reduces them with
// two lane swaps and stores only the pooled value (nn.MaxPool2d((2,2)) fused).
//
// X3 (bf16x3 mode): the same GEMM with every operand split at staging time into
// bf16 (hi, lo) = (bf16(v), bf16(v - hi)), stored k-contiguous ([m][k], [n][k])
// so a lane's 8 consecutive k are one 16-byte MFMA fragment, and each 32-deep
// slice is ONE v_mfma_f32_16x16x32_bf16 step of 3 products (hi*hi + hi*lo +
// lo*hi) per tile pair, fp32 accumulation -- the fp32 1e-4 bar at bf16 MFMA rates.
typedef __bf16 cbf16x8 __attribute__((ext_vector_type(8)));
constexpr int BKP = BK + 8;  // X3 LDS row pitch (bf16): 80 B keeps 16-lane fragment reads conflict-free

template <bool POOL2, bool X3>
__global__ __launch_bounds__(256) void conv_gemm_kernel(GemmArgs a) {
  // fp32: Ws[2][BK][BN + PADM], Xs[2][BK][BM + PADM] (floats)
  // X3:   Wh[2 buf][2 part][BN][BKP], Xh[2 buf][2 part][BM][BKP] (bf16)
  constexpr int WS_BYTES = X3 ? 2 * 2 * BN * BKP * 2 : 2 * BK * (BN + PADM) * 4;
  constexpr int XS_BYTES = X3 ? 2 * 2 * BM * BKP * 2 : 2 * BK * (BM + PADM) * 4;
  __shared__ __attribute__((aligned(16))) char wsm[WS_BYTES];
  __shared__ __attribute__((aligned(16))) char xsm[XS_BYTES];
  float (*Ws)[BK][BN + PADM] = (float (*)[BK][BN + PADM])wsm;
  float (*Xs)[BK][BM + PADM] = (float (*)[BK][BM + PADM])xsm;
  __bf16 (*Wh)[2][BN][BKP] = (__bf16 (*)[2][BN][BKP])wsm;
  __bf16 (*Xh)[2][BM][BKP] = (__bf16 (*)[2][BM][BKP])xsm;
  __shared__ int ktab[KTAB];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int KHW = a.KH * a.KW;
  const bool use_tab = a.K <= KTAB;
  if (use_tab)
    for (int k = tid; k < a.K; k += 256) {
      const int ci = k / KHW, rem = k - ci * KHW;
      const int kh = rem / a.KW, kw = rem - kh * a.KW;
      ktab[k] = (ci * a.H + kh) * a.W + kw;
    }

  // X staging: thread owns pixel column mm = tid % 128 and rows kk = tid/128 + 2r
  // (X3: the 16 consecutive rows 16 (tid/128) + r)
  const int mm = tid & (BM - 1);
  const int kq = tid >> 7;
  const int64_t mglob = m0 + mm;
  const bool mvalid = mglob < a.M;
  int64_t xbase = 0;
  if (mvalid) {
    int oh, ow;
    int64_t b;
    if (POOL2) {
      const int64_t q = mglob >> 2;
      const int sub = (int)(mglob & 3);
      const int PHW = a.PH * a.PW;
      b = q / PHW;
      const int pp = (int)(q - b * PHW);
      const int ph = pp / a.PW, pw = pp - ph * a.PW;
      oh = 2 * ph + (sub >> 1);
      ow = 2 * pw + (sub & 1);
    } else {
      const int OHW = a.OH * a.OW;
      b = mglob / OHW;
      const int pix = (int)(mglob - b * OHW);
      oh = pix / a.OW;
      ow = pix - oh * a.OW;
    }
    xbase = b * ((int64_t)a.Cin * a.H * a.W) + (int64_t)(oh * a.SH) * a.W + ow * a.SW;
  }
  // W staging: thread owns row n = tid/4, columns (tid%4)*8 .. +7
  const int wn_row = tid >> 2;
  const int wk0 = (tid & 3) * 8;
  const bool wvec = (a.K & 3) == 0 && ((((uintptr_t)a.w) & 15) == 0);

  float xr[16], wv[8];
  auto koffset = [&](int k) -> int {
    if (use_tab) return ktab[k];
    const int ci = k / KHW, rem = k - ci * KHW;
    const int kh = rem / a.KW, kw = rem - kh * a.KW;
    return (ci * a.H + kh) * a.W + kw;
  };
  auto load_slice = [&](int k0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = k0 + (X3 ? kq * 16 + r : kq + 2 * r);
      xr[r] = (mvalid && k < a.K) ? a.in[xbase + koffset(k)] : 0.f;
    }
    const int n = n0 + wn_row;
    const int kb = k0 + wk0;
    if (n < a.N && wvec && kb + 8 <= a.K) {
      const f32x4 u = *(const f32x4*)(a.w + (int64_t)n * a.K + kb);
      const f32x4 v = *(const f32x4*)(a.w + (int64_t)n * a.K + kb + 4);
      wv[0] = u[0]; wv[1] = u[1]; wv[2] = u[2]; wv[3] = u[3];
      wv[4] = v[0]; wv[5] = v[1]; wv[6] = v[2]; wv[7] = v[3];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) wv[j] = (n < a.N && kb + j < a.K) ? a.w[(int64_t)n * a.K + kb + j] : 0.f;
    }
  };
  auto store_slice = [&](int buf) {
    if constexpr (X3) {
      cbf16x8 xh[2], xl[2], whv, wlv;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const __bf16 h = (__bf16)xr[r];
        xh[r >> 3][r & 7] = h;
#ifdef HONK_CNN_ABLATE_SPLIT
        xl[r >> 3][r & 7] = h;
#else
        xl[r >> 3][r & 7] = (__bf16)(xr[r] - (float)h);
#endif
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 h = (__bf16)wv[j];
        whv[j] = h;
#ifdef HONK_CNN_ABLATE_SPLIT
        wlv[j] = h;
#else
        wlv[j] = (__bf16)(wv[j] - (float)h);
#endif
      }
      *(cbf16x8*)&Xh[buf][0][mm][kq * 16] = xh[0];
      *(cbf16x8*)&Xh[buf][0][mm][kq * 16 + 8] = xh[1];
      *(cbf16x8*)&Xh[buf][1][mm][kq * 16] = xl[0];
      *(cbf16x8*)&Xh[buf][1][mm][kq * 16 + 8] = xl[1];
      *(cbf16x8*)&Wh[buf][0][wn_row][wk0] = whv;
      *(cbf16x8*)&Wh[buf][1][wn_row][wk0] = wlv;
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) Xs[buf][kq + 2 * r][mm] = xr[r];
#pragma unroll
      for (int j = 0; j < 8; ++j) Ws[buf][wk0 + j][wn_row] = wv[j];
    }
  };

  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // ktab ready
  const int nslices = (a.K + BK - 1) / BK;
  load_slice(0);
  store_slice(0);
  __syncthreads();
  for (int t = 0; t < nslices; ++t) {
    const int buf = t & 1;
    if (t + 1 < nslices) load_slice((t + 1) * BK);
    if constexpr (X3) {
      // one 32-deep k-step: lane (g, i16) holds k = 8g .. 8g+7 of row i16
      const int kc = (lane >> 4) * 8, r16 = lane & 15;
      cbf16x8 aw[2][4], bx[2][2];
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) aw[pt][i] = *(const cbf16x8*)&Wh[buf][pt][i * 16 + r16][kc];
#pragma unroll
        for (int j = 0; j < 2; ++j) bx[pt][j] = *(const cbf16x8*)&Xh[buf][pt][wave * 32 + j * 16 + r16][kc];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[0][i], bx[0][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[0][i], bx[1][j], acc[i][j], 0, 0, 0);
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aw[1][i], bx[0][j], acc[i][j], 0, 0, 0);
        }
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 4; ++ks) {
        const int kk = ks * 4 + (lane >> 4);
        float av[4], bv[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) av[i] = Ws[buf][kk][i * 16 + (lane & 15)];
#pragma unroll
        for (int j = 0; j < 2; ++j) bv[j] = Xs[buf][kk][wave * 32 + j * 16 + (lane & 15)];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
    }
    if (t + 1 < nslices) store_slice(buf ^ 1);
    __syncthreads();
  }

  // epilogue: D[n][m]; lane holds rows n = (lane>>4)*4 + r, column m = lane & 15
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t m = m0 + wave * 32 + j * 16 + (lane & 15);
    const bool mok = m < a.M;
    int64_t obase;
    int64_t plane;
    if (POOL2) {
      const int64_t q = m >> 2;
      const int PHW = a.PH * a.PW;
      const int64_t b = q / PHW;
      obase = b * (int64_t)a.N * PHW + (q - b * PHW);
      plane = PHW;
    } else {
      const int OHW = a.OH * a.OW;
      const int64_t b = m / OHW;
      obase = b * (int64_t)a.N * OHW + (m - b * OHW);
      plane = OHW;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + i * 16 + (lane >> 4) * 4 + r;
        float v = acc[i][j][r] + ((a.bias && n < a.N) ? a.bias[n] : 0.f);
        if (a.relu) v = fmaxf(v, 0.f);
        if (POOL2) {  // max over the 2x2 window = lanes l, l^1, l^2, l^3 (same n)
          v = fmaxf(v, __shfl_xor(v, 1));
          v = fmaxf(v, __shfl_xor(v, 2));
          if ((lane & 3) == 0 && mok && n < a.N) a.out[obase + (int64_t)n * plane] = v;
        } else if (mok && n < a.N) {
          a.out[obase + (int64_t)n * plane] = v;
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

static int launch_gemm(const GemmArgs& a, bool pool2, hipStream_t st, bool x3 = false) {
  if (a.M <= 0 || a.N <= 0) return HONK_OK;
  const int64_t gm = cdiv(a.M, BM);
  if (gm > 0x7fffffff) return fail(HONK_ERR_ARG, "GEMM too large (M=%lld)", (long long)a.M);
  dim3 grid((unsigned)gm, (unsigned)cdiv(a.N, BN));
  TimedLaunch tl(st, 2.0 * (double)a.M * a.N * a.K);
  if (pool2 && x3)
    hipLaunchKernelGGL((conv_gemm_kernel<true, true>), grid, dim3(256), 0, st, a);
  else if (pool2)
    hipLaunchKernelGGL((conv_gemm_kernel<true, false>), grid, dim3(256), 0, st, a);
  else if (x3)
    hipLaunchKernelGGL((conv_gemm_kernel<false, true>), grid, dim3(256), 0, st, a);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<false, false>), grid, dim3(256), 0, st, a);
  tl.done(st);
  HONK_LAUNCH_CHECK("conv_gemm_kernel");
  return HONK_OK;
}

static int conv(const float* in, const float* w, const float* bias, float* out, int64_t batch, int cin,
                int h, int wd, int cout, int kh, int kw, int sh, int sw, int relu, hipStream_t st,
                bool pool2 = false, bool x3 = false) {
  if (kh > h || kw > wd || sh < 1 || sw < 1 || cin < 1 || cout < 1)
    return fail(HONK_ERR_ARG, "bad conv geometry (cin=%d %dx%d k=%dx%d s=%dx%d)", cin, h, wd, kh, kw, sh, sw);
  GemmArgs a;
  a.in = in; a.w = w; a.bias = bias; a.out = out;
  a.Cin = cin; a.H = h; a.W = wd; a.KH = kh; a.KW = kw; a.SH = sh; a.SW = sw;
  a.OH = (h - kh) / sh + 1;
  a.OW = (wd - kw) / sw + 1;
  a.PH = a.OH / 2;
  a.PW = a.OW / 2;
  a.M = pool2 ? batch * a.PH * a.PW * 4 : batch * a.OH * a.OW;
  a.N = cout;
  a.K = cin * kh * kw;
  a.relu = relu;
  if (pool2 && (a.PH < 1 || a.PW < 1)) return fail(HONK_ERR_ARG, "pool larger than conv output");
  return launch_gemm(a, pool2, st, x3);
}

// Linear with few outputs (n <= NB, e.g. cnn-trad-pool2's 26624 -> 4 output
// layer): a GEMV per clip, HBM-bound on x.  One 256-thread block per CPB clips
// walks K with 16-byte loads, every W element read once per block (L2-resident)
// and reused for the CPB clips; wave shuffles + LDS finish the reduction.  The
// GEMM kernel would give such a layer only ceil(m / 128) blocks with the whole
// K serial in each.
template <int NB, int CPB>
__global__ __launch_bounds__(256) void linear_small_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                           const float* __restrict__ b, float* __restrict__ y,
                                                           int64_t m, int K, int N, int relu) {
  __shared__ float red[4][CPB][NB];
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * CPB;
  float acc[CPB][NB];
#pragma unroll
  for (int c = 0; c < CPB; ++c)
#pragma unroll
    for (int n = 0; n < NB; ++n) acc[c][n] = 0.f;
  const bool vec = (K & 3) == 0;
  if (vec) {
    const int K4 = K >> 2;
    for (int k4 = tid; k4 < K4; k4 += 256) {
      float4 xv[CPB];
#pragma unroll
      for (int c = 0; c < CPB; ++c)
        xv[c] = (r0 + c < m) ? ((const float4*)(x + (r0 + c) * K))[k4] : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int n = 0; n < NB; ++n) {
        if (n < N) {
          const float4 wv = ((const float4*)(w + (int64_t)n * K))[k4];
#pragma unroll
          for (int c = 0; c < CPB; ++c)
            acc[c][n] = fmaf(wv.x, xv[c].x, fmaf(wv.y, xv[c].y, fmaf(wv.z, xv[c].z, fmaf(wv.w, xv[c].w, acc[c][n]))));
        }
      }
    }
  } else {
    for (int k = tid; k < K; k += 256) {
      float xv[CPB];
#pragma unroll
      for (int c = 0; c < CPB; ++c) xv[c] = (r0 + c < m) ? x[(r0 + c) * K + k] : 0.f;
#pragma unroll
      for (int n = 0; n < NB; ++n)
        if (n < N) {
          const float wv = w[(int64_t)n * K + k];
#pragma unroll
          for (int c = 0; c < CPB; ++c) acc[c][n] = fmaf(wv, xv[c], acc[c][n]);
        }
    }
  }
#pragma unroll
  for (int c = 0; c < CPB; ++c)
#pragma unroll
    for (int n = 0; n < NB; ++n) {
      float t = acc[c][n];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o);
      if ((tid & 63) == 0) red[tid >> 6][c][n] = t;
    }
  __syncthreads();
  if (tid < CPB * NB) {
    const int c = tid / NB, n = tid - c * NB;
    if (n < N && r0 + c < m) {
      float v = red[0][c][n] + red[1][c][n] + red[2][c][n] + red[3][c][n] + (b ? b[n] : 0.f);
      if (relu) v = fmaxf(v, 0.f);
      y[(r0 + c) * N + n] = v;
    }
  }
}

static int linear(const float* x, const float* w, const float* b, float* y, int64_t m, int k, int n,
                  int relu, hipStream_t st, bool x3 = false) {
  if (n <= 16 && m > 0) {
    constexpr int CPB = 4;
    const unsigned blocks = (unsigned)cdiv(m, CPB);
    if (n <= 4)
      hipLaunchKernelGGL((linear_small_kernel<4, CPB>), dim3(blocks), dim3(256), 0, st, x, w, b, y, m, k, n, relu);
    else if (n <= 8)
      hipLaunchKernelGGL((linear_small_kernel<8, CPB>), dim3(blocks), dim3(256), 0, st, x, w, b, y, m, k, n, relu);
    else
      hipLaunchKernelGGL((linear_small_kernel<16, CPB>), dim3(blocks), dim3(256), 0, st, x, w, b, y, m, k, n, relu);
    HONK_LAUNCH_CHECK("linear_small_kernel");
    return HONK_OK;
  }
  return conv(x, w, b, y, m, k, 1, 1, n, 1, 1, 1, 1, relu, st, false, x3);
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
  if (k < 1 || n < 1 || m < 0) return fail(HONK_ERR_ARG, "bad linear shape");
  if (m == 0) return HONK_OK;
  if (!x || !w || !y) return fail(HONK_ERR_ARG, "null pointer argument");
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
  if (d->precision != HONK_PREC_F32 && d->precision != HONK_PREC_BF16X3)
    return fail(HONK_ERR_UNSUPPORTED, "cnn path precision %d (f32 or bf16x3)", d->precision);
  const bool x3 = d->precision == HONK_PREC_BF16X3;
  hipStream_t st = (hipStream_t)stream;
  const int64_t chunk = chunk_clips(s, batch);
  float* A = (float*)workspace;
  float* B = A + chunk * per_clip_floats(s);

  for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
    const int64_t n = (batch - c0 < chunk) ? batch - c0 : chunk;
    const float* xin = x + c0 * d->height * d->width;
    // conv1 + ReLU (model.py:187) -> A ; pool1 (:189) -> B (skip when 1x1)
    const bool fuse1 = d->p1_h == 2 && d->p1_w == 2;  // conv1 + ReLU + MaxPool2d(2,2) in one kernel
    rc = conv(xin, t[0], t[1], A, n, 1, d->height, d->width, d->c1_out, d->c1_kh, d->c1_kw, d->c1_sh, d->c1_sw, 1,
              st, fuse1, x3);
    if (rc) return rc;
    const float* cur = A;
    float* other = B;
    if (!fuse1 && d->p1_h * d->p1_w > 1) {
      rc = maxpool(A, B, n * d->c1_out, s.oh1, s.ow1, d->p1_h, d->p1_w, st);
      if (rc) return rc;
      cur = B;
      other = A;
    }
    if (d->has_conv2) {  // model.py:190-193
      const bool fuse2 = d->p2_h == 2 && d->p2_w == 2;
      rc = conv(cur, t[2], t[3], other, n, d->c1_out, s.ph1, s.pw1, d->c2_out, d->c2_kh, d->c2_kw, d->c2_sh,
                d->c2_sw, 1, st, fuse2, x3);
      if (rc) return rc;
      const float* c2 = other;
      float* o2 = (float*)cur;
      if (!fuse2 && d->p2_h * d->p2_w > 1) {
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
      rc = linear(cur, t[4], t[5], other, n, width, 32, 0, st, x3);
      if (rc) return rc;
      width = 32;
      float* tmp = other; other = (float*)cur; cur = tmp;
    }
    if (d->dnn1) {       // :197-201
      rc = linear(cur, t[6], t[7], other, n, width, d->dnn1, d->dnn1_relu, st, x3);
      if (rc) return rc;
      width = d->dnn1;
      float* tmp = other; other = (float*)cur; cur = tmp;
    }
    if (d->dnn2) {       // :202-204
      rc = linear(cur, t[8], t[9], other, n, width, d->dnn2, 0, st, x3);
      if (rc) return rc;
      width = d->dnn2;
      float* tmp = other; other = (float*)cur; cur = tmp;
    }
    rc = linear(cur, t[10], t[11], logits + c0 * d->n_labels, n, width, d->n_labels, 0, st, x3);  // :205
    if (rc) return rc;
  }
  return HONK_OK;
}

}  // extern "C"
