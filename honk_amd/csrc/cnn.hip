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
  int DH, DW;        // dilation (1: the SpeechModel convs; the res block convs of honk_conv_same_f32)
  int PH, PW;        // pooled output dims (pool2 fused)
  int relu;
  int nhwc_x3;       // POOL2 only: 1 = store [B][PH][PW][hi N | lo N] bf16 (conv2x3_kernel's input),
                     // 2 = [B][PH][PW][N] fp32 (conv2f_kernel's input), instead of NCHW fp32
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
typedef __bf16 bf16x4c __attribute__((ext_vector_type(4)));
constexpr int BKP = BK + 8;  // X3 LDS row pitch (bf16): 80 B keeps 16-lane fragment reads conflict-free

// max / relu with torch's NaN behaviour (a NaN propagates)
__device__ __forceinline__ float nanmax(float m, float v) { return (v > m || v != v) ? v : m; }
__device__ __forceinline__ float relu_nan(float v) { return v <= 0.f ? 0.f : v; }

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
      ktab[k] = (ci * a.H + kh * a.DH) * a.W + kw * a.DW;
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
    return (ci * a.H + kh * a.DH) * a.W + kw * a.DW;
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
        xl[r >> 3][r & 7] = (__bf16)(xr[r] - (float)h);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const __bf16 h = (__bf16)wv[j];
        whv[j] = h;
        wlv[j] = (__bf16)(wv[j] - (float)h);
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
      float pooled[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + i * 16 + (lane >> 4) * 4 + r;
        float v = acc[i][j][r] + ((a.bias && n < a.N) ? a.bias[n] : 0.f);
        if (a.relu) v = v <= 0.f ? 0.f : v;  // NaN passes, as torch.relu
        if (POOL2) {  // max over the 2x2 window = lanes l, l^1, l^2, l^3 (same n); NaN propagates
          v = nanmax(v, __shfl_xor(v, 1));
          v = nanmax(v, __shfl_xor(v, 2));
          if (a.nhwc_x3) pooled[r] = v;
          else if ((lane & 3) == 0 && mok && n < a.N) a.out[obase + (int64_t)n * plane] = v;
        } else if (mok && n < a.N) {
          a.out[obase + (int64_t)n * plane] = v;
        }
      }
      if (POOL2 && a.nhwc_x3 == 2 && (lane & 3) == 0 && mok) {
        // the lane's 4 consecutive channels of its pooled pixel: one 16-B NHWC store
        const int n = n0 + i * 16 + (lane >> 4) * 4;
        if (n + 3 < a.N)
          *(f32x4*)(a.out + (m >> 2) * (int64_t)a.N + n) = f32x4{pooled[0], pooled[1], pooled[2], pooled[3]};
      }
      if (POOL2 && a.nhwc_x3 == 1 && (lane & 3) == 0 && mok) {
        // the lane's 4 consecutive channels of its pooled pixel, split into bf16
        // (hi, lo) runs of the [hi N | lo N] pixel (N == 64: host-checked)
        const int n = n0 + i * 16 + (lane >> 4) * 4;
        bf16x4c hv, lv;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          hv[r] = (__bf16)pooled[r];
          lv[r] = (__bf16)(pooled[r] - (float)hv[r]);
        }
        __bf16* px = (__bf16*)a.out + (m >> 2) * (int64_t)(2 * a.N);
        *(bf16x4c*)(px + n) = hv;
        *(bf16x4c*)(px + a.N + n) = lv;
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


// ---------------------------------------------------------------------------- //
// conv2 of cnn-trad-pool2 (64 -> <= 64 channels, stride 1, no pool after it) in
// bf16x3 on an NHWC hi/lo input: the whole clip is one tile.
//
// The input (conv1 + ReLU + MaxPool2d(2,2) output, written by conv_gemm_kernel's
// nhwc_x3 epilogue as [B][PH][PW][hi 64 | lo 64] bf16) is staged per clip in two
// 32-channel halves: one LDS image of PH*PW pixels x 128 B ([hi 32 | lo 32]) per
// half, filled by LDS-DMA, its 16-B chunks XOR-swizzled by pixel (chunk c of
// pixel P at slot P*8 + (c ^ (P & 7))) so a fragment read spreads over the banks.
// Implicit GEMM, weights as the MFMA A operand (16 out channels x 32 k), the
// image as B (32 k x 16 output pixels): k-step s = (half, tap kh*KW + kw) over
// the half's 32 channels, lane group g holding channels 8g .. 8g+7.
// 4 waves (one per SIMD): wave = (n-group: out tiles 2ng, 2ng+1) x (m-group: MT
// consecutive 16-pixel tiles of the clip's OH*OW outputs).  Each k-step reads
// the wave's MT A fragment pairs from LDS and its 4 weight fragments (hi, lo of
// 2 out tiles, pre-split by pack_conv2x3_kernel, L2-resident) from global, both
// one k-step ahead, and runs 6 MT MFMAs (hi*hi + hi*lo + lo*hi).
// Epilogue: bias + ReLU, NCHW fp32 stores (flatten order of model.py:194).
// ---------------------------------------------------------------------------- //
constexpr int C2X3_IMG = 96 * 1024;  // LDS bytes of one half image (PH*PW*128 <= this)
// (ablations, round 1: no image DMA -10 %, no A-fragment reads -9 %, L1-resident
// weights -5 %, all three -26 %)

struct Conv2X3Args {
  const __bf16* in;    // [B][PH][PW][hi 64 | lo 64]
  const uint4* wfrag;  // [2*ntap k-steps][4 out tiles][2 parts][64 lanes] x 16 B
  const float* bias;   // [N]
  float* out;          // [B][N][OH][OW]
  int B, PH, PW, KW, ntap, OH, OW, N;
};

template <int MT>
__global__ __launch_bounds__(256, 1) void conv2x3_kernel(Conv2X3Args a) {
  __shared__ __attribute__((aligned(16))) char img[C2X3_IMG];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ng = wave & 1, mg = wave >> 1;
  const int g = lane >> 4, i16 = lane & 15;
  const int npx = a.PH * a.PW;
  const int ohw = a.OH * a.OW;
  const int chunks = npx * 8;
  const int pieces = (chunks + 63) / 64;
  const int clip_bytes = npx * 256;

  // per m-tile: the lane's output pixel -> its input pixel at tap (0, 0)
  int P0[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = (mg * MT + m) * 16 + i16;
    const int oh = p / a.OW, ow = p - oh * a.OW;
    P0[m] = p < ohw ? oh * a.PW + ow : 0;
  }
  const uint4* wl = a.wfrag + ng * 2 * 2 * 64 + lane;  // (s, nt = 2 ng + j, part) -> wl[(s*4 + j)*... ]

  typedef uint4 AFr[MT][2];
  typedef uint4 WFr[2][2];
  auto loadA = [&](AFr& A, int delta) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int P = P0[m] + delta;
      const int ad = ((P << 3) + (g ^ (P & 7))) << 4;
      A[m][0] = *(const uint4*)(img + ad);
      A[m][1] = *(const uint4*)(img + (ad ^ 64));
    }
  };
  auto loadW = [&](WFr& Wr, int s) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int pt = 0; pt < 2; ++pt) Wr[j][pt] = wl[((s * 4 + j) * 2 + pt) * 64];
  };
  f32x4 acc[MT][2];
  auto mma = [&](const AFr& A, const WFr& Wr) {
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, Wr[j][t == 2 ? 1 : 0]),
                                                              __builtin_bit_cast(cbf16x8, A[m][t == 1 ? 1 : 0]),
                                                              acc[m][j], 0, 0, 0);
  };
  auto delta = [&](int t) {
    const int kh = t / a.KW;
    return kh * a.PW + (t - kh * a.KW);
  };

  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.in + (size_t)b * clip_bytes), (short)0, clip_bytes, 0x00020000);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int h = 0; h < 2; ++h) {
      __syncthreads();  // every wave is done reading the previous image
      for (int pc = wave; pc < pieces; pc += 4) {
        const int st = __builtin_amdgcn_readfirstlane(min(pc * 64, chunks - 64));
        const int L = st + lane;
        const int P = L >> 3, c = (L & 7) ^ (P & 7);
        const unsigned voff = (unsigned)(P * 256 + (c >> 2) * 128 + h * 64 + (c & 3) * 16);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + st * 16), 16,
                                                 voff, 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's pieces landed
      __syncthreads();                     // ... and every wave's
      const int s0 = h * a.ntap;
      AFr A0, A1;
      WFr W0, W1;
      loadW(W0, s0);
      loadA(A0, 0);
      for (int t = 0; t < a.ntap; t += 2) {  // ntap even (host-checked)
        loadW(W1, s0 + t + 1);
        loadA(A1, delta(t + 1));
        mma(A0, W0);
        if (t + 2 < a.ntap) {
          loadW(W0, s0 + t + 2);
          loadA(A0, delta(t + 2));
        }
        mma(A1, W1);
      }
    }
    // epilogue: lane (g, i16) holds out channels (2 ng + j) 16 + 4 g + r of pixel p
    float* ob = a.out + (size_t)b * a.N * ohw;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int p = (mg * MT + m) * 16 + i16;
      if (p < ohw) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = (2 * ng + j) * 16 + 4 * g + r;
            if (n < a.N) ob[(size_t)n * ohw + p] = relu_nan(acc[m][j][r] + a.bias[n]);
          }
      }
    }
  }
}

// conv2 weights [N][64][KH][KW] fp32 -> conv2x3_kernel's fragments: k-step
// s = half * ntap + tap, out tile nt, part (hi, lo), lane (g, i16):
// 8 bf16 of W[16 nt + i16][32 half + 8 g + j][tap] (zero past N)
__global__ void pack_conv2x3_kernel(const float* __restrict__ w, __bf16* __restrict__ frag, int N, int ntap) {
  const int total = 2 * ntap * 4 * 2 * 64 * 8;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int r = i;
  const int j = r & 7; r >>= 3;
  const int lane = r & 63; r >>= 6;
  const int pt = r & 1; r >>= 1;
  const int nt = r & 3; r >>= 2;
  const int s = r;
  const int h = s / ntap, t = s - h * ntap;
  const int co = nt * 16 + (lane & 15);
  const int ci = 32 * h + 8 * (lane >> 4) + j;
  const float v = co < N ? w[((size_t)co * 64 + ci) * ntap + t] : 0.f;
  const __bf16 hi = (__bf16)v;
  frag[i] = pt == 0 ? hi : (__bf16)(v - (float)hi);
}


// ---------------------------------------------------------------------------- //
// The same conv2 in fp32 (HONK_PREC_F32, config C2 as BASELINE.json names it) on
// v_mfma_f32_16x16x4_f32: the conv2x3_kernel design -- the whole clip one tile, two
// 32-channel half images by LDS-DMA (fp32 NHWC input from conv_gemm_kernel's
// nhwc_x3 = 2 epilogue: the half image is 128 B per pixel, the bf16 hi/lo one's
// size), 16-B chunks XOR-swizzled by pixel, 4 waves = 2 out-tile pairs x 2 groups
// of MT m-tiles, accumulators for the whole clip in VGPRs.
//   k-chunk (tap t, q): lane group g reads chunk 4q + g of its pixel (channels
//   32h + 16q + 4g .. +3 as one 16-B read); MFMA e = 0..3 takes element e, so one
//   read feeds 4 MFMAs per out tile; the weight A operand of MFMA e is
//   W[co][32h + 16q + 4g + e][t], pre-packed per lane as one float4 per chunk and
//   out tile (pack_conv2f_kernel, L2-resident), loaded one chunk ahead with the
//   activations.  fp32 products and accumulation: the fmaf chain of the reference
//   conv in another order (1e-4 parity).
// ---------------------------------------------------------------------------- //
struct Conv2FArgs {
  const float* in;      // [B][PH][PW][64] fp32
  const f32x4* wfrag;   // [2 h][ntap][2 q][4 out tiles][64 lanes]
  const float* bias;    // [N]
  float* out;           // [B][N][OH][OW]
  int B, PH, PW, KW, ntap, OH, OW, N;
};

template <int MT>
__global__ __launch_bounds__(256, 1) void conv2f_kernel(Conv2FArgs a) {
  __shared__ __attribute__((aligned(16))) char img[C2X3_IMG];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ng = wave & 1, mg = wave >> 1;
  const int g = lane >> 4, i16 = lane & 15;
  const int npx = a.PH * a.PW;
  const int ohw = a.OH * a.OW;
  const int chunks = npx * 8;
  const int pieces = (chunks + 63) / 64;
  const int clip_bytes = npx * 256;

  int P0[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = (mg * MT + m) * 16 + i16;
    const int oh = p / a.OW, ow = p - oh * a.OW;
    P0[m] = p < ohw ? oh * a.PW + ow : 0;
  }
  const f32x4* wl = a.wfrag + ng * 2 * 64 + lane;

  typedef f32x4 BFr[MT];
  typedef f32x4 WFr[2];
  auto loadB = [&](BFr& Bv, int delta, int q) {
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int P = P0[m] + delta;
      Bv[m] = *(const f32x4*)(img + (((P << 3) + ((4 * q + g) ^ (P & 7))) << 4));
    }
  };
  auto loadW = [&](WFr& Wv, int c) {  // c = (h * ntap + t) * 2 + q
#pragma unroll
    for (int j = 0; j < 2; ++j) Wv[j] = wl[(c * 4 + j) * 64];
  };
  f32x4 acc[MT][2];
  auto mma = [&](const BFr& Bv, const WFr& Wv) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[m][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(Wv[j][e], Bv[m][e], acc[m][j], 0, 0, 0);
  };
  auto delta = [&](int t) {
    const int kh = t / a.KW;
    return kh * a.PW + (t - kh * a.KW);
  };

  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)((const char*)a.in + (size_t)b * clip_bytes), (short)0, clip_bytes, 0x00020000);
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int h = 0; h < 2; ++h) {
      __syncthreads();  // every wave is done reading the previous image
      for (int pc = wave; pc < pieces; pc += 4) {
        const int st = __builtin_amdgcn_readfirstlane(min(pc * 64, chunks - 64));
        const int L = st + lane;
        const int P = L >> 3, c = (L & 7) ^ (P & 7);
        const unsigned voff = (unsigned)(P * 256 + h * 128 + c * 16);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(img + st * 16), 16,
                                                 voff, 0, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's pieces landed
      __syncthreads();                     // ... and every wave's
      const int nch = 2 * a.ntap;          // chunks of this half: (tap, q)
      const int c0 = h * nch;
      BFr B0, B1;
      WFr W0, W1;
      loadW(W0, c0);
      loadB(B0, 0, 0);
      for (int c = 0; c < nch; c += 2) {  // chunk c: tap c / 2, q = 0; c + 1: q = 1
        const int dt = delta(c >> 1);
        loadW(W1, c0 + c + 1);
        loadB(B1, dt, 1);
        mma(B0, W0);
        if (c + 2 < nch) {
          loadW(W0, c0 + c + 2);
          loadB(B0, delta((c >> 1) + 1), 0);
        }
        mma(B1, W1);
      }
    }
    float* ob = a.out + (size_t)b * a.N * ohw;
#pragma unroll
    for (int m = 0; m < MT; ++m) {
      const int p = (mg * MT + m) * 16 + i16;
      if (p < ohw) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = (2 * ng + j) * 16 + 4 * g + r;
            if (n < a.N) ob[(size_t)n * ohw + p] = relu_nan(acc[m][j][r] + a.bias[n]);
          }
      }
    }
  }
}

// conv2 weights [N][64][KH][KW] fp32 -> conv2f_kernel's fragments: chunk
// c = (h * ntap + t) * 2 + q, out tile nt, lane (g, i16): the float4
// W[16 nt + i16][32 h + 16 q + 4 g + e][t], e = 0..3 (zero past N)
__global__ void pack_conv2f_kernel(const float* __restrict__ w, float* __restrict__ frag, int N, int ntap) {
  const int total = 2 * ntap * 2 * 4 * 64 * 4;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int r = i;
  const int e = r & 3; r >>= 2;
  const int lane = r & 63; r >>= 6;
  const int nt = r & 3; r >>= 2;
  const int c = r;  // (h * ntap + t) * 2 + q
  const int q = c & 1, ht = c >> 1;
  const int h = ht / ntap, t = ht - h * ntap;
  const int co = nt * 16 + (lane & 15);
  const int ci = 32 * h + 16 * q + 4 * (lane >> 4) + e;
  frag[i] = co < N ? w[((size_t)co * 64 + ci) * ntap + t] : 0.f;
}

// ---------------------------------------------------------------------------- //
// conv1 + ReLU + MaxPool2d(2,2) of cnn-trad-pool2 (1 -> 64 channels, 20 x 8
// filter, stride 1) in bf16x3, writing conv2x3_kernel's NHWC hi/lo input.
// One clip per tile, 8 waves = 2 n-groups (out tiles 2ng, 2ng+1) x 4 m-groups.
//   K = 160 = 5 k-steps: lane group g of k-step s holds kh = 4s + g, kw = 0..7,
//   i.e. 8 consecutive input pixels of one row.  The clip is staged in LDS as a
//   "shifted-row" image: entry (r, c) = x[r][c .. c+7] as 8 bf16, hi and lo in
//   separate planes, c = 0 .. 31 (the pooled output's columns), entry slot
//   r*32 + ((c + 8 r) & 31) (16-B entries: conflict-free fragment reads), so an
//   A fragment is ONE aligned 16-B read and k-step s adds a fixed 2 KiB offset.
//   Weights: the wave's 2 out tiles x 5 k-steps x (hi, lo) fragments live in
//   VGPRs for the whole launch (W[co][kh][0..7] is 8 contiguous floats).
//   M = pooled members (ph, pw, 2x2 member) so the 4 members of a window sit in
//   lanes l .. l^3 of one MFMA column group: bias, ReLU, 2 lane-swap maxes, then
//   the lane with member 0 stores 4 channels' hi and lo runs (8 B each).
// ---------------------------------------------------------------------------- //
constexpr int C1X3_KH = 20, C1X3_KW = 8, C1X3_COLS = 32, C1X3_HMAX = 101;
// (prefetching the next clip's rows during this clip's MFMAs measured 0.4 % slower:
// 15 VGPR spills)
constexpr int C1X3_PLANE = C1X3_HMAX * C1X3_COLS * 16;  // bytes of one (hi or lo) plane

struct Conv1X3Args {
  const float* x;     // [B][H][W]
  const float* w;     // [64][1][20][8]
  const float* bias;  // [64]
  __bf16* out;        // [B][PH][PW][hi 64 | lo 64]
  int B, H, W, PH, PW;
};

__global__ __launch_bounds__(512, 1) void conv1x3_kernel(Conv1X3Args a) {
  __shared__ __attribute__((aligned(16))) char img[2 * C1X3_PLANE];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ng = wave & 1, mg = wave >> 1;
  const int g = lane >> 4, i16 = lane & 15;
  const int nmt = a.PH * a.PW / 4;  // 16-row m-tiles of pooled members (PH*PW % 4 == 0: host-checked)
  const int clip_floats = a.H * a.W;
  const int entries = a.H * C1X3_COLS;

  // weight fragments in registers: [k-step][out tile j][part]
  uint4 wf[5][2][2];
#pragma unroll
  for (int s = 0; s < 5; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = (2 * ng + j) * 16 + i16;
      const float* src = a.w + ((size_t)co * C1X3_KH + 4 * s + g) * C1X3_KW;
      const f32x4 u = *(const f32x4*)src, v = *(const f32x4*)(src + 4);
      cbf16x8 h, l;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float f = e < 4 ? u[e] : v[e - 4];
        h[e] = (__bf16)f;
        l[e] = (__bf16)(f - (float)h[e]);
      }
      wf[s][j][0] = __builtin_bit_cast(uint4, h);
      wf[s][j][1] = __builtin_bit_cast(uint4, l);
    }
  float bias[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = a.bias[(2 * ng + j) * 16 + 4 * g + r];

  // the lane's A-fragment byte offset (hi plane, k-step 0) for m-tile mt
  auto aoff = [&](int mt) {
    const int q = 4 * mt + (i16 >> 2), mem = i16 & 3;
    const int ph = q / a.PW, pw = q - ph * a.PW;
    const int r = 2 * ph + (mem >> 1) + g, c = 2 * pw + (mem & 1);
    return (r * C1X3_COLS + ((c + 8 * r) & (C1X3_COLS - 1))) * 16;
  };
  typedef uint4 AFr[5][2];
  auto loadA = [&](AFr& A, int off) {
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      A[s][0] = *(const uint4*)(img + off + s * 4 * C1X3_COLS * 16);
      A[s][1] = *(const uint4*)(img + C1X3_PLANE + off + s * 4 * C1X3_COLS * 16);
    }
  };
  auto tile = [&](const AFr& A, int mt, __bf16* ob) {
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = f32x4{bias[j][0], bias[j][1], bias[j][2], bias[j][3]};
#pragma unroll
    for (int s = 0; s < 5; ++s)
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(cbf16x8, wf[s][j][t == 2 ? 1 : 0]),
                                                           __builtin_bit_cast(cbf16x8, A[s][t == 1 ? 1 : 0]),
                                                           acc[j], 0, 0, 0);
    const int q = 4 * mt + (i16 >> 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf16x4c hv, lv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = relu_nan(acc[j][r]);
        v = nanmax(v, __shfl_xor(v, 1));
        v = nanmax(v, __shfl_xor(v, 2));
        hv[r] = (__bf16)v;
        lv[r] = (__bf16)(v - (float)hv[r]);
      }
      if ((i16 & 3) == 0) {
        __bf16* px = ob + (size_t)q * 128 + (2 * ng + j) * 16 + 4 * g;
        *(bf16x4c*)px = hv;
        *(bf16x4c*)(px + 64) = lv;
      }
    }
  };

  // the next clip's raw rows are loaded into registers while this clip computes
  // (NE entries of 8 floats per thread), converted and written at its start
  constexpr int NE = (C1X3_HMAX * C1X3_COLS + 511) / 512;
  f32x4 pu[NE], pv[NE];
  auto fetch = [&](int bb) {
    const bool ok = bb < a.B;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.x + (size_t)(ok ? bb : 0) * clip_floats), (short)0, ok ? clip_floats * 4 : 0, 0x00020000);
#pragma unroll
    for (int n = 0; n < NE; ++n) {
      const int e = tid + n * 512;
      const int r = e / C1X3_COLS, c = e - r * C1X3_COLS;
      const int o = e < entries ? (r * a.W + c) * 4 : 0x40000000;
      pu[n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
      pv[n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o + 16, 0, 0));
    }
  };
  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    __syncthreads();  // every wave is done with the previous clip's image
    fetch(b);
#pragma unroll
    for (int n = 0; n < NE; ++n) {
      const int e = tid + n * 512;
      if (e >= entries) break;
      const int r = e / C1X3_COLS, c = e - r * C1X3_COLS;
      const f32x4 u = pu[n], v = pv[n];
      cbf16x8 h, l;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = k < 4 ? u[k] : v[k - 4];
        h[k] = (__bf16)f;
        l[k] = (__bf16)(f - (float)h[k]);
      }
      const int slot = (r * C1X3_COLS + ((c + 8 * r) & (C1X3_COLS - 1))) * 16;
      *(cbf16x8*)(img + slot) = h;
      *(cbf16x8*)(img + C1X3_PLANE + slot) = l;
    }
    __syncthreads();
    __bf16* ob = a.out + (size_t)b * a.PH * a.PW * 128;
    AFr A0, A1;
    int mt = mg;
    if (mt < nmt) loadA(A0, aoff(mt));
    while (mt < nmt) {
      const int m1 = mt + 4;
      if (m1 < nmt) loadA(A1, aoff(m1));
      tile(A0, mt, ob);
      if (m1 >= nmt) break;
      const int m2 = m1 + 4;
      if (m2 < nmt) loadA(A0, aoff(m2));
      tile(A1, m1, ob);
      mt = m2;
    }
  }
}

// ---------------------------------------------------------------------------- //
// conv1 + ReLU + MaxPool2d(2,2) of cnn-trad-pool2 in fp32 (the conv1x3_kernel
// design on v_mfma_f32_16x16x4_f32), writing conv2f_kernel's NHWC fp32 input.
// One clip per tile, 8 waves = 2 n-groups x 4 m-groups.  K = 160 = 10 chunks of
// 16: lane group g of chunk s holds kh = 2s + (g >> 1), kw = 4 (g & 1) + e for
// MFMA e = 0..3.  The clip is staged as a "shifted-row" image of 16-B entries,
// entry (r, c) = x[r][c .. c+3] (c = 0 .. 35), so an operand read is ONE 16-B
// read feeding 4 MFMAs per out tile; the weights W[co][kh][4 (g & 1) .. +3] are 16
// contiguous bytes of the OIHW tensor, held in VGPRs for the launch.  M order
// (pooled pixel, 2x2 member): ReLU, two lane-swap maxes, one 16-B store per lane
// group.  The next clip's rows load into registers during this clip's MFMAs.
// ---------------------------------------------------------------------------- //
constexpr int C1F_COLS = 36;  // entries per image row (the pooled region's 32 columns + kw 0..7 in runs of 4)

struct Conv1FArgs {
  const float* x;     // [B][H][W]
  const float* w;     // [64][1][20][8]
  const float* bias;  // [64]
  float* out;         // [B][PH][PW][64]
  int B, H, W, PH, PW;
};

__global__ __launch_bounds__(512, 1) void conv1f_kernel(Conv1FArgs a) {
  __shared__ __attribute__((aligned(16))) char img[C1X3_HMAX * C1F_COLS * 16];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ng = wave & 1, mg = wave >> 1;
  const int g = lane >> 4, i16 = lane & 15;
  const int nmt = a.PH * a.PW / 4;  // 16-row m-tiles of pooled members (host-checked: PH*PW % 4 == 0)
  const int clip_floats = a.H * a.W;
  const int entries = a.H * C1F_COLS;

  f32x4 wf[10][2];
#pragma unroll
  for (int s = 0; s < 10; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int co = (2 * ng + j) * 16 + i16;
      wf[s][j] = *(const f32x4*)(a.w + ((size_t)co * C1X3_KH + 2 * s + (g >> 1)) * C1X3_KW + 4 * (g & 1));
    }
  float bias[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = a.bias[(2 * ng + j) * 16 + 4 * g + r];

  // the lane's entry offset at chunk 0 for m-tile mt (chunk s adds 2 rows)
  auto aoff = [&](int mt) {
    const int q = 4 * mt + (i16 >> 2), mem = i16 & 3;
    const int ph = q / a.PW, pw = q - ph * a.PW;
    const int r = 2 * ph + (mem >> 1) + (g >> 1), c = 2 * pw + (mem & 1) + 4 * (g & 1);
    return (r * C1F_COLS + c) * 16;
  };
  typedef f32x4 BFr[10];
  auto loadB = [&](BFr& Bv, int off) {
#pragma unroll
    for (int s = 0; s < 10; ++s) Bv[s] = *(const f32x4*)(img + off + s * 2 * C1F_COLS * 16);
  };
  auto tile = [&](const BFr& Bv, int mt, float* ob) {
    f32x4 acc[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[j] = f32x4{bias[j][0], bias[j][1], bias[j][2], bias[j][3]};
#pragma unroll
    for (int s = 0; s < 10; ++s)
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf[s][j][e], Bv[s][e], acc[j], 0, 0, 0);
    const int q = 4 * mt + (i16 >> 2);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      f32x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = relu_nan(acc[j][r]);
        t = nanmax(t, __shfl_xor(t, 1));
        v[r] = nanmax(t, __shfl_xor(t, 2));
      }
      if ((i16 & 3) == 0) *(f32x4*)(ob + (size_t)q * 64 + (2 * ng + j) * 16 + 4 * g) = v;
    }
  };

  constexpr int NE = (C1X3_HMAX * C1F_COLS + 511) / 512;
  f32x4 pu[NE];
  auto fetch = [&](int bb) {
    const bool ok = bb < a.B;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(a.x + (size_t)(ok ? bb : 0) * clip_floats), (short)0, ok ? clip_floats * 4 : 0, 0x00020000);
#pragma unroll
    for (int n = 0; n < NE; ++n) {
      const int e = tid + n * 512;
      const int r = e / C1F_COLS, c = e - r * C1F_COLS;
      const int o = e < entries ? (r * a.W + c) * 4 : 0x40000000;
      pu[n] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0));
    }
  };
  fetch(blockIdx.x);
  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    __syncthreads();  // every wave is done with the previous clip's image
#pragma unroll
    for (int n = 0; n < NE; ++n) {
      const int e = tid + n * 512;
      if (e < entries) *(f32x4*)(img + e * 16) = pu[n];
    }
    __syncthreads();
    fetch(b + gridDim.x);  // the next clip's rows, landing during this clip's MFMAs
    float* ob = a.out + (size_t)b * a.PH * a.PW * 64;
    BFr B0, B1;
    int mt = mg;
    if (mt < nmt) loadB(B0, aoff(mt));
    while (mt < nmt) {
      const int m1 = mt + 4;
      if (m1 < nmt) loadB(B1, aoff(m1));
      tile(B0, mt, ob);
      if (m1 >= nmt) break;
      const int m2 = m1 + 4;
      if (m2 < nmt) loadB(B0, aoff(m2));
      tile(B1, m1, ob);
      mt = m2;
    }
  }
}

// conv1 in fp32 with conv2f following: trad-pool2's conv1 geometry
static bool conv1f_applies(const honk_cnn_desc* d, int oh1, int ph1, int pw1) {
  if (const char* e = getenv("HONK_CNN_C1F"))
    if (atoi(e) == 0) return false;
  return d->c1_kh == C1X3_KH && d->c1_kw == C1X3_KW && d->c1_sh == 1 && d->c1_sw == 1 && d->c1_out == 64 &&
         2 * pw1 + 4 <= C1F_COLS && d->width >= C1F_COLS + 3 && d->height <= C1X3_HMAX && (ph1 * pw1) % 4 == 0 &&
         oh1 >= 2 * ph1;
}

// conv1 on the fast path: bf16x3 with conv2x3 following, trad-pool2's conv1
// geometry (20 x 8 filter, stride 1, 64 maps, 2x2 pool, 32 pooled-window columns)
static bool conv1x3_applies(const honk_cnn_desc* d, int oh1, int ph1, int pw1) {
  if (const char* e = getenv("HONK_CNN_C1X3"))
    if (atoi(e) == 0) return false;
  return d->c1_kh == C1X3_KH && d->c1_kw == C1X3_KW && d->c1_sh == 1 && d->c1_sw == 1 && d->c1_out == 64 &&
         2 * pw1 == C1X3_COLS && d->width >= C1X3_COLS + C1X3_KW - 1 && d->height <= C1X3_HMAX &&
         (ph1 * pw1) % 4 == 0 && oh1 >= 2 * ph1;
}

// cnn-trad-pool2-class conv2 on the fast path: bf16x3, conv1 pooled 2x2 with 64
// maps (its GEMM writes the NHWC split input), conv2 64 -> <= 64, stride 1, no
// pool after it, an even tap count, a half image within C2X3_IMG and OH*OW
// within the instantiated 2 * 13 m-tiles
constexpr int C2X3_MT = 13;
static bool conv2x3_applies(const honk_cnn_desc* d, int ph1, int pw1, int oh2, int ow2) {
  if (d->precision != HONK_PREC_BF16X3 || !d->has_conv2) return false;
  if (const char* e = getenv("HONK_CNN_C2X3"))
    if (atoi(e) == 0) return false;
  return d->p1_h == 2 && d->p1_w == 2 && d->c1_out == 64 && d->c2_out <= 64 && d->c2_sh == 1 && d->c2_sw == 1 &&
         d->p2_h == 1 && d->p2_w == 1 && (d->c2_kh * d->c2_kw) % 2 == 0 && ph1 * pw1 * 128 <= C2X3_IMG &&
         oh2 * ow2 > 16 * C2X3_MT && oh2 * ow2 <= 32 * C2X3_MT;
}
static size_t conv2x3_frag_bytes(const honk_cnn_desc* d) { return (size_t)2 * d->c2_kh * d->c2_kw * 4 * 2 * 64 * 16; }
// the fp32 counterpart (conv2f_kernel): the same geometry in HONK_PREC_F32
constexpr int C2F_MT = 13;
static bool conv2f_applies(const honk_cnn_desc* d, int ph1, int pw1, int oh2, int ow2) {
  if (d->precision != HONK_PREC_F32 || !d->has_conv2) return false;
  if (const char* e = getenv("HONK_CNN_C2F"))
    if (atoi(e) == 0) return false;
  return d->p1_h == 2 && d->p1_w == 2 && d->c1_out == 64 && d->c2_out <= 64 && d->c2_sh == 1 && d->c2_sw == 1 &&
         d->p2_h == 1 && d->p2_w == 1 && ph1 * pw1 * 128 <= C2X3_IMG && oh2 * ow2 > 16 * C2F_MT &&
         oh2 * ow2 <= 32 * C2F_MT;
}
static size_t conv2f_frag_bytes(const honk_cnn_desc* d) { return (size_t)2 * d->c2_kh * d->c2_kw * 2 * 4 * 64 * 16; }

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
                bool pool2 = false, bool x3 = false, int nhwc_x3 = 0, int dil = 1) {
  if ((kh - 1) * dil + 1 > h || (kw - 1) * dil + 1 > wd || sh < 1 || sw < 1 || cin < 1 || cout < 1 || dil < 1)
    return fail(HONK_ERR_ARG, "bad conv geometry (cin=%d %dx%d k=%dx%d s=%dx%d)", cin, h, wd, kh, kw, sh, sw);
  GemmArgs a;
  a.in = in; a.w = w; a.bias = bias; a.out = out;
  a.Cin = cin; a.H = h; a.W = wd; a.KH = kh; a.KW = kw; a.SH = sh; a.SW = sw;
  a.DH = a.DW = dil;
  a.OH = (h - (kh - 1) * dil - 1) / sh + 1;
  a.OW = (wd - (kw - 1) * dil - 1) / sw + 1;
  a.PH = a.OH / 2;
  a.PW = a.OW / 2;
  a.M = pool2 ? batch * a.PH * a.PW * 4 : batch * a.OH * a.OW;
  a.N = cout;
  a.K = cin * kh * kw;
  a.relu = relu;
  a.nhwc_x3 = nhwc_x3;
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
      if (relu) v = relu_nan(v);
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


// ---------------------------------------------------------------------------- //
// SpeechModel training (utils/train.py:123-135 on the cnn configs: the backward of
// model.py:186-193).  The forward reuses conv_gemm_kernel (conv + bias + ReLU,
// pre-pool output kept for the backward) and maxpool_kernel; dropout stays
// PyTorch's own op between them (the reference's RNG stream and mask semantics).
//   * max-pool backward: the gradient of each window goes to its first maximum in
//     scan order (the forward's rule, v > m || isnan(v): torch's max_pool2d index);
//   * weight + bias gradient: dW[n][k] = sum_m g'[n][m] X[k][m], k = (ci, kh, kw),
//     m = (clip, oh, ow), g' = the output gradient through the ReLU (act > 0), X
//     gathered from the NCHW input (the forward's im2col), on fp32 MFMA with m as
//     the reduction; the m range is split over workgroups (one partial each) and
//     the partials are summed in a fixed order: deterministic;
//   * input gradient (stride 1): the full correlation of g' with the flipped,
//     transposed weights = conv_gemm_kernel over g' zero-padded by (KH-1, KW-1).
// ---------------------------------------------------------------------------- //
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const float* __restrict__ in, const float* __restrict__ gout,
                                                          float* __restrict__ gin, int64_t planes, int H, int W,
                                                          int KH, int KW) {
  const int PH = H / KH, PW = W / KW;
  const int64_t total = planes * H * W;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % W);
    const int64_t t = i / W;
    const int y = (int)(t % H);
    const int64_t pl = t / H;
    const int ph = y / KH, pw = x / KW;
    float g = 0.f;
    if (ph < PH && pw < PW) {
      const float* p = in + pl * H * W + (int64_t)(ph * KH) * W + pw * KW;
      float m = p[0];
      int best = 0;
      for (int u = 0; u < KH; ++u)
        for (int v = 0; v < KW; ++v) {
          const float e = p[u * W + v];
          if (e > m || e != e) {
            m = e;
            best = u * KW + v;
          }
        }
      if (best == (y - ph * KH) * KW + (x - pw * KW)) g = gout[(pl * PH + ph) * PW + pw];
    }
    gin[i] = g;
  }
}

constexpr int WG_BN = 64;  // out channels per workgroup
constexpr int WG_BK = 64;  // (ci, kh, kw) columns per workgroup
constexpr int WG_BM = 32;  // reduction (m) per LDS stage

struct ConvWgradArgs {
  const float* in;   // [B][Cin][H][W]
  const float* gy;   // [B][N][OH][OW]
  const float* act;  // [B][N][OH][OW] ReLU output (g' = act <= 0 ? 0 : gy), or nullptr
  float* part;       // [S][N][K]
  float* pbias;      // [S][N] or nullptr
  int64_t M, mper;   // B*OH*OW; m per split (multiple of WG_BM)
  int N, K, Cin, H, W, KH, KW, SH, SW, OH, OW;
  int D;             // dilation
};

// 256 threads = 4 waves; wave w owns out channels n0 + 16w .. +15 and all 4
// 16-column tiles of the workgroup's 64 k (4 accumulators).  A stage stages 32 m
// of g' ([m][n]) and X ([m][k]) in LDS, the next stage's global loads in flight
// during the 8 k-steps of v_mfma_f32_16x16x4_f32.  Staging: thread = m column
// (tid & 31) x 8 rows (tid >> 5) + 8j, one (clip, pixel) decomposition per stage.
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvWgradArgs a) {
  __shared__ float Gs[2][WG_BM][WG_BN + 4];
  __shared__ float Xs[2][WG_BM][WG_BK + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * WG_BN, k0 = blockIdx.y * WG_BK, sp = blockIdx.z;
  const int64_t mbeg = (int64_t)sp * a.mper;
  const int64_t mend = mbeg + a.mper < a.M ? mbeg + a.mper : a.M;
  const int mc = tid & 31, r8 = tid >> 5;
  const int KHW = a.KH * a.KW, OHW = a.OH * a.OW;
  int koff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = k0 + r8 + 8 * j;
    if (k < a.K) {
      const int ci = k / KHW, rem = k - ci * KHW;
      const int kh = rem / a.KW, kw = rem - kh * a.KW;
      koff[j] = (ci * a.H + kh * a.D) * a.W + kw * a.D;
    } else {
      koff[j] = -1;
    }
  }
  const bool do_bias = a.pbias != nullptr && blockIdx.y == 0;
  float gv[8], xv[8], bsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
  auto load = [&](int64_t m0) {
    const int64_t m = m0 + mc;
    const bool ok = m < mend;
    int64_t gbase = 0, xbase = 0;
    if (ok) {
      const int64_t b = m / OHW;
      const int pix = (int)(m - b * OHW);
      const int oh = pix / a.OW, ow = pix - oh * a.OW;
      gbase = b * (int64_t)a.N * OHW + pix;
      xbase = b * (int64_t)a.Cin * a.H * a.W + (int64_t)(oh * a.SH) * a.W + ow * a.SW;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + r8 + 8 * j;
      float g = 0.f;
      if (ok && n < a.N) {
        const int64_t o = gbase + (int64_t)n * OHW;
        g = a.gy[o];
        if (a.act && a.act[o] <= 0.f) g = 0.f;  // threshold_backward: NaN passes
      }
      gv[j] = g;
      xv[j] = (ok && koff[j] >= 0) ? a.in[xbase + koff[j]] : 0.f;
    }
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 8; ++j) bsum[j] += gv[j];
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      Gs[buf][mc][r8 + 8 * j] = gv[j];
      Xs[buf][mc][r8 + 8 * j] = xv[j];
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nst = mend > mbeg ? (mend - mbeg + WG_BM - 1) / WG_BM : 0;
  if (nst > 0) {
    load(mbeg);
    store(0);
  }
  __syncthreads();
  for (int64_t t = 0; t < nst; ++t) {
    const int buf = (int)(t & 1);
    if (t + 1 < nst) load(mbeg + (t + 1) * WG_BM);
#pragma unroll
    for (int ks = 0; ks < WG_BM / 4; ++ks) {
      const int kk = ks * 4 + (lane >> 4);
      const float av = Gs[buf][kk][wave * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Xs[buf][kk][j * 16 + (lane & 15)], acc[j], 0, 0, 0);
    }
    if (t + 1 < nst) store(buf ^ 1);
    __syncthreads();
  }
  // D[i][jj]: lane holds rows i = (lane >> 4) * 4 + r (out channel), column jj = lane & 15 (k)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = k0 + j * 16 + (lane & 15);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = n0 + wave * 16 + (lane >> 4) * 4 + r;
      if (n < a.N && k < a.K) a.part[((int64_t)sp * a.N + n) * a.K + k] = acc[j][r];
    }
  }
  if (do_bias) {
    // the 32 lanes of a half-wave share r8: tree over the m columns
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = bsum[j];
#pragma unroll
      for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o);
      const int n = n0 + r8 + 8 * j;
      if (mc == 0 && n < a.N) a.pbias[(int64_t)sp * a.N + n] = v;
    }
  }
}

// out[i] = sum over s of part[s][i], s ascending (fixed order: deterministic)
__global__ __launch_bounds__(256) void split_sum_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                        int64_t n, int S) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = 0.f;
  for (int s = 0; s < S; ++s) v += part[(int64_t)s * n + i];
  out[i] = v;
}

// gp[pl][y][x] = g'[pl][y - (KH-1)][x - (KW-1)] inside the map, else 0 (g' = ReLU-masked gy)
__global__ __launch_bounds__(256) void dgrad_pad_kernel(const float* __restrict__ gy, const float* __restrict__ act,
                                                        float* __restrict__ gp, int64_t planes, int OH, int OW,
                                                        int PHp, int PWp, int KH, int KW) {
  const int64_t total = planes * PHp * PWp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int x = (int)(i % PWp);
    const int64_t t = i / PWp;
    const int y = (int)(t % PHp);
    const int64_t pl = t / PHp;
    const int oy = y - (KH - 1), ox = x - (KW - 1);
    float g = 0.f;
    if (oy >= 0 && oy < OH && ox >= 0 && ox < OW) {
      const int64_t o = (pl * OH + oy) * OW + ox;
      g = gy[o];
      if (act && act[o] <= 0.f) g = 0.f;
    }
    gp[i] = g;
  }
}

// wf[ci][n][kh][kw] = w[n][ci][KH-1-kh][KW-1-kw]
__global__ __launch_bounds__(256) void flip_weights_kernel(const float* __restrict__ w, float* __restrict__ wf, int N,
                                                           int Cin, int KH, int KW) {
  const int KHW = KH * KW;
  const int64_t total = (int64_t)N * Cin * KHW;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int t = (int)(i % KHW);
  const int64_t q = i / KHW;
  const int n = (int)(q % N);
  const int ci = (int)(q / N);
  wf[i] = w[((int64_t)n * Cin + ci) * KHW + (KHW - 1 - t)];
}

struct WgradPlanC {
  int tn, tk, S;
  int64_t M, mper;
};
static WgradPlanC wgrad_plan_c(int64_t batch, int cin, int h, int w, int cout, int kh, int kw, int sh, int sw,
                               int dil = 1) {
  WgradPlanC p;
  const int oh = (h - (kh - 1) * dil - 1) / sh + 1, ow = (w - (kw - 1) * dil - 1) / sw + 1;
  p.M = batch * oh * ow;
  p.tn = (int)cdiv(cout, WG_BN);
  p.tk = (int)cdiv((int64_t)cin * kh * kw, WG_BK);
  int64_t S = cdiv(1024, (int64_t)p.tn * p.tk);          // ~4 workgroups per CU
  const int64_t smax = cdiv(p.M, 8 * WG_BM);             // >= 8 stages per split
  if (S > smax) S = smax;
  if (S > 4096) S = 4096;
  if (S < 1) S = 1;
  p.mper = cdiv(cdiv(p.M, S), WG_BM) * WG_BM;
  p.S = (int)cdiv(p.M, p.mper);
  if (p.S < 1) p.S = 1;
  return p;
}


// the weight / bias gradient launches (conv_wgrad_kernel + the fixed-order split sums)
static int wgrad_launch(const float* in, const float* gy, const float* act, float* dw, float* db, int64_t batch,
                        int cin, int h, int w, int cout, int kh, int kw, int sh, int sw, int dil, float* part,
                        hipStream_t st) {
  const int64_t K = (int64_t)cin * kh * kw;
  const WgradPlanC p = wgrad_plan_c(batch, cin, h, w, cout, kh, kw, sh, sw, dil);
  ConvWgradArgs a;
  a.in = in; a.gy = gy; a.act = act;
  a.part = part;
  a.pbias = db ? a.part + (int64_t)p.S * cout * K : nullptr;
  a.M = p.M; a.mper = p.mper;
  a.N = cout; a.K = (int)K; a.Cin = cin; a.H = h; a.W = w; a.KH = kh; a.KW = kw; a.SH = sh; a.SW = sw;
  a.OH = (h - (kh - 1) * dil - 1) / sh + 1; a.OW = (w - (kw - 1) * dil - 1) / sw + 1;
  a.D = dil;
  {
    TimedLaunch tl(st, 2.0 * (double)p.M * cout * K);
    hipLaunchKernelGGL(conv_wgrad_kernel, dim3(p.tn, p.tk, p.S), dim3(256), 0, st, a);
    tl.done(st);
  }
  HONK_LAUNCH_CHECK("conv_wgrad_kernel");
  const int64_t nw = (int64_t)cout * K;
  hipLaunchKernelGGL(split_sum_kernel, dim3((unsigned)cdiv(nw, 256)), dim3(256), 0, st, a.part, dw, nw, p.S);
  if (db)
    hipLaunchKernelGGL(split_sum_kernel, dim3((unsigned)cdiv(cout, 256)), dim3(256), 0, st, a.pbias, db,
                       (int64_t)cout, p.S);
  HONK_LAUNCH_CHECK("split_sum_kernel");
  return HONK_OK;
}

// xp[pl][y][x] = x[pl][y - d][x - d] inside the map, else 0 (the "same" conv's zero padding)
__global__ __launch_bounds__(256) void pad_same_kernel(const float* __restrict__ x, float* __restrict__ xp,
                                                       int64_t planes, int H, int W, int d) {
  const int Hp = H + 2 * d, Wp = W + 2 * d;
  const int64_t total = planes * Hp * Wp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int xx = (int)(i % Wp);
    const int64_t t = i / Wp;
    const int yy = (int)(t % Hp);
    const int64_t pl = t / Hp;
    const int sy = yy - d, sx = xx - d;
    xp[i] = (sy >= 0 && sy < H && sx >= 0 && sx < W) ? x[(pl * H + sy) * W + sx] : 0.f;
  }
}
static int pad_same(const float* x, float* xp, int64_t planes, int h, int w, int d, hipStream_t st) {
  const int64_t total = planes * (int64_t)(h + 2 * d) * (w + 2 * d);
  const int64_t blocks = cdiv(total, 256) < 65536 ? cdiv(total, 256) : 65536;
  hipLaunchKernelGGL(pad_same_kernel, dim3((unsigned)blocks), dim3(256), 0, st, x, xp, planes, h, w, d);
  HONK_LAUNCH_CHECK("pad_same_kernel");
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

int honk_maxpool2d_bwd_f32(const float* in, const float* gout, float* gin, int64_t batch, int32_t c, int32_t h,
                           int32_t w, int32_t kh, int32_t kw, void* stream) {
  if (!in || !gout || !gin) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 0 || c < 1 || kh < 1 || kw < 1 || kh > h || kw > w)
    return fail(HONK_ERR_ARG, "bad pool %dx%d on %dx%d", kh, kw, h, w);
  const int64_t total = batch * c * h * w;
  if (total == 0) return HONK_OK;
  const int64_t blocks = cdiv(total, 256) < 65536 ? cdiv(total, 256) : 65536;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, in, gout, gin,
                     batch * c, h, w, kh, kw);
  HONK_LAUNCH_CHECK("maxpool_bwd_kernel");
  return HONK_OK;
}

static int conv_train_check(int64_t batch, int cin, int h, int w, int cout, int kh, int kw, int sh, int sw) {
  if (batch < 0 || cin < 1 || cout < 1 || kh < 1 || kw < 1 || sh < 1 || sw < 1 || kh > h || kw > w)
    return fail(HONK_ERR_ARG, "bad conv geometry (cin=%d %dx%d k=%dx%d s=%dx%d cout=%d)", cin, h, w, kh, kw, sh, sw,
                cout);
  return HONK_OK;
}

size_t honk_conv2d_wgrad_workspace_bytes(int64_t batch, int32_t cin, int32_t h, int32_t w, int32_t cout, int32_t kh,
                                         int32_t kw, int32_t sh, int32_t sw) {
  if (batch < 1 || conv_train_check(batch, cin, h, w, cout, kh, kw, sh, sw) != HONK_OK) return 0;
  const WgradPlanC p = wgrad_plan_c(batch, cin, h, w, cout, kh, kw, sh, sw);
  return (size_t)p.S * ((size_t)cout * cin * kh * kw + cout) * sizeof(float);
}

int honk_conv2d_wgrad_f32(const float* in, const float* gy, const float* act, float* dw, float* db, int64_t batch,
                          int32_t cin, int32_t h, int32_t w, int32_t cout, int32_t kh, int32_t kw, int32_t sh,
                          int32_t sw, void* workspace, size_t ws_bytes, void* stream) {
  int rc = conv_train_check(batch, cin, h, w, cout, kh, kw, sh, sw);
  if (rc) return rc;
  if (!in || !gy || !dw) return fail(HONK_ERR_ARG, "null pointer argument");
  hipStream_t st = (hipStream_t)stream;
  const int64_t K = (int64_t)cin * kh * kw;
  if (batch == 0) {
    HONK_HIP_CHECK(hipMemsetAsync(dw, 0, (size_t)cout * K * sizeof(float), st));
    if (db) HONK_HIP_CHECK(hipMemsetAsync(db, 0, (size_t)cout * sizeof(float), st));
    return HONK_OK;
  }
  const size_t need = honk_conv2d_wgrad_workspace_bytes(batch, cin, h, w, cout, kh, kw, sh, sw);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  return wgrad_launch(in, gy, act, dw, db, batch, cin, h, w, cout, kh, kw, sh, sw, 1, (float*)workspace, st);
}

size_t honk_conv2d_dgrad_workspace_bytes(int64_t batch, int32_t cin, int32_t h, int32_t w, int32_t cout, int32_t kh,
                                         int32_t kw) {
  if (batch < 1 || conv_train_check(batch, cin, h, w, cout, kh, kw, 1, 1) != HONK_OK) return 0;
  const int64_t oh = h - kh + 1, ow = w - kw + 1;
  const int64_t php = oh + 2 * (kh - 1), pwp = ow + 2 * (kw - 1);
  return (size_t)(batch * cout * php * pwp + (int64_t)cout * cin * kh * kw) * sizeof(float);
}

int honk_conv2d_dgrad_f32(const float* gy, const float* act, const float* w, float* dx, int64_t batch, int32_t cin,
                          int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw, void* workspace,
                          size_t ws_bytes, void* stream) {
  int rc = conv_train_check(batch, cin, h, w_, cout, kh, kw, 1, 1);
  if (rc) return rc;
  if (!gy || !w || !dx) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch == 0) return HONK_OK;
  const size_t need = honk_conv2d_dgrad_workspace_bytes(batch, cin, h, w_, cout, kh, kw);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int oh = h - kh + 1, ow = w_ - kw + 1;
  const int php = oh + 2 * (kh - 1), pwp = ow + 2 * (kw - 1);
  float* gp = (float*)workspace;
  float* wf = gp + batch * cout * (int64_t)php * pwp;
  const int64_t np = batch * cout * (int64_t)php * pwp;
  const int64_t blocks = cdiv(np, 256) < 65536 ? cdiv(np, 256) : 65536;
  hipLaunchKernelGGL(dgrad_pad_kernel, dim3((unsigned)blocks), dim3(256), 0, st, gy, act, gp, batch * cout, oh, ow,
                     php, pwp, kh, kw);
  HONK_LAUNCH_CHECK("dgrad_pad_kernel");
  const int64_t nw = (int64_t)cout * cin * kh * kw;
  hipLaunchKernelGGL(flip_weights_kernel, dim3((unsigned)cdiv(nw, 256)), dim3(256), 0, st, w, wf, cout, cin, kh, kw);
  HONK_LAUNCH_CHECK("flip_weights_kernel");
  return conv(gp, wf, nullptr, dx, batch, cout, php, pwp, cin, kh, kw, 1, 1, 0, st);
}

// ---- the res block conv for any channel count (model.py:94-98: 3x3, padding =
// dilation = d, no bias), the training kernels' general path: the input zero-padded
// into the workspace, then the implicit GEMM with dilation ----
static int same_check(const void* a, const void* b, const void* c, int64_t batch, int32_t ch, int32_t h, int32_t w,
                      int32_t d) {
  if (!a || !b || !c) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 0 || ch < 1 || h < 1 || w < 1 || d < 1 || d > 1024)
    return fail(HONK_ERR_ARG, "bad same-conv shape (B=%lld C=%d H=%d W=%d d=%d)", (long long)batch, ch, h, w, d);
  if ((int64_t)ch * 9 > 0x7fffffff / 4) return fail(HONK_ERR_UNSUPPORTED, "same-conv: C=%d too large", ch);
  return HONK_OK;
}

size_t honk_conv_same_workspace_bytes(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil) {
  if (batch < 1 || c < 1 || h < 1 || w_ < 1 || dil < 1) return 0;
  const int hp = h + 2 * dil, wp = w_ + 2 * dil;
  const size_t pad = (size_t)batch * c * hp * wp;
  const WgradPlanC p = wgrad_plan_c(batch, c, hp, wp, c, 3, 3, 1, 1, dil);
  size_t extra = (size_t)p.S * c * c * 9;
  if ((size_t)c * c * 9 > extra) extra = (size_t)c * c * 9;
  return (pad + extra) * sizeof(float);
}

int honk_conv_same_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c, int32_t h, int32_t w_,
                       int32_t dil, int32_t flip, void* workspace, size_t ws_bytes, void* stream) {
  int rc = same_check(x, w, y, batch, c, h, w_, dil);
  if (rc) return rc;
  if (batch == 0) return HONK_OK;
  const size_t need = honk_conv_same_workspace_bytes(batch, c, h, w_, dil);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int hp = h + 2 * dil, wp = w_ + 2 * dil;
  float* xp = (float*)workspace;
  float* wf = xp + (size_t)batch * c * hp * wp;
  rc = pad_same(x, xp, batch * c, h, w_, dil, st);
  if (rc) return rc;
  const float* wk = w;
  if (flip) {  // input gradient: the flipped, transposed kernel, w'[i][o][t] = w[o][i][8 - t]
    const int64_t nw = (int64_t)c * c * 9;
    hipLaunchKernelGGL(flip_weights_kernel, dim3((unsigned)cdiv(nw, 256)), dim3(256), 0, st, w, wf, c, c, 3, 3);
    HONK_LAUNCH_CHECK("flip_weights_kernel");
    wk = wf;
  }
  return conv(xp, wk, nullptr, y, batch, c, hp, wp, c, 3, 3, 1, 1, 0, st, false, false, 0, dil);
}

int honk_conv_same_wgrad_f32(const float* x, const float* dy, float* dw, int64_t batch, int32_t c, int32_t h,
                             int32_t w_, int32_t dil, void* workspace, size_t ws_bytes, void* stream) {
  int rc = same_check(x, dy, dw, batch, c, h, w_, dil);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (batch == 0) {
    HONK_HIP_CHECK(hipMemsetAsync(dw, 0, (size_t)c * c * 9 * sizeof(float), st));
    return HONK_OK;
  }
  const size_t need = honk_conv_same_workspace_bytes(batch, c, h, w_, dil);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  const int hp = h + 2 * dil, wp = w_ + 2 * dil;
  float* xp = (float*)workspace;
  float* part = xp + (size_t)batch * c * hp * wp;
  rc = pad_same(x, xp, batch * c, h, w_, dil, st);
  if (rc) return rc;
  return wgrad_launch(xp, dy, nullptr, dw, nullptr, batch, c, hp, wp, c, 3, 3, 1, 1, dil, part, st);
}

size_t honk_cnn_workspace_bytes(const honk_cnn_desc* d, int64_t batch) {
  Shapes s;
  if (shapes(d, &s) != HONK_OK || batch < 1) return 0;
  size_t b = (size_t)2 * chunk_clips(s, batch) * per_clip_floats(s) * sizeof(float);
  if (conv2x3_applies(d, s.ph1, s.pw1, s.oh2, s.ow2)) b += conv2x3_frag_bytes(d);  // packed conv2 fragments
  if (conv2f_applies(d, s.ph1, s.pw1, s.oh2, s.ow2)) b += conv2f_frag_bytes(d);
  return b;
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
  const bool c2x3 = conv2x3_applies(d, s.ph1, s.pw1, s.oh2, s.ow2);
  uint4* c2frag = (uint4*)(B + chunk * per_clip_floats(s));
  if (c2x3) {  // conv2 weights -> hi/lo fragments (one small launch per call)
    const int ntap = d->c2_kh * d->c2_kw;
    const int total = 2 * ntap * 4 * 2 * 64 * 8;
    hipLaunchKernelGGL(pack_conv2x3_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, t[2],
                       (__bf16*)c2frag, d->c2_out, ntap);
    HONK_LAUNCH_CHECK("pack_conv2x3_kernel");
  }
  const bool c2f = conv2f_applies(d, s.ph1, s.pw1, s.oh2, s.ow2);
  if (c2f) {  // conv2 weights -> fp32 fragments (one small launch per call)
    const int ntap = d->c2_kh * d->c2_kw;
    const int total = 2 * ntap * 2 * 4 * 64 * 4;
    hipLaunchKernelGGL(pack_conv2f_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, st, t[2], (float*)c2frag,
                       d->c2_out, ntap);
    HONK_LAUNCH_CHECK("pack_conv2f_kernel");
  }

  for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
    const int64_t n = (batch - c0 < chunk) ? batch - c0 : chunk;
    const float* xin = x + c0 * d->height * d->width;
    // conv1 + ReLU (model.py:187) -> A ; pool1 (:189) -> B (skip when 1x1)
    const bool fuse1 = d->p1_h == 2 && d->p1_w == 2;  // conv1 + ReLU + MaxPool2d(2,2) in one kernel
    if (c2f && conv1f_applies(d, s.oh1, s.ph1, s.pw1)) {
      Conv1FArgs c;
      c.x = xin;
      c.w = t[0];
      c.bias = t[1];
      c.out = A;
      c.B = (int)n;
      c.H = d->height;
      c.W = d->width;
      c.PH = s.ph1;
      c.PW = s.pw1;
      if (n > 0x7fffffff) return fail(HONK_ERR_ARG, "chunk too large");
      const unsigned grid = (unsigned)(n < cu_count() ? n : cu_count());
      TimedLaunch tl(st, 2.0 * (double)n * s.ph1 * s.pw1 * 4 * 64 * C1X3_KH * C1X3_KW);
      hipLaunchKernelGGL(conv1f_kernel, dim3(grid), dim3(512), 0, st, c);
      tl.done(st);
      HONK_LAUNCH_CHECK("conv1f_kernel");
    } else if (c2x3 && conv1x3_applies(d, s.oh1, s.ph1, s.pw1)) {
      Conv1X3Args c;
      c.x = xin;
      c.w = t[0];
      c.bias = t[1];
      c.out = (__bf16*)A;
      c.B = (int)n;
      c.H = d->height;
      c.W = d->width;
      c.PH = s.ph1;
      c.PW = s.pw1;
      if (n > 0x7fffffff) return fail(HONK_ERR_ARG, "chunk too large");
      const unsigned grid = (unsigned)(n < cu_count() ? n : cu_count());
      TimedLaunch tl(st, 2.0 * (double)n * s.ph1 * s.pw1 * 4 * 64 * C1X3_KH * C1X3_KW);
      hipLaunchKernelGGL(conv1x3_kernel, dim3(grid), dim3(512), 0, st, c);
      tl.done(st);
      HONK_LAUNCH_CHECK("conv1x3_kernel");
    } else {
      rc = conv(xin, t[0], t[1], A, n, 1, d->height, d->width, d->c1_out, d->c1_kh, d->c1_kw, d->c1_sh, d->c1_sw, 1,
                st, fuse1, x3, c2x3 ? 1 : c2f ? 2 : 0);
      if (rc) return rc;
    }
    const float* cur = A;
    float* other = B;
    if (!fuse1 && d->p1_h * d->p1_w > 1) {
      rc = maxpool(A, B, n * d->c1_out, s.oh1, s.ow1, d->p1_h, d->p1_w, st);
      if (rc) return rc;
      cur = B;
      other = A;
    }
    if (c2x3) {  // model.py:190-193 on the fast path (pool2 is 1x1)
      Conv2X3Args c;
      c.in = (const __bf16*)A;
      c.wfrag = c2frag;
      c.bias = t[3];
      c.out = B;
      c.B = (int)n;
      c.PH = s.ph1;
      c.PW = s.pw1;
      c.KW = d->c2_kw;
      c.ntap = d->c2_kh * d->c2_kw;
      c.OH = s.oh2;
      c.OW = s.ow2;
      c.N = d->c2_out;
      if (n > 0x7fffffff) return fail(HONK_ERR_ARG, "chunk too large");
      const unsigned grid = (unsigned)(n < cu_count() ? n : cu_count());
      TimedLaunch tl(st, 2.0 * (double)n * s.oh2 * s.ow2 * d->c2_out * 64 * c.ntap);
      hipLaunchKernelGGL((conv2x3_kernel<C2X3_MT>), dim3(grid), dim3(256), 0, st, c);
      tl.done(st);
      HONK_LAUNCH_CHECK("conv2x3_kernel");
      cur = B;
      other = A;
    } else if (c2f) {  // model.py:190-193, fp32, on the NHWC pooled conv1 output
      Conv2FArgs c;
      c.in = A;
      c.wfrag = (const f32x4*)c2frag;
      c.bias = t[3];
      c.out = B;
      c.B = (int)n;
      c.PH = s.ph1;
      c.PW = s.pw1;
      c.KW = d->c2_kw;
      c.ntap = d->c2_kh * d->c2_kw;
      c.OH = s.oh2;
      c.OW = s.ow2;
      c.N = d->c2_out;
      if (n > 0x7fffffff) return fail(HONK_ERR_ARG, "chunk too large");
      const unsigned grid = (unsigned)(n < cu_count() ? n : cu_count());
      TimedLaunch tl(st, 2.0 * (double)n * s.oh2 * s.ow2 * d->c2_out * 64 * c.ntap);
      hipLaunchKernelGGL((conv2f_kernel<C2F_MT>), dim3(grid), dim3(256), 0, st, c);
      tl.done(st);
      HONK_LAUNCH_CHECK("conv2f_kernel");
      cur = B;
      other = A;
    } else if (d->has_conv2) {  // model.py:190-193
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
