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

// ---------------------------------------------------------------------------- //
// Training-mode 3x3 convolutions of the res block stack (dilation d, padding d,
// no bias; model.py:94-98: d = 1 for res8/res26, 2**(i//3) for res15), fp32 NCHW
// like the PyTorch tensors around them (train-mode BatchNorm, ReLU, residual and
// the loss stay PyTorch ops on the device):
//   conv3x3_kernel<C,NP>: y = conv(x, w) (flip 0) or the input gradient
//     dx = conv(dy, w'), w'[o][i][t] = w[i][o][8-t] (flip 1) -- the transform is
//     applied while the weights are staged into LDS as [in][tap][out].
//   wgrad3x3_kernel<C>: per-workgroup partial dW over its tiles; wsum_kernel adds
//     the partials in a fixed order (deterministic, no atomics).
// VALU direct convolution: 19 (45) channels are far from an MFMA tile (19 -> 32
// is 2.8x the work), and gfx950's fp32 VALU FMA rate equals its fp32 MFMA rate.
// A dilated 3x3 conv couples row h only with rows h -/+ d, so the rows of one
// residue class r = h mod d are an independent problem (the inference row-band
// kernel's decomposition).  A tile is a band of TH class rows (rows r + (k TH + j) d)
// of one clip at full width: its (TH+2) x (W+2d) zero-padded input rows of every
// channel are staged in LDS once (one halo class row above/below, d zero columns
// left/right); tap (ky, kx) of staged pixel (j, w) is (j + ky, w + kx d).  Each
// thread owns NP output pixels x all C outputs (weights read as LDS broadcasts,
// 4 per ds_read_b128).  d = 1 is the plain band of TH rows.
// ---------------------------------------------------------------------------- //
constexpr int TC_XL = 64 * 1024;  // bytes of the staged input tile (wgrad: and of its dy tile)
constexpr int TC_XLC = 64 * 1024;  // conv3x3_kernel's input tile (19 maps); 96 KB = whole clips, 4 px/thread, 1 block/CU: 23 % slower step

template <int C>
struct TC {
  static constexpr int CW = (C + 3) & ~3;  // output channels padded to a float4
  static constexpr int WL = C * 9 * CW;    // floats of the staged weights
};

// class-band geometry of one clip (dilation d, TH class rows per band): classes
// r < rem hold H/d + 1 rows (nb1 bands), the others H/d rows (nb0 bands)
struct ClassBands {
  int d, TH, rem, nb1, nb0, nband;  // nband = bands per clip
};
static inline ClassBands class_bands(int H, int d, int TH) {
  ClassBands g;
  const int q = H / d;
  g.d = d;
  g.TH = TH;
  g.rem = H - q * d;
  g.nb1 = (q + 1 + TH - 1) / TH;
  g.nb0 = (q + TH - 1) / TH;
  g.nband = g.rem * g.nb1 + (d - g.rem) * g.nb0;
  return g;
}
// band bi of a clip -> residue class r, first class row k0, rows in the band
__device__ __forceinline__ void band_of(const ClassBands& g, int H, int bi, int& r, int& k0, int& th) {
  int k;
  if (bi < g.rem * g.nb1) {
    r = bi / g.nb1;
    k = bi - r * g.nb1;
  } else {
    const int bj = bi - g.rem * g.nb1;
    const int rr = bj / g.nb0;
    k = bj - rr * g.nb0;
    r = g.rem + rr;
  }
  const int rows = (H - r + g.d - 1) / g.d;  // class rows of class r
  k0 = k * g.TH;
  th = min(g.TH, rows - k0);
}

struct Conv3Args {
  const float* x;  // [B][C][H][W]
  const float* w;  // OIHW [C][C][3][3]
  float* y;        // [B][C][H][W]
  int B, H, W, flip;
  ClassBands g;
  // conv3x3d_kernel's BatchNorm statistics epilogue (MODE 1 / 2), else unused:
  const float* aux;  // MODE 1: the residual old (may be null); MODE 2: the BN output y
  double* part;      // [C][gridDim.x][2] per-workgroup partial sums
  // MODE 1 only, may be null: y receives s = relu(conv) [+ aux] instead of conv, and
  // mask[b][p] bit o = !(conv[b][o][p] <= 0) (the ReLU's backward mask, torch's
  // threshold_backward; one 32-bit word per pixel, C <= 20)
  unsigned* mask;
  // the layer below's train BatchNorm folded in (conv3x3d_kernel, may be null): MODE 1
  // convolves y = (x - fm[c]) fi[c] (x holds that layer's s), MODE 2 reads its aux the
  // same way -- y is never written to HBM
  const float* fm = nullptr;
  const float* fi = nullptr;
};

typedef float tf2 __attribute__((ext_vector_type(2)));

template <int C, int NP>
__global__ __launch_bounds__(256) void conv3x3_kernel(Conv3Args a) {
  constexpr int CW = TC<C>::CW;
  __shared__ __attribute__((aligned(16))) float wl[TC<C>::WL];
  __shared__ __attribute__((aligned(16))) float xl[(C <= 20 ? TC_XLC : TC_XL) / 4];
  const int tid = threadIdx.x;
  for (int i = tid; i < TC<C>::WL; i += 256) {
    const int o = i % CW, it = i / CW, in = it / 9, t = it - in * 9;
    float v = 0.f;
    if (o < C) v = a.flip ? a.w[(in * C + o) * 9 + 8 - t] : a.w[(o * C + in) * 9 + t];
    wl[i] = v;
  }
  const int d = a.g.d, Wp = a.W + 2 * d;
  for (int tile = blockIdx.x; tile < a.B * a.g.nband; tile += gridDim.x) {
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, a.H, tile - b * a.g.nband, r, k0, th);
    const int rows = th + 2, plane = rows * Wp;
    __syncthreads();  // previous tile's readers done (and the weights staged)
    const float* xb = a.x + (size_t)b * C * a.H * a.W;
    for (int i0 = tid; i0 < C * plane; i0 += 8 * 256) {  // 8 loads in flight per thread
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 256;
        const int c = i / plane, rc = i - c * plane, rr = rc / Wp, col = rc - rr * Wp;
        const int h = r + (k0 - 1 + rr) * d, w = col - d;
        v[u] = (i < C * plane && h >= 0 && h < a.H && w >= 0 && w < a.W) ? xb[((size_t)c * a.H + h) * a.W + w] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + u * 256 < C * plane) xl[i0 + u * 256] = v[u];
    }
    __syncthreads();
    // packed fp32 FMA (v_pk_fma_f32): output channel pairs share the pixel's input
    tf2 acc[NP][CW / 2];
    int base[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int q = tid + k * 256;
      const int j = q / a.W, col = q - j * a.W;
      base[k] = q < th * a.W ? j * Wp + col : 0;
#pragma unroll
      for (int o = 0; o < CW / 2; ++o) acc[k][o] = tf2{0.f, 0.f};
    }
    for (int ci = 0; ci < C; ++ci) {
      const float* xc = xl + ci * plane;
      const float4* wc = (const float4*)(wl + ci * 9 * CW);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int toff = (t / 3) * Wp + (t % 3) * d;
        tf2 xv[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const float v = xc[base[k] + toff];
          xv[k] = tf2{v, v};
        }
#pragma unroll
        for (int j = 0; j < CW / 4; ++j) {
          const float4 w4 = wc[t * (CW / 4) + j];
          const tf2 wa = tf2{w4.x, w4.y}, wb = tf2{w4.z, w4.w};
#pragma unroll
          for (int k = 0; k < NP; ++k) {
            acc[k][2 * j] = __builtin_elementwise_fma(xv[k], wa, acc[k][2 * j]);
            acc[k][2 * j + 1] = __builtin_elementwise_fma(xv[k], wb, acc[k][2 * j + 1]);
          }
        }
      }
    }
    float* yb = a.y + (size_t)b * C * a.H * a.W;
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      const int q = tid + k * 256;
      if (q < th * a.W) {
        const int j = q / a.W, col = q - j * a.W;
        const size_t pix = (size_t)(r + (k0 + j) * d) * a.W + col;
#pragma unroll
        for (int o = 0; o < C; ++o) yb[(size_t)o * a.H * a.W + pix] = acc[k][o >> 1][o & 1];
      }
    }
  }
}

// ---------------------------------------------------------------------------- //
// conv3x3m_kernel<C> (C <= 20): the same convolution (forward / input gradient) as
// conv3x3_kernel on v_mfma_f32_16x16x4_f32, as an implicit GEMM D[o][p] = sum_k
// W'[o][k] X[k][p] over k = 9 c + t (input channel c, tap t) -- the order of
// conv3x3_kernel's FMA chain, and the MFMA is an fmaf chain over its 4 k: the two
// kernels agree bit for bit.  (Training is ill-conditioned where train-mode
// BatchNorm meets a nearly dead channel: a different summation order in one
// layer moved res15-narrow's gradients by 1e-2 from float64.)  Lane (pixel p, kk)
// reads X[4 s + kk][p] = plane c, tap t of the staged band: a per-lane offset per
// k-step (16-bit, packed two per VGPR) plus the pixel's base.  The layer's weight
// operand (ceil(9C / 4) k-steps x 2 out-tiles floats per lane) stays in VGPRs;
// two workgroups per CU.  Output lane (p, g) holds channels 16 n + 4 g .. +3.
// ---------------------------------------------------------------------------- //
constexpr int TM_XL = 64 * 1024;  // staged tile bytes (2 workgroups per CU; 3 would spill the weight operand)

// Stage nrows image rows of W floats into LDS with the workgroup's 256 threads:
// row i comes from src(i) (nullptr: zeros) and lands at LDS offset dst(i).  Each
// thread keeps 8 loads in flight (the tile is latency-bound otherwise: a serial walk
// waits out the HBM latency on every row); rows whose W is a multiple of 4 move as
// float4s (16 B per lane, 4x the bytes in flight of the scalar walk).
template <typename Src, typename Dst>
__device__ __forceinline__ void stage_rows(float* __restrict__ lds, int nrows, int W, Src src, Dst dst) {
  const int tid = threadIdx.x;
  if ((W & 3) == 0) {
    const int W4 = W >> 2, SR = 256 / W4, rl0 = tid / W4, c4 = 4 * (tid - rl0 * W4);
    if (rl0 >= SR) return;
    for (int row0 = rl0; row0 < nrows; row0 += 8 * SR) {
      float4 v[8];
      int o[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int row = row0 + u * SR;
        const float* p = row < nrows ? src(row) : nullptr;
        v[u] = p ? *(const float4*)(p + c4) : float4{0.f, 0.f, 0.f, 0.f};
        o[u] = row < nrows ? dst(row) + c4 : -1;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (o[u] >= 0) {
          lds[o[u]] = v[u].x;
          lds[o[u] + 1] = v[u].y;
          lds[o[u] + 2] = v[u].z;
          lds[o[u] + 3] = v[u].w;
        }
    }
    return;
  }
  const int SR = 256 / W, rl0 = tid / W, col = tid - rl0 * W;
  if (rl0 >= SR) return;
  for (int row0 = rl0; row0 < nrows; row0 += 8 * SR) {
    float v[8];
    int o[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = row0 + u * SR;
      const float* p = row < nrows ? src(row) : nullptr;
      v[u] = p ? p[col] : 0.f;
      o[u] = row < nrows ? dst(row) + col : -1;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (o[u] >= 0) lds[o[u]] = v[u];
  }
}

// row / R for row < 2^16 through the float reciprocal, corrected to exact
__device__ __forceinline__ int div_small(int row, int R, float invR) {
  int c = (int)((float)row * invR);
  c += (row - c * R >= R) ? 1 : ((row - c * R < 0) ? -1 : 0);
  return c;
}
__host__ __device__ inline int tm_ps(int rows, int Wp) {  // plane stride (floats), = 16 mod 32
  const int f = rows * Wp;
  return f + ((16 - f % 32) + 32) % 32;
}

typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <int C>
__global__ __launch_bounds__(256, 2) void conv3x3m_kernel(Conv3Args a) {
  static_assert(C <= 20, "conv3x3m_kernel: C <= 20");
  constexpr int K = 9 * C, KS = (K + 3) / 4;
  __shared__ __attribute__((aligned(16))) float xl[TM_XL / 4];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, kk = lane >> 4;
  const int d = a.g.d, Wp = a.W + 2 * d;
  const int PS = tm_ps(a.g.TH + 2, Wp);  // every tile's planes at the longest band's stride
  // the weight operand wr[s][n] = W'[16 n + i16][4 s + kk] and the lane's LDS offset
  // of k = 4 s + kk (c PS + row / column shift of tap t; the K pad reads plane 0 x 0)
  float wr[KS][2];
  unsigned koff[(KS + 1) / 2];
#pragma unroll
  for (int s = 0; s < (KS + 1) / 2; ++s) koff[s] = 0;
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    const int k = 4 * s + kk, c = k / 9, t = k - 9 * c;
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int o = 16 * n + i16;
      float v = 0.f;
      if (o < C && k < K) v = a.flip ? a.w[(c * C + o) * 9 + 8 - t] : a.w[(o * C + c) * 9 + t];
      wr[s][n] = v;
    }
    const unsigned off = k < K ? (unsigned)(c * PS + (t / 3) * Wp + (t % 3) * d) : 0u;
    koff[s >> 1] |= off << (16 * (s & 1));
  }
  // staging (stage_rows): the d halo columns of every row are zeroed once here and
  // never written again (every tile stages the longest band's R rows)
  const int R = a.g.TH + 2;
  const float invR = 1.0f / (float)R;
  for (int i = tid; i < C * R * 2 * d; i += 256) {
    const int row = i / (2 * d), e = i - row * (2 * d);
    const int c = row / R, rr = row - c * R;
    xl[c * PS + rr * Wp + (e < d ? e : a.W + e)] = 0.f;
  }
  for (int tile = blockIdx.x; tile < a.B * a.g.nband; tile += gridDim.x) {
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, a.H, tile - b * a.g.nband, r, k0, th);
    __syncthreads();  // previous tile's readers done
    {
      const float* xb = a.x + (size_t)b * C * a.H * a.W;
      const int H = a.H, W = a.W, hr = r + (k0 - 1) * d;
      // staged row = (channel c, band row rr): image row hr + rr d (zeros outside)
      stage_rows(
          xl, C * R, W,
          [&](int row) -> const float* {
            const int c = div_small(row, R, invR), h = hr + (row - c * R) * d;
            return h >= 0 && h < H ? xb + ((size_t)c * H + h) * W : nullptr;
          },
          [&](int row) {
            const int c = div_small(row, R, invR);
            return c * PS + (row - c * R) * Wp + d;
          });
    }
    __syncthreads();
    const int npx = th * a.W, nmt = (npx + 15) >> 4;
    float* yb = a.y + (size_t)b * C * a.H * a.W;
    for (int m = wave; m < nmt; m += 4) {
      const int p = 16 * m + i16;
      const bool pv = p < npx;
      const int j = pv ? p / a.W : 0, col = pv ? p - j * a.W : 0;
      const float* xp = xl + j * Wp + col;
      f32x4_t acc[2] = {f32x4_t{0.f, 0.f, 0.f, 0.f}, f32x4_t{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const float xv = xp[(koff[s >> 1] >> (16 * (s & 1))) & 0xffffu];
        acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[s][0], xv, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(wr[s][1], xv, acc[1], 0, 0, 0);
      }
      if (pv) {
        const size_t pix = (size_t)(r + (k0 + j) * d) * a.W + col;
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int o = 16 * n + 4 * kk + i;
            if (o < C) yb[(size_t)o * a.H * a.W + pix] = acc[n][i];
          }
      }
    }
  }
}

// ---------------------------------------------------------------------------- //
// conv3x3d_kernel<C> (C <= 20, d <= 4, W a multiple of 4): conv3x3m_kernel's MFMA
// loop (same k order, bit-identical) on a double-buffered tile staged by LDS-DMA
// (buffer_load ... lds, 16 B per lane): while the 8 waves multiply tile t out of one
// buffer, the DMA fills the other with tile t + grid, so HBM latency never stalls
// the MFMAs.  An LDS row is [4 zeros | W pixels | 4 zeros] (TD_PAD = 4 >= d), a
// plane R rows at a stride = 16 mod 32 floats, every 16-B chunk either an HBM chunk
// of the clip or an out-of-range buffer offset (the bounds check returns zeros:
// the halo columns, rows outside the image and plane padding).  One workgroup of
// 512 threads per CU (two 60-KB buffers).
// ---------------------------------------------------------------------------- //
constexpr int TD_PAD = 4;           // zero floats left / right of every staged row
constexpr int TD_BUF = 64 * 1024;   // bytes per buffer (two per workgroup)
constexpr int TD_ITER = 8;          // DMA instructions per wave per tile (8 waves x 8 x 1 KB)

__device__ __forceinline__ void td_wait_vm0() { __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8)); }

struct TdGeo {
  int Wr, PS, R, nchunk;  // padded row floats, plane stride, rows per plane, chunks per buffer (mult. of 64)
};
__host__ __device__ inline TdGeo td_geo(int C, int W, int TH) {
  TdGeo g;
  g.Wr = W + 2 * TD_PAD;
  g.R = TH + 2;
  const int f = g.R * g.Wr;
  g.PS = f + ((16 - f % 32) + 32) % 32;  // a multiple of 4 (Wr is): whole chunks
  g.nchunk = (C * g.PS / 4 + 63) / 64 * 64;
  return g;
}

// The folded BatchNorm on a staged tile (conv3x3d_kernel MODE 1, wgrad3x3d/q_kernel):
// each lane rewrites the 16-B chunks its own LDS-DMA instructions wrote (chunk e = base_e
// + 64 i at float 4 e, of plane c = 4 e / PS: the mapping is tile-invariant), right after
// its own vmcnt wait and before the tile's barrier -- no barrier of its own.  An in-image x
// chunk (ok[i]) holds the layer below's s and becomes (s - mean[c]) invstd[c] (mv[i] =
// {mean, invstd} of its plane), tail_fwd_kernel's fp32 expression: bit-identical to the y
// it would have written; pad columns and out-of-image rows stay zero (the conv's zero
// padding of y).
template <int N>
__device__ __forceinline__ void td_bn_fold(float* buf, int base_e, const bool (&ok)[N], const float2 (&mv)[N]) {
  float4 v[N];
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (ok[i]) v[i] = *(const float4*)(buf + 4 * (base_e + 64 * i));
#pragma unroll
  for (int i = 0; i < N; ++i)
    if (ok[i]) {
      const float m = mv[i].x, iv = mv[i].y;
      *(float4*)(buf + 4 * (base_e + 64 * i)) =
          float4{(v[i].x - m) * iv, (v[i].y - m) * iv, (v[i].z - m) * iv, (v[i].w - m) * iv};
    }
}

// f(std::integral_constant<int, 0>{}) .. f(std::integral_constant<int, N - 1>{}): a
// compile-time index (an MFMA's ABID must be a constant)
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// 16-lane row transpose and the broadcast 4x4x1 MFMA (wgrad3x3d_kernel's output
// channels 16..C-1; conv3x3d_kernel's every channel).
__device__ __forceinline__ void tr4_rows(float& x0, float& x1, float& x2, float& x3) {
  // on exit 16-lane row g of x_q holds row q of x_g (on entry)
  const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(x0), __float_as_uint(x2), false, false);
  const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(x1), __float_as_uint(x3), false, false);
  const auto r = __builtin_amdgcn_permlane16_swap(p[0], q[0], false, false);
  const auto u = __builtin_amdgcn_permlane16_swap(p[1], q[1], false, false);
  x0 = __uint_as_float(r[0]);
  x1 = __uint_as_float(r[1]);
  x2 = __uint_as_float(u[0]);
  x3 = __uint_as_float(u[1]);
}

// acc += A(block abid, broadcast to all 16 blocks) x b, abid a constant after unrolling
__device__ __forceinline__ f32x4_t mfma4_bc(float a, float b, f32x4_t c, int abid) {
  switch (abid & 15) {
#define HONK_MF4(i) \
  case i:           \
    return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, i, 0);
    HONK_MF4(0) HONK_MF4(1) HONK_MF4(2) HONK_MF4(3) HONK_MF4(4) HONK_MF4(5) HONK_MF4(6) HONK_MF4(7)
    HONK_MF4(8) HONK_MF4(9) HONK_MF4(10) HONK_MF4(11) HONK_MF4(12) HONK_MF4(13) HONK_MF4(14)
    default: return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 4, 15, 0);
#undef HONK_MF4
  }
}

// conv3x3d_kernel: every output channel on v_mfma_f32_4x4x1_16b_f32 (16 blocks of
// 4 x 4).  A wave takes a super tile of 64 pixels, lane l = pixel l; per k = 9 c + t
// one LDS read (x at tap t of plane c, a uniform offset) feeds ceil(C/4) MFMAs, the
// weights of 4 channels for k broadcast from the block that holds them (CBSZ = 4,
// ABID = k mod 16; lane 4 b + r of wt[g][j] = w[4 g + r][16 j + b]).  19 channels use
// 20 MFMA rows (a 16x16x4 tile pair would use 32), and the operands need neither a
// transpose nor a second read.  Each output accumulates k in ascending order, one
// fmaf per k: bit-identical to the VALU kernel's chain.
// MODE (the statistics epilogue; partial sums per workgroup, fixed-order reductions):
//   0: none;
//   1: the res tail's forward statistics of s = relu(h) [+ old] (tail_partial_kernel's
//      sums: s and s*s) -- the pass over h and old that kernel makes is skipped;
//   2: the BatchNorm backward statistics of gy = this (input-gradient) conv's output with
//      the BN output y (bn_partial_kernel's sums: gy and gy*y).
// Per lane fp32 sums over its pixels, then double across lanes and waves.
// FW, FD, FTH (all > 0): the tile geometry (map width, dilation, class rows per tile)
// fixed at compile time, so every k's operand offset is an immediate of its ds_read
// (res26-narrow's 20-pixel maps at d = 1); 0: read from the arguments.
// FOLD: a.fm / a.fi are set (the folded BatchNorm, Conv3Args::fm; compile-time so the
// plain instances keep their register allocation)
template <int C, int MODE, int FW = 0, int FD = 0, int FTH = 0, bool FOLD = false>
__global__ __launch_bounds__(512, 1) void conv3x3d_kernel(Conv3Args a) {
  static_assert(C <= 20, "conv3x3d_kernel: C <= 20");
  constexpr int K = 9 * C, KT = (K + 15) / 16, NG = (C + 3) / 4, PF = 8;  // PF: reads in flight
  __shared__ __attribute__((aligned(16))) float tdl[2 * TD_BUF / 4];
  __shared__ float2 bnf[20];  // the folded BatchNorm's {mean, invstd} per channel (a.fm)
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr bool FIX = FW > 0 && FD > 0 && FTH > 0;
  const int d = FIX ? FD : a.g.d, W = FIX ? FW : a.W, H = a.H;
  const TdGeo G = td_geo(C, W, FIX ? FTH : a.g.TH);
  constexpr bool fold = FOLD && MODE != 0;
  // MODE 2: lane o < C holds channel o's mean / invstd, read out with v_readlane (no
  // memory operation among the k loop's counted LDS reads)
  float fmv = 0.f, fiv = 0.f;
  if (fold) {
    if (MODE == 1 && tid < C) bnf[tid] = float2{a.fm[tid], a.fi[tid]};
    if (MODE == 2 && lane < C) {
      fmv = a.fm[lane];
      fiv = a.fi[lane];
    }
    __syncthreads();
  }
  float wt[NG][KT];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int j = 0; j < KT; ++j) {
      const int o = 4 * g + (lane & 3), k = 16 * j + (lane >> 2);
      float v = 0.f;
      if (o < C && k < K) {
        const int c = k / 9, t = k - 9 * c;
        v = a.flip ? a.w[(c * C + o) * 9 + 8 - t] : a.w[(o * C + c) * 9 + t];
      }
      wt[g][j] = v;
    }
  // per lane and DMA instruction i: chunk e = (wave TD_ITER + i) 64 + lane of the
  // buffer -> (plane c, row rr, 16-B column cc); tile-invariant byte offset of the
  // chunk in its clip (row 0), or -1 for a zero chunk
  int cbase[TD_ITER], crow[TD_ITER];
#pragma unroll
  for (int i = 0; i < TD_ITER; ++i) {
    const int e = (wave * TD_ITER + i) * 64 + lane;
    const int c = e * 4 / G.PS, rem = e * 4 - c * G.PS, rr = rem / G.Wr, col = rem - rr * G.Wr - TD_PAD;
    const bool ok = e < G.nchunk && c < C && rr < G.R && col >= 0 && col < W;
    cbase[i] = ok ? (c * H * W + col) * 4 : -1;
    crow[i] = rr;
  }
  const int ntile = a.B * a.g.nband;
  const size_t clip = (size_t)C * H * W;
  auto issue = [&](int tile, float* buf) {
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, H, tile - b * a.g.nband, r, k0, th);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (size_t)b * clip), (short)0, (int)(clip * 4), 0x00020000);
    const int hr = r + (k0 - 1) * d;
#pragma unroll
    for (int i = 0; i < TD_ITER; ++i) {
      const int h = hr + crow[i] * d;
      const unsigned voff =
          (cbase[i] >= 0 && h >= 0 && h < H) ? (unsigned)(cbase[i] + h * W * 4) : 0x80000000u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(buf + __builtin_amdgcn_readfirstlane((wave * TD_ITER + i) * 256)),
          16, voff, 0, 0, 0);
    }
  };
  // uniform LDS offset of tap t of plane c
  const int PS = G.PS, Wr = G.Wr;
  auto kof = [&](int k) {
    const int c = k / 9, t = k - 9 * c;
    return c * PS + (t / 3) * Wr + (t % 3) * d;
  };
  float sa[MODE ? C : 1], sb[MODE ? C : 1];  // per-lane statistics (MODE 1 / 2)
#pragma unroll
  for (int o = 0; o < (MODE ? C : 1); ++o) sa[o] = sb[o] = 0.f;
  // MODE 1: the lane's sums are of s - piv[o], piv = the lane's first s of the channel,
  // so a channel whose mean is large against its spread (a residual sum) keeps its
  // variance digits in fp32; the lane's (count, sums) are turned back into sums of s and
  // s^2 in double before the cross-lane reduction
  float piv[MODE == 1 ? C : 1];
#pragma unroll
  for (int o = 0; o < (MODE == 1 ? C : 1); ++o) piv[o] = 0.f;
  int pcnt = 0;  // MODE 1: valid pixels this lane has summed
  // Deferred epilogue: a super tile's outputs (stores, statistics) go out during the
  // MFMAs of the wave's next super tile -- one channel every 8 k -- instead of after
  // its own loop, where the 8 waves (one super tile each per band tile) would all sit
  // in their epilogues together with the matrix pipes idle.  Per lane the super tiles
  // and channels are still summed in the same order: bit-identical statistics.
  f32x4_t pacc[NG];  // the pending super tile's accumulators
  float pav[MODE ? C : 1];
#pragma unroll
  for (int g = 0; g < NG; ++g) pacc[g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < (MODE ? C : 1); ++o) pav[o] = 0.f;
  float* pyb = a.y;
  size_t ppix = 0;
  bool ppv = false;  // the pending super tile has a valid pixel in this lane
  unsigned pbits = 0u;  // MODE 1 with a mask: the pending pixel's ReLU bits so far
  auto epi = [&](int o) {
    if (o < C && ppv) {
      const float v = pacc[o >> 2][o & 3];
      if constexpr (MODE == 1) {
        float sv = v <= 0.f ? 0.f : v;  // relu_f: NaN passes, as torch.relu
        if (a.aux) sv = sv + pav[o];
        if (a.mask) {
          pyb[(size_t)o * H * W + ppix] = sv;
          pbits |= (v <= 0.f ? 0u : 1u) << o;
          if (o == C - 1) a.mask[(size_t)(pyb - a.y) / C + ppix] = pbits;  // the pixel's word, once
        } else {
          pyb[(size_t)o * H * W + ppix] = v;
        }
        piv[o] = pcnt == 0 ? sv : piv[o];
        const float dv = sv - piv[o];
        sa[o] += dv;
        sb[o] += dv * dv;
        if (o == C - 1) ++pcnt;
      } else {
        pyb[(size_t)o * H * W + ppix] = v;
      }
      if constexpr (MODE == 2) {
        float yv = pav[o];
        if (fold) {  // aux is the layer below's s: its y as tail_fwd_kernel makes it (at use: the
                     // load's latency stays hidden behind a super tile)
          const float m = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, fmv), o));
          const float iv = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, fiv), o));
          yv = (yv - m) * iv;
        }
        sa[o] += v;
        sb[o] += v * yv;
      }
    }
  };
  constexpr int EK0 = 4, EKS = 8;  // channel o's epilogue at k = EK0 + EKS o
  static_assert(EK0 + EKS * (C - 1) < K, "epilogue inside the k loop");
  float* buf0 = tdl;
  float* buf1 = tdl + TD_BUF / 4;
  if ((int)blockIdx.x < ntile) issue(blockIdx.x, buf0);
  int it = 0;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x, ++it) {
    float* cur = (it & 1) ? buf1 : buf0;
    float* nxt = (it & 1) ? buf0 : buf1;
    td_wait_vm0();
    if (MODE == 1 && fold) {  // the input is the layer below's s: its y in place (own chunks)
      const int b = tile / a.g.nband;
      int r, k0, th;
      band_of(a.g, H, tile - b * a.g.nband, r, k0, th);
      const int hr = r + (k0 - 1) * d;
      bool ok[TD_ITER];
      float2 mv[TD_ITER];
#pragma unroll
      for (int i = 0; i < TD_ITER; ++i) {
        const int h = hr + crow[i] * d;
        ok[i] = cbase[i] >= 0 && h >= 0 && h < H;
        mv[i] = ok[i] ? bnf[4 * ((wave * TD_ITER + i) * 64 + lane) / PS] : float2{0.f, 0.f};
      }
      td_bn_fold(cur, wave * TD_ITER * 64 + lane, ok, mv);
    }
    __syncthreads();  // this tile's DMA landed everywhere; nobody reads nxt any more
    if (tile + (int)gridDim.x < ntile) issue(tile + gridDim.x, nxt);
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, H, tile - b * a.g.nband, r, k0, th);
    const int npx = th * W, nst = (npx + 63) >> 6;
    float* yb = a.y + (size_t)b * clip;
    for (int m = wave; m < nst; m += 8) {  // super tile m: pixels 64 m .. 64 m + 63 of the band
      const int p = 64 * m + lane;
      const bool pv = p < npx;
      const int j = pv ? p / W : 0, col = pv ? p - j * W : 0;
      const float* xp = cur + j * Wr + col + TD_PAD - d;
      f32x4_t acc[NG];
#pragma unroll
      for (int g = 0; g < NG; ++g) acc[g] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      // the statistics epilogue's operand (old / y at this lane's pixel), read now: it is
      // used a whole super tile later
      float av[MODE ? C : 1];
      const size_t pix = (size_t)(r + (k0 + j) * d) * W + col;
      if constexpr (MODE != 0) {
        const float* ab = a.aux ? a.aux + (size_t)b * clip + pix : nullptr;
#pragma unroll
        for (int o = 0; o < C; ++o) av[o] = (ab && pv) ? ab[(size_t)o * H * W] : 0.f;
      }
      float xr[PF];  // ring of operands read PF k ahead (PF divides 16: slots are compile-time)
#pragma unroll
      for (int k = 0; k < PF; ++k) xr[k] = xp[kof(k)];
      static_for<KT>([&](auto jc) {
        constexpr int JJ = decltype(jc)::value;
        static_for<16>([&](auto bc) {
          constexpr int B = decltype(bc)::value;
          constexpr int k = 16 * JJ + B;
          if constexpr (k < K) {
            const float xv = xr[B % PF];
            xr[B % PF] = xp[kof(k + PF < K ? k + PF : K - 1)];
#pragma unroll
            for (int g = 0; g < NG; ++g) acc[g] = __builtin_amdgcn_mfma_f32_4x4x1f32(wt[g][JJ], xv, acc[g], 4, B, 0);
            if constexpr (k >= EK0 && (k - EK0) % EKS == 0 && (k - EK0) / EKS < C) epi((k - EK0) / EKS);
            __builtin_amdgcn_sched_barrier(0);  // keeps each read PF k ahead of its use
          }
        });
      });
      // this super tile becomes the pending one
#pragma unroll
      for (int g = 0; g < NG; ++g) pacc[g] = acc[g];
      if constexpr (MODE != 0) {
#pragma unroll
        for (int o = 0; o < C; ++o) pav[o] = av[o];
      }
      pyb = yb;
      ppix = pix;
      ppv = pv;
      pbits = 0u;
    }
  }
  // the last super tile's epilogue
#pragma unroll
  for (int o = 0; o < C; ++o) epi(o);
  td_wait_vm0();  // no DMA left in flight when the workgroup retires
  if constexpr (MODE != 0) {
    __shared__ double red[8][C][2];
#pragma unroll
    for (int o = 0; o < C; ++o) {
      double u = sa[o], v = sb[o];
      if constexpr (MODE == 1) {  // sums of s and s^2 from the pivoted ones
        const double p = piv[o], n = pcnt;
        v = v + 2.0 * p * u + n * p * p;
        u = u + n * p;
      }
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) {
        u += __shfl_xor(u, m);
        v += __shfl_xor(v, m);
      }
      if (lane == 0) {
        red[wave][o][0] = u;
        red[wave][o][1] = v;
      }
    }
    __syncthreads();
    if (tid < C) {
      double u = 0.0, v = 0.0;
#pragma unroll
      for (int w8 = 0; w8 < 8; ++w8) {
        u += red[w8][tid][0];
        v += red[w8][tid][1];
      }
      a.part[((size_t)tid * gridDim.x + blockIdx.x) * 2] = u;
      a.part[((size_t)tid * gridDim.x + blockIdx.x) * 2 + 1] = v;
    }
  }
}

// class rows per conv3x3d_kernel tile (0: not applicable): the largest band whose
// buffer fits TD_BUF with TD_ITER DMA instructions per wave, balanced over the class
static int td_rows(int C, int H, int W, int d) {
  if (d > TD_PAD || (W & 3) || W > 256 || C > 20) return 0;
  const int hc = (H + d - 1) / d;
  int th = 0;
  for (int t = 1; t <= hc; ++t) {
    const TdGeo g = td_geo(C, W, t);
    if (g.nchunk * 16 > TD_BUF || g.nchunk > 8 * TD_ITER * 64 || C * g.PS >= 65536) break;
    th = t;
  }
  if (th < 1) return 0;
  const int nb = (hc + th - 1) / th;
  return (hc + nb - 1) / nb;
}

// the compile-time geometry instance (res26-narrow: 20-pixel maps, d = 1, 25-row tiles)
// applies; HONK_TD_FIXED=0 turns it off (A/B)
static bool td_fixed(const Conv3Args& a) {
  const char* e = getenv("HONK_TD_FIXED");
  return !(e && e[0] == '0') && a.W == 20 && a.g.d == 1 && a.g.TH == 25;
}

// class rows per conv3x3m_kernel tile: C planes of (TH + 2) x (W + 2d) (+ pad) in TM_XL
static int tm_rows(int C, int H, int W, int d) {
  const int Wp = W + 2 * d;
  int th = (TM_XL / 4 / C - 32) / Wp - 2;
  const int hc = (H + d - 1) / d;
  if (th > hc) th = hc;
  if (th < 1 || W > 256 || (long)C * (th + 2) * Wp >= 65536) return 0;  // 16-bit k-step offsets
  const int nb = (hc + th - 1) / th;
  return (hc + nb - 1) / nb;
}

struct WgradArgs {
  const float* x;   // [B][C][H][W]
  const float* dy;  // [B][C][H][W]
  float* part;      // [gridDim.x][C][C][9] partial sums
  int B, H, W;
  ClassBands g;
  // wgrad3x3d/q_kernel, may be null: x holds the layer below's s, the kernel reads its
  // BatchNorm output (x - fm[c]) fi[c] (Conv3Args::fm)
  const float* fm = nullptr;
  const float* fi = nullptr;
};

// wgrad: 512 threads = NG groups of TG threads (+ idle); group g takes the tile's
// pixels p = g, g + NG, ..; thread (g, u) owns PJ consecutive weight columns
// j = (in ci, tap t) = PJ u .. PJ u + PJ-1 for all C outputs.  Per pixel: PJ x
// reads + CW/4 dy reads ([pixel][out] in LDS) for PJ*CW FMAs (packed).
template <int C>
struct WG {
  // weight columns per thread: 8 for 19 maps (+1.3 % on the res26-narrow step vs 4,
  // 2: -4 %), 4 for 45 maps (8 spills)
  static constexpr int PJ = C <= 20 ? 8 : 4;
  static constexpr int TG = (C * 9 + PJ - 1) / PJ;  // threads per group
  static constexpr int NG = 512 / TG;                     // pixel groups
};

template <int C>
__global__ __launch_bounds__(512) void wgrad3x3_kernel(WgradArgs a) {
  constexpr int CW = TC<C>::CW, TG = WG<C>::TG, NG = WG<C>::NG, PJ = WG<C>::PJ;
  __shared__ __attribute__((aligned(16))) float xl[TC_XL / 4];
  __shared__ __attribute__((aligned(16))) float dl[TC_XL / 4];
  const int tid = threadIdx.x;
  const int grp = tid / TG, u = tid - grp * TG;
  const bool active = grp < NG;
  const int d = a.g.d, Wp = a.W + 2 * d;
  tf2 acc[PJ][CW / 2];
  int jo[PJ];  // per owned column: LDS offset of (ci, tap) in the tile (row 0, col 0), -1 if none
#pragma unroll
  for (int n = 0; n < PJ; ++n) {
#pragma unroll
    for (int o = 0; o < CW / 2; ++o) acc[n][o] = tf2{0.f, 0.f};
  }
  for (int tile = blockIdx.x; tile < a.B * a.g.nband; tile += gridDim.x) {
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, a.H, tile - b * a.g.nband, r, k0, th);
    const int rows = th + 2, plane = rows * Wp, npx = th * a.W;
    __syncthreads();
    // staging with 8 loads in flight per thread (a serial load-store loop waits out
    // the HBM latency on every element)
    const float* xb = a.x + (size_t)b * C * a.H * a.W;
    for (int i0 = tid; i0 < C * plane; i0 += 8 * 512) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 512;
        const int c = i / plane, rc = i - c * plane, rr = rc / Wp, col = rc - rr * Wp;
        const int h = r + (k0 - 1 + rr) * d, w = col - d;
        v[u] = (i < C * plane && h >= 0 && h < a.H && w >= 0 && w < a.W) ? xb[((size_t)c * a.H + h) * a.W + w] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (i0 + u * 512 < C * plane) xl[i0 + u * 512] = v[u];
    }
    const float* db = a.dy + (size_t)b * C * a.H * a.W;
    for (int i0 = tid; i0 < CW * npx; i0 += 8 * 512) {  // dy transposed to [pixel][out]
      float v[8];
      int dst[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 512;
        const int o = i / npx, p = i - o * npx;
        const int j = p / a.W, col = p - j * a.W;
        v[u] = (i < CW * npx && o < C) ? db[(size_t)o * a.H * a.W + (size_t)(r + (k0 + j) * d) * a.W + col] : 0.f;
        dst[u] = i < CW * npx ? p * CW + o : -1;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (dst[u] >= 0) dl[dst[u]] = v[u];
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int n = 0; n < PJ; ++n) {
        const int j = PJ * u + n;
        const int ci = j / 9, t = j - ci * 9;
        jo[n] = j < C * 9 ? ci * plane + (t / 3) * Wp + (t % 3) * d : 0;
      }
      for (int p = grp; p < npx; p += NG) {
        const int j = p / a.W, col = p - j * a.W;
        const int po = j * Wp + col;
        tf2 xv[PJ];
#pragma unroll
        for (int n = 0; n < PJ; ++n) {
          const float v = xl[jo[n] + po];
          xv[n] = tf2{v, v};
        }
        const float4* d4 = (const float4*)(dl + p * CW);
#pragma unroll
        for (int q = 0; q < CW / 4; ++q) {
          const float4 d = d4[q];
          const tf2 da = tf2{d.x, d.y}, dbv = tf2{d.z, d.w};
#pragma unroll
          for (int n = 0; n < PJ; ++n) {
            acc[n][2 * q] = __builtin_elementwise_fma(xv[n], da, acc[n][2 * q]);
            acc[n][2 * q + 1] = __builtin_elementwise_fma(xv[n], dbv, acc[n][2 * q + 1]);
          }
        }
      }
    }
  }
  // the NG groups' columns summed in LDS (fixed order), 4 output channels at a time
  __syncthreads();  // every group is done with the tile images
  float* red = xl;  // NG x (C*9) x 4 floats
  float* pb = a.part + (size_t)blockIdx.x * C * C * 9;
#pragma unroll
  for (int q = 0; q < CW / 4; ++q) {
    if (active) {
#pragma unroll
      for (int n = 0; n < PJ; ++n) {
        const int j = PJ * u + n;
        if (j < C * 9)
          *(float4*)(red + ((size_t)grp * C * 9 + j) * 4) =
              float4{acc[n][2 * q].x, acc[n][2 * q].y, acc[n][2 * q + 1].x, acc[n][2 * q + 1].y};
      }
    }
    __syncthreads();
    for (int idx = tid; idx < C * 9 * 4; idx += 512) {
      float v = 0.f;
      for (int g = 0; g < NG; ++g) v += red[(size_t)g * C * 9 * 4 + idx];
      const int o = 4 * q + (idx & 3), j = idx >> 2;
      if (o < C) pb[o * C * 9 + j] = v;  // [o][ci][t]: j = ci*9 + t
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------- //
// wgrad3x3m_kernel<C> (C <= 20): the weight gradient on v_mfma_f32_16x16x4_f32 as
// a GEMM D[o][j] = sum_p dy[o][p] X[j][p] over the tile's pixels p (k of the MFMA),
// j = 9 ci + t (input channel, tap) -- the [o][ci][t] layout of dW.  M = output
// channels (C -> 2 tiles of 16), N = 9C columns (171 -> 11 tiles), so one wave holds
// 22 accumulator tiles and reads 2 A + 11 B floats per 4 pixels (22 MFMAs).  A band of
// TH class rows is staged as in conv3x3m_kernel (x with a one-row / d-column zero
// halo at a fixed plane stride; dy as [o][TH W]), 2 workgroups per CU so one
// stages while the other multiplies.  The 4 waves take interleaved k-steps; their
// partials are summed in LDS in wave order and each workgroup writes one partial
// dW, which wsum_kernel adds in a fixed order (deterministic, no atomics).
// ---------------------------------------------------------------------------- //
// staged x / dy bytes per workgroup (2 workgroups per CU; 3 would spill the accumulators)
constexpr int TW_XL = 36 * 1024, TW_DL = 28 * 1024;

template <int C>
__global__ __launch_bounds__(256, 2) void wgrad3x3m_kernel(WgradArgs a) {
  static_assert(C <= 20, "wgrad3x3m_kernel: C <= 20");
  constexpr int K9 = 9 * C, NJ = (K9 + 15) / 16, NO = (C + 15) / 16;
  __shared__ __attribute__((aligned(16))) float lds[(TW_XL + TW_DL) / 4];
  float* xl = lds;
  float* dl = lds + TW_XL / 4;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, kk = lane >> 4;
  const int d = a.g.d, Wp = a.W + 2 * d, TH = a.g.TH;
  const int R = TH + 2, PS = R * Wp, DS = TH * a.W;  // x plane stride, dy plane stride
  int joff[NJ];  // B lanes: LDS offset of column j = 16 n + i16 (pad columns read plane 0)
#pragma unroll
  for (int n = 0; n < NJ; ++n) {
    const int j = 16 * n + i16, ci = j / 9, t = j - 9 * ci;
    joff[n] = j < K9 ? ci * PS + (t / 3) * Wp + (t % 3) * d : 0;
  }
  f32x4_t acc[NO][NJ];
#pragma unroll
  for (int m = 0; m < NO; ++m)
#pragma unroll
    for (int n = 0; n < NJ; ++n) acc[m][n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  // halo columns zeroed once (every tile writes only the W interior columns)
  for (int i = tid; i < C * R * 2 * d; i += 256) {
    const int row = i / (2 * d), e = i - row * (2 * d);
    const int c = row / R, rr = row - c * R;
    xl[c * PS + rr * Wp + (e < d ? e : a.W + e)] = 0.f;
  }
  const float invR = 1.0f / (float)R, invT = 1.0f / (float)TH, invW = 1.0f / (float)a.W;
  for (int tile = blockIdx.x; tile < a.B * a.g.nband; tile += gridDim.x) {
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, a.H, tile - b * a.g.nband, r, k0, th);
    __syncthreads();  // previous tile's readers done
    {
      // one pass over the C R x rows (channel c, band row rr: image row hr + rr d)
      // and then the C TH dy rows (channel o, band row jr < th), so the x tail's
      // loads overlap the first dy loads
      const float* xb = a.x + (size_t)b * C * a.H * a.W;
      const float* db = a.dy + (size_t)b * C * a.H * a.W;
      const int H = a.H, W = a.W, hr = r + (k0 - 1) * d, NX = C * R;
      stage_rows(
          lds, NX + C * TH, W,
          [&](int row) -> const float* {
            if (row < NX) {
              const int c = div_small(row, R, invR), h = hr + (row - c * R) * d;
              return h >= 0 && h < H ? xb + ((size_t)c * H + h) * W : nullptr;
            }
            const int o = div_small(row - NX, TH, invT), jr = row - NX - o * TH;
            return jr < th ? db + ((size_t)o * H + r + (k0 + jr) * d) * W : nullptr;
          },
          [&](int row) {
            if (row < NX) {
              const int c = div_small(row, R, invR);
              return c * PS + (row - c * R) * Wp + d;
            }
            const int o = div_small(row - NX, TH, invT);
            return TW_XL / 4 + o * DS + (row - NX - o * TH) * W;
          });
    }
    __syncthreads();
    const int npx = th * a.W, nks = (npx + 3) >> 2;
    for (int s = wave; s < nks; s += 4) {
      const int p = 4 * s + kk;
      const bool pv = p < npx;  // k beyond the band: A = 0 (B reads pixel 0, finite)
      const int pp = pv ? p : 0;
      const int row = div_small(pp, a.W, invW), col = pp - row * a.W;
      const float* xp = xl + row * Wp + col;
      float av[NO], bv[NJ];
#pragma unroll
      for (int m = 0; m < NO; ++m) {
        const int o = 16 * m + i16;
        av[m] = (pv && o < C) ? dl[o * DS + pp] : 0.f;
      }
#pragma unroll
      for (int n = 0; n < NJ; ++n) bv[n] = xp[joff[n]];
#pragma unroll
      for (int m = 0; m < NO; ++m)
#pragma unroll
        for (int n = 0; n < NJ; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m], bv[n], acc[m][n], 0, 0, 0);
    }
  }
  // the 4 waves' partials summed in wave order, one 16-row output tile at a time:
  // red[w][i][j], i = row in the tile (lane (j, g) holds rows 4 g .. 4 g + 3)
  float* pb = a.part + (size_t)blockIdx.x * C * K9;
  constexpr int NJP = NJ * 16;
#pragma unroll
  for (int m = 0; m < NO; ++m) {
    __syncthreads();
#pragma unroll
    for (int n = 0; n < NJ; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) lds[(wave * 16 + 4 * kk + i) * NJP + 16 * n + i16] = acc[m][n][i];
    __syncthreads();
    for (int idx = tid; idx < 16 * K9; idx += 256) {
      const int i = idx / K9, j = idx - i * K9, o = 16 * m + i;
      const float v = ((lds[i * NJP + j] + lds[(16 + i) * NJP + j]) + lds[(32 + i) * NJP + j]) + lds[(48 + i) * NJP + j];
      if (o < C) pb[o * K9 + j] = v;
    }
  }
}

// ---------------------------------------------------------------------------- //
// wgrad3x3d_kernel<C> (C <= 20, d <= 4, W a multiple of 4): wgrad3x3m_kernel's GEMM
// on conv3x3d_kernel's double-buffered LDS-DMA staging.  A buffer holds the x band
// (TdGeo planes) followed by the dy band ([o][TH W] at a plane stride = 4 mod 64, so
// the 16 A lanes of a read hit 16 banks); 8 waves take interleaved k-steps; their
// partials are summed in wave order, one partial per workgroup (wsum_kernel).
// ---------------------------------------------------------------------------- //
// 9 DMA instructions per wave per tile: two 72-KB buffers (144 of the CU's 160 KB), a
// 17-row band for res26-narrow (8 k-steps of 4 px per wave were 8 -> 10.6 per tile)
constexpr int TWD_ITER = 9;
constexpr int TWD_BUF = 8 * TWD_ITER * 1024;

__host__ __device__ inline int twd_ds(int TH, int W) {  // dy plane stride (floats)
  const int f = TH * W;
  return f + ((4 - f % 64) + 64) % 64;
}
__host__ __device__ inline int twd_nchunk(int C, int W, int TH) {
  const TdGeo g = td_geo(C, W, TH);
  return (C * g.PS / 4 + C * twd_ds(TH, W) / 4 + 63) / 64 * 64;
}

// The staging of one weight-gradient tile (wgrad3x3d_kernel, wgrad3x3q_kernel): per
// lane and DMA instruction i, chunk e -> x chunk (plane c, row rr: image row hr + rr d)
// or dy chunk (plane o, band row jr: image row r + (k0 + jr) d), as the byte offset in
// its clip tensor at row 0 and the band row; kind 0 = zero chunk
struct TwdStage {
  int cbase[TWD_ITER], crow[TWD_ITER], ckind[TWD_ITER];
};
__device__ __forceinline__ void twd_stage_init(TwdStage& s, int C, int H, int W, int TH, const TdGeo& G, int wave,
                                               int lane) {
  const int DS = twd_ds(TH, W), XF = C * G.PS, nch = twd_nchunk(C, W, TH);
#pragma unroll
  for (int i = 0; i < TWD_ITER; ++i) {
    const int e = (wave * TWD_ITER + i) * 64 + lane, f = e * 4;
    s.cbase[i] = 0;
    s.crow[i] = 0;
    s.ckind[i] = 0;
    if (e < nch && f < XF) {
      const int c = f / G.PS, rem = f - c * G.PS, rr = rem / G.Wr, col = rem - rr * G.Wr - TD_PAD;
      if (rr < G.R && col >= 0 && col < W) {
        s.cbase[i] = (c * H * W + col) * 4;
        s.crow[i] = rr - 1;
        s.ckind[i] = 1;
      }
    } else if (e < nch && f - XF < C * DS) {
      const int g = f - XF, o = g / DS, rem = g - o * DS, jr = rem / W, col = rem - jr * W;
      if (jr < TH) {
        s.cbase[i] = (o * H * W + col) * 4;
        s.crow[i] = jr;
        s.ckind[i] = 2;
      }
    }
  }
}
// DMA of tile `tile` (x band + dy band of one clip) into buf
__device__ __forceinline__ void twd_issue(const TwdStage& s, const WgradArgs& a, int C, int H, int W, int d, int tile,
                                          float* buf, int wave) {
  const int b = tile / a.g.nband;
  int r, k0, th;
  band_of(a.g, H, tile - b * a.g.nband, r, k0, th);
  const size_t clip = (size_t)C * H * W;
  const __amdgpu_buffer_rsrc_t rx =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.x + (size_t)b * clip), (short)0, (int)(clip * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd =
      __builtin_amdgcn_make_buffer_rsrc((void*)(a.dy + (size_t)b * clip), (short)0, (int)(clip * 4), 0x00020000);
  const int hb = r + k0 * d;
#pragma unroll
  for (int i = 0; i < TWD_ITER; ++i) {
    const int h = hb + s.crow[i] * d;
    const bool ok = s.ckind[i] != 0 && h >= 0 && h < H && (s.ckind[i] == 1 || s.crow[i] < th);
    const unsigned voff = ok ? (unsigned)(s.cbase[i] + h * W * 4) : 0x80000000u;
    // one LDS slot per lane: a lane's chunk comes from dy (rd) or x / zeros (rx); the
    // instruction that straddles the x / dy boundary runs twice under complementary
    // exec masks, every slot written once
    if (s.ckind[i] == 2)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rd, (__attribute__((address_space(3))) void*)(buf + __builtin_amdgcn_readfirstlane((wave * TWD_ITER + i) * 256)),
          16, voff, 0, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rx, (__attribute__((address_space(3))) void*)(buf + __builtin_amdgcn_readfirstlane((wave * TWD_ITER + i) * 256)),
          16, voff, 0, 0, 0);
  }
}

// td_bn_fold on this lane's x chunks of tile `tile` (kind 1, in-image rows)
__device__ __forceinline__ void twd_bn_fold(const TwdStage& s, const WgradArgs& a, int H, int d, int tile, float* buf,
                                            const float2 (&mv)[TWD_ITER], int wave, int lane) {
  const int b = tile / a.g.nband;
  int r, k0, th;
  band_of(a.g, H, tile - b * a.g.nband, r, k0, th);
  const int hb = r + k0 * d;
  bool ok[TWD_ITER];
#pragma unroll
  for (int i = 0; i < TWD_ITER; ++i) {
    const int h = hb + s.crow[i] * d;
    ok[i] = s.ckind[i] == 1 && h >= 0 && h < H;
  }
  td_bn_fold(buf, wave * TWD_ITER * 64 + lane, ok, mv);
}
// the {mean, invstd} of this lane's x chunks' planes (tile-invariant), {0, 0} elsewhere
__device__ __forceinline__ void twd_bn_mv(float2 (&mv)[TWD_ITER], const TwdStage& s, const WgradArgs& a, int wave,
                                         int lane, int PS) {
#pragma unroll
  for (int i = 0; i < TWD_ITER; ++i) {
    const int c = 4 * ((wave * TWD_ITER + i) * 64 + lane) / PS;
    mv[i] = s.ckind[i] == 1 ? float2{a.fm[c], a.fi[c]} : float2{0.f, 0.f};
  }
}

// FW, FD, FTH (all > 0): compile-time tile geometry, as conv3x3d_kernel's
template <int C, int FW = 0, int FD = 0, int FTH = 0>
__global__ __launch_bounds__(512, 1) void wgrad3x3d_kernel(WgradArgs a) {
  static_assert(C > 16 && C <= 20, "wgrad3x3d_kernel: 16 < C <= 20");
  constexpr int K9 = 9 * C, NJ = (K9 + 15) / 16, NH = (K9 + 63) / 64;
  __shared__ __attribute__((aligned(16))) float tdl[2 * TWD_BUF / 4];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i16 = lane & 15, kk = lane >> 4;
  constexpr bool FIX = FW > 0 && FD > 0 && FTH > 0;
  const int d = FIX ? FD : a.g.d, W = FIX ? FW : a.W, H = a.H, TH = FIX ? FTH : a.g.TH;
  const TdGeo G = td_geo(C, W, TH);
  const int DS = twd_ds(TH, W), XF = C * G.PS;  // dy planes start at float XF
  int joff[NJ];
#pragma unroll
  for (int n = 0; n < NJ; ++n) {
    const int j = 16 * n + i16, ci = j / 9, t = j - 9 * ci;
    joff[n] = j < K9 ? ci * G.PS + (t / 3) * G.Wr + (t % 3) * d : 0;
  }
  // outputs 0..15: 16x16x4 tiles acc[n] (rows o, columns j = 16 n + i16); outputs 16..C-1:
  // 4x4x1 blocks acc4[h] (block b, column c: j = 64 h + 4 b + c), the dy of one pixel
  // for 4 outputs broadcast from block 4 q (conv3x3d_kernel's scheme)
  f32x4_t acc[NJ], acc4[NH];
#pragma unroll
  for (int n = 0; n < NJ; ++n) acc[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < NH; ++h) acc4[h] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  TwdStage stg;
  twd_stage_init(stg, C, H, W, TH, G, wave, lane);
  float2 fmv[TWD_ITER];
  if (a.fm) twd_bn_mv(fmv, stg, a, wave, lane, G.PS);
  const int ntile = a.B * a.g.nband;
  auto issue = [&](int tile, float* buf) { twd_issue(stg, a, C, H, W, d, tile, buf, wave); };
  float* buf0 = tdl;
  float* buf1 = tdl + TWD_BUF / 4;
  if ((int)blockIdx.x < ntile) issue(blockIdx.x, buf0);
  const float invW = 1.0f / (float)W;
  int it = 0;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x, ++it) {
    float* cur = (it & 1) ? buf1 : buf0;
    float* nxt = (it & 1) ? buf0 : buf1;
    td_wait_vm0();
    if (a.fm) twd_bn_fold(stg, a, H, d, tile, cur, fmv, wave, lane);
    __syncthreads();
    if (tile + (int)gridDim.x < ntile) issue(tile + gridDim.x, nxt);
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, H, tile - b * a.g.nband, r, k0, th);
    const int npx = th * W, nks = (npx + 3) >> 2;
    const float* dl = cur + XF;
    // operands of k-step s + 8 (this wave's next) are read before step s's MFMAs; the
    // 4x4 MFMAs interleave with the 16x16x4 ones (acc4[h] in q order)
    auto ld = [&](int s, float& a0, float& a1, float* bv) {
      const int p = 4 * s + kk;
      const bool pv = p < npx;
      const int pp = pv ? p : 0;
      const int row = div_small(pp, W, invW), col = pp - row * W;
      const float* xp = cur + row * G.Wr + col + TD_PAD - d;
      // a0 lane (kk, i16) = dy(o = i16, pixel 4 s + kk); a1 the same for o = 16 + i16,
      // read by lanes i16 < 4 (block 4 kk of the 4x4 MFMA)
      a0 = pv ? dl[i16 * DS + pp] : 0.f;
      a1 = (pv && i16 < 4 && 16 + i16 < C) ? dl[(16 + i16) * DS + pp] : 0.f;
#pragma unroll
      for (int n = 0; n < NJ; ++n) bv[n] = xp[joff[n]];
#pragma unroll
      for (int n = NJ; n < 4 * NH; ++n) bv[n] = 0.f;
    };
    auto step = [&](float a0, float a1, const float* bv) {
      float bt[4 * NH];
#pragma unroll
      for (int n = 0; n < 4 * NH; ++n) bt[n] = bv[n];
#pragma unroll
      for (int h = 0; h < NH; ++h)
        tr4_rows(bt[4 * h], bt[4 * h + 1], bt[4 * h + 2], bt[4 * h + 3]);  // lane l: x(j = 64 h + l, pixel 4 s + q)
#pragma unroll
      for (int n = 0; n < 4 * NH; ++n) {
        if (n < NJ) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, bv[n], acc[n], 0, 0, 0);
        const int h = n % NH, q = n / NH;
        acc4[h] = mfma4_bc(a1, bt[4 * h + q], acc4[h], 4 * q);
      }
    };
    // two operand sets in turn (no register moves between steps)
    float e0 = 0.f, e1 = 0.f, ev[4 * NH], o0 = 0.f, o1 = 0.f, ov[4 * NH];
    if (wave < nks) ld(wave, e0, e1, ev);
    for (int s = wave; s < nks; s += 16) {
      ld(s + 8 < nks ? s + 8 : s, o0, o1, ov);
      step(e0, e1, ev);
      if (s + 8 >= nks) break;
      ld(s + 16 < nks ? s + 16 : s, e0, e1, ev);
      step(o0, o1, ov);
    }
  }
  td_wait_vm0();
  float* pb = a.part + (size_t)blockIdx.x * C * K9;
  constexpr int NJP = NJ * 16;
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    __syncthreads();
    if (m == 0) {
#pragma unroll
      for (int n = 0; n < NJ; ++n)
#pragma unroll
        for (int i = 0; i < 4; ++i) tdl[(wave * 16 + 4 * kk + i) * NJP + 16 * n + i16] = acc[n][i];
    } else {
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (64 * h + lane < NJP) tdl[(wave * 16 + i) * NJP + 64 * h + lane] = acc4[h][i];
    }
    __syncthreads();
    for (int idx = tid; idx < 16 * K9; idx += 512) {
      const int i = idx / K9, j = idx - i * K9, o = 16 * m + i;
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += tdl[(16 * w + i) * NJP + j];
      if (o < C) pb[o * K9 + j] = v;
    }
  }
}

// ---------------------------------------------------------------------------- //
// wgrad3x3q_kernel<C> (16 < C <= 20, d <= 4, W a multiple of 4): the weight gradient
// as one rank-1 update per pixel, dW[o][j] += dy[o][p] x_j[p] (j = 9 ci + t), on
// broadcast 4x4x1 blocks only -- conv3x3d_kernel's scheme turned around: block b of
// a v_mfma_f32_4x4x1_16b_f32 multiplies the 4 outputs o = 4 g .. 4 g + 3 (A, broadcast
// from the block that holds them) by the 4 columns j = 64 h + 4 b .. 64 h + 4 b + 3 (B,
// lane = column), so one pixel is NG x NH = 5 x 3 MFMAs of 8 cycles over 20 x 192
// padded outputs (0.85 of the pipe useful for 19 maps; wgrad3x3d's 16x16x4 + 4x4x1 mix
// is 0.91 but needs two transposed operand copies).  A k-step is 4 pixels of one row (W
// % 4 = 0): its operands are 2 A registers (dy of (g, q) in block 4 g + q; g = 4 in
// block q of the second) and NH x 4 B values (x of column j at pixels q = 0..3: two
// ds_read2_b32 per h at immediate offsets), 8 LDS instructions for 60 MFMAs, read one
// step ahead (no address arithmetic but 5 adds of a wave-uniform base).  Staging, tile
// loop and the per-workgroup partials as wgrad3x3d_kernel; every output is the same
// sequence of fp32 FMAs over the wave's pixels as there (bit-identical).
//   HY (hybrid): outputs 0..15 on 16x16x4 tiles instead (lane (kk, i16): dy(o = i16) and
// x(j = 16 n + i16) at pixel 4 s + kk, one ds_read_b32 each: 11 tiles for 171 columns),
// outputs 16..19 on the 4x4x1 blocks as above -- 11 x 36 + 12 x 10 cycles per step
// against 60 x 10 (measured issue rates, exp/mfma44.hip), 12 more reads.  Measured no
// faster on res26-narrow's tiles (0.379 vs 0.382 ms per 4096-clip call) and slower on
// 40-pixel maps (0.48 vs 0.41 ms, exp/wgrad_ab.py): kept for A/B only (HONK_WGRAD=h).
// ---------------------------------------------------------------------------- //
template <int C, bool HY, int FW = 0, int FD = 0, int FTH = 0>
__global__ __launch_bounds__(512, 1) void wgrad3x3q_kernel(WgradArgs a) {
  static_assert(C > 16 && C <= 20, "wgrad3x3q_kernel: 16 < C <= 20");
  constexpr int K9 = 9 * C, NH = (K9 + 63) / 64, NG = (C + 3) / 4, NJP = 64 * NH, NJ = (K9 + 15) / 16;
  static_assert(8 * 4 * NG * NJP <= 2 * TWD_BUF / 4, "wgrad3x3q_kernel: partials exceed the LDS buffers");
  static_assert(16 * NJ <= NJP, "wgrad3x3q_kernel: tile columns exceed the partial rows");
  __shared__ __attribute__((aligned(16))) float tdl[2 * TWD_BUF / 4];
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr bool FIX = FW > 0 && FD > 0 && FTH > 0;
  const int d = FIX ? FD : a.g.d, W = FIX ? FW : a.W, H = a.H, TH = FIX ? FTH : a.g.TH;
  const TdGeo G = td_geo(C, W, TH);
  const int DS = twd_ds(TH, W), XF = C * G.PS;  // dy planes start at float XF
  // B: column j = 64 h + lane -> x(ci, tap t) relative to the pixel's slot (columns past
  // K9 read column K9 - 1: their products land in discarded outputs)
  int boff[NH];
#pragma unroll
  for (int h = 0; h < NH; ++h) {
    const int j = min(64 * h + lane, K9 - 1), ci = j / 9, t = j - 9 * ci;
    boff[h] = ci * G.PS + (t / 3) * G.Wr + (t % 3) * d + TD_PAD - d;
  }
  // A: lane 4 b + i of register 0 holds dy(o = 4 g + i, pixel q) with block b = 4 g + q;
  // register 1 holds o = 16 + i for two k-steps, this wave's s (block q, lanes < 16) and
  // s + 8 (block 4 + q, lanes 16..31: pixel + 32).  Rows o >= C (discarded) read o = C - 1.
  const int q = (lane >> 2) & 3;
  const int aoff0 = (4 * (lane >> 4) + (lane & 3)) * DS + q;
  const int o1 = min(16 + (lane & 3), C - 1);
  const int aoff1 = XF + o1 * DS, apx1 = q + ((lane >> 4) & 1) * 32;
  // HY: lane (kk, i16) of the 16x16x4 operands: dy(o = i16) and x(j = 16 n + i16) at pixel + kk
  const int i16 = lane & 15, kk = lane >> 4;
  const int aoff16 = XF + i16 * DS + kk;
  int boff16[HY ? NJ : 1];
#pragma unroll
  for (int n = 0; n < (HY ? NJ : 1); ++n) {
    const int j = min(16 * n + i16, K9 - 1), ci = j / 9, t = j - 9 * ci;
    boff16[n] = ci * G.PS + (t / 3) * G.Wr + (t % 3) * d + TD_PAD - d + kk;
  }
  f32x4_t acc[NG][NH], acc16[HY ? NJ : 1];
#pragma unroll
  for (int g = 0; g < NG; ++g)
#pragma unroll
    for (int h = 0; h < NH; ++h) acc[g][h] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int n = 0; n < (HY ? NJ : 1); ++n) acc16[n] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  TwdStage stg;
  twd_stage_init(stg, C, H, W, TH, G, wave, lane);
  float2 fmv[TWD_ITER];
  if (a.fm) twd_bn_mv(fmv, stg, a, wave, lane, G.PS);
  const int ntile = a.B * a.g.nband;
  float* buf0 = tdl;
  float* buf1 = tdl + TWD_BUF / 4;
  if ((int)blockIdx.x < ntile) twd_issue(stg, a, C, H, W, d, blockIdx.x, buf0, wave);
  struct Ops {
    float a0, b[4][NH], b16[HY ? NJ : 1];
  };
  int it = 0;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x, ++it) {
    float* cur = (it & 1) ? buf1 : buf0;
    float* nxt = (it & 1) ? buf0 : buf1;
    td_wait_vm0();
    if (a.fm) twd_bn_fold(stg, a, H, d, tile, cur, fmv, wave, lane);  // x: the layer below's s -> y
    __syncthreads();
    if (tile + (int)gridDim.x < ntile) twd_issue(stg, a, C, H, W, d, tile + gridDim.x, nxt, wave);
    const int b = tile / a.g.nband;
    int r, k0, th;
    band_of(a.g, H, tile - b * a.g.nband, r, k0, th);
    const int nks = th * W / 4;
    // the load cursor: k-step ls = pixel 4 ls of the band, at (lrow, lcol); this wave's
    // steps are wave, wave + 8, ..
    int lrow = (4 * wave) / W, lcol = 4 * wave - lrow * W;
    // 7 LDS instructions per step (register 1 every other step): with the next step's
    // in flight, at most 15 outstanding -- the lgkmcnt range, so each step waits for its
    // own reads only
    auto ld = [&](Ops& o) {
      const float* xp = cur + lrow * G.Wr + lcol;
      if constexpr (HY) {
        o.a0 = cur[aoff16 + lrow * W + lcol];
#pragma unroll
        for (int n = 0; n < NJ; ++n) o.b16[n] = xp[boff16[n]];
      } else {
        o.a0 = cur[XF + aoff0 + lrow * W + lcol];
      }
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int u = 0; u < 4; ++u) o.b[u][h] = xp[boff[h] + u];
      lcol += 32;
      while (lcol >= W) {
        lcol -= W;
        ++lrow;
      }
    };
    const int npx1 = th * W - 1;
    auto ld1 = [&](int s) { return cur[aoff1 + min(4 * s + apx1, npx1)]; };
    // a step's operands are complete when it starts (read a step earlier); the reads of
    // the next step go out after its first pixel's 15 MFMAs (`next`), so they never
    // share the lgkm counter with reads still awaited
    auto step = [&](const Ops& o, float a1, auto ab, auto&& next) {
      if constexpr (HY) {
        // 16x16x4 tile n, then the 4x4x1 block of (pixel u, h) = divmod(n, NH), in turn;
        // the next step's reads after the first 3 + 3
        static_for<4 * NH>([&](auto m) {
          constexpr int u = m / NH, h = m % NH;
          if constexpr (m < NJ) acc16[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(o.a0, o.b16[m], acc16[m], 0, 0, 0);
          acc[NG - 1][h] =
              __builtin_amdgcn_mfma_f32_4x4x1f32(a1, o.b[u][h], acc[NG - 1][h], 4, decltype(ab)::value + u, 0);
          if constexpr (m == NH - 1) {
            __builtin_amdgcn_sched_barrier(0);
            next();
            __builtin_amdgcn_sched_barrier(0);
          }
        });
        return;
      }
      static_for<4>([&](auto u) {
#pragma unroll
        for (int h = 0; h < NH; ++h) {
          static_for<NG>([&](auto g) {
            if constexpr (g < 4)
              acc[g][h] = __builtin_amdgcn_mfma_f32_4x4x1f32(o.a0, o.b[u][h], acc[g][h], 4, 4 * g + u, 0);
            else
              acc[g][h] = __builtin_amdgcn_mfma_f32_4x4x1f32(a1, o.b[u][h], acc[g][h], 4, decltype(ab)::value + u, 0);
          });
        }
        if constexpr (u == 0) {
          __builtin_amdgcn_sched_barrier(0);
          next();
          __builtin_amdgcn_sched_barrier(0);
        }
      });
    };
    // four steps per trip: register 1 alternates between a1a and a1b without a copy
    Ops e, o;
    float a1a = 0.f, a1b = 0.f;
    if (wave < nks) {
      ld(e);
      a1a = ld1(wave);
    }
    constexpr std::integral_constant<int, 0> B0{};
    constexpr std::integral_constant<int, 4> B4{};
    for (int s = wave; s < nks; s += 32) {
      step(e, a1a, B0, [&] {
        if (s + 8 < nks) ld(o);
      });
      if (s + 8 >= nks) break;
      step(o, a1a, B4, [&] {
        if (s + 16 < nks) {
          ld(e);
          a1b = ld1(s + 16);
        }
      });
      if (s + 16 >= nks) break;
      step(e, a1b, B0, [&] {
        if (s + 24 < nks) ld(o);
      });
      if (s + 24 >= nks) break;
      step(o, a1b, B4, [&] {
        if (s + 32 < nks) {
          ld(e);
          a1a = ld1(s + 32);
        }
      });
    }
  }
  td_wait_vm0();
  __syncthreads();
  // per-wave partials [wave][4 g + i][j], summed in wave order
#pragma unroll
  for (int g = HY ? NG - 1 : 0; g < NG; ++g)
#pragma unroll
    for (int h = 0; h < NH; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i) tdl[(wave * 4 * NG + 4 * g + i) * NJP + 64 * h + lane] = acc[g][h][i];
  if constexpr (HY) {
#pragma unroll
    for (int n = 0; n < NJ; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) tdl[(wave * 4 * NG + 4 * kk + i) * NJP + 16 * n + i16] = acc16[n][i];
  }
  __syncthreads();
  float* pb = a.part + (size_t)blockIdx.x * C * K9;
  for (int idx = tid; idx < C * K9; idx += 512) {
    const int o = idx / K9, j = idx - o * K9;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < 8; ++w) v += tdl[(4 * NG * w + o) * NJP + j];
    pb[idx] = v;
  }
}

// class rows per wgrad3x3d_kernel tile (0: not applicable)
static int twd_rows(int C, int H, int W, int d) {
  if (d > TD_PAD || (W & 3) || W > 256 || C > 20) return 0;
  const int hc = (H + d - 1) / d;
  int th = 0;
  for (int t = 1; t <= hc; ++t) {
    if (twd_nchunk(C, W, t) > 8 * TWD_ITER * 64 || C * td_geo(C, W, t).PS >= 65536) break;
    th = t;
  }
  if (th < 1) return 0;
  const int nb = (hc + th - 1) / th;
  return (hc + nb - 1) / nb;
}

// wgrad3x3d_kernel's compile-time geometry instance (res26-narrow: W = 20, d = 1, 17-row
// bands); HONK_TD_FIXED=0 turns it off (A/B)
static bool twd_fixed(const WgradArgs& a) {
  const char* e = getenv("HONK_TD_FIXED");
  return !(e && e[0] == '0') && a.W == 20 && a.g.d == 1 && a.g.TH == 17;
}

// class rows per wgrad3x3m_kernel tile: C x planes of (TH + 2) x (W + 2d) in TW_XL,
// C dy planes of TH x W in TW_DL, the 4 waves' 64 x 16 NJ partial sums in both
static int tw_rows(int C, int H, int W, int d) {
  const int Wp = W + 2 * d;
  int th = TW_XL / 4 / C / Wp - 2;
  const int byd = TW_DL / 4 / C / W;
  if (th > byd) th = byd;
  const int hc = (H + d - 1) / d;
  if (th > hc) th = hc;
  if (th < 1 || W > 256 || (long)C * (th + 2) * Wp >= 65536) return 0;
  const int nb = (hc + th - 1) / th;
  return (hc + nb - 1) / nb;
}

// dw[i] = sum over the nblk per-workgroup partials, fixed order: 16 outputs per
// workgroup, 16 strands over k (k = strand mod 16, 8 loads in flight per strand)
// combined in strand order in LDS
constexpr int WSUM_OUT = 16;
__global__ __launch_bounds__(256) void wsum_kernel(const float* __restrict__ part, float* __restrict__ dw, int n,
                                                   int nblk) {
  __shared__ float red[16][WSUM_OUT + 1];
  const int il = threadIdx.x & (WSUM_OUT - 1), strand = threadIdx.x / WSUM_OUT;
  const int i = blockIdx.x * WSUM_OUT + il;
  float s = 0.f;
  if (i < n) {
#pragma unroll 8
    for (int k = strand; k < nblk; k += 16) s += part[(size_t)k * n + i];
  }
  red[strand][il] = s;
  __syncthreads();
  if (strand == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][il];
    dw[i] = t;
  }
}

// ---------------------------------------------------------------------------- //
// Train-mode BatchNorm2d(affine=False) of the res blocks (model.py:100,117-118 in
// training): batch statistics over (B, H, W) per channel, running-stat update,
// normalisation; backward dx = invstd (dy - mean(dy) - y mean(dy y)) with y = the
// normalised output (affine=False: y IS x-hat).  PyTorch's NCHW kernels take one
// workgroup row per channel (19 channels -> 9 ms per layer per 4096 clips);
// here a channel's B planes are split over S workgroups, each reducing in fp64,
// and a per-channel pass combines the S partials in a fixed order.
// ---------------------------------------------------------------------------- //
__device__ __forceinline__ double bn_block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wv] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// part[c][s] = (sum a, sum a*b) over planes b of slice s of channel c, a = p[.], b = q[.]
// (q == nullptr: b = a, i.e. the sum of squares)
__global__ __launch_bounds__(256) void bn_partial_kernel(const float* __restrict__ p, const float* __restrict__ q,
                                                         double* __restrict__ part, int B, int C, int HW, int S) {
  __shared__ double red[4];
  const int c = blockIdx.x, s = blockIdx.y;
  const int b0 = (int)((int64_t)B * s / S), b1 = (int)((int64_t)B * (s + 1) / S);
  double sa = 0.0, sab = 0.0;
  if ((HW & 3) == 0) {  // one flat float4 sweep over the slice's planes (more loads in flight)
    const int hw4 = HW >> 2;
    const int n4 = (b1 - b0) * hw4;
    for (int k = threadIdx.x; k < n4; k += 256) {
      const int pl = k / hw4, o4 = k - pl * hw4;
      const size_t off = ((size_t)(b0 + pl) * C + c) * HW + 4 * o4;
      const float4 a = *(const float4*)(p + off);
      const float4 bb = q ? *(const float4*)(q + off) : a;
      sa += (double)((a.x + a.y) + (a.z + a.w));
      sab += (double)a.x * bb.x + (double)a.y * bb.y + (double)a.z * bb.z + (double)a.w * bb.w;
    }
  } else {
    for (int b = b0; b < b1; ++b) {
      const size_t base = ((size_t)b * C + c) * HW;
      for (int i = threadIdx.x; i < HW; i += 256) {
        const float a = p[base + i];
        const float bb = q ? q[base + i] : a;
        sa += (double)a;
        sab += (double)a * (double)bb;
      }
    }
  }
  sa = bn_block_sum(sa, red);
  sab = bn_block_sum(sab, red);
  if (threadIdx.x == 0) {
    part[((size_t)c * S + s) * 2] = sa;
    part[((size_t)c * S + s) * 2 + 1] = sab;
  }
}

// the S (sum a, sum ab) partials of channel c = blockIdx.x, summed by one workgroup:
// thread t takes slices t, t + 256, .. in order, then a fixed LDS tree
__device__ __forceinline__ void bn_combine(const double* __restrict__ part, int S, double& s1, double& s2) {
  __shared__ double r1[256], r2[256];
  const int c = blockIdx.x, t = threadIdx.x;
  double a = 0.0, b = 0.0;
  for (int s = t; s < S; s += 256) {
    a += part[((size_t)c * S + s) * 2];
    b += part[((size_t)c * S + s) * 2 + 1];
  }
  r1[t] = a;
  r2[t] = b;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (t < w) {
      r1[t] += r1[t + w];
      r2[t] += r2[t + w];
    }
    __syncthreads();
  }
  s1 = r1[0];
  s2 = r2[0];
}

// forward: mean, invstd per channel; running stats (momentum, unbiased variance).
// One workgroup of 256 threads per channel.
__global__ __launch_bounds__(256) void bn_stats_kernel(const double* __restrict__ part, float* __restrict__ mean,
                                                       float* __restrict__ invstd, float* __restrict__ rmean,
                                                       float* __restrict__ rvar, int C, int S, double n,
                                                       float momentum, float eps) {
  double s1, s2;
  bn_combine(part, S, s1, s2);
  const int c = blockIdx.x;
  if (threadIdx.x != 0) return;
  const double m = s1 / n;
  double var = s2 / n - m * m;
  if (var < 0.0) var = 0.0;
  mean[c] = (float)m;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (rmean) {
    rmean[c] = (float)((1.0 - momentum) * (double)rmean[c] + momentum * m);
    rvar[c] = (float)((1.0 - momentum) * (double)rvar[c] + momentum * var * n / (n > 1.0 ? n - 1.0 : 1.0));
  }
}

// backward: per-channel mean(dy), mean(dy*y); one workgroup per channel
__global__ __launch_bounds__(256) void bn_bstats_kernel(const double* __restrict__ part, float* __restrict__ mdy,
                                                        float* __restrict__ mdyy, int C, int S, double n) {
  double s1, s2;
  bn_combine(part, S, s1, s2);
  if (threadIdx.x != 0) return;
  mdy[blockIdx.x] = (float)(s1 / n);
  mdyy[blockIdx.x] = (float)(s2 / n);
}

// out = (a - u[c]) * v[c]                         (forward: y = (x - mean) invstd)
// out = v[c] * (a - u[c] - b * w[c])              (backward: dx, a = dy, b = y)
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                       const float* __restrict__ u, const float* __restrict__ v,
                                                       const float* __restrict__ w, float* __restrict__ out,
                                                       int64_t total, int C, int HW) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((HW & 3) == 0) {  // float4 per thread (a float4 never crosses a channel plane)
    const int64_t i4 = 4 * i;
    if (i4 >= total) return;
    const int c = (int)((i4 / HW) % C);
    const float4 av = *(const float4*)(a + i4);
    float4 r;
    if (b) {
      const float4 bv = *(const float4*)(b + i4);
      r = float4{v[c] * (av.x - u[c] - bv.x * w[c]), v[c] * (av.y - u[c] - bv.y * w[c]),
                 v[c] * (av.z - u[c] - bv.z * w[c]), v[c] * (av.w - u[c] - bv.w * w[c])};
    } else {
      r = float4{(av.x - u[c]) * v[c], (av.y - u[c]) * v[c], (av.z - u[c]) * v[c], (av.w - u[c]) * v[c]};
    }
    *(float4*)(out + i4) = r;
    return;
  }
  if (i >= total) return;
  const int c = (int)((i / HW) % C);
  out[i] = b ? v[c] * (a[i] - u[c] - b[i] * w[c]) : (a[i] - u[c]) * v[c];
}

// ---------------------------------------------------------------------------- //
// The res block tail fused around the train-mode BatchNorm (model.py:111-118):
//   s = relu(h) [+ old]   (h = the block conv's output, old = the residual stream)
//   y = (s - mean) * invstd, batch statistics of s
// and its backward
//   g = invstd (gy - mean(gy) - y mean(gy y)) [+ gs]   (gs: grad of s as the next residual)
//   gold = g,  gh = g where h > 0 else 0
// so that ReLU, the residual add, its gradient accumulation and ReLU's backward
// never round-trip HBM on their own.  Every value is the same fp32 operation the
// unfused PyTorch graph performs (relu, add, BatchNorm kernels above, autograd's
// accumulation, threshold_backward): bit-identical to it.
// ---------------------------------------------------------------------------- //
__device__ __forceinline__ float relu_f(float h) { return h <= 0.f ? 0.f : h; }  // NaN passes, as torch.relu

__global__ __launch_bounds__(256) void tail_partial_kernel(const float* __restrict__ h, const float* __restrict__ old,
                                                           double* __restrict__ part, int B, int C, int HW, int S) {
  __shared__ double red[4];
  const int c = blockIdx.x, s = blockIdx.y;
  const int b0 = (int)((int64_t)B * s / S), b1 = (int)((int64_t)B * (s + 1) / S);
  double sa = 0.0, sab = 0.0;
  if ((HW & 3) == 0) {
    const int hw4 = HW >> 2;
    const int n4 = (b1 - b0) * hw4;
    for (int k = threadIdx.x; k < n4; k += 256) {
      const int pl = k / hw4, o4 = k - pl * hw4;
      const size_t off = ((size_t)(b0 + pl) * C + c) * HW + 4 * o4;
      const float4 hv = *(const float4*)(h + off);
      float4 a = float4{relu_f(hv.x), relu_f(hv.y), relu_f(hv.z), relu_f(hv.w)};
      if (old) {
        const float4 ov = *(const float4*)(old + off);
        a = float4{a.x + ov.x, a.y + ov.y, a.z + ov.z, a.w + ov.w};
      }
      sa += (double)((a.x + a.y) + (a.z + a.w));
      sab += (double)a.x * a.x + (double)a.y * a.y + (double)a.z * a.z + (double)a.w * a.w;
    }
  } else {
    for (int b = b0; b < b1; ++b) {
      const size_t base = ((size_t)b * C + c) * HW;
      for (int i = threadIdx.x; i < HW; i += 256) {
        float a = relu_f(h[base + i]);
        if (old) a = a + old[base + i];
        sa += (double)a;
        sab += (double)a * (double)a;
      }
    }
  }
  sa = bn_block_sum(sa, red);
  sab = bn_block_sum(sab, red);
  if (threadIdx.x == 0) {
    part[((size_t)c * S + s) * 2] = sa;
    part[((size_t)c * S + s) * 2 + 1] = sab;
  }
}

// y = (relu(h) [+ old] - mean[c]) * invstd[c]; s_out (may be null) = relu(h) [+ old]
// (s_in: h already holds s = relu(h) [+ old], made by the conv's epilogue: y = (h - mean) * invstd)
template <bool S_IN>
__global__ __launch_bounds__(256) void tail_fwd_kernel(const float* __restrict__ h, const float* __restrict__ old,
                                                       const float* __restrict__ u, const float* __restrict__ v,
                                                       float* __restrict__ y, float* __restrict__ s_out, int64_t total,
                                                       int C, int HW) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((HW & 3) == 0) {
    const int64_t i4 = 4 * i;
    if (i4 >= total) return;
    const int c = (int)((i4 / HW) % C);
    const float4 hv = *(const float4*)(h + i4);
    if constexpr (S_IN) {
      *(float4*)(y + i4) = float4{(hv.x - u[c]) * v[c], (hv.y - u[c]) * v[c], (hv.z - u[c]) * v[c], (hv.w - u[c]) * v[c]};
      return;
    }
    float4 a = float4{relu_f(hv.x), relu_f(hv.y), relu_f(hv.z), relu_f(hv.w)};
    if (old) {
      const float4 ov = *(const float4*)(old + i4);
      a = float4{a.x + ov.x, a.y + ov.y, a.z + ov.z, a.w + ov.w};
    }
    if (s_out) *(float4*)(s_out + i4) = a;
    *(float4*)(y + i4) = float4{(a.x - u[c]) * v[c], (a.y - u[c]) * v[c], (a.z - u[c]) * v[c], (a.w - u[c]) * v[c]};
    return;
  }
  if (i >= total) return;
  const int c = (int)((i / HW) % C);
  if constexpr (S_IN) {
    y[i] = (h[i] - u[c]) * v[c];
    return;
  }
  float a = relu_f(h[i]);
  if (old) a = a + old[i];
  if (s_out) s_out[i] = a;
  y[i] = (a - u[c]) * v[c];
}

// g = v[c] (gy - u[c] - y w[c]) [+ gs]; gold (may be null) = g; gh = h > 0 ? g : 0
// (MASK: the conv epilogue's bit mask in place of h: word [b][p], bit c = !(h <= 0))
// (FOLD: y holds the tail's s, the BatchNorm output is (s - ym[c]) v[c] -- tail_fwd_kernel's
// expression; the tail wrote no y, its next conv folded it in)
template <bool MASK, bool FOLD = false>
__global__ __launch_bounds__(256) void tail_bwd_kernel(const float* __restrict__ gy, const float* __restrict__ y,
                                                       const float* __restrict__ gs, const void* __restrict__ hm,
                                                       const float* __restrict__ u, const float* __restrict__ v,
                                                       const float* __restrict__ w, float* __restrict__ gh,
                                                       float* __restrict__ gold, int64_t total, int C, int HW,
                                                       const float* __restrict__ ym) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float* h = (const float*)hm;
  const unsigned* mk = (const unsigned*)hm;
  if ((HW & 3) == 0) {
    const int64_t i4 = 4 * i;
    if (i4 >= total) return;
    const int64_t bc = i4 / HW;
    const int c = (int)(bc % C);
    const float4 av = *(const float4*)(gy + i4);
    float4 bv = *(const float4*)(y + i4);
    if constexpr (FOLD) bv = float4{(bv.x - ym[c]) * v[c], (bv.y - ym[c]) * v[c], (bv.z - ym[c]) * v[c], (bv.w - ym[c]) * v[c]};
    float4 hv;
    if constexpr (MASK) {
      // the 4 pixels' words (pixel p = i4 - bc HW of clip b = bc / C)
      const uint4 mw = *(const uint4*)(mk + (bc / C) * HW + (i4 - bc * HW));
      hv = float4{((mw.x >> c) & 1u) ? 1.f : 0.f, ((mw.y >> c) & 1u) ? 1.f : 0.f, ((mw.z >> c) & 1u) ? 1.f : 0.f,
                  ((mw.w >> c) & 1u) ? 1.f : 0.f};
    } else {
      hv = *(const float4*)(h + i4);
    }
    float4 g = float4{v[c] * (av.x - u[c] - bv.x * w[c]), v[c] * (av.y - u[c] - bv.y * w[c]),
                      v[c] * (av.z - u[c] - bv.z * w[c]), v[c] * (av.w - u[c] - bv.w * w[c])};
    if (gs) {
      const float4 sv = *(const float4*)(gs + i4);
      g = float4{g.x + sv.x, g.y + sv.y, g.z + sv.z, g.w + sv.w};
    }
    if (gold) *(float4*)(gold + i4) = g;
    *(float4*)(gh + i4) = float4{hv.x <= 0.f ? 0.f : g.x, hv.y <= 0.f ? 0.f : g.y, hv.z <= 0.f ? 0.f : g.z,
                                 hv.w <= 0.f ? 0.f : g.w};
    return;
  }
  if (i >= total) return;
  const int64_t bc = i / HW;
  const int c = (int)(bc % C);
  const float yv = FOLD ? (y[i] - ym[c]) * v[c] : y[i];
  float g = v[c] * (gy[i] - u[c] - yv * w[c]);
  if (gs) g = g + gs[i];
  if (gold) gold[i] = g;
  if constexpr (MASK) gh[i] = ((mk[(bc / C) * HW + (i - bc * HW)] >> c) & 1u) ? g : 0.f;
  else gh[i] = h[i] <= 0.f ? 0.f : g;
}

// ---------------------------------------------------------------------------- //
// The res stem in training (model.py:104-110): y = AvgPool2d(ph, pw)(relu(conv0(x)))
// (no pool: ph = pw = 1), conv0 = Conv2d(1, C, 3, padding 1, no bias), and its
// weight gradient (the input needs none).  One workgroup per clip at a time: the
// clip's [H][W] map is staged into LDS with a zero border; thread (o, q) owns output
// channel o (its 9 weights in registers) and every Q-th output pixel.  The pool sums
// its window in row-major order and divides, as avg_pool2d's kernels do.  Backward
// recomputes the conv (9 FMAs) for the ReLU mask instead of keeping the pre-pool map;
// each thread accumulates its channel's 9 weight gradients, summed over the Q
// threads of a channel in a fixed order into one partial per workgroup (wsum_kernel).
// ---------------------------------------------------------------------------- //
constexpr int STEM_XL = 8192;  // floats of the staged (H+2) x (W+2) map (static LDS kernels)
// maps past STEM_XL (the wide eval fallback, e.g. 101 x 160 inputs): stem_kernel with the
// image and the reduction buffer in dynamic LDS, up to the CU's 160 KiB
constexpr int STEM_XL_DYN = 160 * 256 - 256 * 9;  // floats

struct StemArgs {
  const float* x;   // [B][H][W]
  const float* w;   // [C][1][3][3]
  const float* gy;  // backward: [B][C][Hp][Wp]
  float* y;         // forward: [B][C][Hp][Wp]
  float* part;      // backward: [gridDim.x][C][9]
  int B, C, H, W, ph, pw;
};

__device__ __forceinline__ float stem_conv(const float* xs, int Ws, int h, int w, const float (&wr)[9]) {
  float acc = 0.f;
#pragma unroll
  for (int t = 0; t < 9; ++t) acc = fmaf(wr[t], xs[(h + t / 3) * Ws + w + t % 3], acc);
  return acc;
}

// the clip's map into the bordered LDS image, 8 loads in flight per thread (float4s
// when rows are whole float4s)
__device__ __forceinline__ void stem_stage(float* xs, const float* xb, int H, int W) {
  const int Ws = W + 2;
  if ((W & 3) == 0) {
    const int n4 = H * W / 4;
    for (int i0 = threadIdx.x; i0 < n4; i0 += 8 * 256) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 256;
        v[u] = i < n4 ? *(const float4*)(xb + 4 * i) : float4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 256;
        if (i < n4) {
          const int h = 4 * i / W, w = 4 * i - h * W;
          float* d = xs + (h + 1) * Ws + w + 1;
          d[0] = v[u].x; d[1] = v[u].y; d[2] = v[u].z; d[3] = v[u].w;
        }
      }
    }
    return;
  }
  for (int i0 = threadIdx.x; i0 < H * W; i0 += 8 * 256) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 256;
      v[u] = i < H * W ? xb[i] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 256;
      if (i < H * W) {
        const int h = i / W, w = i - h * W;
        xs[(h + 1) * Ws + w + 1] = v[u];
      }
    }
  }
}

__device__ __forceinline__ void stem_border(float* xs, int H, int W) {
  const int Ws = W + 2;
  for (int i = threadIdx.x; i < (H + 2) * Ws; i += 256) {
    const int h = i / Ws, w = i - h * Ws;
    if (h == 0 || h == H + 1 || w == 0 || w == W + 1) xs[i] = 0.f;
  }
}

template <bool BWD, bool DYN = false>
__global__ __launch_bounds__(256) void stem_kernel(StemArgs a) {
  __shared__ float xs_s[DYN ? 1 : STEM_XL];
  __shared__ float red_s[DYN ? 1 : 256 * 9];
  extern __shared__ float dyn_lds[];
  float* xs = DYN ? dyn_lds + 256 * 9 : xs_s;
  float* red = DYN ? dyn_lds : red_s;
  const int Q = 256 / a.C, o = threadIdx.x / Q, q = threadIdx.x - o * Q;
  const bool act = o < a.C;
  float wr[9], dw[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    wr[t] = act ? a.w[o * 9 + t] : 0.f;
    dw[t] = 0.f;
  }
  const int Ws = a.W + 2, Hp = a.H / a.ph, Wq = a.W / a.pw, np = a.ph * a.pw;
  stem_border(xs, a.H, a.W);
  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    __syncthreads();  // previous clip's readers done (and the border written)
    stem_stage(xs, a.x + (size_t)b * a.H * a.W, a.H, a.W);
    __syncthreads();
    if (!act) continue;
    const size_t ob = ((size_t)b * a.C + o) * Hp * Wq;
    if (!BWD) {
      for (int px = q; px < Hp * Wq; px += Q) {
        const int i = px / Wq, j = px - i * Wq;
        float s = 0.f;
        for (int u = 0; u < a.ph; ++u)
          for (int v = 0; v < a.pw; ++v) s += relu_f(stem_conv(xs, Ws, i * a.ph + u, j * a.pw + v, wr));
        a.y[ob + px] = np == 1 ? s : s / (float)np;
      }
    } else {
      for (int px = q; px < a.H * a.W; px += Q) {
        const int h = px / a.W, w = px - h * a.W, i = h / a.ph, j = w / a.pw;
        if (i >= Hp || j >= Wq) continue;              // rows / columns the floor pooling drops
        if (stem_conv(xs, Ws, h, w, wr) <= 0.f) continue;  // ReLU's backward
        const float g0 = a.gy[ob + i * Wq + j];
        const float g = np == 1 ? g0 : g0 / (float)np;
#pragma unroll
        for (int t = 0; t < 9; ++t) dw[t] = fmaf(g, xs[(h + t / 3) * Ws + w + t % 3], dw[t]);
      }
    }
  }
  if (!BWD) return;
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 9; ++t) red[threadIdx.x * 9 + t] = dw[t];
  __syncthreads();
  if (act && q == 0) {
    float* pb = a.part + (size_t)blockIdx.x * a.C * 9 + o * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float s = 0.f;
      for (int k = 0; k < Q; ++k) s += red[(threadIdx.x + k) * 9 + t];
      pb[t] = s;
    }
  }
}

// stem_kernel with the pool window fixed at compile time: a thread item is SW
// horizontally adjacent pooled outputs (SW = 4 without pool, where each output is
// one conv pixel), read once as a (PH + 2) x (SW PW + 2) register patch: 16 LDS
// reads for a 2x2 window instead of 36, and one index computation per item.  Same
// arithmetic as stem_kernel: the 9-tap fmaf chain per conv pixel, the window summed
// row-major then divided; backward accumulates each thread's dW in item order.
template <bool BWD, int PH, int PW, int SW>
__global__ __launch_bounds__(256) void stem_tile_kernel(StemArgs a) {
  constexpr int PR = PH + 2, PC = SW * PW + 2, NP = PH * PW;
  __shared__ float xs[STEM_XL];
  __shared__ float red[256 * 9];
  const int Q = 256 / a.C, o = threadIdx.x / Q, q = threadIdx.x - o * Q;
  const bool act = o < a.C;
  float wr[9], dw[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    wr[t] = act ? a.w[o * 9 + t] : 0.f;
    dw[t] = 0.f;
  }
  const int Ws = a.W + 2, Hp = a.H / PH, Wq = a.W / PW, ipr = Wq / SW;  // host: SW divides Wq
  const float inv_ipr = 1.0f / (float)ipr;
  stem_border(xs, a.H, a.W);
  for (int b = blockIdx.x; b < a.B; b += gridDim.x) {
    __syncthreads();
    stem_stage(xs, a.x + (size_t)b * a.H * a.W, a.H, a.W);
    __syncthreads();
    if (!act) continue;
    const size_t ob = ((size_t)b * a.C + o) * Hp * Wq;
    for (int it = q; it < Hp * ipr; it += Q) {
      const int i = div_small(it, ipr, inv_ipr), j0 = (it - i * ipr) * SW;
      float pt[PR][PC];
      const float* src = xs + i * PH * Ws + j0 * PW;
#pragma unroll
      for (int u = 0; u < PR; ++u)
#pragma unroll
        for (int v = 0; v < PC; ++v) pt[u][v] = src[u * Ws + v];
#pragma unroll
      for (int sw = 0; sw < SW; ++sw) {
        float g = 0.f;
        if (BWD) {
          const float g0 = a.gy[ob + (size_t)i * Wq + j0 + sw];
          g = NP == 1 ? g0 : g0 / (float)NP;
        }
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < PH; ++u)
#pragma unroll
          for (int v = 0; v < PW; ++v) {
            const int c0 = sw * PW + v;
            float acc = 0.f;
#pragma unroll
            for (int t = 0; t < 9; ++t) acc = fmaf(wr[t], pt[u + t / 3][c0 + t % 3], acc);
            if (!BWD) {
              s += relu_f(acc);
            } else if (!(acc <= 0.f)) {  // ReLU's backward (as stem_kernel)
#pragma unroll
              for (int t = 0; t < 9; ++t) dw[t] = fmaf(g, pt[u + t / 3][c0 + t % 3], dw[t]);
            }
          }
        if (!BWD) a.y[ob + (size_t)i * Wq + j0 + sw] = NP == 1 ? s : s / (float)NP;
      }
    }
  }
  if (!BWD) return;
  __syncthreads();
#pragma unroll
  for (int t = 0; t < 9; ++t) red[threadIdx.x * 9 + t] = dw[t];
  __syncthreads();
  if (act && q == 0) {
    float* pb = a.part + (size_t)blockIdx.x * a.C * 9 + o * 9;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      float s = 0.f;
      for (int k = 0; k < Q; ++k) s += red[(threadIdx.x + k) * 9 + t];
      pb[t] = s;
    }
  }
}

// launch the stem pass: a compile-time window for res26/res8 pools and no pool
template <bool BWD>
static void stem_launch(const StemArgs& a, int grid, hipStream_t st) {
  const int Wq = a.W / a.pw;
  const int xl = (a.H + 2) * (a.W + 2);
  if (xl > STEM_XL) {
    const unsigned bytes = (unsigned)(256 * 9 + xl) * 4u;
    (void)hipFuncSetAttribute((const void*)stem_kernel<BWD, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)bytes);
    hipLaunchKernelGGL((stem_kernel<BWD, true>), dim3(grid), dim3(256), bytes, st, a);
  } else if (a.ph == 2 && a.pw == 2) hipLaunchKernelGGL((stem_tile_kernel<BWD, 2, 2, 1>), dim3(grid), dim3(256), 0, st, a);
  else if (a.ph == 4 && a.pw == 3) hipLaunchKernelGGL((stem_tile_kernel<BWD, 4, 3, 1>), dim3(grid), dim3(256), 0, st, a);
  else if (a.ph == 1 && a.pw == 1 && Wq % 4 == 0)
    hipLaunchKernelGGL((stem_tile_kernel<BWD, 1, 1, 4>), dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(stem_kernel<BWD>, dim3(grid), dim3(256), 0, st, a);
}

static int bn_slices(int B, int C) {
  int S = (4 * 256 + C - 1) / C;  // ~4 workgroups per CU in total
  if (S > B) S = B;
  return S < 1 ? 1 : S;
}

// class rows per tile: the staged input (C planes of (TH+2) x (W+2d)) and (wgrad)
// its dy within TC_XL, at most 1024 pixels (4 per thread); bands balanced over the
// (longest) class
static int tc_rows(int C, int H, int W, int d, bool conv = false) {
  int th = (conv && C <= 20 ? TC_XLC : TC_XL) / 4 / (C * (W + 2 * d)) - 2;
  const int byp = (C <= 20 ? 1024 : 512) / W;  // conv3x3_kernel: NP <= 4 (19 maps) / 2 (45 maps)
  if (th > byp) th = byp;
  if (!conv) {
    const int byd = TC_XL / 4 / (((C + 3) & ~3) * W);
    if (th > byd) th = byd;
  }
  const int hc = (H + d - 1) / d;  // rows of the longest class
  if (th > hc) th = hc;
  if (th < 1) return 0;
  const int nb = (hc + th - 1) / th;
  return (hc + nb - 1) / nb;
}
static int tc_grid(int64_t tiles) {
  const int64_t g = 2 * (int64_t)cu_count();
  return (int)(tiles < g ? tiles : g);
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

namespace {
int tc_check(const void* a, const void* b, const void* c, int64_t batch, int32_t ch, int32_t h, int32_t w,
             int32_t d) {
  if (!a || !b || !c) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 0 || h < 1 || w < 1) return fail(HONK_ERR_ARG, "bad conv3x3 shape (B=%lld H=%d W=%d)", (long long)batch, h, w);
  if (d < 1 || d > 64) return fail(HONK_ERR_ARG, "conv3x3: dilation %d (1..64)", d);
  if (ch != 19 && ch != 45) return fail(HONK_ERR_UNSUPPORTED, "conv3x3 training kernels: C=%d (19 or 45)", ch);
  if (train::tc_rows(ch, h, w, d) < 1 || train::tc_rows(ch, h, w, d, true) < 1)
    return fail(HONK_ERR_UNSUPPORTED, "conv3x3: width %d at dilation %d too large", w, d);
  if (batch * (int64_t)h > 0x3fffffff) return fail(HONK_ERR_ARG, "conv3x3: batch too large");
  return HONK_OK;
}
}  // namespace

extern "C" int honk_conv3x3_check(int32_t c, int32_t h, int32_t w_, int32_t dil) {
  static const float dummy = 0.f;
  return tc_check(&dummy, &dummy, &dummy, 1, c, h, w_, dil);
}

extern "C" int honk_conv3x3_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c, int32_t h,
                                int32_t w_, int32_t dil, int32_t flip, void* stream) {
  int rc = tc_check(x, w, y, batch, c, h, w_, dil);
  if (rc) return rc;
  if (batch == 0) return HONK_OK;
  train::Conv3Args a;
  a.x = x; a.w = w; a.y = y;
  a.B = (int)batch; a.H = h; a.W = w_; a.flip = flip ? 1 : 0;
  a.g = train::class_bands(h, dil, train::tc_rows(c, h, w_, dil, true));
  const int grid = train::tc_grid((int64_t)a.B * a.g.nband);
  hipStream_t st = (hipStream_t)stream;
  TimedLaunch tl(st, 2.0 * (double)batch * h * w_ * c * c * 9);
  const int np = (int)cdiv((int64_t)a.g.TH * w_, 256);  // output pixels per thread
  // 19 maps: the LDS-DMA double-buffered MFMA kernel where it applies (d <= 4, W % 4 == 0),
  // else the register-staged one; HONK_TRAIN_CONV=m / v forces conv3x3m / the VALU kernel
  // (tests compare all three bitwise)
  const char* ke = getenv("HONK_TRAIN_CONV");
  const int tdr = c == 19 && !(ke && (ke[0] == 'v' || ke[0] == 'm')) ? train::td_rows(c, h, w_, dil) : 0;
  if (tdr > 0) {
    a.g = train::class_bands(h, dil, tdr);
    const int gd = (int)std::min<int64_t>((int64_t)a.B * a.g.nband, cu_count());
    if (train::td_fixed(a)) hipLaunchKernelGGL((train::conv3x3d_kernel<19, 0, 20, 1, 25>), dim3(gd), dim3(512), 0, st, a);
    else hipLaunchKernelGGL((train::conv3x3d_kernel<19, 0>), dim3(gd), dim3(512), 0, st, a);
  } else if (c == 19 && !(ke && ke[0] == 'v') && train::tm_rows(c, h, w_, dil) > 0) {
    a.g = train::class_bands(h, dil, train::tm_rows(c, h, w_, dil));
    const int gm = train::tc_grid((int64_t)a.B * a.g.nband);
    hipLaunchKernelGGL((train::conv3x3m_kernel<19>), dim3(gm), dim3(256), 0, st, a);
  } else if (c == 19) {
    if (np <= 1) hipLaunchKernelGGL((train::conv3x3_kernel<19, 1>), dim3(grid), dim3(256), 0, st, a);
    else if (np == 2) hipLaunchKernelGGL((train::conv3x3_kernel<19, 2>), dim3(grid), dim3(256), 0, st, a);
    else if (np == 3) hipLaunchKernelGGL((train::conv3x3_kernel<19, 3>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((train::conv3x3_kernel<19, 4>), dim3(grid), dim3(256), 0, st, a);
  } else {
    if (np <= 1) hipLaunchKernelGGL((train::conv3x3_kernel<45, 1>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((train::conv3x3_kernel<45, 2>), dim3(grid), dim3(256), 0, st, a);
  }
  tl.done(st);
  HONK_LAUNCH_CHECK("conv3x3_kernel");
  return HONK_OK;
}

namespace {
// the weight-gradient kernel for a shape: the MFMA one for 19 maps (HONK_TRAIN_CONV=v
// selects the VALU kernel, for tests), its class-band geometry and grid
struct WgradPlan {
  bool mfma, dma;
  train::ClassBands g;
  int grid;
};
WgradPlan wgrad_plan(int64_t batch, int c, int h, int w_, int dil) {
  WgradPlan p;
  const char* ke = getenv("HONK_TRAIN_CONV");
  const int td = c == 19 && !(ke && (ke[0] == 'v' || ke[0] == 'm')) ? train::twd_rows(c, h, w_, dil) : 0;
  const int tw = c == 19 && !(ke && ke[0] == 'v') ? train::tw_rows(c, h, w_, dil) : 0;
  p.dma = td > 0;
  p.mfma = !p.dma && tw > 0;
  p.g = train::class_bands(h, dil, p.dma ? td : p.mfma ? tw : train::tc_rows(c, h, w_, dil));
  p.grid = p.dma ? (int)std::min<int64_t>(batch * p.g.nband, cu_count()) : train::tc_grid(batch * p.g.nband);
  return p;
}
}  // namespace

extern "C" size_t honk_conv3x3_wgrad_workspace_bytes(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil) {
  if (batch < 1 || (c != 19 && c != 45) || h < 1 || w_ < 1 || dil < 1 || dil > 64) return 0;
  if (train::tc_rows(c, h, w_, dil) < 1) return 0;
  // the largest grid of any kernel choice (the environment may switch kernels between
  // this query and the call)
  int64_t t = batch * train::class_bands(h, dil, train::tc_rows(c, h, w_, dil)).nband;
  const int tw = c == 19 ? train::tw_rows(c, h, w_, dil) : 0;
  if (tw > 0) t = std::max<int64_t>(t, batch * train::class_bands(h, dil, tw).nband);
  const int td = c == 19 ? train::twd_rows(c, h, w_, dil) : 0;  // grid <= CUs < tc_grid's 2 CUs
  if (td > 0) t = std::max<int64_t>(t, batch * train::class_bands(h, dil, td).nband);
  return (size_t)train::tc_grid(t) * c * c * 9 * sizeof(float);
}

namespace {
int conv3x3_wgrad(const float* x, const float* dy, float* dw, int64_t batch, int32_t c, int32_t h, int32_t w_,
                  int32_t dil, const float* fm, const float* fi, void* workspace, size_t ws_bytes, void* stream) {
  int rc = tc_check(x, dy, dw, batch, c, h, w_, dil);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  const int n = c * c * 9;
  if (batch == 0) {
    HONK_HIP_CHECK(hipMemsetAsync(dw, 0, (size_t)n * sizeof(float), st));
    return HONK_OK;
  }
  const size_t need = honk_conv3x3_wgrad_workspace_bytes(batch, c, h, w_, dil);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  train::WgradArgs a;
  a.x = x; a.dy = dy; a.part = (float*)workspace;
  a.B = (int)batch; a.H = h; a.W = w_;
  a.fm = fm; a.fi = fi;
  const WgradPlan wp = wgrad_plan(batch, c, h, w_, dil);
  if (fm && !wp.dma) return fail(HONK_ERR_UNSUPPORTED, "conv3x3 wgrad: folded BatchNorm needs the DMA-staged kernels");
  a.g = wp.g;
  const int grid = wp.grid;
  TimedLaunch tl(st, 2.0 * (double)batch * h * w_ * c * c * 9);
  // HONK_WGRAD=d: wgrad3x3d_kernel instead of wgrad3x3q_kernel (A/B, tests)
  const char* we = getenv("HONK_WGRAD");
  const bool wq = !(we && we[0] == 'd');
  const bool wh = we && we[0] == 'h';  // HONK_WGRAD=h: the hybrid (16x16x4 for outputs 0..15)
  if (wp.dma && wq && wh && train::twd_fixed(a))
    hipLaunchKernelGGL((train::wgrad3x3q_kernel<19, true, 20, 1, 17>), dim3(grid), dim3(512), 0, st, a);
  else if (wp.dma && wq && wh) hipLaunchKernelGGL((train::wgrad3x3q_kernel<19, true>), dim3(grid), dim3(512), 0, st, a);
  else if (wp.dma && wq && train::twd_fixed(a))
    hipLaunchKernelGGL((train::wgrad3x3q_kernel<19, false, 20, 1, 17>), dim3(grid), dim3(512), 0, st, a);
  else if (wp.dma && wq) hipLaunchKernelGGL((train::wgrad3x3q_kernel<19, false>), dim3(grid), dim3(512), 0, st, a);
  else if (wp.dma && train::twd_fixed(a)) hipLaunchKernelGGL((train::wgrad3x3d_kernel<19, 20, 1, 17>), dim3(grid), dim3(512), 0, st, a);
  else if (wp.dma) hipLaunchKernelGGL((train::wgrad3x3d_kernel<19>), dim3(grid), dim3(512), 0, st, a);
  else if (wp.mfma) hipLaunchKernelGGL((train::wgrad3x3m_kernel<19>), dim3(grid), dim3(256), 0, st, a);
  else if (c == 19) hipLaunchKernelGGL((train::wgrad3x3_kernel<19>), dim3(grid), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((train::wgrad3x3_kernel<45>), dim3(grid), dim3(512), 0, st, a);
  tl.done(st);
  HONK_LAUNCH_CHECK("wgrad3x3_kernel");
  hipLaunchKernelGGL(train::wsum_kernel, dim3((unsigned)cdiv(n, train::WSUM_OUT)), dim3(256), 0, st, (const float*)workspace, dw,
                     n, grid);
  HONK_LAUNCH_CHECK("wsum_kernel");
  return HONK_OK;
}
}  // namespace

extern "C" int honk_conv3x3_wgrad_f32(const float* x, const float* dy, float* dw, int64_t batch, int32_t c,
                                      int32_t h, int32_t w_, int32_t dil, void* workspace, size_t ws_bytes,
                                      void* stream) {
  return conv3x3_wgrad(x, dy, dw, batch, c, h, w_, dil, nullptr, nullptr, workspace, ws_bytes, stream);
}

extern "C" int honk_conv3x3_wgrad_bn_f32(const float* x, const float* dy, float* dw, int64_t batch, int32_t c,
                                         int32_t h, int32_t w_, int32_t dil, const float* fold_mean,
                                         const float* fold_invstd, void* workspace, size_t ws_bytes, void* stream) {
  if (!fold_mean || !fold_invstd) return fail(HONK_ERR_ARG, "null pointer argument");
  return conv3x3_wgrad(x, dy, dw, batch, c, h, w_, dil, fold_mean, fold_invstd, workspace, ws_bytes, stream);
}

// SyncBN (honk_amd/syncbn.py): the ranks' statistics partials are all-reduced before a
// BatchNorm finalises them, and the element count is the whole job's -- this rank's times
// the scale (the ranks' equal batches; thread-local, 1 outside a synchronised training)
namespace {
thread_local double g_bn_nscale = 1.0;
double bn_count(int64_t batch, int64_t hw) { return (double)batch * (double)hw * g_bn_nscale; }
}  // namespace

extern "C" int honk_bn_count_scale(double k) {
  if (!(k >= 1.0 && k <= 65536.0)) return fail(HONK_ERR_ARG, "BatchNorm count scale %g outside [1, 65536]", k);
  g_bn_nscale = k;
  return HONK_OK;
}

// The (sum a, sum a*b) partials of a BatchNorm statistic over [batch][c][hw] (b null: a*a)
// into part ([c][S][2] doubles, S = the bn_slices count honk_bn_train_workspace_bytes sizes),
// for a caller that reduces them itself (SyncBN: all-reduced across ranks, then handed to
// honk_res_tail_bwd_mask*_f32 with dil = -1)
extern "C" int honk_bn_partials_f32(const float* a, const float* b, void* part, size_t part_bytes, int64_t batch,
                                    int32_t c, int64_t hw, void* stream) {
  if (!a || !part) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 1 || c < 1 || hw < 1 || hw > 0x7fffffff || batch > 0x7fffffff) return fail(HONK_ERR_ARG, "bad batchnorm shape");
  const int S = train::bn_slices((int)batch, c);
  if (part_bytes < (size_t)c * S * 2 * sizeof(double)) return fail(HONK_ERR_WORKSPACE, "partials buffer too small");
  hipLaunchKernelGGL(train::bn_partial_kernel, dim3(c, S), dim3(256), 0, (hipStream_t)stream, a, b, (double*)part,
                     (int)batch, c, (int)hw, S);
  HONK_LAUNCH_CHECK("bn_partial_kernel");
  return HONK_OK;
}

extern "C" size_t honk_bn_train_workspace_bytes(int64_t batch, int32_t c, int64_t hw) {
  if (batch < 1 || c < 1 || hw < 1) return 0;
  return (size_t)c * train::bn_slices((int)batch, c) * 2 * sizeof(double) + (size_t)4 * c * sizeof(float);
}

extern "C" int honk_bn_train_fwd_f32(const float* x, float* y, float* mean, float* invstd, float* running_mean,
                                     float* running_var, int64_t batch, int32_t c, int64_t hw, float momentum,
                                     float eps, void* workspace, size_t ws_bytes, void* stream) {
  if (!x || !y || !mean || !invstd || (!running_mean != !running_var)) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 1 || c < 1 || hw < 1 || hw > 0x7fffffff || batch > 0x7fffffff) return fail(HONK_ERR_ARG, "bad batchnorm shape");
  const size_t need = honk_bn_train_workspace_bytes(batch, c, hw);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int S = train::bn_slices((int)batch, c);
  double* part = (double*)workspace;
  hipLaunchKernelGGL(train::bn_partial_kernel, dim3(c, S), dim3(256), 0, st, x, (const float*)nullptr, part,
                     (int)batch, c, (int)hw, S);
  HONK_LAUNCH_CHECK("bn_partial_kernel");
  hipLaunchKernelGGL(train::bn_stats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)part, mean,
                     invstd, running_mean, running_var, c, S, bn_count(batch, hw), momentum, eps);
  HONK_LAUNCH_CHECK("bn_stats_kernel");
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  hipLaunchKernelGGL(train::bn_apply_kernel, dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, x,
                     (const float*)nullptr, (const float*)mean, (const float*)invstd, (const float*)nullptr, y, total,
                     c, (int)hw);
  HONK_LAUNCH_CHECK("bn_apply_kernel");
  return HONK_OK;
}

extern "C" int honk_bn_train_bwd_f32(const float* dy, const float* y, const float* invstd, float* dx, int64_t batch,
                                     int32_t c, int64_t hw, void* workspace, size_t ws_bytes, void* stream) {
  if (!dy || !y || !invstd || !dx) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 1 || c < 1 || hw < 1 || hw > 0x7fffffff || batch > 0x7fffffff) return fail(HONK_ERR_ARG, "bad batchnorm shape");
  const size_t need = honk_bn_train_workspace_bytes(batch, c, hw);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int S = train::bn_slices((int)batch, c);
  double* part = (double*)workspace;
  float* m = (float*)(part + (size_t)c * S * 2);
  hipLaunchKernelGGL(train::bn_partial_kernel, dim3(c, S), dim3(256), 0, st, dy, y, part, (int)batch, c, (int)hw, S);
  HONK_LAUNCH_CHECK("bn_partial_kernel");
  hipLaunchKernelGGL(train::bn_bstats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)part, m,
                     m + c, c, S, bn_count(batch, hw));
  HONK_LAUNCH_CHECK("bn_bstats_kernel");
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  hipLaunchKernelGGL(train::bn_apply_kernel, dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, dy, y,
                     (const float*)m, invstd, (const float*)(m + c), dx, total, c, (int)hw);
  HONK_LAUNCH_CHECK("bn_apply_kernel");
  return HONK_OK;
}

extern "C" int honk_res_tail_fwd_f32(const float* h, const float* old, float* s, float* y, float* mean, float* invstd,
                                     float* running_mean, float* running_var, int64_t batch, int32_t c, int64_t hw,
                                     float momentum, float eps, void* workspace, size_t ws_bytes, void* stream) {
  if (!h || !y || !mean || !invstd || (!running_mean != !running_var)) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 1 || c < 1 || hw < 1 || hw > 0x7fffffff || batch > 0x7fffffff) return fail(HONK_ERR_ARG, "bad batchnorm shape");
  const size_t need = honk_bn_train_workspace_bytes(batch, c, hw);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int S = train::bn_slices((int)batch, c);
  double* part = (double*)workspace;
  hipLaunchKernelGGL(train::tail_partial_kernel, dim3(c, S), dim3(256), 0, st, h, old, part, (int)batch, c, (int)hw, S);
  HONK_LAUNCH_CHECK("tail_partial_kernel");
  hipLaunchKernelGGL(train::bn_stats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)part, mean,
                     invstd, running_mean, running_var, c, S, bn_count(batch, hw), momentum, eps);
  HONK_LAUNCH_CHECK("bn_stats_kernel");
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  hipLaunchKernelGGL(train::tail_fwd_kernel<false>, dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, h, old,
                     (const float*)mean, (const float*)invstd, y, s, total, c, (int)hw);
  HONK_LAUNCH_CHECK("tail_fwd_kernel");
  return HONK_OK;
}

extern "C" int honk_res_tail_bwd_f32(const float* gy, const float* gs, const float* y, const float* invstd,
                                     const float* h, float* gh, float* gold, int64_t batch, int32_t c, int64_t hw,
                                     void* workspace, size_t ws_bytes, void* stream) {
  if (!gy || !y || !invstd || !h || !gh) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 1 || c < 1 || hw < 1 || hw > 0x7fffffff || batch > 0x7fffffff) return fail(HONK_ERR_ARG, "bad batchnorm shape");
  const size_t need = honk_bn_train_workspace_bytes(batch, c, hw);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int S = train::bn_slices((int)batch, c);
  double* part = (double*)workspace;
  float* m = (float*)(part + (size_t)c * S * 2);
  hipLaunchKernelGGL(train::bn_partial_kernel, dim3(c, S), dim3(256), 0, st, gy, y, part, (int)batch, c, (int)hw, S);
  HONK_LAUNCH_CHECK("bn_partial_kernel");
  hipLaunchKernelGGL(train::bn_bstats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)part, m,
                     m + c, c, S, bn_count(batch, hw));
  HONK_LAUNCH_CHECK("bn_bstats_kernel");
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  hipLaunchKernelGGL(train::tail_bwd_kernel<false>, dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, gy, y, gs, h,
                     (const float*)m, invstd, (const float*)(m + c), gh, gold, total, c, (int)hw,
                     (const float*)nullptr);
  HONK_LAUNCH_CHECK("tail_bwd_kernel");
  return HONK_OK;
}

// ---- the statistics epilogue (conv3x3d_kernel MODE 1 / 2) and the tails that take
// its partial sums instead of their own pass over the tensors ----
namespace {
int stats_grid(int64_t batch, int c, int h, int w_, int dil) {
  if (batch < 1 || c != 19 || h < 1 || w_ < 1 || dil < 1 || dil > 64) return 0;
  const char* ke = getenv("HONK_TRAIN_CONV");
  if (ke && (ke[0] == 'v' || ke[0] == 'm')) return 0;
  const int tdr = train::td_rows(c, h, w_, dil);
  if (tdr <= 0) return 0;
  return (int)std::min<int64_t>(batch * train::class_bands(h, dil, tdr).nband, cu_count());
}
}  // namespace

namespace {
// conv3x3d_kernel with the statistics epilogue: mode 1 / 2, the fixed-geometry instance
// where it applies, the folded-BatchNorm instance when a.fm is set
void launch_conv_stats(const train::Conv3Args& a, int mode, int S, hipStream_t st) {
  const bool fx = train::td_fixed(a), fo = a.fm != nullptr;
#define HONK_CS(M, FO)                                                                                           \
  if (fx) hipLaunchKernelGGL((train::conv3x3d_kernel<19, M, 20, 1, 25, FO>), dim3(S), dim3(512), 0, st, a); \
  else hipLaunchKernelGGL((train::conv3x3d_kernel<19, M, 0, 0, 0, FO>), dim3(S), dim3(512), 0, st, a);
  if (mode == 1 && fo) { HONK_CS(1, true) }
  else if (mode == 1) { HONK_CS(1, false) }
  else if (fo) { HONK_CS(2, true) }
  else { HONK_CS(2, false) }
#undef HONK_CS
}
}  // namespace

extern "C" size_t honk_conv3x3_stats_bytes(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil) {
  const int S = stats_grid(batch, c, h, w_, dil);
  return S > 0 ? (size_t)c * S * 2 * sizeof(double) + (size_t)4 * c * sizeof(float) : 0;
}

extern "C" int honk_conv3x3_stats_bn_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c,
                                         int32_t h, int32_t w_, int32_t dil, int32_t flip, int32_t mode,
                                         const float* aux, const float* fold_mean, const float* fold_invstd,
                                         void* stats, size_t stats_bytes, void* stream) {
  if (!fold_mean != !fold_invstd) return fail(HONK_ERR_ARG, "null pointer argument");
  int rc = tc_check(x, w, y, batch, c, h, w_, dil);
  if (rc) return rc;
  if (mode != 1 && mode != 2) return fail(HONK_ERR_ARG, "conv3x3 statistics mode %d (1 or 2)", mode);
  if (mode == 2 && !aux) return fail(HONK_ERR_ARG, "conv3x3 statistics mode 2 needs the BN output");
  const int S = stats_grid(batch, c, h, w_, dil);
  if (S <= 0) return fail(HONK_ERR_UNSUPPORTED, "conv3x3 statistics epilogue: shape outside conv3x3d_kernel");
  if (!stats || stats_bytes < honk_conv3x3_stats_bytes(batch, c, h, w_, dil))
    return fail(HONK_ERR_WORKSPACE, "statistics buffer %zu B < required %zu B", stats_bytes,
                honk_conv3x3_stats_bytes(batch, c, h, w_, dil));
  train::Conv3Args a;
  a.x = x; a.w = w; a.y = y;
  a.B = (int)batch; a.H = h; a.W = w_; a.flip = flip ? 1 : 0;
  a.g = train::class_bands(h, dil, train::td_rows(c, h, w_, dil));
  a.aux = aux;
  a.part = (double*)stats;
  a.mask = nullptr;
  a.fm = fold_mean; a.fi = fold_invstd;
  hipStream_t st = (hipStream_t)stream;
  TimedLaunch tl(st, 2.0 * (double)batch * h * w_ * c * c * 9);
  launch_conv_stats(a, mode, S, st);
  tl.done(st);
  HONK_LAUNCH_CHECK("conv3x3d_kernel");
  return HONK_OK;
}

extern "C" int honk_conv3x3_stats_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c, int32_t h,
                                      int32_t w_, int32_t dil, int32_t flip, int32_t mode, const float* aux,
                                      void* stats, size_t stats_bytes, void* stream) {
  return honk_conv3x3_stats_bn_f32(x, w, y, batch, c, h, w_, dil, flip, mode, aux, nullptr, nullptr, stats,
                                   stats_bytes, stream);
}

extern "C" int honk_conv3x3_tail_bn_f32(const float* x, const float* w, float* s, uint32_t* mask, int64_t batch,
                                        int32_t c, int32_t h, int32_t w_, int32_t dil, const float* old,
                                        const float* fold_mean, const float* fold_invstd, void* stats,
                                        size_t stats_bytes, void* stream) {
  if (!fold_mean != !fold_invstd) return fail(HONK_ERR_ARG, "null pointer argument");
  int rc = tc_check(x, w, s, batch, c, h, w_, dil);
  if (rc) return rc;
  if (!mask) return fail(HONK_ERR_ARG, "null pointer argument");
  const int S = stats_grid(batch, c, h, w_, dil);
  if (S <= 0) return fail(HONK_ERR_UNSUPPORTED, "conv3x3 tail epilogue: shape outside conv3x3d_kernel");
  if (!stats || stats_bytes < honk_conv3x3_stats_bytes(batch, c, h, w_, dil))
    return fail(HONK_ERR_WORKSPACE, "statistics buffer %zu B < required %zu B", stats_bytes,
                honk_conv3x3_stats_bytes(batch, c, h, w_, dil));
  train::Conv3Args a;
  a.x = x; a.w = w; a.y = s;
  a.B = (int)batch; a.H = h; a.W = w_; a.flip = 0;
  a.g = train::class_bands(h, dil, train::td_rows(c, h, w_, dil));
  a.aux = old;
  a.part = (double*)stats;
  a.mask = mask;
  a.fm = fold_mean; a.fi = fold_invstd;
  hipStream_t st = (hipStream_t)stream;
  TimedLaunch tl(st, 2.0 * (double)batch * h * w_ * c * c * 9);
  launch_conv_stats(a, 1, S, st);
  tl.done(st);
  HONK_LAUNCH_CHECK("conv3x3d_kernel (tail epilogue)");
  return HONK_OK;
}

extern "C" int honk_conv3x3_tail_f32(const float* x, const float* w, float* s, uint32_t* mask, int64_t batch,
                                     int32_t c, int32_t h, int32_t w_, int32_t dil, const float* old, void* stats,
                                     size_t stats_bytes, void* stream) {
  return honk_conv3x3_tail_bn_f32(x, w, s, mask, batch, c, h, w_, dil, old, nullptr, nullptr, stats, stats_bytes,
                                  stream);
}

extern "C" int honk_conv3x3_bn_fold_check(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil) {
  if (stats_grid(batch, c, h, w_, dil) <= 0 || !wgrad_plan(batch, c, h, w_, dil).dma)
    return fail(HONK_ERR_UNSUPPORTED, "conv3x3: no folded BatchNorm for this shape");
  return HONK_OK;
}

extern "C" int honk_res_tail_fwd_s_f32(const float* s, float* y, float* mean, float* invstd, float* running_mean,
                                       float* running_var, const void* stats, int64_t batch, int32_t c, int32_t hh,
                                       int32_t ww, int32_t dil, float momentum, float eps, void* stream) {
  if (!s || !mean || !invstd || !stats || (!running_mean != !running_var))
    return fail(HONK_ERR_ARG, "null pointer argument");
  const int S = stats_grid(batch, c, hh, ww, dil);
  if (S <= 0) return fail(HONK_ERR_UNSUPPORTED, "res tail: no statistics epilogue for this shape");
  hipStream_t st = (hipStream_t)stream;
  const int64_t hw = (int64_t)hh * ww;
  hipLaunchKernelGGL(train::bn_stats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)stats,
                     mean, invstd, running_mean, running_var, c, S, bn_count(batch, hw), momentum, eps);
  HONK_LAUNCH_CHECK("bn_stats_kernel");
  if (!y) return HONK_OK;  // the next conv folds the BatchNorm in (honk_conv3x3_tail_bn_f32)
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  hipLaunchKernelGGL(train::tail_fwd_kernel<true>, dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, s,
                     (const float*)nullptr, (const float*)mean, (const float*)invstd, y, (float*)nullptr, total, c,
                     (int)hw);
  HONK_LAUNCH_CHECK("tail_fwd_kernel");
  return HONK_OK;
}

namespace {
int res_tail_bwd_mask(const float* gy, const float* gs, const float* y, const float* ym, const float* invstd,
                      const uint32_t* mask, float* gh, float* gold, int64_t batch, int32_t c, int32_t hh, int32_t ww,
                      int32_t dil, void* stats, size_t stats_bytes, void* stream) {
  if (!gy || !y || !invstd || !mask || !gh || !stats) return fail(HONK_ERR_ARG, "null pointer argument");
  if (ym && dil == 0) return fail(HONK_ERR_UNSUPPORTED, "res tail: a folded BatchNorm needs the conv's statistics");
  if (batch < 1 || c < 1 || hh < 1 || ww < 1 || batch > 0x7fffffff || (int64_t)hh * ww > 0x7fffffff)
    return fail(HONK_ERR_ARG, "bad res tail shape");
  hipStream_t st = (hipStream_t)stream;
  const int64_t hw = (int64_t)hh * ww;
  double* part = (double*)stats;
  int S;
  if (dil > 0) {  // the input-gradient conv's epilogue summed them (its grid's partials)
    S = stats_grid(batch, c, hh, ww, dil);
    if (S <= 0) return fail(HONK_ERR_UNSUPPORTED, "res tail: no statistics epilogue for this shape");
    if (stats_bytes < honk_conv3x3_stats_bytes(batch, c, hh, ww, dil))
      return fail(HONK_ERR_WORKSPACE, "statistics buffer %zu B < required %zu B", stats_bytes,
                  honk_conv3x3_stats_bytes(batch, c, hh, ww, dil));
  } else if (dil < 0) {  // the caller's partials (honk_bn_partials_f32; SyncBN: all-reduced)
    const size_t need = honk_bn_train_workspace_bytes(batch, c, hw);
    if (stats_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", stats_bytes, need);
    S = train::bn_slices((int)batch, c);
  } else {  // dil = 0: no conv consumed the gradient (the last block): sum them here
    const size_t need = honk_bn_train_workspace_bytes(batch, c, hw);
    if (stats_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", stats_bytes, need);
    S = train::bn_slices((int)batch, c);
    hipLaunchKernelGGL(train::bn_partial_kernel, dim3(c, S), dim3(256), 0, st, gy, y, part, (int)batch, c, (int)hw,
                       S);
    HONK_LAUNCH_CHECK("bn_partial_kernel");
  }
  float* m = (float*)(part + (size_t)c * S * 2);
  hipLaunchKernelGGL(train::bn_bstats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)part, m,
                     m + c, c, S, bn_count(batch, hw));
  HONK_LAUNCH_CHECK("bn_bstats_kernel");
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  if (ym)
    hipLaunchKernelGGL((train::tail_bwd_kernel<true, true>), dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, gy, y,
                       gs, (const void*)mask, (const float*)m, invstd, (const float*)(m + c), gh, gold, total, c,
                       (int)hw, ym);
  else
    hipLaunchKernelGGL((train::tail_bwd_kernel<true>), dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, gy, y, gs,
                       (const void*)mask, (const float*)m, invstd, (const float*)(m + c), gh, gold, total, c, (int)hw,
                       (const float*)nullptr);
  HONK_LAUNCH_CHECK("tail_bwd_kernel");
  return HONK_OK;
}
}  // namespace

extern "C" int honk_res_tail_bwd_mask_f32(const float* gy, const float* gs, const float* y, const float* invstd,
                                          const uint32_t* mask, float* gh, float* gold, int64_t batch, int32_t c,
                                          int32_t hh, int32_t ww, int32_t dil, void* stats, size_t stats_bytes,
                                          void* stream) {
  return res_tail_bwd_mask(gy, gs, y, nullptr, invstd, mask, gh, gold, batch, c, hh, ww, dil, stats, stats_bytes,
                           stream);
}

extern "C" int honk_res_tail_bwd_mask_bn_f32(const float* gy, const float* gs, const float* s, const float* mean,
                                             const float* invstd, const uint32_t* mask, float* gh, float* gold,
                                             int64_t batch, int32_t c, int32_t hh, int32_t ww, int32_t dil,
                                             void* stats, size_t stats_bytes, void* stream) {
  if (!mean) return fail(HONK_ERR_ARG, "null pointer argument");
  return res_tail_bwd_mask(gy, gs, s, mean, invstd, mask, gh, gold, batch, c, hh, ww, dil, stats, stats_bytes,
                           stream);
}

extern "C" int honk_res_tail_fwd_part_f32(const float* h, const float* old, float* s, float* y, float* mean,
                                          float* invstd, float* running_mean, float* running_var,
                                          const void* stats, int64_t batch, int32_t c, int32_t hh, int32_t ww,
                                          int32_t dil, float momentum, float eps, void* stream) {
  if (!h || !y || !mean || !invstd || !stats || (!running_mean != !running_var))
    return fail(HONK_ERR_ARG, "null pointer argument");
  const int S = stats_grid(batch, c, hh, ww, dil);
  if (S <= 0) return fail(HONK_ERR_UNSUPPORTED, "res tail: no statistics epilogue for this shape");
  hipStream_t st = (hipStream_t)stream;
  const int64_t hw = (int64_t)hh * ww;
  hipLaunchKernelGGL(train::bn_stats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)stats,
                     mean, invstd, running_mean, running_var, c, S, bn_count(batch, hw), momentum, eps);
  HONK_LAUNCH_CHECK("bn_stats_kernel");
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  hipLaunchKernelGGL(train::tail_fwd_kernel<false>, dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, h, old,
                     (const float*)mean, (const float*)invstd, y, s, total, c, (int)hw);
  HONK_LAUNCH_CHECK("tail_fwd_kernel");
  return HONK_OK;
}

extern "C" int honk_res_tail_bwd_part_f32(const float* gy, const float* gs, const float* y, const float* invstd,
                                          const float* h, float* gh, float* gold, void* stats, int64_t batch,
                                          int32_t c, int32_t hh, int32_t ww, int32_t dil, void* stream) {
  if (!gy || !y || !invstd || !h || !gh || !stats) return fail(HONK_ERR_ARG, "null pointer argument");
  const int S = stats_grid(batch, c, hh, ww, dil);
  if (S <= 0) return fail(HONK_ERR_UNSUPPORTED, "res tail: no statistics epilogue for this shape");
  hipStream_t st = (hipStream_t)stream;
  const int64_t hw = (int64_t)hh * ww;
  double* part = (double*)stats;
  float* m = (float*)(part + (size_t)c * S * 2);
  hipLaunchKernelGGL(train::bn_bstats_kernel, dim3((unsigned)c), dim3(256), 0, st, (const double*)part, m,
                     m + c, c, S, bn_count(batch, hw));
  HONK_LAUNCH_CHECK("bn_bstats_kernel");
  const int64_t total = batch * c * hw;
  const int64_t nthr = (hw & 3) == 0 ? total / 4 : total;
  hipLaunchKernelGGL(train::tail_bwd_kernel<false>, dim3((unsigned)cdiv(nthr, 256)), dim3(256), 0, st, gy, y, gs, h,
                     (const float*)m, invstd, (const float*)(m + c), gh, gold, total, c, (int)hw,
                     (const float*)nullptr);
  HONK_LAUNCH_CHECK("tail_bwd_kernel");
  return HONK_OK;
}

namespace {
int stem_check(const void* x, const void* w, const void* y, int64_t batch, int32_t c, int32_t h, int32_t w_,
               int32_t ph, int32_t pw) {
  if (!x || !w || !y) return fail(HONK_ERR_ARG, "null pointer argument");
  if (batch < 0 || batch > 0x7fffffff || h < 1 || w_ < 1 || ph < 1 || pw < 1 || ph > h || pw > w_)
    return fail(HONK_ERR_ARG, "bad stem shape (B=%lld H=%d W=%d pool %dx%d)", (long long)batch, h, w_, ph, pw);
  if (c < 1 || c > 64) return fail(HONK_ERR_UNSUPPORTED, "stem: %d feature maps (1..64)", c);
  if ((int64_t)(h + 2) * (w_ + 2) > train::STEM_XL_DYN)
    return fail(HONK_ERR_UNSUPPORTED, "stem: %dx%d input too large ((H+2)(W+2) <= %d)", h, w_, train::STEM_XL_DYN);
  return HONK_OK;
}
int stem_grid(int64_t batch) { return (int)std::min<int64_t>(batch, 3 * (int64_t)cu_count()); }
}  // namespace

extern "C" int honk_res_stem_fwd_f32(const float* x, const float* w0, float* y, int64_t batch, int32_t c, int32_t h,
                                     int32_t w_, int32_t ph, int32_t pw, void* stream) {
  int rc = stem_check(x, w0, y, batch, c, h, w_, ph, pw);
  if (rc) return rc;
  if (batch == 0) return HONK_OK;
  train::StemArgs a{x, w0, nullptr, y, nullptr, (int)batch, c, h, w_, ph, pw};
  train::stem_launch<false>(a, stem_grid(batch), (hipStream_t)stream);
  HONK_LAUNCH_CHECK("stem_kernel");
  return HONK_OK;
}

extern "C" size_t honk_res_stem_wgrad_workspace_bytes(int64_t batch, int32_t c) {
  if (batch < 1 || c < 1 || c > 64) return 0;
  return (size_t)stem_grid(batch) * c * 9 * sizeof(float);
}

extern "C" int honk_res_stem_wgrad_f32(const float* x, const float* w0, const float* gy, float* dw, int64_t batch,
                                       int32_t c, int32_t h, int32_t w_, int32_t ph, int32_t pw, void* workspace,
                                       size_t ws_bytes, void* stream) {
  int rc = stem_check(x, w0, dw, batch, c, h, w_, ph, pw);
  if (rc) return rc;
  if (!gy) return fail(HONK_ERR_ARG, "null pointer argument");
  hipStream_t st = (hipStream_t)stream;
  if (batch == 0) {
    HONK_HIP_CHECK(hipMemsetAsync(dw, 0, (size_t)c * 9 * sizeof(float), st));
    return HONK_OK;
  }
  const size_t need = honk_res_stem_wgrad_workspace_bytes(batch, c);
  if (!workspace || ws_bytes < need) return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  const int grid = stem_grid(batch);
  train::StemArgs a{x, w0, gy, nullptr, (float*)workspace, (int)batch, c, h, w_, ph, pw};
  train::stem_launch<true>(a, grid, st);
  HONK_LAUNCH_CHECK("stem_kernel");
  const int n = c * 9;
  hipLaunchKernelGGL(train::wsum_kernel, dim3((unsigned)cdiv(n, train::WSUM_OUT)), dim3(256), 0, st, (const float*)workspace, dw,
                     n, grid);
  HONK_LAUNCH_CHECK("wsum_kernel");
  return HONK_OK;
}
