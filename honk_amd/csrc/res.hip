// SpeechResModel forward (res8/15/26[-narrow]) for gfx950, fp32.
//
// Reference: /root/reference/utils/model.py:82-121.  The per-layer schedule
// (model.py:104-121) is
//     y = relu(conv_i(x)); i==0: y = pool(y), old = y
//     i>0 even: x = y + old, old = x    else: x = y
//     i>0: x = bn_i(x)                  (eval: (x-mean)/sqrt(var+1e-5))
//     logits = Linear(mean_hw(x))
//
// HBM layout: activations are NHWC with the channel dim padded to CP = 16*NT
// (CP = 48 for 45 maps, 32 for 19 maps); padded channels are kept at exactly 0.
// Three activation buffers per batch chunk:
//     R   pre-BN residual stream ("old_x"; written in place by even layers)
//     X0/X1  BN-applied layer outputs = the next conv's input (ping-pong)
// so every conv reads an already-normalised input (zero padding is then exactly
// the reference's post-BN zero padding) and the epilogue fuses ReLU, residual
// add, BN and both stores.
//
// Kernels
//   conv0_kernel   1->C 3x3 pad 1 + ReLU + optional avg-pool, VALU (1.6 MMAC/clip)
//   block_kernel   C->C 3x3 dilated conv as an implicit GEMM on fp32 MFMA
//                  (v_mfma_f32_16x16x4_f32): M = pixels of a row band, N = CP
//                  out-channels, K = 9 taps x CP in-channels.  Persistent grid,
//                  one 64*4*NT-thread workgroup per CU; wave (nt, mg) owns
//                  out-channel tile nt and MT 16-pixel m-tiles; its B operand
//                  (the layer's weights for tile nt) is streamed from L2 one
//                  row-offset (3 taps, 3*CP/4 VGPRs) per stage.  The A operand is staged per
//                  (tile, dy) as a band of TH full rows shifted by (dy-1)*dil,
//                  copied HBM/L2 -> LDS by buffer_load...lds (16 B per lane)
//                  double-buffered against the MFMA work; the dx shift and the
//                  column zero padding are folded into per-lane LDS addresses
//                  (an out-of-range column reads a zero pixel kept in LDS); row
//                  padding comes from the buffer bounds check (reads as 0).
//   tail           spatial mean + Linear(C, n_labels) (model.py:119-121): the
//                  last block layer sums its BN output per channel in the
//                  epilogue (no activation store); tail_sum_kernel finishes the
//                  mean and the Linear.
#include "common.h"

#include <cstring>

namespace honk {
namespace res {
constexpr int MW = 4;  // waves along M per workgroup

template <int NT, int MT>
struct Geo {
  static constexpr int CP = 16 * NT;          // padded channels
  static constexpr int Q = CP / 16;           // 16-channel k-quads per tap (= NT)
  static constexpr int CH4 = CP / 4;          // 16-byte chunks per pixel
  static constexpr int NWAVES = NT * MW;
  static constexpr int NTHREADS = 64 * NWAVES;
  static constexpr int MP = 16 * MT * MW;     // max pixels per tile
  static constexpr int ZOFF = MP * CP;        // zero pixel (floats); MP*CP*4 = MT*NWAVES KiB
  static constexpr int BUF = ZOFF + CP;       // floats per LDS stage buffer
  static constexpr int LDS_FLOATS = 2 * BUF;
  // VMEM ops a wave issues per stage after its glds: B refills (3*NT) and, in
  // the tile's last stage, residual loads (MT) + pre/BN stores (2*MT)
  static constexpr int VM_AFTER_GLDS = 3 * NT;
  static constexpr int VM_AFTER_GLDS_LAST = 3 * NT + 3 * MT;
};

struct BlockArgs {
  const float* in;        // [n][H][W][CP]  BN-applied input
  const float* res;       // [n][H][W][CP]  residual (pre-BN) or nullptr
  float* out_pre;         // pre-BN output (residual stream) or nullptr
  float* out_bn;          // BN-applied output
  const float* wfrag;     // [NT][9][Q][64][4] B fragments
  const float* bn_scale;  // [CP]
  const float* bn_shift;  // [CP]
  float* chsum;           // last layer only: [ntiles][MW][CP] partial channel sums of the
                          // BN output over valid pixels (fused spatial mean), or nullptr
  int H, W, dil, TH, nbands, ntiles;
};

// s_waitcnt vmcnt(N) (expcnt/lgkmcnt untouched), visible to the compiler's waitcnt pass
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// A-operand staging: one (tile, dy) band of TH rows x W pixels x CP channels,
// HBM/L2 -> LDS by buffer_load ... lds (16 B per lane, LDS image lane-linear).
// Every wave issues exactly MT pieces of 1 KiB (the band buffer holds
// MT*NWAVES KiB), so the barrier's vmcnt count is a compile-time constant.
// Rows outside [0, H) and pieces past the band get an out-of-range offset: the
// buffer bounds check returns zeros (= the reference's zero padding).
template <int NT, int MT>
__device__ __forceinline__ void issue_stage(const BlockArgs& a, int tile, int dy, float* buf, int wave,
                                            const unsigned (&gpack)[MT]) {
  using G = Geo<NT, MT>;
  const int b = tile / a.nbands;
  const int h0 = (tile - b * a.nbands) * a.TH;
  const int clip_floats = a.H * a.W * G::CP;
  __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.in + (size_t)b * clip_floats), (short)0, clip_floats * 4, 0x00020000);
  const int rbase = h0 + (dy - 1) * a.dil;   // wave-uniform
  const unsigned row_bytes = (unsigned)(a.W * G::CP * 4);
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int pc = wave + i * G::NWAVES;
    // gpack: (band row << 16) | byte offset within the row; row 0xffff = past the band
    const int grow = rbase + (int)(gpack[i] >> 16);
    const unsigned voff = ((unsigned)grow < (unsigned)a.H) ? (unsigned)grow * row_bytes + (gpack[i] & 0xffffu)
                                                           : 0x80000000u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(buf + (pc << 8)),
                                             16, voff, 0, 0, 0);
  }
}

// per-lane, tile-invariant part of the staging addresses (see issue_stage)
template <int NT, int MT>
__device__ __forceinline__ void make_gpack(const BlockArgs& a, int wave, int lane, unsigned (&gpack)[MT]) {
  using G = Geo<NT, MT>;
  const int total = a.TH * a.W * G::CH4;
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const int ci = ((wave + i * G::NWAVES) << 6) + lane;
    const int pix = ci / G::CH4;
    const int ch = ci - pix * G::CH4;
    const int r = pix / a.W;
    const int w = pix - r * a.W;
    gpack[i] = (ci < total) ? ((unsigned)r << 16) | (unsigned)((w * G::CP + ch * 4) * 4) : 0xffff0000u;
  }
}

// B fragments of tap (dy, dx): frag[nt][tap][q][lane][4] via a buffer descriptor
template <int NT>
__device__ __forceinline__ void load_b_dx(__amdgpu_buffer_rsrc_t wr, int dy, int dx, int lane16, f32x4 (&b)[NT]) {
#pragma unroll
  for (int q = 0; q < NT; ++q)
    b[q] = __builtin_bit_cast(
        f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, lane16, ((dy * 3 + dx) * NT + q) * 1024, 0));
}

// One (dx, q) step of a stage: reads the A fragments of step K+1 while the
// MFMAs of step K run; after the last q of a dx, that dx's B registers are
// refilled with the next stage's fragments (row offset NDY) so the L2 latency
// hides under the remaining MFMAs.  Template recursion keeps register indices static.
template <int NT, int MT, int NDY, int K, typename Mid>
__device__ __forceinline__ void stage_step(const char* base, const int (&aoff)[3][MT], f32x4 (&bcur)[3][NT],
                                           f32x4 (&acc)[MT], f32x4 (&a0)[MT], f32x4 (&a1)[MT],
                                           __amdgpu_buffer_rsrc_t wr, int lane16, Mid& mid) {
  constexpr int NK = 3 * NT;
  if constexpr (K < NK) {
    constexpr int dx = K / NT, q = K % NT;
    f32x4 (&cur)[MT] = (K & 1) ? a1 : a0;
    f32x4 (&nxt)[MT] = (K & 1) ? a0 : a1;
    if constexpr (K + 1 < NK) {
      constexpr int dx1 = (K + 1) / NT, q1 = (K + 1) % NT;
#pragma unroll
      for (int m = 0; m < MT; ++m) nxt[m] = *(const f32x4*)(base + aoff[dx1][m] + q1 * 64);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
      for (int m = 0; m < MT; ++m)
        // weights as the A operand, activations as B: D = W . X^T, so the C/D layout
        // gives each lane 4 consecutive out-channels (rows 4g+r) of pixel i16
        acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(bcur[dx][q][j], cur[m][j], acc[m], 0, 0, 0);
    }
    // after the first step's MFMAs are issued: next-stage LDS-DMA (+ residual
    // prefetch), whose VALU address math then overlaps the other waves' MFMAs.
    // It precedes every B refill, so the barrier's vmcnt count stays exact.
    if constexpr (K == 0) mid();
    if constexpr (q == NT - 1) load_b_dx<NT>(wr, NDY, dx, lane16, bcur[dx]);
    __builtin_amdgcn_sched_barrier(0);
    stage_step<NT, MT, NDY, K + 1>(base, aoff, bcur, acc, a0, a1, wr, lane16, mid);
  }
}

template <int NT, int MT, int NDY, typename Mid>
__device__ __forceinline__ void compute_stage(const float* cur, const int (&aoff)[3][MT], f32x4 (&bcur)[3][NT],
                                              f32x4 (&acc)[MT], __amdgpu_buffer_rsrc_t wr, int lane16, Mid& mid) {
  const char* base = (const char*)cur;
  f32x4 a0[MT], a1[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) a0[m] = *(const f32x4*)(base + aoff[0][m]);
  stage_step<NT, MT, NDY, 0>(base, aoff, bcur, acc, a0, a1, wr, lane16, mid);
}

template <int NT, int MT, bool LAST>
__global__ __launch_bounds__((Geo<NT, MT>::NTHREADS), NT) void block_kernel(BlockArgs a) {
  using G = Geo<NT, MT>;
  // ONE LDS array (a second __shared__ object can de-pipeline glds waits):
  // [stage buffer 0 | stage buffer 1]
  __shared__ __attribute__((aligned(16))) float smem[G::LDS_FLOATS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nt = wave % NT;
  const int mg = wave / NT;
  const int g = lane >> 4;
  const int i16 = lane & 15;

  for (int t = tid; t < G::CP; t += G::NTHREADS) {
    smem[G::ZOFF + t] = 0.f;
    smem[G::BUF + G::ZOFF + t] = 0.f;
  }

  // B operand: the layer's weights for out-channel tile nt, streamed from L2 one
  // row offset (3 taps) per stage (refilled inside compute_stage after last use)
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(a.wfrag + (size_t)nt * 9 * G::Q * 64 * 4), (short)0, 9 * G::Q * 64 * 16, 0x00020000);
  const int lane16 = lane * 16;
  f32x4 bcur[3][NT];

  // A operand addresses (bytes within a stage buffer), one per (dx, m-tile)
  const int TP = a.TH * a.W;
  int aoff[3][MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = (mg * MT + m) * 16 + i16;
    const int r = p / a.W;
    const int w = p - r * a.W;
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
      const int sh = (dx - 1) * a.dil;
      const int col = w + sh;
      const bool ok = (p < TP) && (col >= 0) && (col < a.W);
      aoff[dx][m] = ok ? ((p + sh) * G::CP + g * 4) * 4 : (G::ZOFF + g * 4) * 4;
    }
  }

  // epilogue constants: lane (g, i16) owns pixel i16 of each m-tile and out
  // channels nt*16 + 4g .. +3 (one 16-byte chunk)
  const int c4 = nt * 16 + 4 * g;
  const f32x4 bsc = *(const f32x4*)(a.bn_scale + c4);
  const f32x4 bsh = *(const f32x4*)(a.bn_shift + c4);
  const int eoff = ((mg * MT * 16 + i16) * G::CP + c4) * 4;

  // XCD-aware tile order: blocks sharing an XCD (bid % 8) walk adjacent tiles
  const int GR = gridDim.x;
  const int bid = blockIdx.x;
  const int lb = ((GR & 7) == 0) ? (bid & 7) * (GR >> 3) + (bid >> 3) : bid;
  int tile = lb;
  if (tile >= a.ntiles) return;

  // buffer descriptor over the valid pixels of `tile` in an NHWC(CP) tensor;
  // a null tensor gets 0 records (loads return 0, stores are dropped)
  auto tile_rsrc = [&](const float* t) {
    const int b = tile / a.nbands;
    const int h0 = (tile - b * a.nbands) * a.TH;
    const int vp = min(a.TH, a.H - h0) * a.W;
    const size_t off = ((size_t)b * a.H + h0) * a.W * G::CP;
    return __builtin_amdgcn_make_buffer_rsrc((void*)(t ? t + off : a.out_bn), (short)0, t ? vp * G::CP * 4 : 0,
                                             0x00020000);
  };

  // prologue: stage (tile, dy=0) and its B fragments, fully landed before the loop
  unsigned gpack[MT];
  make_gpack<NT, MT>(a, wave, lane, gpack);
  issue_stage<NT, MT>(a, tile, 0, smem, wave, gpack);
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) load_b_dx<NT>(wr, 0, dx, lane16, bcur[dx]);
  wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  int s = 0;
  f32x4 rv[MT];
  while (true) {
    f32x4 acc[MT];
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};

    // stage DY: wait for this stage's glds (issued one stage ago) in all waves,
    // then prefetch the next stage into the other buffer and run the MFMAs
#define HONK_STAGE(DY)                                                                  \
  {                                                                                     \
    float* cur = smem + (s & 1) * G::BUF;                                               \
    float* nxt = smem + ((s + 1) & 1) * G::BUF;                                         \
    if (DY == 0) wait_vmcnt<G::VM_AFTER_GLDS_LAST>(); else wait_vmcnt<G::VM_AFTER_GLDS>(); \
    __builtin_amdgcn_s_barrier();                                                       \
    auto mid = [&]() {                                                                  \
      if (DY < 2)                                                                       \
        issue_stage<NT, MT>(a, tile, DY + 1, nxt, wave, gpack);                         \
      else if (tile + GR < a.ntiles)                                                    \
        issue_stage<NT, MT>(a, tile + GR, 0, nxt, wave, gpack);                         \
      if (DY == 2 && !LAST) {                                                           \
        const __amdgpu_buffer_rsrc_t rr = tile_rsrc(a.res);                             \
        _Pragma("unroll") for (int m = 0; m < MT; ++m)                                  \
          rv[m] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(      \
              rr, eoff, m * 16 * G::CP * 4, 0));                                        \
      }                                                                                 \
    };                                                                                  \
    compute_stage<NT, MT, (DY + 1) % 3>(cur, aoff, bcur, acc, wr, lane16, mid);         \
    ++s;                                                                                \
  }
    HONK_STAGE(0)
    HONK_STAGE(1)
    HONK_STAGE(2)
#undef HONK_STAGE

    // epilogue: lane (g, i16) holds out channels c4..c4+3 of pixel i16 of each
    // m-tile: ReLU, residual add, pre-BN store (even layers) and BN store, 16 B
    // per lane; stores past the tile's valid pixels are dropped by the bounds
    // check.  In the last layer nothing is stored: the BN output is summed per
    // channel over the tile's valid pixels instead (fused spatial mean).
    {
      const __amdgpu_buffer_rsrc_t bn_r = tile_rsrc(LAST ? nullptr : a.out_bn);
      const __amdgpu_buffer_rsrc_t pre_r = tile_rsrc(a.out_pre);
      const int b = tile / a.nbands;
      const int lim = min(a.TH, a.H - (tile - b * a.nbands) * a.TH) * a.W - (mg * MT * 16 + i16);
      f32x4 csum = {0.f, 0.f, 0.f, 0.f};
      const __amdgpu_buffer_rsrc_t rr = tile_rsrc(a.res);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        if (LAST)  // last layer: residual loaded here (no prefetch registers)
          rv[m] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rr, eoff, m * 16 * G::CP * 4, 0));
        f32x4 v, o;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k] = relu_keepnan(acc[m][k]) + rv[m][k];
          o[k] = fmaf(v[k], bsc[k], bsh[k]);
        }
        const int so = m * 16 * G::CP * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v),
                                               pre_r, eoff, so, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, o),
                                               bn_r, eoff, so, 0);
        if (LAST && m * 16 < lim) csum += o;
      }
      if (LAST) {
        // reduce over the 16 lanes (pixels) holding the same 4 channels
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          csum[k] = sum16_dpp(csum[k]);
        }
        if (i16 == 0) *(f32x4*)(a.chsum + ((size_t)tile * MW + mg) * G::CP + c4) = csum;
      }
    }
    tile += GR;
    if (tile >= a.ntiles) break;
  }
}

// --------------------------------------------------------------------------- //
// conv0: 1 -> C, 3x3, pad 1, ReLU, optional avg-pool (PH x PW); NHWC(CP) out
// --------------------------------------------------------------------------- //
__device__ __forceinline__ void store4(float* o, f32x4 v) { *(f32x4*)o = v; }
__device__ __forceinline__ void store4(__bf16* o, f32x4 v) {
  typedef __bf16 b4 __attribute__((ext_vector_type(4)));
  const b4 b = {(__bf16)v[0], (__bf16)v[1], (__bf16)v[2], (__bf16)v[3]};
  *(b4*)o = b;
}
__device__ __forceinline__ void store4(_Float16* o, f32x4 v) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 b = {(_Float16)v[0], (_Float16)v[1], (_Float16)v[2], (_Float16)v[3]};
  *(h4*)o = b;
}

// Thread = output pixel (weights wave-uniform: scalar loads); the block's 256
// pixels x CP channels are staged in LDS and written back as one contiguous
// span with 16-byte accesses (a direct thread-per-pixel store strides 8-16 B
// accesses by the pixel pitch).  The packed weights are zero for channels >= C.
// ONES: channel C (< CP) holds 1.0 -- the bias channel of the weight-stationary
// bf16 kernels (pack_block16_kernel)
// cscale (may be null): the clips' power-of-two scales of the f16x2 path, as conv0m_kernel
template <int PH, int PW, typename OT, bool SPLIT, bool ONES, int CPM = 48>
__global__ __launch_bounds__(256) void conv0_kernel(const float* __restrict__ x, OT* __restrict__ out,
                                                    const float* __restrict__ w0, int n, int Hin,
                                                    int Win, int H, int W, int C, int CP,
                                                    const float* __restrict__ cscale) {
  // SPLIT (bf16x3 activations): per pixel [hi CP][lo CP] bf16, lo = bf16(v - hi)
  constexpr int PPX = SPLIT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) OT stage[256 * CPM * PPX];  // CPM >= CP
  const int64_t p0 = (int64_t)blockIdx.x * 256;
  const int64_t gid = p0 + threadIdx.x;
  const int64_t total = (int64_t)n * H * W;
  if (gid < total) {
    const int ow = (int)(gid % W);
    const int64_t t = gid / W;
    const int oh = (int)(t % H);
    const int b = (int)(t / H);
    const float* xb = x + (int64_t)b * Hin * Win;
    // input window rows [oh*PH-1, oh*PH+PH], cols [ow*PW-1, ow*PW+PW]
    float win[PH + 2][PW + 2];
#pragma unroll
    for (int r = 0; r < PH + 2; ++r) {
      const int ir = oh * PH - 1 + r;
#pragma unroll
      for (int c = 0; c < PW + 2; ++c) {
        const int ic = ow * PW - 1 + c;
        win[r][c] = (ir >= 0 && ir < Hin && ic >= 0 && ic < Win) ? xb[(int64_t)ir * Win + ic] : 0.f;
      }
    }
    OT* o = stage + threadIdx.x * CP * PPX;
    const float inv = 1.0f / (float)(PH * PW);
    const float cs = cscale ? cscale[b] : 1.f;
    for (int c4 = 0; c4 < CP; c4 += 4) {
      float v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* wc = w0 + (c4 + u) * 9;
        float wr[9];
#pragma unroll
        for (int k = 0; k < 9; ++k) wr[k] = wc[k];
        float s = 0.f;
#pragma unroll
        for (int a = 0; a < PH; ++a)
#pragma unroll
          for (int bb = 0; bb < PW; ++bb) {
            float acc = 0.f;
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
              for (int kx = 0; kx < 3; ++kx) acc = fmaf(win[a + ky][bb + kx], wr[ky * 3 + kx], acc);
            s += relu_keepnan(acc);
          }
        v[u] = ((PH * PW > 1) ? s * inv : s) * cs;
        if (ONES && (c4 + u == C || c4 + u == C + 1)) v[u] = cs;
      }
      const f32x4 vv = {v[0], v[1], v[2], v[3]};
      store4(o + c4, vv);
      if constexpr (SPLIT) {
        f32x4 lo;
#pragma unroll
        for (int u = 0; u < 4; ++u) lo[u] = vv[u] - (float)(OT)vv[u];
        store4(o + CP + c4, lo);
      }
    }
  }
  __syncthreads();
  // contiguous write-back of the block's valid pixels
  const int64_t np = (total - p0 < 256) ? total - p0 : 256;
  const int chunks = (int)(np * CP * PPX * (int)sizeof(OT) / 16);
  const uint4* src = (const uint4*)stage;
  uint4* dst = (uint4*)(out + p0 * CP * PPX);
  for (int i = threadIdx.x; i < chunks; i += 256) dst[i] = src[i];
}

// generic pool shape (any PH, PW): same math, input read through L1
template <typename OT>
__global__ __launch_bounds__(256) void conv0_generic_kernel(const float* __restrict__ x,
                                                            OT* __restrict__ out,
                                                            const float* __restrict__ w0, int n,
                                                            int Hin, int Win, int H, int W, int C,
                                                            int CP, int PH, int PW) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)n * H * W;
  if (gid >= total) return;
  const int ow = (int)(gid % W);
  const int64_t t = gid / W;
  const int oh = (int)(t % H);
  const int b = (int)(t / H);
  const float* xb = x + (int64_t)b * Hin * Win;
  OT* o = out + gid * CP;
  const float inv = 1.0f / (float)(PH * PW);
  for (int c = 0; c < CP; ++c) {
    float s = 0.f;
    if (c < C) {
      for (int a = 0; a < PH; ++a)
        for (int bb = 0; bb < PW; ++bb) {
          float acc = 0.f;
          for (int ky = 0; ky < 3; ++ky)
            for (int kx = 0; kx < 3; ++kx) {
              const int ir = oh * PH + a + ky - 1, ic = ow * PW + bb + kx - 1;
              const float xv = (ir >= 0 && ir < Hin && ic >= 0 && ic < Win) ? xb[(int64_t)ir * Win + ic] : 0.f;
              acc = fmaf(xv, w0[c * 9 + ky * 3 + kx], acc);
            }
          s += relu_keepnan(acc);
        }
      if (PH * PW > 1) s *= inv;
    }
    o[c] = (OT)s;
  }
}

#ifndef HONK_RES_VF_TU  // res_vf.hip: templates only (see there)
// --------------------------------------------------------------------------- //
// tail: logits[b] = Wout . mean_hw(x[b]) + bout      (x already BN-applied)
// --------------------------------------------------------------------------- //
__global__ __launch_bounds__(256) void tail_kernel(const float* __restrict__ x, const float* __restrict__ wout,
                                                   const float* __restrict__ bout, float* __restrict__ logits,
                                                   int HW, int C, int CP, int NL) {
  __shared__ float part[256];
  __shared__ float mean[64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int groups = blockDim.x / CP;  // pixel groups
  const int c = tid % CP;
  const int pg = tid / CP;
  float s = 0.f;
  if (pg < groups) {
    const float* xb = x + (int64_t)b * HW * CP + c;
    for (int p = pg; p < HW; p += groups) s += xb[(int64_t)p * CP];
  }
  part[tid] = s;
  __syncthreads();
  if (tid < CP) {
    float t = 0.f;
    for (int q = 0; q < groups; ++q) t += part[q * CP + tid];
    mean[tid] = t / (float)HW;
  }
  __syncthreads();
  for (int nlab = tid; nlab < NL; nlab += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < C; ++k) acc = fmaf(wout[nlab * C + k], mean[k], acc);
    logits[(int64_t)b * NL + nlab] = acc + bout[nlab];
  }
}

// The head over a stored bf16 activation tensor [n][HW][CP] (CP = 48): the bf16 path's
// last layer when it is the B layer of a fused pair (an even last layer: res8, res26),
// which stores its output like any pair.  One workgroup per clip: thread t sums 16-B chunk
// t % 6 (8 channels) over pixels t / 6, t / 6 + 42, ... in order, 48 threads add the 42
// partials in order (deterministic, independent of the clip's position in the batch), then
// tail_sum_kernel's last BatchNorm on the channel means and the Linear.
__global__ __launch_bounds__(256) void tail_act_kernel(const __bf16* __restrict__ act, const float* __restrict__ wout,
                                                       const float* __restrict__ bout, float* __restrict__ logits,
                                                       int HW, int C, int NL, const float* __restrict__ bn_scale,
                                                       const float* __restrict__ bn_shift) {
  constexpr int CP = 48, NCH = CP / 8, NPG = 256 / NCH;  // 6 chunks, 42 pixel groups
  __shared__ float part[NPG][CP];
  __shared__ float mean[CP];
  const int b = blockIdx.x, t = threadIdx.x;
  const int j = t % NCH, pg = t / NCH;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (pg < NPG) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4* src = (const u4*)(act + (size_t)b * HW * CP) + j;
    for (int p = pg; p < HW; p += NPG) {
      const u4 v = src[(size_t)p * NCH];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        s[2 * e] += __builtin_bit_cast(float, v[e] << 16);
        s[2 * e + 1] += __builtin_bit_cast(float, v[e] & 0xffff0000u);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) part[pg][8 * j + e] = s[e];
  }
  __syncthreads();
  if (t < CP) {
    float v = part[0][t];
    for (int g = 1; g < NPG; ++g) v += part[g][t];
    mean[t] = bn_scale ? fmaf(v / (float)HW, bn_scale[t], bn_shift[t]) : v / (float)HW;
  }
  __syncthreads();
  for (int n = t; n < NL; n += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < C; ++k) acc = fmaf(wout[n * C + k], mean[k], acc);
    logits[(int64_t)b * NL + n] = acc + bout[n];
  }
}

// logits[b] = Wout . (sum of the fused per-tile channel sums) / HW + bout
// bn_scale/bn_shift: the last layer's BatchNorm applied to the channel means
// (bf16 path, whose activations are pre-BN), or nullptr (fp32 path)
__global__ __launch_bounds__(256) void tail_sum_kernel(const float* __restrict__ chsum, const float* __restrict__ wout,
                                                       const float* __restrict__ bout, float* __restrict__ logits,
                                                       int nparts, int HW, int C, int CP, int NL,
                                                       const float* __restrict__ bn_scale,
                                                       const float* __restrict__ bn_shift,
                                                       const float* __restrict__ cscale,
                                                       const float* __restrict__ oscale,
                                                       int* __restrict__ flags, float zmax) {
  // groups of 64 threads sum every ng-th partial (coalesced rows of CP floats), then one
  // thread per channel adds the groups' sums in group order: a fixed order for every clip
  // (the row-band last layer writes 8 waves x MT m-tiles x bands partials per clip; one
  // thread walking all of them serially took 15 us per 4096-clip chunk)
  __shared__ float part[4][64];
  __shared__ float mean[64];
  __shared__ int out_of_range;
  const int b = blockIdx.x;
  const int t = threadIdx.x, c = t & 63, grp = t >> 6, ng = blockDim.x >> 6;
  if (t == 0) out_of_range = 0;
  float s = 0.f;
  if (c < CP) {
    const float* p = chsum + (size_t)b * nparts * CP + c;
    for (int i = grp; i < nparts; i += ng) s += p[(size_t)i * CP];
  }
  part[grp][c] = s;
  __syncthreads();
  if (t < CP) {
    float v = part[0][t];
    for (int g = 1; g < ng; ++g) v += part[g][t];
    // the f16x2 clip scale times the last layer's output exponent (powers of two: exact)
    if (cscale) v /= cscale[b] * *oscale;
    mean[t] = bn_scale ? fmaf(v / (float)HW, bn_scale[t], bn_shift[t]) : v / (float)HW;
    // f16x2 admission (flags != null): the clip's BatchNorm'd last-layer channel means are
    // its distance from the model's calibration, in standard deviations; beyond zmax (or
    // not finite: an fp16 store overflowed) the clip is re-run in bf16x3 (honk_res_forward)
    if (flags && t < C && !(fabsf(mean[t]) <= zmax)) out_of_range = 1;
  }
  __syncthreads();
  // flags[b] == 2: the clip's input is not finite (clip_scale_kernel) -- its NaN logits are
  // the reference's, nothing to re-run
  if (flags && t == 0 && out_of_range && flags[b] != 2) flags[b] = 1;
  for (int n = t; n < NL; n += blockDim.x) {
    float acc = 0.f;
    for (int k = 0; k < C; ++k) acc = fmaf(wout[n * C + k], mean[k], acc);
    logits[(int64_t)b * NL + n] = acc + bout[n];
  }
}

#endif  // HONK_RES_VF_TU

#include "res_bf16.inc"
#include "res_bf16r.inc"
#include "res_bf16w.inc"
#include "res_bf16p.inc"
#include "res_bf16k.inc"
#include "res_bf16n.inc"

// conv0m / conv0p staging: the clip's [Hin][Win] fp32 map through put(r, c, v), 256 threads.
// Rows of whole float4s: a thread's U loads all in flight before its first LDS write (res8 /
// res15: 1010 float4s, 4 per thread -- one HBM latency per clip instead of four in series).
template <typename Put>
__device__ __forceinline__ void c0_stage(const float* __restrict__ xc, int Hin, int Win, Put&& put) {
  if ((Win & 3) == 0) {
    constexpr int U = 4;
    const int w4 = Win >> 2, n4 = Hin * w4;
    for (int i0 = threadIdx.x; i0 < n4; i0 += U * 256) {
      f32x4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * 256;
        v[u] = i < n4 ? *(const f32x4*)(xc + 4 * (size_t)i) : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * 256;
        if (i < n4) {
          const int r = i / w4, c = (i - r * w4) * 4;
#pragma unroll
          for (int e = 0; e < 4; ++e) put(r, c + e, v[u][e]);
        }
      }
    }
  } else {
    for (int i = threadIdx.x; i < Hin * Win; i += 256) {
      const int r = i / Win;
      put(r, i - r * Win, xc[i]);
    }
  }
}

// --------------------------------------------------------------------------- //
// conv0 on the matrix cores (the bf16 / bf16x3 / f16x2 paths): 1 -> CP 3x3 pad 1,
// ReLU, avg-pool PH x PW (model.py:87-89, 107-110), written in the block
// kernels' activation format.  One workgroup per clip (4 waves).
//
// The 9-tap contraction is one v_mfma_f32_16x16x32_bf16 per (16 conv pixels,
// 16 out channels) carrying ALL THREE bf16x3 products in its K = 32:
//   k  0.. 8: w_hi[t] * x_hi[t]      k  9..17: w_hi[t] * x_lo[t]
//   k 18..26: w_lo[t] * x_hi[t]      k 27..31: 0
// (fp32 values as bf16 (hi, lo) pairs, the w_lo * x_lo term dropped: ~2^-17
// relative, as the bf16x3 layers).  The clip's input is staged once into LDS as
// bf16 hi and lo planes with a zero border (the conv's zero padding); a lane's B
// fragment (its pixel, k-chunk 8g..8g+7) is 8 u16 reads at per-lane constant
// offsets.  The weights (A: rows = out channels in the co16 order, so a lane's
// results are aligned channel runs of its pixel) stay in registers.
// Pooling: an m-tile = 16 pooled outputs x ONE member k of their PH x PW window;
// the members are summed (after ReLU, row-major, as avg_pool2d) in the lanes'
// accumulators, then divided by PH * PW.  ONES: channel C = 1.0 (the folded-bias
// channel of the weight-stationary / pair kernels).  FM: 0 bf16, 1 bf16x3
// ([hi CP][lo CP]), 2 fp16 output.
// --------------------------------------------------------------------------- //
// FWB > 0: the bordered plane width Win + 2 at compile time (40-wide inputs: 42), so a
// pool member's tap reads take their offset as an immediate
// cscale (FM 2 only, else null): the clips' power-of-two scales (clip_scale_kernel): the
// output is s * relu(conv0(x)) (pooled) and channel C holds s instead of 1.0.
template <int NT, int PH, int PW, int FM, bool ONES, int FWB = 0>
// (launch bounds: 7 waves per SIMD -- 72 registers, a few 4-byte whole-tuple spills in the
// 4x3-pool instances: res8's conv0m 114 -> 110 us per 4096 clips at 7 workgroups per CU vs 6)
__global__ __launch_bounds__(256, 7) void conv0m_kernel(const float* __restrict__ x, __bf16* __restrict__ out,
                                                     const float* __restrict__ w0, int Hin, int Win, int H, int W,
                                                     int C, const float* __restrict__ cscale) {
  constexpr int CP = 16 * NT, P = PH * PW, SP = FM == 1 ? 2 : 1, CB = CP * 2 * SP;
  extern __shared__ __attribute__((aligned(16))) unsigned short c0lds[];  // hi plane, lo plane
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int clip = blockIdx.x;
  const int Wb = FWB > 0 ? FWB : Win + 2, plane = (Hin + 2) * Wb;
  unsigned short* hp = c0lds;
  unsigned short* lp = c0lds + plane;

  // weights: A fragment of n-tile n = lane (row rho = i16, k-chunk g)
  u32x4 wa[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int co = co16(NT, n, i16);
    unsigned short v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 8 * g + j;
      const int t = k < 9 ? k : k < 18 ? k - 9 : k < 27 ? k - 18 : 0;
      // (w0 = the packed conv0 weights, [CP][9], zero rows past C: unconditional loads)
      const float wl = w0[co * 9 + t];
      const float w = k < 27 ? wl : 0.f;
      const __bf16 wh = (__bf16)w;
      const __bf16 wv = k < 18 ? wh : (__bf16)(w - (float)wh);
      v[j] = __builtin_bit_cast(unsigned short, wv);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[n][j] = (unsigned)v[2 * j] | ((unsigned)v[2 * j + 1] << 16);
  }
  // the lane's 8 B-operand offsets (u16 elements, relative to its window's top-left
  // in the bordered plane): slot j of chunk g = plane hi/lo, tap t.  The padding
  // slots k >= 27 (zero weights) read the window's centre: 0 x a finite value is 0,
  // and no per-lane select or branch guards the reads
  int boff[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int k = 8 * g + j;
    const int t = k < 9 ? k : k < 18 ? k - 9 : k < 27 ? k - 18 : 4;
    const bool lo = k >= 9 && k < 18;
    boff[j] = (lo ? plane : 0) + (t / 3) * Wb + (t % 3);
  }

  // stage the clip: zero both planes (the border = the conv's zero padding), then the
  // interior as bf16 (hi, lo); rows of whole float4s when W % 4 == 0
  const float* xc = x + (size_t)clip * Hin * Win;
  {
    const int n16 = (2 * plane * 2 + 15) / 16;
    for (int i = threadIdx.x; i < n16; i += 256) ((u32x4*)c0lds)[i] = u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();
  auto put = [&](int r, int c, float v) {  // input (r, c) -> bordered (r + 1, c + 1)
    const int i = (r + 1) * Wb + c + 1;
    const __bf16 h = (__bf16)v;
    hp[i] = __builtin_bit_cast(unsigned short, h);
    lp[i] = __builtin_bit_cast(unsigned short, (__bf16)(v - (float)h));
  };
  c0_stage(xc, Hin, Win, put);
  __syncthreads();

  const int npo = H * W;                 // pooled outputs
  const int ngroups = (npo + 15) >> 4;
  char* oc = (char*)out + (size_t)clip * npo * CB;
  float cs = 1.f;
  if constexpr (FM == 2) cs = cscale[clip];
  for (int gi = wave; gi < ngroups; gi += 4) {
    const int q0 = 16 * gi + i16;
    const int q = q0 < npo ? q0 : npo - 1;
    const int ph = q / W, pw = q - ph * W;
    f32x4 pacc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) pacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the lane's 8 read addresses for member 0 (window top-left (ph PH, pw PW), bordered)
    const char* la[8];
    {
      const int base0 = ph * PH * Wb + pw * PW;
#pragma unroll
      for (int j = 0; j < 8; ++j) la[j] = (const char*)c0lds + 2 * (base0 + boff[j]);
    }
    auto member = [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int moff = 2 * ((k / PW) * Wb + k % PW);  // an immediate when FWB > 0
      unsigned short bv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) bv[j] = *(const unsigned short*)(la[j] + moff);
      u32x4 b;
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (unsigned)bv[2 * j] | ((unsigned)bv[2 * j + 1] << 16);
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[n]),
                                                                  __builtin_bit_cast(bf16x8, b),
                                                                  f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) pacc[n][r] += relu_keepnan(acc[r]);
      }
      // (two members between fences: one's reads overlap the other's MFMAs without every
      // member's results live at once -- the empty asm makes the sums materialise here,
      // which a sched_barrier alone does not: the IR moves the arithmetic across it)
      if constexpr (k & 1) {
#pragma unroll
        for (int n = 0; n < NT; ++n) asm volatile("" : "+v"(pacc[n]));
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    static_for<P>(member);
    if (q0 >= npo) continue;
    char* op = oc + (size_t)q0 * CB;
    typedef typename ActT<FM == 2 ? 2 : 0>::T AT;
    typedef typename ActT<FM == 2 ? 2 : 0>::V4 AT4;
    AT4 hv[NT], lv[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // avg_pool2d's sum / count: the reciprocal product with one FMA correction
        float v = pacc[n][r];
        if constexpr (P > 1) {
          constexpr float rp = 1.0f / (float)P;
          const float q = v * rp;
          v = fmaf(fmaf(-q, (float)P, v), rp, q);
        }
        if constexpr (FM == 2) v *= cs;  // exact: a power of two
        if (ONES && (co16(NT, n, 4 * g + r) == C || co16(NT, n, 4 * g + r) == C + 1)) v = cs;
        hv[n][r] = (AT)v;
        if constexpr (SP == 2) lv[n][r] = (AT)(v - (float)hv[n][r]);
      }
#pragma unroll
    for (int pt = 0; pt < SP; ++pt) {
      AT4* vv = pt ? lv : hv;
#pragma unroll
      for (int pr = 0; pr < NT / 2; ++pr) {
        const u32x2 a0 = __builtin_bit_cast(u32x2, vv[2 * pr]), a1 = __builtin_bit_cast(u32x2, vv[2 * pr + 1]);
        *(u32x4*)(op + pt * CP * 2 + 64 * pr + 16 * g) = u32x4{a0[0], a0[1], a1[0], a1[1]};
      }
      if constexpr (NT & 1) *(u32x2*)(op + pt * CP * 2 + 64 * (NT / 2) + 8 * g) = __builtin_bit_cast(u32x2, vv[NT - 1]);
    }
  }
}

// --------------------------------------------------------------------------- //
// conv0 of the bf16 format (FM 0) with an average pool (res8 4x3, res26 2x2; round 6).
// bf16 weights (the format's own) times the input as bf16 (hi, lo): two products, in a K
// layout all four lane groups share -- slot j of lane group g reads plane (g < 2: hi, else
// lo) at tap row dy = 2 (g & 1) + j / 4 and tap column dx = j % 4 (dy or dx = 3: a zero
// weight; the read is an in-image value or the zero border, and a non-finite one only
// lands in a clip whose logits are NaN anyway).  A lane's B operand for pool member (mr,
// mc) is then 4 pairs of ONE plane: patch rows mr, mr + 1, columns mc, mc + 2 (and + 1),
// counted from its window's row 4 ph + 2 (g & 1) -- the same registers in every lane group.
// So an m-tile loads its lane's (PH + 1) x (PW + 3) patch once (res8: 30 LDS reads per 16
// pooled outputs; conv0m_kernel reads 8 u16 per member, 96) and packs each row's pairs once
// (25 packs; conv0m_kernel: 48).  Everything else is conv0m_kernel's.
template <int NT, int PH, int PW, bool ONES, int FWB = 0>
__global__ __launch_bounds__(256, 5) void conv0p_kernel(const float* __restrict__ x, __bf16* __restrict__ out,
                                                     const float* __restrict__ w0, int Hin, int Win, int H, int W,
                                                     int C) {
  constexpr int CP = 16 * NT, CB = CP * 2;
  constexpr int PR = PH + 1, PC = PW + 3;  // patch rows, columns (pairs per row: PC - 1)
  extern __shared__ __attribute__((aligned(16))) unsigned short c0lds[];  // hi plane, lo plane, a zero row
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = lane >> 4, i16 = lane & 15;
  const int clip = blockIdx.x;
  const int Wb = FWB > 0 ? FWB : Win + 2, plane = (Hin + 2) * Wb;
  unsigned short* hp = c0lds;
  unsigned short* lp = c0lds + plane;

  // weights: A fragment of n-tile n (row = out channel co16(NT, n, i16), k-chunk g)
  u32x4 wa[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int co = co16(NT, n, i16);
    unsigned short v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int dy = 2 * (g & 1) + j / 4, dx = j % 4;
      const float w = w0[co * 9 + (dy < 3 && dx < 3 ? dy * 3 + dx : 0)];
      v[j] = __builtin_bit_cast(unsigned short, (__bf16)(dy < 3 && dx < 3 ? w : 0.f));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) wa[n][j] = (unsigned)v[2 * j] | ((unsigned)v[2 * j + 1] << 16);
  }

  // stage the clip (conv0m_kernel's staging), plus one zero row past the lo plane: the
  // patch of the last pooled row reaches one row beyond the bordered image when PH | Hin
  const float* xc = x + (size_t)clip * Hin * Win;
  {
    const int n16 = ((2 * plane + Wb) * 2 + 15) / 16;
    for (int i = threadIdx.x; i < n16; i += 256) ((u32x4*)c0lds)[i] = u32x4{0u, 0u, 0u, 0u};
  }
  __syncthreads();
  auto put = [&](int r, int c, float v) {
    const int i = (r + 1) * Wb + c + 1;
    const __bf16 h = (__bf16)v;
    hp[i] = __builtin_bit_cast(unsigned short, h);
    lp[i] = __builtin_bit_cast(unsigned short, (__bf16)(v - (float)h));
  };
  c0_stage(xc, Hin, Win, put);
  __syncthreads();

  const int npo = H * W;
  const int ngroups = (npo + 15) >> 4;
  char* oc = (char*)out + (size_t)clip * npo * CB;
  for (int gi = wave; gi < ngroups; gi += 4) {
    const int q0 = 16 * gi + i16;
    const int q = q0 < npo ? q0 : npo - 1;
    // (FWB > 0: the pooled width (FWB - 2) / PW is a compile-time divisor)
    const int Wq = FWB > 0 ? (FWB - 2) / PW : W;
    const int ph = q / Wq, pw = q - ph * Wq;
    const unsigned short* pb = c0lds + (g >= 2 ? plane : 0) + (ph * PH + 2 * (g & 1)) * Wb + pw * PW;
    // the patch's pairs: pr[i][c] = (row i column c, row i column c + 1)
    unsigned pr[PR][PC - 1];
#pragma unroll
    for (int i = 0; i < PR; ++i) {
      unsigned short v[PC];
#pragma unroll
      for (int c = 0; c < PC; ++c) v[c] = pb[i * Wb + c];
#pragma unroll
      for (int c = 0; c < PC - 1; ++c) pr[i][c] = (unsigned)v[c] | ((unsigned)v[c + 1] << 16);
    }
    f32x4 pacc[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n) pacc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    // software-pipelined members: member k + 1's MFMAs issue before member k's ReLU + sum
    // reads its results (SQ: 52 % of the wave cycles stalled on an instruction dependency
    // when each member's VALU read its MFMAs right behind them)
    f32x4 am[2][NT];
    auto issue = [&](auto kc) {
      constexpr int k = decltype(kc)::value, mr = k / PW, mc = k % PW;
      const u32x4 b{pr[mr][mc], pr[mr][mc + 2], pr[mr + 1][mc], pr[mr + 1][mc + 2]};
#pragma unroll
      for (int n = 0; n < NT; ++n)
        am[k & 1][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, wa[n]),
                                                              __builtin_bit_cast(bf16x8, b),
                                                              f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
    };
    auto fold = [&](auto kc) {
      constexpr int k = decltype(kc)::value;
#pragma unroll
      for (int n = 0; n < NT; ++n)
#pragma unroll
        for (int r = 0; r < 4; ++r) pacc[n][r] += relu_keepnan(am[k & 1][n][r]);
    };
    issue(std::integral_constant<int, 0>{});
    static_for<PH * PW>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      if constexpr (k + 1 < PH * PW) issue(std::integral_constant<int, k + 1>{});
      __builtin_amdgcn_sched_barrier(0);
      fold(kc);
#pragma unroll
      for (int n = 0; n < NT; ++n) asm volatile("" : "+v"(pacc[n]));
      __builtin_amdgcn_sched_barrier(0);
    });
    if (q0 >= npo) continue;
    char* op = oc + (size_t)q0 * CB;
    typename ActT<0>::V4 hv[NT];
#pragma unroll
    for (int n = 0; n < NT; ++n)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = pacc[n][r];
        constexpr float rp = 1.0f / (float)(PH * PW);
        const float qv = v * rp;
        v = fmaf(fmaf(-qv, (float)(PH * PW), v), rp, qv);
        const int co = co16(NT, n, 4 * g + r);
        if (ONES && (co == C || co == C + 1)) v = 1.f;
        hv[n][r] = (__bf16)v;
      }
#pragma unroll
    for (int p2 = 0; p2 < NT / 2; ++p2) {
      const u32x2 a0 = __builtin_bit_cast(u32x2, hv[2 * p2]), a1 = __builtin_bit_cast(u32x2, hv[2 * p2 + 1]);
      *(u32x4*)(op + 64 * p2 + 16 * g) = u32x4{a0[0], a0[1], a1[0], a1[1]};
    }
    if constexpr (NT & 1) *(u32x2*)(op + 64 * (NT / 2) + 8 * g) = __builtin_bit_cast(u32x2, hv[NT - 1]);
  }
}

#ifndef HONK_RES_VF_TU
// --------------------------------------------------------------------------- //
// weight packing
// --------------------------------------------------------------------------- //
__global__ void pack_conv0_kernel(const float* __restrict__ w, float* __restrict__ out, int C, int CP) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= CP * 9) return;
  const int c = i / 9;
  out[i] = (c < C) ? w[i] : 0.f;
}

// frag[nt][tap][q][lane][j] = W[co = nt*16 + (lane&15)][ci = 16q + 4(lane>>4) + j][tap]
__global__ void pack_block_kernel(const float* __restrict__ w, float* __restrict__ frag, int C, int NT) {
  const int CP = 16 * NT;
  const int Q = CP / 16;
  const int total = NT * 9 * Q * 4 * 64;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int r = i;
  const int j = r & 3; r >>= 2;
  const int lane = r & 63; r >>= 6;
  const int q = r % Q; r /= Q;
  const int tap = r % 9; r /= 9;
  const int nt = r;
  const int co = nt * 16 + (lane & 15);
  const int ci = 16 * q + 4 * (lane >> 4) + j;
  frag[i] = (co < C && ci < C) ? w[((size_t)co * C + ci) * 9 + tap] : 0.f;
}

__global__ void pack_bn_kernel(const float* __restrict__ mean, const float* __restrict__ var,
                               float* __restrict__ scale, float* __restrict__ shift, int C, int CP) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= CP) return;
  if (c < C) {
    const float inv = 1.0f / sqrtf(var[c] + 1e-5f);
    scale[c] = inv;
    shift[c] = -mean[c] * inv;
  } else {
    scale[c] = 1.f;
    shift[c] = 0.f;
  }
}

__global__ void copy_kernel(const float* __restrict__ src, float* __restrict__ dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src ? src[i] : 0.f;
}

// --------------------------------------------------------------------------- //
// f16x2 range and fitness (the numerics record, HONK_NUM_* in include/honk_hip.h)
//
// The f16x2 path stores every pre-BN tensor as ONE fp16: 11 significant bits and a
// range of 2^-14 .. 65504.  Range: every stored tensor of a clip carries one
// power-of-two scale s (the clip's scale, clip_scale_kernel): conv0 writes
// s * relu(conv0(x)) and s itself into the folded-bias channel C, and from there on
// the scale rides along exactly -- the bias weights multiply channel C (= s), the
// odd layers' passthrough keeps it, ReLU is positively homogeneous, the residual
// adds two tensors of the same scale -- so every layer computes s * (its output), a
// power-of-two multiple of the unscaled arithmetic (bit for bit while the values stay
// normal), and tail_sum_kernel divides the channel sums by s.
// s = s_model * 2^-e(clip):
//  * s_model (pack time) puts M = max over the BatchNorm'd tensors and channels of
//    |running_mean| + 8 sqrt(running_var) -- the calibrated size of the stored values
//    (bn2 also bounds conv0's output: relu(conv2) + x0 >= x0) -- just below 2^4, which
//    leaves 2^12 of headroom to fp16's maximum and 2^18 down to its smallest normal;
//  * e(clip) (per clip, from its input) = the binades by which the clip's bound
//    max|x| * max_c sum_t |w0[c][t]| on conv0's output exceeds M: an out-of-range clip
//    (MFCCs of another scale, c0 in the -1e3..-1e4 range) is scaled down before it is
//    stored, not clipped to Inf.
// Fitness (the host policy, honk_res_select_precision): the fp16 rounding of a
// stored value costs 2^-12 |x|, i.e. 2^-12 |x| / std in the next layer's BatchNorm
// units, so the error grows with rho = sqrt(mean_c (mean_c^2 + var_c) / var_c); and
// a folded weight part beyond fp16's range cannot be stored at all (flag).
// --------------------------------------------------------------------------- //
#define HONK_NUM_TARGET_EXP 4  // M * s_model < 2^4
// Weight exponents (f16x2): the folded weights W * invstd of a layer whose input has a
// large spread (e.g. the residual stream of a model fed MFCCs at 1e3..1e4 scale:
// std 1e4 -> invstd 1e-4) fall below fp16's smallest normal (6.1e-5), where the
// (hi, lo) split keeps only ~2^-25 absolute -- a percent of the weight.  So layer i's
// fragments are packed as W * invstd * 2^kw[i]: an odd layer i and the even layer
// i + 1 after it take +k / -k (the odd layer's output X_i is stored at 2^k times the
// residual stream's scale -- its channel-C passthrough and border-bias weights carry
// the same 2^k, so the scale rides along as the clip scale does -- and the even layer
// maps it back onto the residual stream), k balancing the two layers' rms weights
// around their geometric mean, bounded so that X_i keeps the residual stream's fp16
// headroom (|mean| + 8 std of bn_i times s_model times 2^k < 2^5).  A last odd layer
// (its output is only summed, in fp32) aims its rms weight at 2^-4.  Models at unit
// scale get kw = 0 or +-1 (their weights are already O(0.05)).
// One workgroup: per-layer sums of squares over the fp32 fragments (pack_block_kernel
// layout), then thread 0.
__global__ __launch_bounds__(256) void pack_range_kernel(float* __restrict__ rec, const float* __restrict__ bn,
                                                         const float* __restrict__ w0,
                                                         const float* __restrict__ frag32, size_t layer_floats,
                                                         int C, int CP, int NT, int L) {
  __shared__ double red[256];
  float* erms = rec + HONK_NUM_KW + L - 1;  // scratch after kw[]: erms[i], i = 1..L
  const int Q = CP / 16;
  for (int i = 0; i < L; ++i) {
    // rms of the folded weights W[co][ci][t] * invstd_{i-1}[ci] (layer 1: no input BN)
    const float* fr = frag32 + (size_t)i * layer_floats;
    const float* inv = i > 0 ? bn + (size_t)2 * CP * (i - 1) : nullptr;
    double q = 0.0;
    for (size_t e = threadIdx.x; e < layer_floats; e += blockDim.x) {
      const int j = (int)(e & 3), lane = (int)((e >> 2) & 63);
      const int qq = (int)((e >> 8) % Q);
      const int ci = 16 * qq + 4 * (lane >> 4) + j;
      const double v = (double)fr[e] * (inv && ci < C ? (double)inv[ci] : 1.0);
      q += v * v;
    }
    red[threadIdx.x] = q;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
      if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      const double ms = red[0] / ((double)C * C * 9);
      erms[i + 1] = ms > 0 ? (float)(0.5 * log2(ms)) : 0.f;
    }
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  float w0s = 0.f;
  for (int c = 0; c < C; ++c) {
    float s = 0.f;
    for (int t = 0; t < 9; ++t) s += fabsf(w0[c * 9 + t]);
    w0s = fmaxf(w0s, s);
  }
  float M = 0.f, rho = 0.f;
  int rho_layer = 0;
  bool bad = !(w0s <= 3.0e38f);
  for (int i = 0; i < L; ++i) {
    const float* sc = bn + (size_t)2 * CP * i;  // [scale = invstd][shift = -mean * invstd]
    double q = 0.0;
    for (int c = 0; c < C; ++c) {
      const float inv = sc[c], sh = sc[CP + c];
      const float m = (fabsf(sh) + 8.f) / inv;  // |mean| + 8 std
      if (!(m <= 3.0e38f) || !(inv > 0.f)) bad = true;
      else M = fmaxf(M, m);
      q += (double)sh * (double)sh;
    }
    const float r = (float)sqrt(1.0 + q / (C > 0 ? C : 1));
    if (!(r <= 3.0e38f)) bad = true;
    else if (r > rho) {
      rho = r;
      rho_layer = i + 1;
    }
  }
  float s = 1.f;
  if (M > 0.f) {
    int ex;
    (void)frexpf(M, &ex);  // M < 2^ex
    int e = HONK_NUM_TARGET_EXP - ex;
    if (e > 14) e = 14;
    if (e < -24) e = -24;
    s = ldexpf(1.f, e);
  }
  // the per-layer weight exponents (layers 1..L, 1-based)
  float* kw = rec + HONK_NUM_KW;
  int kout = 0;  // exponent of the last layer's output relative to the residual stream
  for (int i = 1; i <= L; ++i) kw[i - 1] = 0.f;
  for (int i = 1; i <= L && !bad; i += 2) {
    if (i + 1 <= L) {
      int k = (int)rintf(0.5f * (erms[i + 1] - erms[i]));
      // X_i's headroom: (|mean| + 8 std of bn_i) * s_model * 2^k < 2^5
      const float* sc = bn + (size_t)2 * CP * (i - 1);
      float mx = 0.f;
      for (int c = 0; c < C; ++c) mx = fmaxf(mx, (fabsf(sc[CP + c]) + 8.f) / sc[c]);
      int ex = -126;
      if (mx * s > 0.f) (void)frexpf(mx * s, &ex);
      if (k > 5 - ex) k = 5 - ex;
      k = k > 20 ? 20 : k < -20 ? -20 : k;
      kw[i - 1] = (float)k;
      kw[i] = (float)-k;
    } else {
      int k = (int)rintf(-4.f - erms[i]);
      k = k > 20 ? 20 : k < -20 ? -20 : k;
      kw[i - 1] = (float)k;
      kout = k;
    }
  }
  rec[HONK_NUM_SCALE] = s;
  rec[HONK_NUM_RANGE] = M;
  rec[HONK_NUM_W0SUM] = w0s;
  rec[HONK_NUM_RHO] = bad ? __builtin_nanf("") : rho;
  // rec[HONK_NUM_F16_OVERFLOW] is set by pack_block16_kernel (which runs after this kernel)
  rec[HONK_NUM_RHO_LAYER] = (float)rho_layer;
  rec[HONK_NUM_OUT_SCALE] = ldexpf(1.f, kout);
  rec[HONK_NUM_VALID] = 1.f;
}

// The clip's power-of-two scale (see above): one wave per clip; a clip with a
// non-finite input keeps s_model (its NaN / Inf propagates as in the reference).
// flags (may be null): [n] the clips' admission flags, initialised here (2: the input is
// not finite, else 0; tail_sum_kernel raises 1).
__global__ __launch_bounds__(256) void clip_scale_kernel(const float* __restrict__ x, const float* __restrict__ rec,
                                                         float* __restrict__ cscale, int n, int hw,
                                                         int* __restrict__ flags) {
  const int lane = threadIdx.x & 63;
  const int clip = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (clip >= n) return;
  const float* xc = x + (size_t)clip * hw;
  float mx = 0.f;
  bool bad = false;
  if ((hw & 3) == 0) {
    const f32x4* x4 = (const f32x4*)xc;
    for (int i = lane; i < (hw >> 2); i += 64) {
      const f32x4 v = x4[i];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float a = fabsf(v[u]);
        bad |= !(a <= 3.4e38f);
        mx = fmaxf(mx, a);
      }
    }
  } else {
    for (int i = lane; i < hw; i += 64) {
      const float a = fabsf(xc[i]);
      bad |= !(a <= 3.4e38f);
      mx = fmaxf(mx, a);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  bad = __any(bad);
  float s = rec[HONK_NUM_SCALE];
  const float M = rec[HONK_NUM_RANGE], bound = mx * rec[HONK_NUM_W0SUM];
  if (!bad && M > 0.f && bound > M) {
    const float r = bound / M;
    int ex = 126;
    if (r <= 1e37f) (void)frexpf(r, &ex);  // r < 2^ex
    s = ldexpf(s, -ex);
  }
  s = fminf(fmaxf(s, 0x1p-24f), 0x1p14f);  // channel C holds s: an exact fp16 value
  if (lane == 0) {
    cscale[clip] = s;
    if (flags) flags[clip] = bad ? 2 : 0;
  }
}

// The f16x2 admission's bookkeeping (honk_res_forward): the flagged clips' indices in
// batch order (one workgroup, a fixed-order scan: the re-run is deterministic), then the
// gather of their inputs and the scatter of their re-run logits.
__global__ __launch_bounds__(1024) void flag_compact_kernel(const int* __restrict__ flags, int64_t n,
                                                            int* __restrict__ list, int* __restrict__ count) {
  __shared__ int part[1024];
  const int t = threadIdx.x;
  const int64_t per = (n + 1023) / 1024, lo = t * per, hi = lo + per < n ? lo + per : n;
  int k = 0;
  for (int64_t i = lo; i < hi; ++i) k += flags[i] == 1;
  part[t] = k;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // inclusive scan (Hillis-Steele)
    const int v = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int w = part[t] - k;
  for (int64_t i = lo; i < hi; ++i)
    if (flags[i] == 1) list[w++] = (int)i;
  if (t == 1023) *count = part[1023];
}

__global__ __launch_bounds__(256) void gather_clips_kernel(const float* __restrict__ x, const int* __restrict__ list,
                                                           int hw, float* __restrict__ out) {
  const float* src = x + (size_t)list[blockIdx.x] * hw;
  float* dst = out + (size_t)blockIdx.x * hw;
  for (int i = threadIdx.x; i < hw; i += blockDim.x) dst[i] = src[i];
}

__global__ __launch_bounds__(64) void scatter_logits_kernel(const float* __restrict__ src,
                                                            const int* __restrict__ list, int n, int NL,
                                                            float* __restrict__ logits) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n * NL) return;
  logits[(size_t)list[i / NL] * NL + i % NL] = src[i];
}

// --------------------------------------------------------------------------- //
// host side
// --------------------------------------------------------------------------- //
struct Layout {
  int C, CP, NT, L, NL, prec;
  int Hin, Win, H, W, ph, pw;
  size_t off_conv0, off_layers, layer_floats, off_bn, off_wout, off_bout, off_zeros, off_frag16, frag16_floats,
      off_fragx3, fragx3_floats, off_fragh, off_bias16, off_range, total;
};

// operand format of the bf16-pipe kernels (res_bf16w.inc): 0 bf16, 1 bf16x3, 2 f16x2;
// activation parts in memory (2 for bf16x3 only)
static int fmt_of(int prec) { return prec == HONK_PREC_BF16X3 ? 1 : prec == HONK_PREC_F16X2 ? 2 : 0; }
static int sp_of(int fm) { return fm == 1 ? 2 : 1; }

static size_t round64(size_t x) { return (x + 63) & ~(size_t)63; }

static int make_layout(const honk_res_desc* d, Layout* L) {
  if (!d) return fail(HONK_ERR_ARG, "null descriptor");
  if (d->n_maps < 1 || d->n_layers < 0 || d->n_labels < 1 || d->height < 1 || d->width < 1)
    return fail(HONK_ERR_ARG, "bad res descriptor (n_maps=%d n_layers=%d n_labels=%d h=%d w=%d)",
                d->n_maps, d->n_layers, d->n_labels, d->height, d->width);
  if (d->n_maps > 64 || (d->n_maps > 48 && d->precision != HONK_PREC_F32))
    return fail(HONK_ERR_UNSUPPORTED,
                "n_feature_maps=%d: the gfx950 kernels take up to 64 maps in precision f32, 48 in bf16 / bf16x3 / f16x2",
                d->n_maps);
  L->C = d->n_maps;
  L->NT = (d->n_maps + 15) / 16;
  L->CP = 16 * L->NT;
  L->L = d->n_layers;
  L->NL = d->n_labels;
  L->Hin = d->height;
  L->Win = d->width;
  L->ph = d->pool_h > 0 ? d->pool_h : 1;
  L->pw = d->pool_w > 0 ? d->pool_w : 1;
  L->H = L->Hin / L->ph;
  L->W = L->Win / L->pw;
  if (L->H < 1 || L->W < 1) return fail(HONK_ERR_ARG, "pool larger than input");
  if (L->W * L->CP * 4 > 65535)  // staging offsets pack the row byte offset in 16 bits
    return fail(HONK_ERR_UNSUPPORTED, "feature-map width %d too large for the staging plan", L->W);
  L->off_conv0 = 0;
  L->off_layers = round64((size_t)L->CP * 9);
  L->layer_floats = (size_t)9 * L->CP * L->CP;
  L->off_bn = L->off_layers + L->layer_floats * L->L;
  L->off_wout = L->off_bn + round64((size_t)2 * L->CP * L->L);
  L->off_bout = L->off_wout + round64((size_t)L->NL * L->C);
  L->off_zeros = L->off_bout + round64((size_t)L->NL);
  // bf16 weight fragments per layer (layout G16R::xfrag: k-steps across the three
  // dy rows) for HONK_PREC_BF16 and the hi/lo pairs for HONK_PREC_BF16X3
  L->off_frag16 = L->off_zeros + 64;
  L->frag16_floats = (size_t)g16_frag_bytes(L->NT, 1) / 4;
  L->off_fragx3 = L->off_frag16 + L->frag16_floats * L->L;
  L->fragx3_floats = (size_t)g16_frag_bytes(L->NT, 2) / 4;
  // fp16 (hi, lo) weight fragments for HONK_PREC_F16X2 (same layout and size as bf16x3's)
  L->off_fragh = L->off_fragx3 + L->fragx3_floats * L->L;
  // folded input-BN bias [L][16 classes][CP] for the bf16 kernel
  L->off_bias16 = L->off_fragh + L->fragx3_floats * L->L;
  // the numerics record (pack_range_kernel, HONK_NUM_*: 64 header floats, kw[L], scratch[L])
  L->off_range = L->off_bias16 + round64((size_t)16 * L->CP * L->L);
  L->total = L->off_range + HONK_NUM_KW + round64((size_t)2 * L->L);
  L->prec = d->precision;
  if (L->prec != HONK_PREC_F32 && L->prec != HONK_PREC_BF16 && L->prec != HONK_PREC_BF16X3 &&
      L->prec != HONK_PREC_F16X2)
    return fail(HONK_ERR_ARG, "unknown precision %d", d->precision);
  return HONK_OK;
}

static int64_t chunk_clips(const Layout& L, int64_t batch) {
  const size_t per_clip = (size_t)L.H * L.W * L.CP * sizeof(float);
  // 4096 clips (3.2 GB per buffer for res15) keeps >200 tiles per CU per launch; pooled maps
  // (res8 25 x 13, res26 50 x 20: <= 256 KiB per clip) take 8192 -- a res8 chunk's six
  // launches are ~0.45 ms at 4096 clips, and C3 measured 9.40M -> 10.07M clips/s at 8192
  // (16384 / 32768 within 0.5 % of it; res15 unchanged at 8192; exp/chunk_ab.sh)
  int64_t ch = per_clip <= ((size_t)256 << 10)   ? 8192
               : per_clip <= ((size_t)1 << 20) ? 4096
                                               : (int64_t)((size_t)4 << 30) / (int64_t)per_clip;
  if (const char* e = getenv("HONK_RES_CHUNK")) ch = atoll(e);
  if (ch < 1) ch = 1;
  return batch < ch ? batch : ch;
}

struct Plan {
  int NT, MT, TH, nbands;
};

// choose MT (m-tiles per wave) and TH (rows per band) to minimise padded work
static Plan plan_block(const Layout& L) {
  Plan best{L.NT, 4, 1, L.H};
  double best_cost = 1e30;
  const int mts[5] = {5, 4, 6, 3, 2};  // preference order on equal cost
  for (int mi = 0; mi < 5; ++mi) {
    const int MT = mts[mi];
    if (L.NT == 3 && MT > 5) continue;  // VGPR budget at 3 waves/SIMD
    if (L.NT == 4 && MT != 2) continue;  // 16 waves (4 per SIMD): MT = 2 fits 128 VGPRs
    const int MP = 16 * MT * MW;
    const int thmax = MP / L.W;
    if (thmax < 1) continue;
    const int nb = (L.H + thmax - 1) / thmax;
    const int th = (L.H + nb - 1) / nb;
    // cost ~ padded pixels per clip (all m-tiles are computed), plus a per-stage
    // fixed overhead (barrier + staging issue ~ 2.5k cycles vs 576*MT MFMA cycles)
    const double cost = (double)nb * MP * (1.0 + 4.3 / MT);
    if (cost < best_cost - 1e-9) {
      best_cost = cost;
      best = Plan{L.NT, MT, th, nb};
    }
  }
  return best;
}

// Row-band kernel plan (res_bf16r.inc): 8 waves x MT m-tiles (g16r_mt); TH rows of
// one dilation class per tile, limited by the tile's pixels and by the staging
// image (TH + 2 rows); TH = 0: the width does not fit the staging plan (the
// bf16 / bf16x3 modes then fail with HONK_ERR_UNSUPPORTED; f32 has no such limit).
struct PlanR {
  int NT, MT, TH;
};
static PlanR plan_block16r(const Layout& L, int SP) {
  PlanR r{L.NT, g16r_mt(L.NT, SP), 0};
  const int MP = 16 * 8 * r.MT;
  const int rpx = g16r_rpx(L.NT, r.MT, SP);
  int th = MP / L.W;
  if (rpx / L.W - 2 < th) th = rpx / L.W - 2;
  if (th < 1 || (th + 2) * L.W * L.CP * 2 * SP / 16 < 64) return r;
  r.TH = th;
  return r;
}
static int max_bands_per_clip(const Layout& L, int TH, int use_dilation) {
  int best = 0;
  for (int i = 1; i <= L.L; ++i) {
    const int n = band_geo(L.H, use_dilation ? (1 << ((i - 1) / 3)) : 1, TH).nbc;
    if (n > best) best = n;
  }
  return best;
}

// Weight-stationary kernel plan (res_bf16w.inc) for one layer at dilation d: the
// band height TH (class rows per tile) minimising a cycle model -- per tile, the
// slowest wave's m-tiles x the MFMA cycles of one m-tile plus a fixed per-tile
// cost (barrier, first operand reads) -- among the heights whose (TH + 2)-row
// image (W + d pixels per row + 1) fits the staging buffer.  0: does not fit.
static int plan_w_th(const Layout& L, int FM, int d) {
  const int SP = sp_of(FM);
  const int imgpx = g16w_img_px(L.NT, SP);
  const int RW = L.W + d;
  int thmax = (imgpx - 1) / RW - 2;
  const int q = L.H / d, rem = L.H - q * d;
  const int nmax = q + (rem ? 1 : 0);
  if (thmax > nmax) thmax = nmax;
  if (thmax < 1) return 0;
  // 16-bit per-lane offsets of the kernel (tap offsets, staging chunks in 16-B
  // units, the separator code 0xffff landing past the clip)
  const long CB = 32L * L.NT * SP, RB = (long)L.W * CB;
  if ((RW + 1) * CB + 16 * (2 * L.NT) >= 32768) return 0;
  if (0xffffL * 16 - (long)d * RB < (long)L.H * RB) return 0;
  while (thmax >= 1 && ((long)(thmax + 1) * d * RB + RB) / 16 >= 0xffff) --thmax;
  if (thmax < 1) return 0;
  const int ksa = (18 * L.NT + 3) / 4;
  const double c_mt = ksa * L.NT * (FM == 1 ? 3 : FM == 2 ? 2 : 1) * 16.0, c_tile = 1500.0;
  int best = 0;
  double best_cost = 1e300;
  for (int th = thmax; th >= 1; --th) {
    double cost = 0;
    for (int cls = 0; cls < d; ++cls) {
      const int n = q + (cls < rem ? 1 : 0);
      for (int k = 0; k * th < n; ++k) {
        const int rows = std::min(th, n - k * th);
        const int nmt = (rows * L.W + 15) / 16;
        const int it = std::max(1, (nmt + 3) / 4);
        cost += it * c_mt + c_tile;
      }
    }
    if (cost < best_cost * (1 - 1e-9)) {
      best_cost = cost;
      best = th;
    }
  }
  return best;
}
static int dil_of(const honk_res_desc* d, int i) { return d->use_dilation ? (1 << ((i - 1) / 3)) : 1; }
// bands per clip of layer i under the weight-stationary plan (0: a layer does not fit)
static int bands_w(const Layout& L, const honk_res_desc* d, int FM, int i) {
  const int dl = dil_of(d, i);
  const int th = plan_w_th(L, FM, dl);
  return th ? band_geo(L.H, dl, th).nbc : 0;
}
// Which bf16 / bf16x3 block kernel runs: the weight-stationary one where it was
// measured faster (45 maps at bf16x3: res15 2.14 vs 2.21 ms per 4096-clip
// launch; it loses 7-20 % on the narrow, pooled and bf16 configurations), the
// row-band one elsewhere.  HONK_RES_KERNEL=w / r forces either (tests run both).
struct PairPlan {
  bool ok;
  int lag, NRA, NRB, slotb, ppr, ppw;  // ppw: DMA pieces per A wave per step
  int padb;                            // f16x2: zero-column bytes each side of a slot's row
  int ns;                              // streams per workgroup (block16p_kernel NS)
  bool tbl;                            // bf16 two streams: the row-table instance (SCA = -1)
  int ks;                              // 2: f16x2 with K split over two waves per SIMD (block16k_kernel)
  bool lin;                            // bf16 two streams, undilated A: linear A-in DMA (block16p_body LIN)
  int ringpad;                         // shared pad columns (Block16PArgs::ringpad)
};
static PairPlan pair_at(const Layout& L, const honk_res_desc* d, int FM, int64_t n, int grid, int i);
static bool use_w_kernel(const Layout& L, const honk_res_desc* d, int FM) {
  // 45-map bf16x3: the weight-stationary path (with fused pairs); bf16: only when
  // pairs fuse (the single weight-stationary layer is slower than the row-band one)
  // (measured: res15 bf16 +4 %; res8's 13-pixel rows lose 20 % -- row-band there);
  // f16x2: always (its only kernels)
  // bf16 on rows < 32 pixels (res8, res26): only an even stack whose every layer pairs on
  // the two-stream kernel (every pair and the last one; measured res8 0.128 ms per pair
  // launch vs 2 x 0.070 row-band layers)
  bool want = FM == 2 || (L.NT == 3 && (FM == 1 || (L.W >= 32 && L.L >= 3 && pair_at(L, d, FM, 4096, 256, 1).ok)));
  if (FM == 0 && L.NT == 3 && L.W < 32 && L.L >= 2 && L.L % 2 == 0) {
    bool all = true;
    for (int i = 1; i < L.L && all; i += 2) {
      const PairPlan pp = pair_at(L, d, FM, 4096, 256, i);
      all = pp.ok && pp.ns == 2;
    }
    want = want || all;
  }
  if (const char* e = getenv("HONK_RES_KERNEL")) {
    if (e[0] == 'r' && FM != 2) return false;
    if (e[0] == 'w' || e[0] == 'p') want = true;
  }
  if (!want) return false;
  if (L.W >= 64) return false;  // m-tile walk steps 64 pixels = at most one row carry
  if (L.C >= L.CP) return false;  // no zero-padding channel for the folded bias
  if (L.ph * L.pw > 1 && !((L.ph == 2 && L.pw == 2) || (L.ph == 4 && L.pw == 3))) return false;  // conv0 shapes
  for (int i = 1; i <= L.L; ++i)
    if (!bands_w(L, d, FM, i)) return false;
  return true;
}

// Fused pair plan (res_bf16p.inc) for layers A (dilation d) and B (tap stride sB
// class rows), at most `cpw` clips per workgroup: B's lag and the ring sizes from
// an exact walk over the steps of the longest stream.  ok = false: does not fit.
static PairPlan plan_pair(const Layout& L, int FM, int d, int sB, int cpw, int nstreams = 1, bool padcols = false,
                          bool tbl = false, int ks = 1, bool lin = false, bool sharedpad = false) {
  PairPlan pp{false, 0, 0, 0, 0, 0, 0, 0, nstreams, tbl, ks, lin, 0};
  const int SP = sp_of(FM);
  const int P = 64, W = L.W, H = L.H;
  const long PXB = g16p_pxb(L.NT, SP);  // LDS pixel pitch
  pp.ppr = (int)((W * PXB + 1023) / 1024);
  // slot pitch: room for the DMA's whole pieces, = W * PXB mod 256 so that
  // stream pixels stay at a constant LDS pitch across a row change
  pp.slotb = (int)(W * PXB + ((pp.ppr * 1024 - W * PXB + 255) / 256) * 256);
  if (lin) pp.slotb = (int)(W * PXB);  // rows contiguous in the ring (block16p_body LIN)
  if ((FM == 2 || FM == 0) && padcols) {
    // the tap-step instances and the last layer on the row table (res_bf16p.inc PADC; f16x2,
    // and bf16's: its one-stream pairs and res15's last layer): zero columns either side of every slot's
    // row, at least the widest tap offset (B's sB d columns), in 256-B units; the DMA's
    // pieces and their zero tail after the left pad
    const long sc = (long)sB * d;
    pp.padb = (int)((sc * PXB + 255) / 256 * 256);
    const long right = W * PXB + pp.padb > pp.ppr * 1024L ? W * PXB + pp.padb : pp.ppr * 1024L;
    pp.slotb = (int)((pp.padb + right + 255) / 256 * 256);
    // shared pads: a slot = its left pad + the row, the right pad being the next slot's left
    // pad (zero too: the DMA's tail zeros land there, hence padb >= the piece tail, 256 B),
    // one more pad after ring B (plan ringpad; ring A's last slot reads ring B's first left pad)
    if (sharedpad && pp.padb >= 256 && (W * PXB) % 256 == 0 && pp.ppr * 1024 - W * PXB <= pp.padb) {
      pp.slotb = (int)(pp.padb + W * PXB);
      pp.ringpad = pp.padb;
    }
  }
  const long total = (long)cpw * H * W, rows_total = (long)cpw * H;
  if (total >= (1L << 24) || sB < 1 || sB > 2) return pp;
  auto rho = [&](long q) { return q / W; };
  auto F = [&](long k) {
    long lp = (k + 2) * P + 32;
    lp = (lp < total ? lp : total) - 1;
    const long f = rho(lp) + 1;
    return f < rows_total - 1 ? f : rows_total - 1;
  };
  // B at step k computes [kP - lag - P, kP - lag) and prefetches the next step's
  // first 32 pixels; everything it reads must be finished by A before the step's
  // barrier: A's pixels below (k - 1) P + 32 (A's last m-tiles defer their
  // epilogue into the next step)
  int lag = -1;
  for (int cand = 0; cand <= 2048 && lag < 0; cand += 16) {
    const long ns = (total + cand + P - 1) / P + 1;
    bool ok = true;
    for (long k = 0; k < ns && ok; ++k) {
      long lo = k * P - cand - P, hi = k * P - cand + 32;
      if (lo < 0) lo = 0;
      if (hi > total) hi = total;
      if (hi <= lo) continue;
      const long done = (k - 1) * P + 32;
      if (done >= total) continue;
      long rmax = rho(hi - 1) + sB;
      if (rmax > rows_total - 1) rmax = rows_total - 1;
      if ((rmax + 1) * W > done) ok = false;
    }
    if (ok) lag = cand;
  }
  if (lag < 0) return pp;
  pp.lag = lag;
  const long ns = (total + lag + P - 1) / P + 1;
  long nra = 0, nrb = 0;
  for (long k = 0; k < ns; ++k) {
    if (k * P < total) {  // A reads rows >= rho(kP) - 1 while step k's DMA fills rows up to F(k)
      const long need = F(k) - (rho(k * P) - 1) + 1;
      if (need > nra) nra = need;
    }
    const long blo = k * P - lag - P;
    if (blo + P + 32 > 0 && blo < total) {  // B reads rows >= rho(blo) - sB while A writes up to rho(kP + 31)
      long wmax = k * P + 31;
      if (wmax > total - 1) wmax = total - 1;
      const long rlo = rho(blo > 0 ? blo : 0) - sB;
      const long need = rho(wmax) - rlo + 1;
      if (need > nrb) nrb = need;
    }
  }
  // rows entering the A-in ring per step: pieces per A wave
  long maxrows = 0;
  for (long k = 0; k < ns; ++k)
    if (F(k) - F(k - 1) > maxrows) maxrows = F(k) - F(k - 1);
  pp.ppw = (int)((maxrows * pp.ppr + 1) / 2);
  if (F(-1) < 0) return pp;
  pp.NRA = (int)(nra > 2 ? nra : 2);
  if (lin) {
    // a ring of whole 1-KiB pieces: NRA a multiple of 1024 / gcd(slot, 1024); the pieces per
    // step from the bytes of rows 0 .. F(k)
    int g = 1024;
    for (int b = pp.slotb; b % 2 == 0 && g > 1; b /= 2) g /= 2;  // 1024 / gcd(slotb, 1024)
    pp.NRA = ((int)nra + 1 + g - 1) / g * g;  // (+1: a step's last piece may start the row after F(k))
    const long ptot = (rows_total * (long)pp.slotb + 1023) / 1024;
    auto pieces = [&](long k) {
      const long p = ((F(k) + 1) * (long)pp.slotb + 1023) / 1024;
      return p < ptot ? p : ptot;
    };
    long mx = 0;
    for (long k = 0; k < ns; ++k)
      if (pieces(k) - pieces(k - 1) > mx) mx = pieces(k) - pieces(k - 1);
    pp.ppw = (int)((mx + 1) / 2);
    if ((long)pp.NRA * pp.slotb / 1024 <= 2 * pp.ppw + pieces(-1)) return pp;  // (the ring must outrun a step)
  }
  pp.NRB = (int)(nrb > 2 ? nrb : 2);
  const long extra = ks == 2 ? g16p_lds_extra(true, 8, pp.slotb) + g16k_xch_bytes()
                             : g16p_lds_extra(FM == 2 || padcols || tbl, 4, pp.slotb);
  if (tbl && nstreams > 1)  // the streams share the zero block, sink and zeroed slot (block16p_body SHZ)
    pp.ok = (long)(pp.NRA + pp.NRB) * pp.slotb + pp.ringpad + 4 * g16p_tr() * g16p_teb() <=
            g16p_stream_bytes(nstreams, pp.slotb + pp.ringpad);
  else
    pp.ok = (long)(pp.NRA + pp.NRB) * pp.slotb + 2L * pp.ringpad + extra <= g16p_lds_bytes() / nstreams;
  return pp;
}

// The fused pair for layers (i, i + 1) of a chunk of n clips on `grid`
// workgroups, or ok = false: i odd, i + 1 not the last layer (the pair kernel has
// no channel-sum epilogue), B's dilation d or 2d of A's, 45-map class bf16x3 on the
// weight-stationary path, an instantiated row pitch, a plan that fits the LDS.
// instantiated block16p_kernel<3, SP, PPR, PPW> (W = 40: res15, 20: res26 2x2 pool,
// 13: res8 4x3 pool) -- the plan's pieces per wave may be fewer than PPW
static int pair_ppw(int SP, int ppr) {
  if (SP == 2) return ppr == 9 ? 9 : ppr == 5 ? 10 : ppr == 3 ? 9 : 0;
  return ppr == 4 ? 4 : ppr == 2 ? 5 : 0;
}
// f16x2 pairs with an instantiated compile-time tap step (block16p_kernel SCA / SCB: res15's
// dilation pairs on 40-pixel rows): their rings carry pad columns (plan_pair padcols)
static bool pair_imm(const Layout& L, int FM, int dA, int dB) {
  if ((FM != 2 && FM != 0) || L.W != 40 || L.NT != 3) return false;
  return (dA == 1 && (dB == 1 || dB == 2)) || (dA == 2 && dB == 2) || (dA == 4 && (dB == 4 || dB == 8)) ||
         (dA == 8 && dB == 8);
}
static PairPlan pair_at(const Layout& L, const honk_res_desc* d, int FM, int64_t n, int grid, int i) {
  const PairPlan no{false, 0, 0, 0, 0, 0, 0, 0, 1, false, 1};
  const int SP = sp_of(FM);
  const char* kenv = getenv("HONK_RES_KERNEL");
  if (L.NT != 3 || (kenv && (kenv[0] == 'w' || kenv[0] == 'r'))) return no;
  // (bf16: B may be an even last layer -- it stores its output like any pair and
  // tail_act_kernel sums it; the other formats keep their fused last-layer sums)
  if (i % 2 == 0 || i + 1 > L.L || (i + 1 == L.L && FM != 0)) return no;
  const int dA = dil_of(d, i), dB = dil_of(d, i + 1);
  const int sB = dB == dA ? 1 : (dB == 2 * dA ? 2 : 0);
  const size_t cb = (size_t)n * L.H * L.W * L.CP * 2 * SP;
  if (!sB || cb >= 0xE0000000ull) return no;
  // bf16 with full 40-pixel rows: two streams per workgroup when both rings fit half the LDS
  const char* nse = getenv("HONK_PAIR_STREAMS");
  // (round 6: on the row-table walk, block16p_kernel<..., 2, 0, -1, -1>: its smaller per-wave
  // state fits 256 registers with 32 weight fragments pinned and no spill -- res15 bf16 408K
  // -> 469K clips/s against the walk-based two-stream kernel (19 spilled values reloaded in
  // its step loop, now removed), 416K with one stream on the tap-step instances, same box;
  // HONK_PAIR_STREAMS=1 selects those)
  if (FM == 0 && !(nse && nse[0] == '1')) {
    // undilated A on narrow rows whose LDS pixel is the HBM pixel: the linear A-in DMA
    // (HONK_PAIR_LIN=0 keeps the row pieces)
    const char* le = getenv("HONK_PAIR_LIN");
    if (dA == 1 && g16p_pxb(3, SP) == 32 * 3 * SP && L.W < 32 && !(le && le[0] == '0')) {
      const PairPlan pl = plan_pair(L, FM, dA, sB, (int)cdiv(cdiv(n, grid), 2), 2, false, true, 1, true);
      if (pl.ok && pl.ppr == 2 && pl.ppw <= 4) return pl;
    }
    // 40-pixel rows: the compile-time tap-step instances where their pad columns fit two
    // streams (res15's (1,1) (1,2) (2,2) (4,4) pairs; HONK_PAIR_IMM2=0 keeps the row table)
    const char* ie = getenv("HONK_PAIR_IMM2");
    if (pair_imm(L, FM, dA, dB) && !(ie && ie[0] == '0')) {
      PairPlan pi = plan_pair(L, FM, dA, sB, (int)cdiv(cdiv(n, grid), 2), 2, true, true);
      pi.tbl = false;
      if (pi.ok && pi.ppr == 4 && pi.ppw <= pair_ppw(SP, pi.ppr)) return pi;
      // the pads shared between neighbouring slots (one pad per slot): (8,8) then fits
      pi = plan_pair(L, FM, dA, sB, (int)cdiv(cdiv(n, grid), 2), 2, true, true, 1, false, true);
      pi.tbl = false;
      if (pi.ok && pi.ringpad > 0 && pi.ppr == 4 && pi.ppw <= pair_ppw(SP, pi.ppr)) return pi;
    }
    const PairPlan p2 = plan_pair(L, FM, dA, sB, (int)cdiv(cdiv(n, grid), 2), 2, false, true);
    if (p2.ok && (p2.ppr == 4 || p2.ppr == 2) && p2.ppw <= pair_ppw(SP, p2.ppr)) return p2;
  }
  const bool imm = pair_imm(L, FM, dA, dB);
  const int ppw = pair_ppw(SP, imm ? 4 : 0);
  if (FM == 2 && imm && getenv("HONK_PAIR_KS") && getenv("HONK_PAIR_KS")[0] == '1') {
    // opt-in: the K split over two waves per SIMD (block16k_kernel, res_bf16k.inc) -- measured
    // 4-5 % slower than the one-wave pair (res15 f16x2 312K vs 327K clips/s, same box;
    // DESIGN.md §3), so the default stays block16p_kernel
    const PairPlan pk = plan_pair(L, FM, dA, sB, (int)cdiv(n, grid), 1, true, false, 2);
    if (pk.ok && pk.ppr == 4 && pk.ppw <= ppw) return pk;
  }
  const PairPlan pp = plan_pair(L, FM, dA, sB, (int)cdiv(n, grid), 1, imm);
  const int ppw1 = pair_ppw(SP, pp.ppr);
  return pp.ok && ppw1 && pp.ppw <= ppw1 ? pp : no;
}

// The last layer on the pair machinery (block16l_kernel: layer A only, fused
// channel sums), or ok = false: an odd last layer (no residual) of the 45-map
// class, full 40-pixel rows (the instantiated row pitches), a ring that fits the
// stream's share of the LDS.  One clip per stream pass: the plan of a 1-clip stream
// (no A-out ring: NRB = 1 unused slot, no lag).  HONK_LAST_KERNEL=w keeps the
// weight-stationary kernel (the pair-vs-w bitwise tests).
static PairPlan last_at(const Layout& L, const honk_res_desc* d, int FM, int i) {
  const PairPlan no{false, 0, 0, 0, 0, 0, 0, 0, 1, false, 1};
  const int SP = sp_of(FM);
  const char* kenv = getenv("HONK_RES_KERNEL");
  const char* lenv = getenv("HONK_LAST_KERNEL");
  if (L.NT != 3 || (kenv && (kenv[0] == 'w' || kenv[0] == 'r')) || (lenv && lenv[0] == 'w')) return no;
  if (i != L.L || i % 2 == 0 || L.W != 40) return no;
  // two streams of 2 A waves: one wave per SIMD (bf16 with four streams, two waves per
  // SIMD at 256 registers, spilled the weights: 3.38 vs 1.65 ms per 4096-clip launch)
  const int ns = 2;
  PairPlan pp = plan_pair(L, FM, dil_of(d, i), 1, 1, ns, true);
  if (pp.NRA < 2 || pp.ppr != (SP == 2 ? 9 : 4) || pp.ppw > pair_ppw(SP, pp.ppr)) return no;
  pp.NRB = 1;
  pp.lag = 0;
  pp.ns = ns;
  pp.ok = (long)(pp.NRA + 1) * pp.slotb + g16p_lds_extra(FM == 2 || (FM == 0 && pp.padb > 0), 2, pp.slotb) <=
          g16p_lds_bytes() / ns;
  return pp.ok ? pp : no;
}

template <int NT, int FM>
static int launch_block16w(const Block16WArgs& a, hipStream_t st) {
  constexpr int SP = FM == 1 ? 2 : 1;
  int grid = cu_count();
  if (grid > a.ntiles) grid = a.ntiles;
  const dim3 gd(grid), bd(G16W<NT, SP, FM>::NTHREADS);
  const bool last = a.chsum != nullptr, res = a.res != nullptr;
  if (last && res) hipLaunchKernelGGL((block16w_kernel<NT, SP, true, true, FM>), gd, bd, 0, st, a);
  else if (last) hipLaunchKernelGGL((block16w_kernel<NT, SP, true, false, FM>), gd, bd, 0, st, a);
  else if (res) hipLaunchKernelGGL((block16w_kernel<NT, SP, false, true, FM>), gd, bd, 0, st, a);
  else hipLaunchKernelGGL((block16w_kernel<NT, SP, false, false, FM>), gd, bd, 0, st, a);
  HONK_LAUNCH_CHECK("res block16w_kernel");
  return HONK_OK;
}
static int dispatch_block16w(int NT, int FM, const Block16WArgs& a, hipStream_t st) {
#define HONK_W(nt, fm) \
  if (NT == nt && FM == fm) return launch_block16w<nt, fm>(a, st);
  HONK_W(1, 0) HONK_W(2, 0) HONK_W(3, 0)
  HONK_W(1, 1) HONK_W(2, 1) HONK_W(3, 1)
  HONK_W(1, 2) HONK_W(2, 2) HONK_W(3, 2)
#undef HONK_W
  return fail(HONK_ERR_UNSUPPORTED, "no weight-stationary kernel for NT=%d format %d", NT, FM);
}

template <int NT, int MT, int SP>
static int launch_block16r(const Block16RArgs& a, hipStream_t st) {
  using G = G16<NT, MT, SP>;
  static_assert(G16R<NT, MT, SP>::LDS <= 160 * 1024, "LDS");
  int grid = cu_count();
  if (grid > a.ntiles) grid = a.ntiles;
  const dim3 gd(grid), bd(G::NTHREADS);
  const bool last = a.chsum != nullptr, res = a.res != nullptr;
  if (last && res) hipLaunchKernelGGL((block16r_kernel<NT, MT, SP, true, true>), gd, bd, 0, st, a);
  else if (last) hipLaunchKernelGGL((block16r_kernel<NT, MT, SP, true, false>), gd, bd, 0, st, a);
  else if (res) hipLaunchKernelGGL((block16r_kernel<NT, MT, SP, false, true>), gd, bd, 0, st, a);
  else hipLaunchKernelGGL((block16r_kernel<NT, MT, SP, false, false>), gd, bd, 0, st, a);
  HONK_LAUNCH_CHECK("res block16r_kernel");
  return HONK_OK;
}

static int dispatch_block16r(const PlanR& p, int SP, const Block16RArgs& a, hipStream_t st) {
  if (SP == 1) {
    if (p.NT == 1 && p.MT == g16r_mt(1, 1)) return launch_block16r<1, g16r_mt(1, 1), 1>(a, st);
    if (p.NT == 2 && p.MT == g16r_mt(2, 1)) return launch_block16r<2, g16r_mt(2, 1), 1>(a, st);
    if (p.NT == 3 && p.MT == g16r_mt(3, 1)) return launch_block16r<3, g16r_mt(3, 1), 1>(a, st);
  } else {
    if (p.NT == 1 && p.MT == g16r_mt(1, 2)) return launch_block16r<1, g16r_mt(1, 2), 2>(a, st);
    if (p.NT == 2 && p.MT == g16r_mt(2, 2)) return launch_block16r<2, g16r_mt(2, 2), 2>(a, st);
    if (p.NT == 3 && p.MT == g16r_mt(3, 2)) return launch_block16r<3, g16r_mt(3, 2), 2>(a, st);
  }
  return fail(HONK_ERR_UNSUPPORTED, "no row-band kernel for NT=%d MT=%d SP=%d", p.NT, p.MT, SP);
}

template <int NT, int MT>
static int launch_block(const BlockArgs& a, hipStream_t st) {
  using G = Geo<NT, MT>;
  int grid = cu_count();
  if (grid > a.ntiles) grid = a.ntiles;
  if (a.chsum)
    hipLaunchKernelGGL((block_kernel<NT, MT, true>), dim3(grid), dim3(G::NTHREADS), 0, st, a);
  else
    hipLaunchKernelGGL((block_kernel<NT, MT, false>), dim3(grid), dim3(G::NTHREADS), 0, st, a);
  HONK_LAUNCH_CHECK("res block_kernel");
  return HONK_OK;
}

static int dispatch_block(const Plan& p, const BlockArgs& a, hipStream_t st) {
#define HONK_CASE(nt, mt) \
  if (p.NT == nt && p.MT == mt) return launch_block<nt, mt>(a, st);
  HONK_CASE(1, 2) HONK_CASE(1, 3) HONK_CASE(1, 4) HONK_CASE(1, 5) HONK_CASE(1, 6)
  HONK_CASE(2, 2) HONK_CASE(2, 3) HONK_CASE(2, 4) HONK_CASE(2, 5) HONK_CASE(2, 6)
  HONK_CASE(3, 2) HONK_CASE(3, 3) HONK_CASE(3, 4) HONK_CASE(3, 5)
  HONK_CASE(4, 2)
#undef HONK_CASE
  return fail(HONK_ERR_UNSUPPORTED, "no block kernel for NT=%d MT=%d", p.NT, p.MT);
}

template <typename OT, bool SPLIT = false, bool ONES = false>
static int launch_conv0(const Layout& L, const float* x, OT* out, const float* w0, int64_t n,
                        hipStream_t st, const float* cscale = nullptr) {
  const int64_t total = n * L.H * L.W;
  const int blocks = (int)cdiv(total, 256);
#define HONK_C0(PH, PW)                                                                               \
  if (L.ph == PH && L.pw == PW) {                                                                     \
    if (L.CP <= 48)                                                                                   \
      hipLaunchKernelGGL((conv0_kernel<PH, PW, OT, SPLIT, ONES>), dim3(blocks), dim3(256), 0, st, x, out, w0, \
                         (int)n, L.Hin, L.Win, L.H, L.W, L.C, L.CP, cscale);                          \
    else                                                                                              \
      hipLaunchKernelGGL((conv0_kernel<PH, PW, OT, SPLIT, ONES, 64>), dim3(blocks), dim3(256), 0, st, x, out, \
                         w0, (int)n, L.Hin, L.Win, L.H, L.W, L.C, L.CP, cscale);                      \
    HONK_LAUNCH_CHECK("res conv0_kernel");                                                            \
    return HONK_OK;                                                                                   \
  }
  HONK_C0(1, 1) HONK_C0(2, 2) HONK_C0(4, 3)
#undef HONK_C0
  if (SPLIT || ONES) return fail(HONK_ERR_UNSUPPORTED, "bf16: avg-pool %dx%d has no conv0 kernel", L.ph, L.pw);
  hipLaunchKernelGGL((conv0_generic_kernel<OT>), dim3(blocks), dim3(256), 0, st, x, out, w0, (int)n, L.Hin,
                     L.Win, L.H, L.W, L.C, L.CP, L.ph, L.pw);
  HONK_LAUNCH_CHECK("res conv0_generic_kernel");
  return HONK_OK;
}

// conv0 of the bf16-pipe formats: the MFMA kernel (conv0m_kernel) where it is
// instantiated (NT <= 3; pools 1x1, 2x2, 4x3; the staged clip within the LDS),
// else the VALU kernel.  HONK_CONV0=v forces the VALU kernel (A/B experiments).
template <int NT, int FM, bool ONES>
static int launch_conv0m_nt(const Layout& L, const float* x, void* out, const float* w0, int64_t n,
                            hipStream_t st, const float* cscale) {
  const unsigned lds = 2u * (unsigned)((L.Hin + 2) * (L.Win + 2)) * 2u;
  // bf16 with a pool: the shared-layout patch kernel (conv0p_kernel); HONK_CONV0=m keeps conv0m_kernel
  const char* ce = getenv("HONK_CONV0");
  if constexpr (FM == 0) {
    if (L.ph * L.pw > 1 && !(ce && ce[0] == 'm')) {
      const unsigned ldsp = lds + 2u * (unsigned)(L.Win + 2);
#define HONK_C0P(ph_, pw_)                                                                                     \
  if (L.ph == ph_ && L.pw == pw_) {                                                                            \
    if (ldsp > 65536)                                                                                          \
      (void)hipFuncSetAttribute((const void*)conv0p_kernel<NT, ph_, pw_, ONES>,                               \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsp);                      \
    if (L.Win == 40)                                                                                           \
      hipLaunchKernelGGL((conv0p_kernel<NT, ph_, pw_, ONES, 42>), dim3((unsigned)n), dim3(256), ldsp, st, x,   \
                         (__bf16*)out, w0, L.Hin, L.Win, L.H, L.W, L.C);                                      \
    else                                                                                                       \
      hipLaunchKernelGGL((conv0p_kernel<NT, ph_, pw_, ONES>), dim3((unsigned)n), dim3(256), ldsp, st, x,       \
                         (__bf16*)out, w0, L.Hin, L.Win, L.H, L.W, L.C);                                      \
    HONK_LAUNCH_CHECK("res conv0p_kernel");                                                                    \
    return HONK_OK;                                                                                            \
  }
      HONK_C0P(2, 2) HONK_C0P(4, 3)
#undef HONK_C0P
    }
  }
#define HONK_C0M(ph_, pw_)                                                                              \
  if (L.ph == ph_ && L.pw == pw_) {                                                                     \
    if (lds > 65536)                                                                                    \
      (void)hipFuncSetAttribute((const void*)conv0m_kernel<NT, ph_, pw_, FM, ONES>,                    \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                \
    if (L.Win == 40)                                                                                    \
      hipLaunchKernelGGL((conv0m_kernel<NT, ph_, pw_, FM, ONES, 42>), dim3((unsigned)n), dim3(256), lds, st, x, \
                         (__bf16*)out, w0, L.Hin, L.Win, L.H, L.W, L.C, cscale);                        \
    else                                                                                                \
      hipLaunchKernelGGL((conv0m_kernel<NT, ph_, pw_, FM, ONES>), dim3((unsigned)n), dim3(256), lds, st, x, \
                         (__bf16*)out, w0, L.Hin, L.Win, L.H, L.W, L.C, cscale);                        \
    HONK_LAUNCH_CHECK("res conv0m_kernel");                                                             \
    return HONK_OK;                                                                                     \
  }
  HONK_C0M(1, 1) HONK_C0M(2, 2) HONK_C0M(4, 3)
#undef HONK_C0M
  return 1;  // no instance
}
template <int FM, bool ONES>
static int launch_conv0_16(const Layout& L, const float* x, void* out, const float* w0, int64_t n, hipStream_t st,
                           const float* cscale = nullptr) {
  const char* e = getenv("HONK_CONV0");
  const bool valu = e && e[0] == 'v';
  const bool fits = 2L * (L.Hin + 3) * (L.Win + 2) * 2 <= 160 * 1024 && n <= 0x7fffffff;
  if (!valu && fits) {
    int rc = 1;
    if (L.NT == 1) rc = launch_conv0m_nt<1, FM, ONES>(L, x, out, w0, n, st, cscale);
    else if (L.NT == 2) rc = launch_conv0m_nt<2, FM, ONES>(L, x, out, w0, n, st, cscale);
    else if (L.NT == 3) rc = launch_conv0m_nt<3, FM, ONES>(L, x, out, w0, n, st, cscale);
    if (rc <= 0) return rc;
  }
  if constexpr (FM == 2) return launch_conv0<_Float16, false, ONES>(L, x, (_Float16*)out, w0, n, st, cscale);
  else return launch_conv0<__bf16, FM == 1, ONES>(L, x, (__bf16*)out, w0, n, st);
}

// the whole-stack kernel (res_bf16n.inc) takes the model: bf16, every layer at
// dilation 1, a zero-padding channel for the folded bias, 2 or 3 out-tiles, a map
// whose image fits its LDS slot, at least one m-tile per wave.  Opt-in
// (HONK_RES_KERNEL=n): on res8 it measured 0.50 ms per 4096-clip launch against the
// row-band kernel's 0.45 ms for the same six layers, so the default stays.
static bool use_n_kernel(const Layout& L, const honk_res_desc* d, int FM) {
  const char* e = getenv("HONK_RES_KERNEL");
  if (!e || e[0] != 'n') return false;
  if (FM != 0 || L.L < 1 || L.C >= L.CP || (L.NT != 2 && L.NT != 3)) return false;
  for (int i = 1; i <= L.L; ++i)
    if (dil_of(d, i) != 1) return false;
  if (!g16n_fits(L.NT, L.H, L.W)) return false;
  return (L.H * L.W + 15) / 16 >= 4;
}

template <int NT>
static int launch_block16n(const Layout& L, const __bf16* in, const float* frb, size_t frl, float* chsum, int64_t n,
                           hipStream_t st) {
  Block16NArgs a;
  a.in = in;
  a.wfrag = (const char*)frb;
  a.wstride = (int)(frl * sizeof(float));
  a.chsum = chsum;
  a.nclips = (int)n;
  a.H = L.H;
  a.W = L.W;
  a.nL = L.L;
  int grid = cu_count();
  if (grid > n) grid = (int)n;
  TimedLaunch tl(st, 2.0 * L.H * L.W * L.C * L.C * 9 * L.L * (double)n);
  hipLaunchKernelGGL((block16n_kernel<NT>), dim3(grid), dim3(256), 0, st, a);
  HONK_LAUNCH_CHECK("res block16n_kernel");
  tl.done(st);
  return HONK_OK;
}

// bf16 driver: same schedule as the fp32 one (R / X0 / X1 buffers, fused mean)
// bf16 schedule: activations stay pre-BN (see res_bf16.inc), so one residual
// stream R (conv0 output, then every even layer's sum, in place) and one odd-layer
// buffer X suffice; each layer writes exactly one tensor.
// res_vf.hip (compiled with its own flags): the pair and last-layer launches
bool launch_pair_vf(int FM, int ppr, bool imm, int dA, int dB, dim3 gd, dim3 bd, hipStream_t st,
                    const Block16PArgs& pa);
void launch_last_vf(int FM, int d, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa);
void launch_pair2t_vf(int ppr, bool lin, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa);
bool launch_pair2i_vf(int dA, int dB, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa);
bool launch_pairk_vf(int dA, int dB, dim3 gd, dim3 bd, hipStream_t st, const Block16PArgs& pa);

// flags (f16x2 only, may be null): [batch] the clips' admission flags (clip_scale_kernel,
// tail_sum_kernel; honk_res_forward re-runs the flagged clips)
static int forward_bf16(const Layout& L, const honk_res_desc* d, const float* packed, const float* x,
                        float* logits, int64_t batch, int64_t chunk, void* workspace, hipStream_t st,
                        int* flags = nullptr) {
  const int FM = fmt_of(L.prec);  // operand format (res_bf16w.inc)
  const int SP = sp_of(FM);       // 16-bit elements per channel value
  const size_t act = (size_t)chunk * L.H * L.W * L.CP * SP;
  // this format's packed weight fragments (per layer)
  const float* frb = FM == 1 ? packed + L.off_fragx3 : FM == 2 ? packed + L.off_fragh : packed + L.off_frag16;
  const size_t frl = FM == 0 ? L.frag16_floats : L.fragx3_floats;
  __bf16* R = (__bf16*)workspace;
  __bf16* X = R + act;
  float* cscale = (float*)(R + 2 * act);  // [chunk] the f16x2 clip scales (clip_scale_kernel)
  float* chsum = cscale + round64((size_t)chunk);
  const float* tail_cs = FM == 2 ? cscale : nullptr;
  const PlanR pr = plan_block16r(L, SP);
  const double layer_flop_per_clip = 2.0 * L.H * L.W * L.C * L.C * 9;
  if (L.L == 0) return fail(HONK_ERR_UNSUPPORTED, "bf16 path needs n_layers >= 1");
  if (pr.TH == 0)
    return fail(HONK_ERR_UNSUPPORTED, "bf16/bf16x3: feature-map width %d exceeds the row-band staging plan "
                "(use precision f32)", L.W);
  int rc;
  if (use_n_kernel(L, d, FM)) {
    // conv0 -> R, then the whole block stack per clip in LDS, then the head
    for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
      const int64_t n = (batch - c0 < chunk) ? batch - c0 : chunk;
      rc = launch_conv0_16<0, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);
      if (rc) return rc;
      rc = L.NT == 3 ? launch_block16n<3>(L, R, frb, frl, chsum, n, st) : launch_block16n<2>(L, R, frb, frl, chsum, n, st);
      if (rc) return rc;
      const float* bn_last = packed + L.off_bn + (size_t)2 * L.CP * (L.L - 1);
      hipLaunchKernelGGL(tail_sum_kernel, dim3((unsigned)n), dim3(256), 0, st, chsum, packed + L.off_wout,
                         packed + L.off_bout, logits + c0 * L.NL, 4, L.H * L.W, L.C, L.CP, L.NL, bn_last,
                         bn_last + L.CP, tail_cs, packed + L.off_range + HONK_NUM_OUT_SCALE, (int*)nullptr, 0.f);
      HONK_LAUNCH_CHECK("res tail_sum_kernel (whole stack)");
    }
    return HONK_OK;
  }
  const bool wpath = use_w_kernel(L, d, FM);
  if (!wpath && FM == 2)
    return fail(HONK_ERR_UNSUPPORTED, "f16x2 runs on the weight-stationary / pair kernels only: %d maps, %dx%d "
                "(pooled) map, pool %dx%d is outside their envelope (use precision f32 or bf16x3)", L.C, L.H, L.W,
                L.ph, L.pw);
  if (wpath) {
    // weight-stationary kernel: tiles = (clip, dilation class, band of TH class rows), TH per dilation
    int parts_last = 0;  // channel-sum partials per clip of the last layer
    for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
      const int64_t n = (batch - c0 < chunk) ? batch - c0 : chunk;
      if (FM == 2) {
        hipLaunchKernelGGL(clip_scale_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, st, x + c0 * L.Hin * L.Win,
                           packed + L.off_range, cscale, (int)n, L.Hin * L.Win, flags ? flags + c0 : nullptr);
        HONK_LAUNCH_CHECK("res clip_scale_kernel");
      }
      rc = (FM == 1) ? launch_conv0_16<1, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st)
           : (FM == 2) ? launch_conv0_16<2, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st, cscale)
                       : launch_conv0_16<0, true>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);
      if (rc) return rc;
      int grid = cu_count();
      if (grid > n) grid = (int)n;
      bool last_stored = false;  // the last layer ran as a pair's B layer (tail_act_kernel sums it)
      for (int i = 1; i <= L.L; ++i) {
        const bool even = (i % 2) == 0;
        {
          const PairPlan pp = pair_at(L, d, FM, n, grid, i);
          if (pp.ok) {
            if (i + 1 == L.L) last_stored = true;
            const int dA = dil_of(d, i);
            const size_t cb = (size_t)n * L.H * L.W * L.CP * 2 * SP;
            Block16PArgs pa;
            pa.R = R;
            pa.chsum = nullptr;
            pa.wA = (const char*)(frb + (size_t)(i - 1) * frl);
            pa.wB = (const char*)(frb + (size_t)i * frl);
            pa.chunk_bytes = (unsigned)cb;
            pa.nclips = (int)n;
            pa.H = L.H;
            pa.W = L.W;
            pa.d = dA;
            pa.lgd = 0;
            while ((1 << pa.lgd) < dA) ++pa.lgd;
            pa.sB = dil_of(d, i + 1) == dA ? 1 : 2;
            pa.lag = pp.lag;
            pa.NRA = pp.NRA;
            pa.NRB = pp.NRB;
            pa.slotb = pp.slotb;
            pa.ppr = pp.ppr;
            pa.padb = pp.padb;
            pa.ringpad = pp.ringpad;
            TimedLaunch tl(st, 2.0 * layer_flop_per_clip * (double)n);
            const dim3 gd(grid), bd(256 * pp.ns * pp.ks);
            if (pp.ks == 2) {
              if (!launch_pairk_vf(dA, dil_of(d, i + 1), gd, bd, st, pa))
                return fail(HONK_ERR_UNSUPPORTED, "block16k: no instance for dilations %d, %d", dA, dil_of(d, i + 1));
            } else if (FM == 0 && pp.ns == 2 && pp.padb > 0) {
              if (!launch_pair2i_vf(dA, dil_of(d, i + 1), gd, bd, st, pa))
                return fail(HONK_ERR_UNSUPPORTED, "block16p: no two-stream tap-step instance for dilations %d, %d", dA,
                            dil_of(d, i + 1));
            } else if (FM == 0 && pp.ns == 2) launch_pair2t_vf(pp.ppr, pp.lin, gd, bd, st, pa);
            else if (!launch_pair_vf(FM, pp.ppr, pp.ppr == 4 && pp.padb > 0, dA, dil_of(d, i + 1), gd, bd, st, pa))
              return fail(HONK_ERR_UNSUPPORTED, "block16p: no tap-step instance for dilations %d, %d", dA,
                          dil_of(d, i + 1));
            HONK_LAUNCH_CHECK("res block16p_kernel");
            tl.done(st);
            ++i;  // layer i + 1 done too
            continue;
          }
          const PairPlan lp = last_at(L, d, FM, i);
          if (lp.ok) {
            Block16PArgs pa;
            pa.R = R;  // the last (odd) layer reads R
            pa.wA = pa.wB = (const char*)(frb + (size_t)(i - 1) * frl);
            pa.chunk_bytes = (unsigned)((size_t)n * L.H * L.W * L.CP * 2 * SP);
            pa.nclips = (int)n;
            pa.H = L.H;
            pa.W = L.W;
            pa.d = dil_of(d, i);
            pa.lgd = 0;
            while ((1 << pa.lgd) < pa.d) ++pa.lgd;
            pa.sB = 1;
            pa.lag = 0;
            pa.NRA = lp.NRA;
            pa.NRB = lp.NRB;
            pa.slotb = lp.slotb;
            pa.ppr = lp.ppr;
            pa.padb = lp.padb;
            pa.ringpad = lp.ringpad;
            pa.chsum = chsum;
            TimedLaunch tl(st, layer_flop_per_clip * (double)n);
            const dim3 gd(grid), bd(128 * lp.ns);
            launch_last_vf(FM, pa.d, gd, bd, st, pa);
            HONK_LAUNCH_CHECK("res block16l_kernel");
            tl.done(st);
            parts_last = 2;
            continue;
          }
        }
        Block16WArgs a;
        a.in = even ? X : R;
        a.res = even ? R : nullptr;
        a.out = (i == L.L) ? nullptr : (even ? R : X);
        a.wfrag = (const char*)(frb + (size_t)(i - 1) * frl);
        a.chsum = (i == L.L) ? chsum : nullptr;
        a.H = L.H;
        a.W = L.W;
        a.dil = dil_of(d, i);
        a.TH = plan_w_th(L, FM, a.dil);
        const BandGeo bg = band_geo(L.H, a.dil, a.TH);
        a.nbc = bg.nbc;
        a.rem = bg.rem;
        a.nb1 = bg.nb1;
        a.nb0 = bg.nb0;
        a.lgd = 0;
        while ((1 << a.lgd) < a.dil) ++a.lgd;
        if ((int64_t)n * a.nbc > 0x7fffffff) return fail(HONK_ERR_ARG, "chunk too large");
        a.ntiles = (int)(n * a.nbc);
        if (i == L.L) parts_last = a.nbc * 4;
        TimedLaunch tl(st, layer_flop_per_clip * (double)n);
        rc = dispatch_block16w(L.NT, FM, a, st);
        tl.done(st);
        if (rc) return rc;
      }
      const float* bn_last = packed + L.off_bn + (size_t)2 * L.CP * (L.L - 1);
      if (last_stored) {
        // the last layer was a pair's B layer (bf16): it stored its output in R
        if (L.CP != 48 || SP != 1) return fail(HONK_ERR_UNSUPPORTED, "tail_act_kernel: 48 bf16 channels only");
        hipLaunchKernelGGL(tail_act_kernel, dim3((unsigned)n), dim3(256), 0, st, R, packed + L.off_wout,
                           packed + L.off_bout, logits + c0 * L.NL, L.H * L.W, L.C, L.NL, bn_last, bn_last + L.CP);
        HONK_LAUNCH_CHECK("res tail_act_kernel");
        continue;
      }
      hipLaunchKernelGGL(tail_sum_kernel, dim3((unsigned)n), dim3(256), 0, st, chsum, packed + L.off_wout,
                         packed + L.off_bout, logits + c0 * L.NL, parts_last, L.H * L.W, L.C, L.CP, L.NL,
                         bn_last, bn_last + L.CP, tail_cs, packed + L.off_range + HONK_NUM_OUT_SCALE,
                         flags ? flags + c0 : nullptr, (float)HONK_F16X2_Z_MAX);
      HONK_LAUNCH_CHECK("res tail_sum_kernel (weight-stationary)");
    }
    return HONK_OK;
  }
  {
    // row-band kernel: tiles = (clip, dilation class, band of TH class rows)
    int nbc_last = 0;
    for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
      const int64_t n = (batch - c0 < chunk) ? batch - c0 : chunk;
      rc = (SP == 2) ? launch_conv0_16<1, false>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st)
                     : launch_conv0_16<0, false>(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);
      if (rc) return rc;
      for (int i = 1; i <= L.L; ++i) {
        const bool even = (i % 2) == 0;
        Block16RArgs a;
        a.in = even ? X : R;
        a.res = even ? R : nullptr;
        a.out = (i == L.L) ? nullptr : (even ? R : X);
        a.bfrag = (const uint4*)(SP == 2 ? packed + L.off_fragx3 + (size_t)(i - 1) * L.fragx3_floats
                                         : packed + L.off_frag16 + (size_t)(i - 1) * L.frag16_floats);
        a.bias = packed + L.off_bias16 + (size_t)16 * L.CP * (i - 1);
        a.chsum = (i == L.L) ? chsum : nullptr;
        a.H = L.H;
        a.W = L.W;
        a.dil = d->use_dilation ? (1 << ((i - 1) / 3)) : 1;
        a.TH = pr.TH;
        const BandGeo bg = band_geo(L.H, a.dil, pr.TH);
        a.nbc = bg.nbc;
        a.rem = bg.rem;
        a.nb1 = bg.nb1;
        a.nb0 = bg.nb0;
        if ((int64_t)n * a.nbc > 0x7fffffff) return fail(HONK_ERR_ARG, "chunk too large");
        a.ntiles = (int)(n * a.nbc);
        if (i == L.L) nbc_last = a.nbc;
        TimedLaunch tl(st, layer_flop_per_clip * (double)n);
        rc = dispatch_block16r(pr, SP, a, st);
        tl.done(st);
        if (rc) return rc;
      }
      const float* bn_last = packed + L.off_bn + (size_t)2 * L.CP * (L.L - 1);
      hipLaunchKernelGGL(tail_sum_kernel, dim3((unsigned)n), dim3(256), 0, st, chsum, packed + L.off_wout,
                         packed + L.off_bout, logits + c0 * L.NL, nbc_last * 8 * pr.MT, L.H * L.W, L.C, L.CP, L.NL,
                         bn_last, bn_last + L.CP, tail_cs, packed + L.off_range + HONK_NUM_OUT_SCALE, (int*)nullptr, 0.f);
      HONK_LAUNCH_CHECK("res tail_sum_kernel (bf16 row-band)");
    }
    return HONK_OK;
  }
}

#endif  // HONK_RES_VF_TU
}  // namespace res
}  // namespace honk
#ifndef HONK_RES_VF_TU

using namespace honk;
using namespace honk::res;

extern "C" {

size_t honk_res_packed_floats(const honk_res_desc* d) {
  Layout L;
  if (make_layout(d, &L) != HONK_OK) return 0;
  return L.total;
}

int honk_res_launch_plan(const honk_res_desc* d, int64_t batch, int32_t n_cus, int32_t* kinds, int32_t max_kinds) {
  Layout L;
  int rc = make_layout(d, &L);
  if (rc) return rc;
  if (batch < 1) return fail(HONK_ERR_ARG, "batch < 1");
  const int64_t n = chunk_clips(L, batch);
  int grid = n_cus > 0 ? n_cus : cu_count();
  if (grid > n) grid = (int)n;
  int cnt = 0;
  auto put = [&](int k) {
    if (kinds && cnt < max_kinds) kinds[cnt] = k;
    ++cnt;
  };
  if (L.prec == HONK_PREC_F32) {
    for (int i = 1; i <= L.L; ++i) put(HONK_KERNEL_BLOCK_F32);
    return cnt;
  }
  const int FM = fmt_of(L.prec), SP = sp_of(FM);
  if (plan_block16r(L, SP).TH == 0) return fail(HONK_ERR_UNSUPPORTED, "width beyond the row-band staging plan");
  if (use_n_kernel(L, d, FM)) {
    put(HONK_KERNEL_NET);
    return cnt;
  }
  if (!use_w_kernel(L, d, FM)) {
    if (FM == 2) return fail(HONK_ERR_UNSUPPORTED, "f16x2: outside the weight-stationary / pair kernels' envelope");
    for (int i = 1; i <= L.L; ++i) put(HONK_KERNEL_ROWBAND);
    return cnt;
  }
  for (int i = 1; i <= L.L; ++i) {
    const PairPlan pp = pair_at(L, d, FM, n, grid, i);
    if (pp.ok) {
      put(pp.ks == 2 ? HONK_KERNEL_PAIR_KS : HONK_KERNEL_PAIR);
      ++i;
    } else if (last_at(L, d, FM, i).ok) {
      put(HONK_KERNEL_LAST);
    } else {
      put(HONK_KERNEL_WSTAT);
    }
  }
  return cnt;
}

}  // extern "C"

// honk_res_workspace_bytes without the f16x2 admission's regions (below)
static size_t ws_bytes_plain(const honk_res_desc* d, int64_t batch) {
  Layout L;
  if (make_layout(d, &L) != HONK_OK || batch < 1) return 0;
  const int64_t ch = chunk_clips(L, batch);
  if (L.prec != HONK_PREC_F32) {
    const int FM = fmt_of(L.prec), SP = sp_of(FM);
    if (L.L < 1) {
      fail(HONK_ERR_UNSUPPORTED, "bf16 / bf16x3 / f16x2 need n_layers >= 1 (use precision f32)");
      return 0;
    }
    if (L.ph * L.pw > 1 && !((L.ph == 2 && L.pw == 2) || (L.ph == 4 && L.pw == 3))) {
      fail(HONK_ERR_UNSUPPORTED, "bf16 / bf16x3 / f16x2: avg-pool %dx%d has no conv0 kernel (1x1, 2x2, 4x3; "
           "use precision f32)", L.ph, L.pw);
      return 0;
    }
    const PlanR pr = plan_block16r(L, SP);
    if (pr.TH == 0) {
      fail(HONK_ERR_UNSUPPORTED, "bf16/bf16x3: feature-map width %d exceeds the row-band staging plan "
           "(use precision f32)", L.W);
      return 0;
    }
    const bool wpath = L.L > 0 && use_w_kernel(L, d, FM);
    if (FM == 2 && !wpath) {
      fail(HONK_ERR_UNSUPPORTED, "f16x2 runs on the weight-stationary / pair kernels only: %d maps, %dx%d (pooled) "
           "map, pool %dx%d is outside their envelope (use precision f32 or bf16x3)", L.C, L.H, L.W, L.ph, L.pw);
      return 0;
    }
    const int nb = max_bands_per_clip(L, pr.TH, d->use_dilation);
    size_t parts = (size_t)nb * 8 * pr.MT;  // row-band kernel: [tile][wave][m-tile] channel sums
    if (wpath) {
      const size_t pw = (size_t)bands_w(L, d, FM, L.L) * 4;  // weight-stationary: [tile][wave]
      if (pw > parts) parts = pw;
    }
    // R, X, the clip scales, the channel-sum partials (forward_bf16)
    return (size_t)2 * ch * L.H * L.W * L.CP * 2 * SP + round64((size_t)ch) * sizeof(float) +
           (size_t)ch * parts * L.CP * sizeof(float);
  }
  const Plan p = plan_block(L);
  return (size_t)3 * ch * L.H * L.W * L.CP * sizeof(float) + (size_t)ch * p.nbands * MW * L.CP * sizeof(float);
}

// The f16x2 admission (HONK_PREC_F16X2, unless HONK_F16X2_RERUN=0): after the f16x2
// pass, the clips tail_sum_kernel flagged are re-run in bf16x3, RC at a time, in the
// f16x2 pass's (then free) activation region.  Workspace: [main | flags[batch] |
// list[batch] | count | gathered inputs [RC] | re-run logits [RC]].
struct F16Check {
  int64_t rc;
  size_t main, flags, list, count, gx, glog, total;
};
static bool f16x2_rerun_on() {
  const char* e = getenv("HONK_F16X2_RERUN");
  return !(e && e[0] == '0');
}
static honk_res_desc rerun_desc(const honk_res_desc* d) {
  honk_res_desc e = *d;
  e.precision = HONK_PREC_BF16X3;
  return e;
}
static bool f16_check_plan(const honk_res_desc* d, int64_t batch, F16Check* p) {
  Layout L;
  if (make_layout(d, &L) != HONK_OK || batch < 1) return false;
  const size_t f16 = ws_bytes_plain(d, batch);
  const honk_res_desc e = rerun_desc(d);
  if (f16 == 0) return false;
  int64_t rc = chunk_clips(L, batch) / 2;
  if (rc < 1) rc = 1;
  while (rc > 1 && ws_bytes_plain(&e, rc) > f16) rc /= 2;
  const size_t r = ws_bytes_plain(&e, rc);
  if (r == 0) {
    fail(HONK_ERR_UNSUPPORTED, "f16x2 admission: the bf16x3 re-run does not take this shape");
    return false;
  }
  auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
  p->rc = rc;
  p->main = up(f16 > r ? f16 : r);
  p->flags = p->main;
  p->list = p->flags + up((size_t)batch * sizeof(int));
  p->count = p->list + up((size_t)batch * sizeof(int));
  p->gx = p->count + 256;
  p->glog = p->gx + up((size_t)rc * L.Hin * L.Win * sizeof(float));
  p->total = p->glog + up((size_t)rc * L.NL * sizeof(float));
  return true;
}

static thread_local int64_t g_rerun = 0;

extern "C" {

size_t honk_res_workspace_bytes(const honk_res_desc* d, int64_t batch) {
  if (d && d->precision == HONK_PREC_F16X2 && f16x2_rerun_on()) {
    F16Check p;
    return f16_check_plan(d, batch, &p) ? p.total : 0;
  }
  return ws_bytes_plain(d, batch);
}

int64_t honk_res_rerun_count(void) { return g_rerun; }

int honk_res_pack(const honk_res_desc* d, const float* const* t, int32_t n_tensors, float* packed,
                  void* stream) {
  Layout L;
  int rc = make_layout(d, &L);
  if (rc) return rc;
  if (!t || !packed) return fail(HONK_ERR_ARG, "null tensors/packed");
  if (n_tensors != 3 * L.L + 3)
    return fail(HONK_ERR_ARG, "honk_res_pack expects %d tensors, got %d", 3 * L.L + 3, n_tensors);
  for (int i = 0; i < n_tensors; ++i)
    if (!t[i]) return fail(HONK_ERR_ARG, "tensor %d is null", i);
  hipStream_t st = (hipStream_t)stream;
  float* rec = packed + L.off_range;
  hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, st, (const float*)nullptr, rec, 64);
  hipLaunchKernelGGL(pack_conv0_kernel, dim3(cdiv(L.CP * 9, 256)), dim3(256), 0, st, t[0],
                     packed + L.off_conv0, L.C, L.CP);
  HONK_LAUNCH_CHECK("pack_conv0");
  const int nfrag = (int)L.layer_floats;
  // pass 1: the fp32 fragments and every layer's BatchNorm (scale, shift)
  for (int i = 0; i < L.L; ++i) {
    hipLaunchKernelGGL(pack_block_kernel, dim3(cdiv(nfrag, 256)), dim3(256), 0, st, t[1 + i],
                       packed + L.off_layers + (size_t)i * L.layer_floats, L.C, L.NT);
    HONK_LAUNCH_CHECK("pack_block");
    float* sc = packed + L.off_bn + (size_t)2 * L.CP * i;
    hipLaunchKernelGGL(pack_bn_kernel, dim3(1), dim3(64), 0, st, t[1 + L.L + 2 * i],
                       t[1 + L.L + 2 * i + 1], sc, sc + L.CP, L.C, L.CP);
    HONK_LAUNCH_CHECK("pack_bn");
  }
  // the numerics record: f16x2 scales, fitness, the per-layer weight exponents
  hipLaunchKernelGGL(pack_range_kernel, dim3(1), dim3(256), 0, st, rec, packed + L.off_bn, packed + L.off_conv0,
                     packed + L.off_layers, L.layer_floats, L.C, L.CP, L.NT, L.L);
  HONK_LAUNCH_CHECK("pack_range");
  // pass 2: the bf16-pipe fragments with the input BatchNorm folded in
  for (int i = 0; i < L.L; ++i) {
    // the input BatchNorm (layer i-1's; none for layer 1) folded into the weights and
    // the border-class bias
    const float* in_bn = (i > 0) ? packed + L.off_bn + (size_t)2 * L.CP * (i - 1) : nullptr;
    const int n16 = ((18 * L.NT + 3) / 4) * L.NT * 64 * 8;
    const float* in_shift = in_bn ? in_bn + L.CP : nullptr;
    const int odd = ((i + 1) & 1);  // layer i + 1 (1-based) is odd
    hipLaunchKernelGGL(pack_block16_kernel, dim3(cdiv(n16, 256)), dim3(256), 0, st, t[1 + i], in_bn, in_shift, odd,
                       (unsigned short*)(packed + L.off_frag16 + (size_t)i * L.frag16_floats), L.C, L.NT, 1, 0,
                       (float*)nullptr, (const float*)nullptr);
    hipLaunchKernelGGL(pack_block16_kernel, dim3(cdiv(n16, 256)), dim3(256), 0, st, t[1 + i], in_bn, in_shift, odd,
                       (unsigned short*)(packed + L.off_fragx3 + (size_t)i * L.fragx3_floats), L.C, L.NT, 2, 0,
                       (float*)nullptr, (const float*)nullptr);
    hipLaunchKernelGGL(pack_block16_kernel, dim3(cdiv(n16, 256)), dim3(256), 0, st, t[1 + i], in_bn, in_shift, odd,
                       (unsigned short*)(packed + L.off_fragh + (size_t)i * L.fragx3_floats), L.C, L.NT, 2, 1,
                       rec + HONK_NUM_F16_OVERFLOW, (const float*)(rec + HONK_NUM_KW + i));
    HONK_LAUNCH_CHECK("pack_block16");
    hipLaunchKernelGGL(pack_bias16_kernel, dim3(cdiv(16 * L.CP, 256)), dim3(256), 0, st, t[1 + i],
                       in_shift, packed + L.off_bias16 + (size_t)16 * L.CP * i, L.C, L.CP);
    HONK_LAUNCH_CHECK("pack_bias16");
  }
  const int nw = L.NL * L.C;
  hipLaunchKernelGGL(copy_kernel, dim3(cdiv(nw, 256)), dim3(256), 0, st, t[1 + 3 * L.L],
                     packed + L.off_wout, nw);
  hipLaunchKernelGGL(copy_kernel, dim3(cdiv(L.NL, 256)), dim3(256), 0, st, t[2 + 3 * L.L],
                     packed + L.off_bout, L.NL);
  hipLaunchKernelGGL(copy_kernel, dim3(1), dim3(64), 0, st, (const float*)nullptr,
                     packed + L.off_zeros, 64);
  HONK_LAUNCH_CHECK("pack_copy");
  return HONK_OK;
}

int honk_res_numerics(const honk_res_desc* d, const float* packed, float* rec, int32_t n, void* stream) {
  Layout L;
  int rc = make_layout(d, &L);
  if (rc) return rc;
  if (!packed || !rec || n < 1) return fail(HONK_ERR_ARG, "null packed / rec or n < 1");
  if (n > HONK_NUM_KW + L.L) n = HONK_NUM_KW + L.L;
  hipStream_t st = (hipStream_t)stream;
  HONK_HIP_CHECK(hipMemcpyAsync(rec, packed + L.off_range, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, st));
  HONK_HIP_CHECK(hipStreamSynchronize(st));
  return HONK_OK;
}

// The precision policy (host-only).  "Supported" = the packed forward takes the
// descriptor in that precision (honk_res_workspace_bytes != 0).
//  * F32 -> F32.  BF16 (top-1 parity, an explicit choice) -> BF16 where supported.
//  * F16X2 / AUTO -> F16X2 where its 1e-4 contract holds: the res15 map class (an
//    unpooled map of >= 4040 pixels -- the spatial mean averages the fp16 rounding --
//    and >= 32 maps), no folded weight beyond fp16's range, rho <= HONK_F16X2_RHO_MAX;
//    otherwise the BF16X3 rule.
//  * BF16X3 -> BF16X3 where supported and rho <= HONK_BF16X3_RHO_MAX, else F32.
// The rho bounds: exp/f16_range_sim.py (float64 simulation of the kernels' roundings):
// f16x2 on res15 stays <= 6.4e-5 up to rho 4.9 and failed the bar only at rho >= 5.1
// (8.4e-5 .. 1.6e-3); bf16x3 carries ~2^5 more significant bits per activation.
#define HONK_F16X2_RHO_MAX 3.5f
#define HONK_BF16X3_RHO_MAX 100.f
static bool prec_supported(const honk_res_desc* d, int p) {
  honk_res_desc e = *d;
  e.precision = p;
  const std::string keep = get_error();
  const bool ok = honk_res_workspace_bytes(&e, 1) != 0 && honk_res_packed_floats(&e) != 0;
  set_error("%s", keep.c_str());
  return ok;
}
int honk_res_select_precision(const honk_res_desc* d, const float* rec, int32_t requested, char* note,
                              size_t note_len) {
  Layout L;
  honk_res_desc e = *d;
  e.precision = HONK_PREC_F32;
  int rc = make_layout(&e, &L);
  if (rc) return rc;
  char buf[256];
  buf[0] = 0;
  auto done = [&](int p) {
    if (note && note_len) snprintf(note, note_len, "%s", buf);
    return p;
  };
  if (requested == HONK_PREC_F32) return done(HONK_PREC_F32);
  if (requested == HONK_PREC_BF16) {
    if (prec_supported(d, HONK_PREC_BF16)) return done(HONK_PREC_BF16);
    snprintf(buf, sizeof buf, "bf16 does not take this shape (%s)", get_error());
    return done(HONK_PREC_F32);
  }
  if (requested != HONK_PREC_F16X2 && requested != HONK_PREC_BF16X3 && requested != HONK_PREC_AUTO)
    return fail(HONK_ERR_ARG, "unknown precision %d", requested);
  if (!rec || rec[HONK_NUM_VALID] != 1.f) return fail(HONK_ERR_ARG, "no numerics record (honk_res_numerics)");
  const float rho = rec[HONK_NUM_RHO];
  if (requested != HONK_PREC_BF16X3) {
    const char* why = nullptr;
    if (!prec_supported(d, HONK_PREC_F16X2)) why = "outside the f16x2 kernels' envelope";
    else if (L.ph * L.pw > 1 || L.H * L.W < 4040 || L.C < 32)
      why = "the 1e-4 contract of f16x2 covers unpooled maps of >= 4040 pixels and >= 32 feature maps (res15)";
    else if (rec[HONK_NUM_F16_OVERFLOW] != 0.f) why = "a folded weight is beyond fp16's range";
    else if (!(rho <= HONK_F16X2_RHO_MAX)) why = "the stored tensors' mean-to-spread ratio rho exceeds f16x2's bound";
    if (!why) return done(HONK_PREC_F16X2);
    snprintf(buf, sizeof buf, "f16x2 not taken: %s (rho %.3g, bound %.3g)", why, (double)rho,
             (double)HONK_F16X2_RHO_MAX);
  }
  if (prec_supported(d, HONK_PREC_BF16X3) && rho <= HONK_BF16X3_RHO_MAX) return done(HONK_PREC_BF16X3);
  const size_t k = strlen(buf);
  snprintf(buf + k, sizeof buf - k, "%sbf16x3 not taken (rho %.3g, bound %.3g, %s)", k ? "; " : "", (double)rho,
           (double)HONK_BF16X3_RHO_MAX, prec_supported(d, HONK_PREC_BF16X3) ? "supported" : "unsupported shape");
  return done(HONK_PREC_F32);
}

int honk_res_forward(const honk_res_desc* d, const float* packed, const float* x, float* logits,
                     int64_t batch, void* workspace, size_t ws_bytes, void* stream) {
  Layout L;
  int rc = make_layout(d, &L);
  if (rc) return rc;
  if (batch < 0) return fail(HONK_ERR_ARG, "negative batch");
  if (batch == 0) return HONK_OK;
  if (!packed || !x || !logits || !workspace) return fail(HONK_ERR_ARG, "null pointer argument");
  const size_t need = honk_res_workspace_bytes(d, batch);
  if (ws_bytes < need)
    return fail(HONK_ERR_WORKSPACE, "workspace %zu B < required %zu B", ws_bytes, need);
  hipStream_t st = (hipStream_t)stream;
  const int64_t chunk = chunk_clips(L, batch);
  g_rerun = 0;
  if (L.prec == HONK_PREC_F16X2 && f16x2_rerun_on()) {
    if (batch > 0x7fffffff) return fail(HONK_ERR_ARG, "f16x2: batch beyond 2^31 clips");
    F16Check p;
    if (!f16_check_plan(d, batch, &p)) return fail(HONK_ERR_UNSUPPORTED, "%s", get_error());
    char* ws = (char*)workspace;
    int* flags = (int*)(ws + p.flags);
    int* list = (int*)(ws + p.list);
    int* count = (int*)(ws + p.count);
    rc = forward_bf16(L, d, packed, x, logits, batch, chunk, workspace, st, flags);
    if (rc) return rc;
    hipLaunchKernelGGL(flag_compact_kernel, dim3(1), dim3(1024), 0, st, flags, batch, list, count);
    HONK_LAUNCH_CHECK("res flag_compact_kernel");
    int flagged = 0;
    HONK_HIP_CHECK(hipMemcpyAsync(&flagged, count, sizeof(int), hipMemcpyDeviceToHost, st));
    HONK_HIP_CHECK(hipStreamSynchronize(st));
    g_rerun = flagged;
    if (flagged == 0) return HONK_OK;
    const honk_res_desc e = rerun_desc(d);
    Layout L3;
    rc = make_layout(&e, &L3);
    if (rc) return rc;
    float* gx = (float*)(ws + p.gx);
    float* glog = (float*)(ws + p.glog);
    for (int64_t o = 0; o < flagged; o += p.rc) {
      const int64_t n = flagged - o < p.rc ? flagged - o : p.rc;
      hipLaunchKernelGGL(gather_clips_kernel, dim3((unsigned)n), dim3(256), 0, st, x, list + o, L.Hin * L.Win, gx);
      HONK_LAUNCH_CHECK("res gather_clips_kernel");
      rc = forward_bf16(L3, &e, packed, gx, glog, n, chunk_clips(L3, n), workspace, st);
      if (rc) return rc;
      hipLaunchKernelGGL(scatter_logits_kernel, dim3((unsigned)cdiv(n * L.NL, 64)), dim3(64), 0, st, glog, list + o,
                         (int)n, L.NL, logits);
      HONK_LAUNCH_CHECK("res scatter_logits_kernel");
    }
    return HONK_OK;
  }
  if (L.prec != HONK_PREC_F32) return forward_bf16(L, d, packed, x, logits, batch, chunk, workspace, st);
  const size_t act = (size_t)chunk * L.H * L.W * L.CP;
  float* R = (float*)workspace;
  float* X[2] = {R + act, R + 2 * act};
  float* chsum = R + 3 * act;  // [chunk][nbands][MW][CP] fused-mean partial sums
  const Plan p = plan_block(L);
  const double layer_flop_per_clip = 2.0 * L.H * L.W * L.C * L.C * 9;

  for (int64_t c0 = 0; c0 < batch; c0 += chunk) {
    const int64_t n = (batch - c0 < chunk) ? batch - c0 : chunk;
    if ((int64_t)n * p.nbands > 0x7fffffff) return fail(HONK_ERR_ARG, "chunk too large");
    rc = launch_conv0(L, x + c0 * L.Hin * L.Win, R, packed + L.off_conv0, n, st);
    if (rc) return rc;
    for (int i = 1; i <= L.L; ++i) {
      BlockArgs a;
      a.in = (i == 1) ? R : X[i & 1];
      const bool even = (i % 2) == 0;
      a.res = even ? R : nullptr;
      a.out_pre = even ? R : nullptr;
      a.out_bn = X[(i + 1) & 1];
      a.wfrag = packed + L.off_layers + (size_t)(i - 1) * L.layer_floats;
      a.bn_scale = packed + L.off_bn + (size_t)2 * L.CP * (i - 1);
      a.bn_shift = a.bn_scale + L.CP;
      a.H = L.H;
      a.W = L.W;
      a.dil = d->use_dilation ? (1 << ((i - 1) / 3)) : 1;
      a.TH = p.TH;
      a.nbands = p.nbands;
      a.ntiles = (int)(n * p.nbands);
      a.chsum = (i == L.L) ? chsum : nullptr;  // last layer: fused spatial mean, no stores
      if (i == L.L) a.out_pre = nullptr;
      TimedLaunch tl(st, layer_flop_per_clip * (double)n);
      rc = dispatch_block(p, a, st);
      tl.done(st);
      if (rc) return rc;
    }
    if (L.L == 0) {  // no block layer: mean of the conv0 output
      hipLaunchKernelGGL(tail_kernel, dim3((unsigned)n), dim3(L.CP * (256 / L.CP)), 0, st, R,
                         packed + L.off_wout, packed + L.off_bout, logits + c0 * L.NL, L.H * L.W, L.C,
                         L.CP, L.NL);
      HONK_LAUNCH_CHECK("res tail_kernel");
    } else {
      hipLaunchKernelGGL(tail_sum_kernel, dim3((unsigned)n), dim3(256), 0, st, chsum, packed + L.off_wout,
                         packed + L.off_bout, logits + c0 * L.NL, p.nbands * MW, L.H * L.W, L.C, L.CP, L.NL,
                         (const float*)nullptr, (const float*)nullptr, (const float*)nullptr,
                         (const float*)nullptr, (int*)nullptr, 0.f);
      HONK_LAUNCH_CHECK("res tail_sum_kernel");
    }
  }
  return HONK_OK;
}

}  // extern "C"
#endif  // HONK_RES_VF_TU
