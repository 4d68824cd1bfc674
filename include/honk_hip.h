/*
 * honk_hip.h -- C ABI of libhonk_hip.so, the MI355X (gfx950) forward path of
 * Honk's keyword-spotting CNNs.
 *
 * The reference (ljj7975/honk) is pure PyTorch; its "FFI" for this path is the
 * nn.Module call made by its callers.  Each entry point below replaces one
 * reference interface:
 *
 *   honk_res_forward  <- SpeechResModel.forward   /root/reference/utils/model.py:104-121
 *   honk_cnn_forward  <- SpeechModel.forward      /root/reference/utils/model.py:186-205
 *   honk_res_pack     <- SerializableModule.load  /root/reference/utils/model.py:79-80
 *                        (state_dict -> kernel layout, done once per weight change)
 *   honk_*_desc       <- the config dicts          /root/reference/utils/model.py:381-414
 *
 * Conventions: every pointer named x/logits/packed/tensors[i]/workspace is a
 * DEVICE pointer (hipMalloc / torch caching allocator); `stream` is a
 * hipStream_t passed as void*.  Work is enqueued on `stream`; no call
 * synchronises or allocates device memory.  Global state: a thread-local
 * last-error string, a per-device CU-count cache, and the mutex-guarded
 * timing window of honk_timing_enable/read (off unless enabled; a diagnostic,
 * not used by the forward itself).  Status: 0 = ok, <0 = error, see
 * honk_last_error().
 * Arithmetic: fp32 inputs/outputs everywhere; the res and cnn forwards take a
 * precision field (HONK_PREC_F32: IEEE fp32 MFMA; HONK_PREC_BF16X3: fp32 values
 * as bf16 hi + lo pairs, 3 bf16 MFMA products per MAC, fp32 accumulation -- both
 * meet the 1e-4 logit bar; HONK_PREC_BF16: bf16, top-1 parity); every other
 * entry point is IEEE fp32 (MFMA / FMA), the BatchNorm statistics fp64.
 */
#ifndef HONK_HIP_H
#define HONK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HONK_OK 0
#define HONK_ERR_ARG (-1)        /* bad descriptor / shape / null pointer        */
#define HONK_ERR_UNSUPPORTED (-2) /* configuration outside the kernels' envelope */
#define HONK_ERR_WORKSPACE (-3)  /* workspace too small                          */
#define HONK_ERR_HIP (-4)        /* a HIP runtime call failed                    */

/* ---- SpeechResModel (res8/15/26[-narrow]); utils/model.py:82-121 ------------- */
typedef struct honk_res_desc {
  int32_t n_labels;       /* config["n_labels"]                                  */
  int32_t n_maps;         /* config["n_feature_maps"] (1..64 in f32, 1..48 bf16*) */
  int32_t n_layers;       /* config["n_layers"]                                  */
  int32_t use_dilation;   /* config["use_dilation"]: conv{i} dilation 2**((i-1)//3) */
  int32_t pool_h, pool_w; /* config["res_pool"], or 0,0 when absent              */
  int32_t height, width;  /* input frames x MFCC coefficients (101, 40)          */
  int32_t precision;      /* HONK_PREC_F32 (IEEE fp32 MFMA, 1e-4 parity),
                             HONK_PREC_BF16 (bf16 activations/weights, fp32
                             accumulate; top-1 parity) or HONK_PREC_BF16X3
                             (fp32 values as bf16 hi + lo pairs, products
                             hi*hi + hi*lo + lo*hi on bf16 MFMA, fp32
                             accumulate; 1e-4 parity) -- same packed buffer.
                             BF16 / BF16X3: the row-band staging plan bounds
                             the (pooled) width -- 66 for 45-map bf16x3, 154
                             for 45-map bf16 -- HONK_ERR_UNSUPPORTED beyond */
} honk_res_desc;

#define HONK_PREC_F32 0
#define HONK_PREC_BF16 1
#define HONK_PREC_BF16X3 2
/* fp16 activations (RNE), weights (input BN folded) as fp16 hi + lo, products
   w_hi*x + w_lo*x on fp16 MFMA, fp32 accumulate: ~11-bit activations, each clip's
   stored tensors scaled by a power of two that keeps them inside fp16's range (see
   HONK_NUM_SCALE).  Runs on the weight-stationary / pair kernels only (n_maps <= 48
   with a zero-padding channel, (pooled) width < 64; HONK_ERR_UNSUPPORTED otherwise).
   Logit error: within the 1e-4 bar on res15 (simulated <= 3.8e-5, measured on the
   goldens); up to ~2e-4 on the pooled res8 / res26 maps, which average over fewer
   pixels -- honk_res_select_precision routes those to BF16X3. */
#define HONK_PREC_F16X2 3
/* Not a kernel format: honk_res_select_precision's request for "the fastest mode that
   holds the 1e-4 logit bar for this model" (f16x2 -> bf16x3 -> f32). */
#define HONK_PREC_AUTO 4

/* number of floats of the packed (kernel-layout) weight buffer */
size_t honk_res_packed_floats(const honk_res_desc* d);
/* bytes of scratch needed by honk_res_forward for `batch` clips */
size_t honk_res_workspace_bytes(const honk_res_desc* d, int64_t batch);
/*
 * The block-layer launches honk_res_forward makes per batch chunk, in order: kinds[i]
 * = HONK_KERNEL_* (up to max_kinds written).  Returns the launch count (> 0), or a
 * (negative) HONK_ERR_* status code.  n_cus = 0: the current device's CU count (the pair kernel's plan
 * depends on clips per workgroup).  Host-only; no GPU work.
 */
#define HONK_KERNEL_BLOCK_F32 1 /* fp32-MFMA layer (block_kernel)                        */
#define HONK_KERNEL_ROWBAND 2   /* bf16 / bf16x3 row-band layer (block16r_kernel)          */
#define HONK_KERNEL_WSTAT 3     /* bf16 / bf16x3 weight-stationary layer (block16w_kernel) */
#define HONK_KERNEL_PAIR 4      /* fused odd + even layer pair (block16p_kernel)           */
#define HONK_KERNEL_LAST 5      /* last (odd) layer, fused channel sums (block16l_kernel)  */
#define HONK_KERNEL_NET 6       /* every block layer of a clip in LDS (block16n_kernel), bf16 */
#define HONK_KERNEL_PAIR_KS 7   /* f16x2 pair, K split over two waves per SIMD (block16k_kernel) */
int honk_res_launch_plan(const honk_res_desc* d, int64_t batch, int32_t n_cus, int32_t* kinds, int32_t max_kinds);
/*
 * Pack a state_dict into kernel layout.  tensors[] (device, fp32, contiguous),
 * in this order (n_tensors = 3*n_layers + 3):
 *   conv0.weight [C,1,3,3], conv1.weight .. conv{L}.weight [C,C,3,3],
 *   bn1.running_mean, bn1.running_var, .., bn{L}.running_mean, bn{L}.running_var [C],
 *   output.weight [n_labels,C], output.bias [n_labels]
 */
int honk_res_pack(const honk_res_desc* d, const float* const* tensors, int32_t n_tensors,
                  float* packed, void* stream);
/*
 * The numerics record honk_res_pack writes into `packed` (device; read by the f16x2
 * forward, and by the host through honk_res_numerics):
 *   HONK_NUM_SCALE    s_model, the power-of-two activation scale of the f16x2 path:
 *                     M * s_model < 2^4 (each clip stores s * (its pre-BN tensors) with
 *                     s = s_model, lowered by the binades its input's conv0 bound
 *                     max|x| * HONK_NUM_W0SUM exceeds M -- fp16's range follows the clip)
 *   HONK_NUM_RANGE    M = max over layers / channels of |running_mean| + 8 sqrt(running_var)
 *   HONK_NUM_W0SUM    max_c sum_t |conv0.weight[c][0][t]|
 *   HONK_NUM_RHO      max over layers of sqrt(mean_c (mean_c^2 + var_c) / var_c): the RMS
 *                     size of a stored tensor in its own BatchNorm units (the factor by
 *                     which the storage rounding grows in the next layer); NaN if a
 *                     statistic is not finite
 *   HONK_NUM_F16_OVERFLOW  1 if a folded weight (W * invstd, or a border-bias weight)
 *                     has no finite fp16 (hi, lo) split
 *   HONK_NUM_RHO_LAYER the layer (1-based) of HONK_NUM_RHO
 *   HONK_NUM_VALID    1 once the record is written
 *   HONK_NUM_OUT_SCALE 2^kw[L] for an odd n_layers (the last layer's output relative to
 *                     the residual stream's scale), else 1
 *   [HONK_NUM_KW + i] kw[i+1], the f16x2 weight exponent of conv{i+1}: its folded weights
 *                     are packed times 2^kw, an odd layer and the even layer after it
 *                     taking +k / -k (keeps weights of layers fed by a wide-spread tensor
 *                     out of fp16's subnormal range; 0 / +-1 at unit scale)
 */
#define HONK_NUM_SCALE 0
#define HONK_NUM_RANGE 1
#define HONK_NUM_W0SUM 2
#define HONK_NUM_RHO 3
#define HONK_NUM_F16_OVERFLOW 4
#define HONK_NUM_RHO_LAYER 5
#define HONK_NUM_VALID 6
#define HONK_NUM_OUT_SCALE 7
#define HONK_NUM_COUNT 8
#define HONK_NUM_KW 64
/* Copy the first n (at most HONK_NUM_KW + n_layers) record entries to HOST memory rec[]:
   enqueues the copy on `stream` and SYNCHRONISES it (once per pack, not on the forward
   path). */
int honk_res_numerics(const honk_res_desc* d, const float* packed, float* rec, int32_t n, void* stream);
/*
 * Host-only precision policy: the precision honk_res_forward should run for the
 * `requested` one (HONK_PREC_*, HONK_PREC_AUTO) given the model's record (rec from
 * honk_res_numerics; may be NULL for F32 / BF16).  F32 -> F32; BF16 (top-1 parity, an
 * explicit choice) -> BF16 where the kernels take the shape, else F32; F16X2 / AUTO ->
 * F16X2 where its 1e-4 contract holds (unpooled maps of >= 4040 pixels and >= 32 maps,
 * no folded weight beyond fp16's range, HONK_NUM_RHO <= 3.5), else as BF16X3; BF16X3
 * -> BF16X3 where supported and HONK_NUM_RHO <= 100, else F32.  note (may be NULL)
 * receives why a requested format was not taken ("" when it was).  Returns the
 * precision (>= 0) or a HONK_ERR_* code.
 */
int honk_res_select_precision(const honk_res_desc* d, const float* rec, int32_t requested, char* note,
                              size_t note_len);
/*
 * x: [batch, height, width] fp32;  logits: [batch, n_labels] fp32 (eval-mode forward)
 *
 * HONK_PREC_F16X2 admits every clip on its own (per batch, not once per model): after the
 * f16x2 pass, a clip whose last-layer BatchNorm'd channel means lie beyond
 * HONK_F16X2_Z_MAX standard deviations of the model's calibration (an input far outside
 * the distribution the running statistics describe: f16x2's rounding is no longer
 * averaged away there), or whose f16x2 logits are not finite while its input is, is
 * re-run in BF16X3 and its logits replaced.  This is the one honk_res_forward mode that
 * SYNCHRONISES `stream` (once per call, to read the flagged-clip count; not capturable
 * in a hipGraph).  HONK_F16X2_RERUN=0 in the environment turns the admission off (raw
 * f16x2: kernel tests).  The workspace (honk_res_workspace_bytes) includes its buffers.
 */
int honk_res_forward(const honk_res_desc* d, const float* packed, const float* x, float* logits,
                     int64_t batch, void* workspace, size_t workspace_bytes, void* stream);
#define HONK_F16X2_Z_MAX 8
/* The clips the calling thread's last honk_res_forward re-ran in bf16x3 (0 unless F16X2). */
int64_t honk_res_rerun_count(void);

/* ---- SpeechModel (cnn-*); utils/model.py:123-205 ------------------------------ */
typedef struct honk_cnn_desc {
  int32_t height, width, n_labels;
  int32_t c1_out, c1_kh, c1_kw, c1_sh, c1_sw, p1_h, p1_w;   /* conv1 + pool1         */
  int32_t has_conv2, c2_out, c2_kh, c2_kw, c2_sh, c2_sw, p2_h, p2_w;
  int32_t has_lin;                                        /* Linear(flat, 32), no ReLU */
  int32_t dnn1, dnn2;                                     /* 0 = absent              */
  int32_t dnn1_relu;                                      /* 1 unless tf_variant     */
  int32_t precision;  /* HONK_PREC_F32 or HONK_PREC_BF16X3 (convs and >16-output Linears on the
                         bf16 MFMA pipe with hi/lo-split operands; 1e-4 parity)  */
} honk_cnn_desc;

size_t honk_cnn_workspace_bytes(const honk_cnn_desc* d, int64_t batch);
/*
 * tensors[] (device fp32, contiguous; NULL for absent layers), fixed order of 12:
 *   conv1.weight, conv1.bias, conv2.weight, conv2.bias, lin.weight, lin.bias,
 *   dnn1.weight, dnn1.bias, dnn2.weight, dnn2.bias, output.weight, output.bias
 * No separate pack call: OIHW weights are the [N][K] operand of the generic implicit GEMM; the
 * bf16x3 cnn-trad-pool2 path splits conv2's weights into hi/lo fragments inside the workspace
 * on every call (one small launch) and conv1's while staging them into registers.
 */
int honk_cnn_forward(const honk_cnn_desc* d, const float* const* tensors, const float* x,
                     float* logits, int64_t batch, void* workspace, size_t workspace_bytes,
                     void* stream);

/* ---- layer-level operators (used by the cnn driver; exported for tests) ------- */
/* out[b][n][oh][ow] = act(bias[n] + sum_{ci,kh,kw} in[b][ci][oh*sh+kh][ow*sw+kw] * w[n][ci][kh][kw]) */
int honk_conv2d_f32(const float* in, const float* w, const float* bias, float* out, int64_t batch,
                    int32_t cin, int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw,
                    int32_t sh, int32_t sw, int32_t relu, void* stream);
/* nn.MaxPool2d((kh,kw)) on NCHW, stride = kernel, floor */
int honk_maxpool2d_f32(const float* in, float* out, int64_t batch, int32_t c, int32_t h, int32_t w,
                       int32_t kh, int32_t kw, void* stream);
/* y[m][n] = act(b[n] + sum_k x[m][k] * w[n][k])  (nn.Linear) */
int honk_linear_f32(const float* x, const float* w, const float* b, float* y, int64_t m, int32_t k,
                    int32_t n, int32_t relu, void* stream);

/* ---- SpeechModel training (utils/train.py:123-135 on the cnn configs) ----------- */
/*
 * The backward of model.py:186-193 (relu(conv) -> dropout -> max-pool; the forward is
 * honk_conv2d_f32 with relu = 1 and honk_maxpool2d_f32), replacing the cuDNN/MIOpen
 * convolution backward and max_pool2d_with_indices_backward autograd runs there.
 * g' below is the output gradient gy through the ReLU: g' = (act <= 0 ? 0 : gy), act =
 * the forward's ReLU output (act may be NULL: g' = gy) -- torch's threshold_backward.
 *
 * Max-pool backward (MaxPool2d((kh,kw)), stride = kernel, floor): gin = gout at each
 * window's first maximum in scan order (v > m || isnan(v): torch's index), 0 elsewhere.
 */
int honk_maxpool2d_bwd_f32(const float* in, const float* gout, float* gin, int64_t batch, int32_t c, int32_t h,
                           int32_t w, int32_t kh, int32_t kw, void* stream);
/* dw[n][ci][kh][kw] = sum_{b,oh,ow} g'[b][n][oh][ow] * in[b][ci][oh*sh+kh][ow*sw+kw]; db[n] = sum g' (db may
 * be NULL).  fp32 MFMA; deterministic (per-split partials in the workspace, summed in fixed order). */
size_t honk_conv2d_wgrad_workspace_bytes(int64_t batch, int32_t cin, int32_t h, int32_t w, int32_t cout, int32_t kh,
                                         int32_t kw, int32_t sh, int32_t sw);
int honk_conv2d_wgrad_f32(const float* in, const float* gy, const float* act, float* dw, float* db, int64_t batch,
                          int32_t cin, int32_t h, int32_t w, int32_t cout, int32_t kh, int32_t kw, int32_t sh,
                          int32_t sw, void* workspace, size_t workspace_bytes, void* stream);
/* stride 1: dx[b][ci][y][x] = sum_{n,kh,kw} g'[b][n][y-kh][x-kw] * w[n][ci][kh][kw] (zero outside g'),
 * dx [batch][cin][h][w]; the full correlation as an fp32-MFMA implicit GEMM over g' padded in the workspace */
size_t honk_conv2d_dgrad_workspace_bytes(int64_t batch, int32_t cin, int32_t h, int32_t w, int32_t cout, int32_t kh,
                                         int32_t kw);
int honk_conv2d_dgrad_f32(const float* gy, const float* act, const float* w, float* dx, int64_t batch, int32_t cin,
                          int32_t h, int32_t w_, int32_t cout, int32_t kh, int32_t kw, void* workspace,
                          size_t workspace_bytes, void* stream);

/*
 * The res block conv for ANY channel count C (3x3, padding = dilation = dil, no bias,
 * NCHW fp32; model.py:94-98) -- the general path under honk_conv3x3_f32's
 * {19, 45}-map kernels: the input zero-padded into the workspace, then the fp32-MFMA
 * implicit GEMM with dilation.  flip = 1: the input gradient (w'[i][o][t] =
 * w[o][i][8-t], as honk_conv3x3_f32).  The weight gradient as
 * honk_conv3x3_wgrad_f32 (deterministic).  Workspace: honk_conv_same_workspace_bytes.
 */
size_t honk_conv_same_workspace_bytes(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil);
int honk_conv_same_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c, int32_t h, int32_t w_,
                       int32_t dil, int32_t flip, void* workspace, size_t workspace_bytes, void* stream);
int honk_conv_same_wgrad_f32(const float* x, const float* dy, float* dw, int64_t batch, int32_t c, int32_t h,
                             int32_t w_, int32_t dil, void* workspace, size_t workspace_bytes, void* stream);

/* ---- MFCC front-end (AudioPreprocessor.compute_mfccs, utils/manage_audio.py:30-42) ---- */
/*
 * pcm [batch][samples] f32 -> out [batch][1 + samples/hop][n_dct] f32 (the
 * [B,101,40] model input for 1 s @ 16 kHz, hop 160, n_fft 480, 40 mels/DCT).
 * window [n_fft], mel_weights [n_mels][n_fft/2+1], dct [n_dct][n_mels] are the
 * librosa-0.6 Hann window / Slaney mel basis / DCT basis (device, f32).
 * Centre reflect padding, power spectrum, log of positive entries.  batch <= 65535.
 */
int honk_mfcc_f32(const float* pcm, int64_t batch, int32_t samples, const float* window, int32_t n_fft,
                  int32_t hop, const float* mel_weights, int32_t n_mels, const float* dct, int32_t n_dct,
                  float* out, void* stream);

/* ---- training (data-parallel train(), utils/train.py:99-135) -------------------- */
/*
 * One torch.optim.SGD step (dampening 0) over a flat fp32 parameter bucket whose
 * gradients were summed across ranks; grad_scale = 1/world_size.  momentum_buf
 * (zero-initialised by the caller, re-zeroed when the reference re-creates its
 * optimizer at a schedule boundary, train.py:137-141) may be NULL iff momentum == 0.
 */
int honk_sgd_step_f32(float* params, const float* grads, float* momentum_buf, int64_t n, float lr,
                      float momentum, float weight_decay, float grad_scale, int32_t nesterov, void* stream);

/*
 * Training-mode 3x3 convolutions of the res block stack (dilation d, padding d, no
 * bias: model.py:94-98 -- d = 1 for res8/res26 and -narrow, d = 2**(i//3) for
 * res15 and res15-narrow), replacing the nn.Conv2d forward/backward that
 * utils/train.py:131-134 runs through autograd.  NCHW fp32, channels C in {19, 45};
 * w is the OIHW [C][C][3][3] conv weight; 1 <= dil <= 64.
 *   flip = 0: y = conv(x, w)                                (forward)
 *   flip = 1: y = conv(x, w'), w'[o][i][t] = w[i][o][8-t]   (input gradient: x = dy)
 */
int honk_conv3x3_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c, int32_t h, int32_t w_,
                     int32_t dil, int32_t flip, void* stream);
/* Host-only: HONK_OK when honk_conv3x3_f32 / honk_conv3x3_wgrad_f32 cover (C, H, W, dil),
 * else the status (and honk_last_error text) those calls would return. */
int honk_conv3x3_check(int32_t c, int32_t h, int32_t w_, int32_t dil);
/* dw[o][i][ky][kx] = sum_{b,h,w} dy[b][o][h][w] * x[b][i][h+(ky-1)d][w+(kx-1)d] (zero padded);
 * deterministic: per-workgroup partials in the workspace, summed in a fixed order. */
size_t honk_conv3x3_wgrad_workspace_bytes(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil);
int honk_conv3x3_wgrad_f32(const float* x, const float* dy, float* dw, int64_t batch, int32_t c, int32_t h,
                           int32_t w_, int32_t dil, void* workspace, size_t workspace_bytes, void* stream);
/*
 * Train-mode BatchNorm2d(affine=False) (model.py:100 in training, nn.BatchNorm2d
 * semantics): y = (x - mean) * invstd with the biased batch variance over (B, H, W);
 * running stats (may both be NULL) <- (1 - momentum) running + momentum * batch
 * (unbiased variance); mean/invstd [C] are saved for the backward:
 * dx = invstd * (dy - mean(dy) - y * mean(dy * y)).  NCHW fp32, hw = H * W.
 */
size_t honk_bn_train_workspace_bytes(int64_t batch, int32_t c, int64_t hw);
/*
 * SyncBN (optional; honk_amd/syncbn.py): the caller all-reduces every
 * statistics-partials buffer across the data-parallel ranks before the BatchNorm that
 * finalises it, and sets the element-count scale k (the ranks' equal batches: k = world
 * size; thread-local, 1 by default) so the mean / variance / running statistics are the
 * whole job's.  honk_bn_partials_f32 writes the (sum a, sum a*b) partials ([c][S][2]
 * doubles, b NULL: a*a; S as honk_bn_train_workspace_bytes sizes) for a caller that reduces
 * them itself; honk_res_tail_bwd_mask*_f32 takes them with dil = -1.
 */
int honk_bn_count_scale(double k);
int honk_bn_partials_f32(const float* a, const float* b, void* part, size_t part_bytes, int64_t batch, int32_t c,
                         int64_t hw, void* stream);
int honk_bn_train_fwd_f32(const float* x, float* y, float* mean, float* invstd, float* running_mean,
                          float* running_var, int64_t batch, int32_t c, int64_t hw, float momentum, float eps,
                          void* workspace, size_t workspace_bytes, void* stream);
int honk_bn_train_bwd_f32(const float* dy, const float* y, const float* invstd, float* dx, int64_t batch,
                          int32_t c, int64_t hw, void* workspace, size_t workspace_bytes, void* stream);
/*
 * The res block tail around that BatchNorm, fused (model.py:111-118 in training:
 * x = relu(conv(x)); x = x + old_x on even layers; x = bn(x)), replacing the
 * relu / add / BatchNorm2d / threshold_backward / gradient-accumulation kernels
 * autograd runs for it (utils/train.py:131-134):
 *   forward:  s = relu(h) [+ old]  (old may be NULL; s written only when non-NULL),
 *             y = (s - mean) * invstd, batch statistics of s, running stats as above;
 *   backward: g = invstd * (gy - mean(gy) - y * mean(gy * y)) [+ gs]  (gs may be NULL:
 *             the gradient of s through its use as the next residual),
 *             gold = g (may be NULL), gh = (h > 0 ? g : 0).
 * Bit-identical to the unfused operations.  Workspace: honk_bn_train_workspace_bytes.
 */
int honk_res_tail_fwd_f32(const float* h, const float* old, float* s, float* y, float* mean, float* invstd,
                          float* running_mean, float* running_var, int64_t batch, int32_t c, int64_t hw,
                          float momentum, float eps, void* workspace, size_t workspace_bytes, void* stream);
int honk_res_tail_bwd_f32(const float* gy, const float* gs, const float* y, const float* invstd, const float* h,
                          float* gh, float* gold, int64_t batch, int32_t c, int64_t hw, void* workspace,
                          size_t workspace_bytes, void* stream);
/*
 * The tails' statistics computed in the producing conv's epilogue (the 19-map LDS-DMA
 * kernel's shapes: honk_conv3x3_stats_bytes > 0), so the tails skip their own pass:
 *   honk_conv3x3_stats_f32 = honk_conv3x3_f32 that also writes per-workgroup partial sums
 *   into `stats` -- mode 1 (forward conv, aux = old or NULL): of s = relu(y) [+ aux] and
 *   s*s; mode 2 (input-gradient conv, flip = 1, aux = the BN output y of the layer below):
 *   of the conv's output gy and gy*aux;
 *   honk_res_tail_fwd_part_f32 / honk_res_tail_bwd_part_f32 = honk_res_tail_fwd/bwd_f32
 *   taking those partials (mode 1 / mode 2 of the same shape; the backward also uses the
 *   buffer's tail as scratch).  Per-lane fp32 sums, then double in a fixed order: the
 *   statistics agree with the two-pass tails to fp32 rounding (not bit for bit).
 */
/*
 * The forward conv of a res block with the tail's elementwise head in its epilogue (the
 * statistics epilogue's shapes): s = relu(conv(x, w)) [+ old] is written instead of the
 * conv output (NCHW, as x), the ReLU's backward mask as one 32-bit word per pixel
 * (mask[b][h][w] bit o = !(conv[b][o][h][w] <= 0): NaN counts as > 0, as in torch's
 * threshold_backward; these shapes have c <= 20), and the statistics
 * of s as honk_conv3x3_stats_f32 mode 1.  Then honk_res_tail_fwd_s_f32 makes
 * y = BatchNorm_train(s) from s alone, and honk_res_tail_bwd_mask_f32 is
 * honk_res_tail_bwd_part_f32 with the mask in place of the conv output: the tails read
 * neither the conv output nor old, and write no separate s.  Same fp32 operations as the
 * unfused tails (bit-identical given the same statistics).
 */
int honk_conv3x3_tail_f32(const float* x, const float* w, float* s, uint32_t* mask, int64_t batch, int32_t c,
                          int32_t h, int32_t w_, int32_t dil, const float* old, void* stats, size_t stats_bytes,
                          void* stream);
int honk_res_tail_fwd_s_f32(const float* s, float* y, float* mean, float* invstd, float* running_mean,
                            float* running_var, const void* stats, int64_t batch, int32_t c, int32_t hh, int32_t ww,
                            int32_t dil, float momentum, float eps, void* stream);
/* dil >= 1: `stats` = the input-gradient conv's partials (honk_conv3x3_stats_f32 mode 2 at
 * dilation dil); dil = 0: `stats` is a workspace of honk_bn_train_workspace_bytes(batch, c,
 * hh * ww) and the statistics are summed here (a block whose output feeds no conv);
 * dil = -1: that workspace already holds honk_bn_partials_f32(gy, y) (SyncBN). */
int honk_res_tail_bwd_mask_f32(const float* gy, const float* gs, const float* y, const float* invstd,
                               const uint32_t* mask, float* gh, float* gold, int64_t batch, int32_t c,
                               int32_t hh, int32_t ww, int32_t dil, void* stats, size_t stats_bytes, void* stream);
size_t honk_conv3x3_stats_bytes(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil);
int honk_conv3x3_stats_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c, int32_t h,
                           int32_t w_, int32_t dil, int32_t flip, int32_t mode, const float* aux, void* stats,
                           size_t stats_bytes, void* stream);
/*
 * The train BatchNorm of a res block folded into the next conv (res26-narrow's C5 step:
 * one HBM pass less per block -- the tail writes no y).  honk_res_tail_fwd_s_f32 with
 * y = NULL computes only mean / invstd / the running statistics; the consumers of y then
 * take that block's s with its (fold_mean, fold_invstd) and make y = (s - mean) * invstd
 * where they read it, tail_fwd's fp32 expression (bit-identical to the materialized y):
 *   honk_conv3x3_tail_bn_f32 / honk_conv3x3_stats_bn_f32 mode 1 -- the forward conv's
 *   input x (its staged tile, in LDS; the conv's zero padding stays zero);
 *   honk_conv3x3_stats_bn_f32 mode 2 -- the input-gradient conv's aux;
 *   honk_conv3x3_wgrad_bn_f32 -- the weight-gradient conv's x;
 *   honk_res_tail_bwd_mask_bn_f32 -- the tail backward's y (s = that tail's s, mean its
 *   mean; dil >= 1 only: a folded block always feeds an input-gradient conv).
 * The NULL-fold forms are the entry points above.  honk_conv3x3_bn_fold_check: HONK_OK when
 * the shape has all four (the statistics epilogue's shapes whose weight gradient runs on
 * the LDS-DMA kernels).  Replaces no reference call: the reference's bn (model.py:117-118)
 * is one module the drop-in keeps; this is the same arithmetic in a different kernel.
 */
int honk_conv3x3_bn_fold_check(int64_t batch, int32_t c, int32_t h, int32_t w_, int32_t dil);
int honk_conv3x3_tail_bn_f32(const float* x, const float* w, float* s, uint32_t* mask, int64_t batch, int32_t c,
                             int32_t h, int32_t w_, int32_t dil, const float* old, const float* fold_mean,
                             const float* fold_invstd, void* stats, size_t stats_bytes, void* stream);
int honk_conv3x3_stats_bn_f32(const float* x, const float* w, float* y, int64_t batch, int32_t c, int32_t h,
                              int32_t w_, int32_t dil, int32_t flip, int32_t mode, const float* aux,
                              const float* fold_mean, const float* fold_invstd, void* stats, size_t stats_bytes,
                              void* stream);
int honk_conv3x3_wgrad_bn_f32(const float* x, const float* dy, float* dw, int64_t batch, int32_t c, int32_t h,
                              int32_t w_, int32_t dil, const float* fold_mean, const float* fold_invstd,
                              void* workspace, size_t ws_bytes, void* stream);
int honk_res_tail_bwd_mask_bn_f32(const float* gy, const float* gs, const float* s, const float* mean,
                                  const float* invstd, const uint32_t* mask, float* gh, float* gold, int64_t batch,
                                  int32_t c, int32_t hh, int32_t ww, int32_t dil, void* stats, size_t stats_bytes,
                                  void* stream);
int honk_res_tail_fwd_part_f32(const float* h, const float* old, float* s, float* y, float* mean, float* invstd,
                               float* running_mean, float* running_var, const void* stats, int64_t batch, int32_t c,
                               int32_t h_, int32_t w_, int32_t dil, float momentum, float eps, void* stream);
int honk_res_tail_bwd_part_f32(const float* gy, const float* gs, const float* y, const float* invstd, const float* h,
                               float* gh, float* gold, void* stats, int64_t batch, int32_t c, int32_t h_, int32_t w_,
                               int32_t dil, void* stream);
/*
 * The res stem in training (model.py:104-110 in training: y = relu(conv0(x)), then
 * AvgPool2d((ph, pw)) when the config has res_pool; ph = pw = 1 without pool),
 * replacing the conv0 / relu / avg_pool2d kernels autograd runs and their backward
 * (utils/train.py:131-134).  x [B][H][W] fp32 (the MFCC input, no gradient), w0 the
 * [C][1][3][3] conv0 weight, y / gy [B][C][H/ph][W/pw]; 1 <= C <= 64, (H+2)(W+2) <= 8192.
 * honk_res_stem_wgrad_f32: dw0 = d(sum gy * y)/d w0 (the ReLU mask recomputed from x),
 * deterministic (per-workgroup partials summed in a fixed order).
 */
int honk_res_stem_fwd_f32(const float* x, const float* w0, float* y, int64_t batch, int32_t c, int32_t h, int32_t w_,
                          int32_t ph, int32_t pw, void* stream);
size_t honk_res_stem_wgrad_workspace_bytes(int64_t batch, int32_t c);
int honk_res_stem_wgrad_f32(const float* x, const float* w0, const float* gy, float* dw0, int64_t batch, int32_t c,
                            int32_t h, int32_t w_, int32_t ph, int32_t pw, void* workspace, size_t workspace_bytes,
                            void* stream);

/*
 * The training step's head (utils/train.py:129-131 with model.py:119-121): the
 * spatial mean z[r] = sum_i x[r][i] / hw over rows r = (b, c) (x.view(B, C, -1) then
 * torch.mean(x, 2)) and its backward gx[r][i] = gz[r] / hw; nn.CrossEntropyLoss()
 * (mean reduction): *loss = mean_b (logsumexp(z_b) - z_b[labels_b]) (a label outside
 * [0, n) gives NaN), and dlogits = (softmax(z_b) - onehot(labels_b)) * (*grad_loss) / batch
 * (grad_loss: the device scalar upstream gradient).  Fixed-order reductions.
 */
int honk_spatial_mean_f32(const float* x, float* z, int64_t rows, int32_t hw, void* stream);
int honk_spatial_mean_bwd_f32(const float* gz, float* gx, int64_t rows, int32_t hw, void* stream);
int honk_cross_entropy_f32(const float* logits, const int64_t* labels, float* loss, int64_t batch, int32_t n,
                           void* stream);
int honk_cross_entropy_bwd_f32(const float* logits, const int64_t* labels, const float* grad_loss, float* dlogits,
                               int64_t batch, int32_t n, void* stream);

/*
 * Training-set audio augmentation (SpeechDataset.load_audio, utils/model.py:282-306,
 * with _timeshift_audio :264-270), the per-clip transform on a batch of PCM
 * audio/out [batch][len] (the clips right-padded to len); the random draws are the
 * caller's (honk_amd/augment.py draws them on the reference's `random` stream):
 *   v[i] = (flags & HONK_AUG_SILENCE) ? 0 : (0 <= i + shift < len ? audio[i + shift] : 0)
 *   out[i] = (flags & HONK_AUG_NOISE) ? clip(amp * noise[noise_off + i] + v[i], -1, 1) : v[i]
 * in float32 (product rounded, then the sum; NaN kept).  shift/noise_off/amp/flags are
 * [batch] device arrays; noise is the concatenated background-noise bank
 * [noise_len] (NULL iff noise_len == 0; reads outside it are 0).  batch <= 65535.
 */
#define HONK_AUG_SILENCE 1
#define HONK_AUG_NOISE 2
int honk_augment_f32(const float* audio, const float* noise, const int32_t* shift, const int64_t* noise_off,
                     const float* amp, const int32_t* flags, float* out, int64_t batch, int32_t len,
                     int64_t noise_len, void* stream);

/* ---- diagnostics --------------------------------------------------------------- */
const char* honk_last_error(void);
const char* honk_version(void);
/*
 * Per-launch timing of the dominant kernel (res block conv) with hipEvents
 * recorded on the launch stream.  enable=1 starts a window (clears it);
 * honk_timing_read synchronises the recorded events and returns the summed
 * kernel time (ms), the launch count and the summed algorithmic FLOP.
 */
int honk_timing_enable(int32_t enable);
int honk_timing_read(double* total_ms, int64_t* launches, double* flop);

#ifdef __cplusplus
}
#endif
#endif /* HONK_HIP_H */
