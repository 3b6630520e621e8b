/* libmauv_hip — C-ABI of the MI355X (gfx950) hot path of sams-tom/Multimodal-AUV.
 *
 * The reference is pure Python: its hot path calls into third-party framework kernels
 * (bayesian-torch 0.5.0 reparameterisation layers -> F.conv2d / F.linear / normal_ /
 * log1p(exp) on cuDNN/cuBLAS/curand).  Each entry point below replaces one of those call
 * sites (file:line in /root/reference/src/Multimodal_AUV unless noted) and is bound from
 * Python with ctypes by multimodal-auv_amd/mauv/_lib.py.
 *
 * Conventions:
 *  - every pointer is a DEVICE pointer owned by the caller (PyTorch caching allocator);
 *    the library never allocates device memory — workspace sizes come from *_workspace_*;
 *  - every call takes the hipStream_t to launch on (torch.cuda.current_stream()) and is
 *    asynchronous (no host synchronisation);
 *  - return 0 on success, < 0 on error (-1 bad argument, -2 launch failure);
 *    mauv_last_error() returns a thread-local message;
 *  - stateless and re-entrant; one process per GPU.
 *  - MC groups: G = number of Monte-Carlo samples processed by ONE launch (the reference's
 *    `for _ in range(num_mc): model(...)` loop, train/multimodal.py:107-112,
 *    inference/predictors.py:54-61, collapsed onto blockIdx.z).
 *  - layouts: activations NHWC [G][B][H][W][C] fp32; sampled weights KRSC [G][Cout][R][S][Cin];
 *    parameters/gradients in the reference's OIHW layout (bayesian-torch state_dict shapes).
 */
#ifndef MAUV_H
#define MAUV_H

#include <hip/hip_runtime.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- housekeeping ---------------------------------------------------------------------- */
const char* mauv_last_error(void);
int mauv_abi_version(void);

/* Kernel routing: ONE process-wide record, the only state the library keeps besides the
 * thread-local error message.  Every launch reads it; change it only while no other thread of
 * the process launches (a test or an A/B run between launches, or once at start-up).  Each
 * field selects between kernels that compute the same operation (outputs bit-identical, or — for
 * f32_math and the reparam backward — the same fp32 maths in another summation order); none
 * replaces a reference call site, so the defaults need never change.
 *   f32_math        arithmetic of the fp32 convs (mauv_conv2d_*_f32, mauv_stem_fwd_f32):
 *                   6 split (default): every fp32 operand split exactly into three bf16 planes
 *                   x = h + m + l, the six plane products h*h, h*m, m*h, h*l, l*h, m*m on
 *                   v_mfma_f32_32x32x16_bf16 with fp32 accumulation — the dropped terms are
 *                   <= 2^-24 |a*b|: fp32-grade results at 2.67x the f32-MFMA rate;
 *                   5 split1 (one accumulator everywhere); 3 split3 (planes h, m; products
 *                   h*h, h*m, m*h: ~2^-16 |a*b|, opt-in); 0 exact (v_mfma_f32_32x32x2_f32).
 *                   Initial value from MAUV_F32_MATH=split|split1|split3|exact.
 *   halo3           16-bit 3x3 / stride-1 convs over 64 -> 64 channels through an LDS image of
 *                   the input rows (conv_halo16.hip): 1 (default) / 0 the implicit GEMM.
 *   big16, big16_min_k  16-bit forwards on 256-row LDS-DMA tiles (conv_big16.hip): 1 (default)
 *                   the shapes where they measured faster (1x1, no pending BN, K >= 512,
 *                   N >= 256, >= 512 tiles), 2 every covered forward with K >= big16_min_k
 *                   (default and minimum 512: the K range its tests cover), 0 none.
 *   haloc16         16-bit 3x3 / stride-1 forwards and data gradients over 128-512 channels
 *                   through the chunked LDS row image (conv_haloc16.hip): 1 (default) with
 *                   32 x 64 wave tiles, 2 with 64 x 64 wave tiles, 3 the forwards only, 0 none.
 *   expand16        16-bit 1x1 expansion forwards (K = 64 / 128 / 256) through the
 *                   weight-stationary kernel (conv_expand16.hip): 1 (default) where it measured
 *                   faster, 2 every covered shape, 3 as 2 with 32-column waves at K = 128, 0 none.
 *   reparam_kernels bit 0: sampling by (output channel, channel range) blocks with vector KRSC
 *                   stores (bit-identical to the per-element kernel); bit 1: the reparameterisation
 *                   backward with 16-byte slab loads (another fixed sum order).  Default 3.
 * mauv_set_route validates every field and changes nothing on an error (-1). */
typedef struct MauvRoute {
  int f32_math;
  int halo3;
  int big16;
  int big16_min_k;
  int haloc16;
  int expand16;
  int reparam_kernels;
  int reserved[9];
} MauvRoute;
int mauv_get_route(MauvRoute* out);
int mauv_set_route(const MauvRoute* in);

/* ---- implicit-GEMM convolution on MFMA (conv_gemm.hip) ---------------------------------
 * Replaces F.conv2d inside bayesian-torch Conv2dReparameterization.forward for every conv of
 * the three torchvision ResNet-50 trunks (models/base_models.py:15-18,
 * models/model_utils.py:57-61) and F.linear in LinearReparameterization.forward (attention
 * q/k/v/score, fc, fc1, fc2: models/base_models.py:38-41,60-65) as the 1x1, H=W=1 case.
 * x_strides (host pointer, nullable): element strides {group, batch, h, w, c} of x; NULL =
 * dense NHWC.  Group stride 0 = one input shared by all G samples (the stems read the
 * caller's NCHW images this way). */
/* x_scale/x_shift (nullable, [G][Cin]) + x_relu: the producing layer's BatchNorm(+ReLU)
 * applied while loading x (its normalised activation is never stored).
 * st_mean/st_m2/st_cnt (nullable): per-m-tile BatchNorm statistics of y written by the
 * epilogue ([G][nblk][Cout], [G][nblk][Cout], [G][nblk]; nblk from
 * mauv_conv2d_fwd_stat_blocks) for mauv_bn_stats_finalize. */
int mauv_conv2d_fwd_f32(const float* x, const long long* x_strides, const float* x_scale,
                        const float* x_shift, int x_relu, const float* w, const float* bias,
                        float* y, int G, int B, int H, int W, int Cin, int Cout, int R, int S,
                        int stride, int pad, float* st_mean, float* st_m2, float* st_cnt,
                        hipStream_t stream);
int mauv_conv2d_fwd_stat_blocks(int G, int B, int H, int W, int Cin, int Cout, int R, int S,
                                int stride, int pad);
/* cuDNN dgrad in loss.backward() (train/multimodal.py:138): dx = conv^T(dy, W_g)
 * (+ addend) (+ dx if accumulate); one launch per output-parity class (stride^2).
 * bn_* (nullable): dx is the output gradient of a BatchNorm(+ReLU) whose backward partial
 * sums (sum dz, sum dz*xhat per channel; [G][nblk][Cin], nblk from
 * mauv_conv2d_bwd_data_stat_blocks) the epilogue writes for mauv_bn_bwd's pre_p1/pre_p2;
 * the ReLU mask comes from bn_mask bits (mauv_bn_apply_mask), else bn_out, else from
 * bn_y*bn_scale+bn_shift.  addend_mask
 * (nullable): the addend counts only where these ReLU-mask bits ([G][B*H*W][Cin] / 8,
 * mauv_bn_apply_mask) are set — a block output's residual gradient dres = dout * mask added
 * without being stored. */
int mauv_conv2d_bwd_data_f32(const float* dy, const float* w, float* dx, const float* addend,
                             const unsigned char* addend_mask,
                             int accumulate, int G, int B, int H, int W, int Cin, int Cout,
                             int R, int S, int stride, int pad, const float* bn_y,
                             const float* bn_out, const unsigned char* bn_mask,
                             const float* bn_scale, const float* bn_shift,
                             const float* bn_mean, const float* bn_invstd, int bn_relu,
                             float* bn_p1, float* bn_p2, hipStream_t stream);
int mauv_conv2d_bwd_data_stat_blocks(int G, int B, int H, int W, int Cin, int Cout, int R,
                                     int S, int stride, int pad);
/* cuDNN wgrad (train/multimodal.py:138): split-K partial slabs ws[splits][G][Cout][R*S*Cin],
 * reduced deterministically by mauv_reparam_bwd.  mauv_conv2d_wgrad_splits sizes them. */
int mauv_conv2d_wgrad_splits(int G, int B, int H, int W, int Cin, int Cout, int R, int S,
                             int stride, int pad);
int mauv_conv2d_bwd_weight_f32(const float* x, const long long* x_strides, const float* x_scale,
                               const float* x_shift, int x_relu, const float* dy, float* ws,
                               int splits, int G, int B, int H, int W, int Cin, int Cout, int R,
                               int S, int stride, int pad, hipStream_t stream);
/* Their arithmetic: MauvRoute.f32_math (housekeeping section). */

/* ---- 16-bit implicit-GEMM convs (conv_gemm16.hip) -----------------------------------------
 * Same three GEMM views on v_mfma_f32_32x32x16_{bf16,f16}: dtype 0 = bf16 (BASELINE configs[2]
 * training), 1 = f16 (the reference predictor's torch.amp.autocast on a GPU,
 * inference/predictors.py:55).  x / w / y / dy / dx / addend are 16-bit words, statistics
 * partials and weight-gradient slabs fp32.  Cin and Cout must be multiples of 8 (the stems
 * run as GEMMs over im2col rows, mauv_stem_*; their former 8-channel padded form remains
 * valid), dgrad needs Cout % 32 == 0; x strides
 * are channel-contiguous multiples of 8.  Statistics partials: mauv_conv2d_fwd_stat_blocks.
 * y_shift (nullable, [Cout] fp32): y is STORED centred, y[.., c] = round16(conv - y_shift[c]):
 * the fp32 accumulators start at -y_shift[c], so the statistics partials are those of the stored
 * values too; pass the consuming BatchNorm's centre (its running mean where that dominates the
 * channel's spread, else 0) here and to mauv_bn_stats_finalize — the 16-bit rounding error of the
 * stored tensor then scales with the batch spread |y - mean| instead of |y|, the error the BN's
 * 1/std amplifies when a channel's mean is large.  Every route (the
 * implicit GEMM, 3x3 row images, LDS-DMA tiles, weight-stationary expansion) gives the same bits
 * for the same y_shift. */
int mauv_conv2d_fwd_h16(int dtype, const void* x, const long long* x_strides,
                        const float* x_scale, const float* x_shift, int x_relu, const void* w,
                        void* y, int G, int B, int H, int W, int Cin, int Cout, int R, int S,
                        int stride, int pad, float* st_mean, float* st_m2, float* st_cnt,
                        const float* y_shift, hipStream_t stream);
/* A bottleneck's conv1 (1x1, stride 1, no padding) whose input is the previous bottleneck's
 * output, formed while conv1's tiles are loaded (replaces bn3 + residual add + ReLU, the
 * `out += identity; out = relu(out)` of torchvision's Bottleneck.forward under
 * models/base_models.py:74-90, followed by the next block's conv1):
 *   out = relu(y*scale + shift + r),  r = res, or res*res_scale + res_shift (the downsample
 *   branch's BN, res_scale / res_shift both non-NULL), per (group, channel) [G][Cin] parameters;
 * `out` ([G][B][H][W][Cin], written once) gets exactly mauv_bn_apply's values (out_mask,
 * nullable: mauv_bn_apply_mask's ReLU bits of it, for a training step) and y1 / the
 * statistics partials exactly mauv_conv2d_fwd_h16's on that `out`.  y, res: contiguous
 * [G][B][H][W][Cin]; Cin % 64 == 0, Cin <= 2048.  Returns 0 when launched, 1 when the shape is
 * outside the kernel (nothing launched: run mauv_bn_apply, then mauv_conv2d_fwd_h16), < 0 on an
 * argument error.  y1_shift: mauv_conv2d_fwd_h16's y_shift for y1. */
int mauv_conv2d_fwd_fold_h16(int dtype, const void* y, const float* scale, const float* shift,
                             const void* res, const float* res_scale, const float* res_shift,
                             void* out, unsigned char* out_mask, const void* w, void* y1, int G,
                             int B, int H, int W, int Cin, int Cout, float* st_mean,
                             float* st_m2, float* st_cnt, const float* y1_shift,
                             hipStream_t stream);
int mauv_conv2d_bwd_data_h16(int dtype, const void* dy, const void* w, void* dx,
                             const void* addend, int accumulate, int G, int B, int H, int W,
                             int Cin, int Cout, int R, int S, int stride, int pad,
                             hipStream_t stream);
/* mauv_conv2d_bwd_data_h16 whose epilogue also writes the BatchNorm-backward partial sums of
 * the BN whose output gradient dx is (bn_p1 = sum dz, bn_p2 = sum dz*xhat, [G][nblk][Cin], nblk
 * = mauv_conv2d_bwd_data_stat_blocks), for mauv_bn_bwd_ex's pre_p1/pre_p2: the standalone
 * partial pass over (y, dout) of models/resnet50_variational.py's BN backward disappears.
 * ReLU mask: bn_mask bits (mauv_bn_apply_mask) else bn_out > 0 else bn_y*bn_scale+bn_shift > 0.
 * addend_mask as in mauv_conv2d_bwd_data_f32.  bn_p1 and addend_mask NULL =
 * mauv_conv2d_bwd_data_h16.  Cout % 64 == 0 with partials or addend_mask. */
int mauv_conv2d_bwd_data_bn_h16(int dtype, const void* dy, const void* w, void* dx,
                                const void* addend, int accumulate, int G, int B, int H, int W,
                                int Cin, int Cout, int R, int S, int stride, int pad,
                                const unsigned char* addend_mask, const void* bn_y, const void* bn_out,
                                const unsigned char* bn_mask, const float* bn_scale,
                                const float* bn_shift, const float* bn_mean,
                                const float* bn_invstd, int bn_relu, float* bn_p1, float* bn_p2,
                                hipStream_t stream);
int mauv_conv2d_bwd_weight_h16(int dtype, const void* x, const long long* x_strides,
                               const float* x_scale, const float* x_shift, int x_relu,
                               const void* dy, float* ws, int splits, int G, int B, int H, int W,
                               int Cin, int Cout, int R, int S, int stride, int pad,
                               hipStream_t stream);

/* ---- variational sampling / KL (reparam.hip) --------------------------------------------
 * bayesian-torch Conv2dReparameterization/LinearReparameterization.forward:
 *   sigma = log1p(exp(rho)); eps.normal_(); w = mu + sigma*eps      (per MC sample g)
 * eps from Philox4x32-10(seed, sample0+g, layer, quad) — or the explicit eps [G][numel]
 * (parameter order) when non-NULL (parity tests).  out_gstride 0 = numel. */
int mauv_reparam_sample(const float* mu, const float* rho, const float* eps,
                        unsigned long long seed, unsigned long long sample0, unsigned int layer,
                        int G, int Cout, int Cin, int RS, float* out, long long out_gstride,
                        hipStream_t stream);
/* Backward of the above: dmu += sum_g dW_g; drho += sum_g dW_g * eps_g' * sigmoid(rho),
 * g' = g (fixed_sample < 0) or the sample `fixed_sample` for every g (bayesian-torch 0.5.0
 * semantics: its eps buffer is overwritten in place by later MC forwards while autograd
 * still references it).  dw element (s, g, i) at dw[s*dw_sstride + g*dw_gstride + i], i in
 * KRSC order with dw_cin (>= Cin; the 16-bit stems' padded channel count) channels. */
int mauv_reparam_bwd(const float* dw, int splits, long long dw_gstride, long long dw_sstride,
                     const float* mu, const float* rho, const float* eps,
                     unsigned long long seed, unsigned long long sample0, unsigned int layer,
                     int G, int Cout, int Cin, int RS, int dw_cin, float* dmu, float* drho,
                     long long fixed_sample, hipStream_t stream);
/* Their kernel forms: MauvRoute.reparam_kernels (housekeeping section). */
/* 16-bit sampled weights (dtype 0 = bf16, 1 = f16) for the 16-bit convs: KRSC with cin_pad
 * (>= Cin) input channels; pad channels are not written (zero-fill them once).  The sampling
 * arithmetic is fp32, only the stored weight is rounded.  out_gstride 0 = Cout*RS*cin_pad. */
int mauv_reparam_sample_h16(int dtype, const float* mu, const float* rho, const float* eps,
                            unsigned long long seed, unsigned long long sample0,
                            unsigned int layer, int G, int Cout, int Cin, int RS, int cin_pad,
                            void* out, long long out_gstride, hipStream_t stream);
/* The three sampling forms in one entry (dtype -1 = fp32, 0 = bf16, 1 = f16; KRSC with cin_pad
 * >= Cin channels, pad untouched) whose MC sample index is sample0 + *sample_base + g when
 * sample_base (nullable device counter) is given: a HIP graph captured around a forward
 * replays with fresh samples after the caller updates the counter. */
int mauv_reparam_sample_ex(int dtype, const float* mu, const float* rho, const float* eps,
                           unsigned long long seed, unsigned long long sample0,
                           const unsigned long long* sample_base, unsigned int layer, int G,
                           int Cout, int Cin, int RS, int cin_pad, void* out,
                           long long out_gstride, hipStream_t stream);
/* fp32 counterpart of mauv_reparam_sample_h16's padded layout (the fp32 stems' 4-channel KRSC
 * weights); same sampling as mauv_reparam_sample, pad channels not written. */
int mauv_reparam_sample_padded(const float* mu, const float* rho, const float* eps,
                               unsigned long long seed, unsigned long long sample0,
                               unsigned int layer, int G, int Cout, int Cin, int RS, int cin_pad,
                               float* out, long long out_gstride, hipStream_t stream);

/* get_kl_loss (bayesian-torch 0.5.0; called at train/multimodal.py:114,284 and
 * train/unimodal.py:130,262): sum over entries of mean(log s_p - log s + (s^2 + (mu-m_p)^2)
 * / (2 s_p^2) - 1/2), s = softplus(rho).  `table` is a device array of MauvKlEntry. */
typedef struct MauvKlEntry {
  const float* mu;
  const float* rho;
  float* dmu;
  float* drho;
  long long numel;
  float prior_mu;
  float prior_sigma;
} MauvKlEntry;
int mauv_kl_workspace_bytes(int n_entries);
int mauv_kl_fwd(const MauvKlEntry* table, int n, double* workspace, float scale, float* out,
                hipStream_t stream);
/* dmu/drho += (coef_dev ? *coef_dev : 1) * scale * dKL/d(mu, rho) (coef_dev: device scalar,
 * the upstream gradient — no host sync). */
int mauv_kl_bwd(const MauvKlEntry* table, int n, const float* coef_dev, float scale,
                hipStream_t stream);
/* test hook: raw Philox words [nq][4] and the derived normals [nq][4] */
int mauv_philox_raw(unsigned long long seed, unsigned long long sample, unsigned int layer,
                    int nq, unsigned int* out_u32x4, float* out_normal4, hipStream_t stream);

/* ---- fused Adam (adam.hip) ------------------------------------------------------------------
 * torch.optim.Adam as the reference builds it (train/loop_utils.py:45-61: amsgrad=False,
 * maximize=False, L2 weight_decay) stepped for a whole table of fp32 tensors in one launch;
 * step = the (shared) 1-based step count used for bias correction. */
typedef struct MauvAdamEntry {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  long long numel;
} MauvAdamEntry;
int mauv_adam_step(const MauvAdamEntry* table, int n, float lr, float beta1, float beta2,
                   float eps, float weight_decay, long long step, hipStream_t stream);
/* The step decision of train/multimodal.py:133-145 (skip on a non-finite loss; skip the step
 * AND the zero_grad on non-finite gradients; otherwise step + zero_grad) taken on the device, so
 * a training step has no host round trip.  64-byte device struct; the caller zero-initialises
 * it, writes ok_loss (1 = the loss is finite on every rank) before the backward and counts
 * the gradient arena's non-finite elements into `nonfinite` after it.  mode / step_size /
 * bc2_sqrt are written by mauv_adam_step_gated; step is the Adam step count (bias correction);
 * poisoned = the arena still holds a skipped step's non-finite gradients. */
typedef struct MauvStepGate {
  int ok_loss, nonfinite, poisoned, mode;
  int step, stepped, skipped_loss, skipped_grad;
  float step_size, bc2_sqrt;
  int reserved[6];   /* untouched by the library (mauv.train counts non-finite inputs in [5]) */
} MauvStepGate;
int mauv_adam_step_gated(const MauvAdamEntry* table, int n, float lr, float beta1, float beta2,
                         float eps, float weight_decay, MauvStepGate* gate, hipStream_t stream);

/* ---- BatchNorm2d (training mode, per MC group) + residual + ReLU (bn.hip) ---------------
 * torchvision Bottleneck bn1..3 / downsample.1 / stem bn1 in .train() for every MC pass
 * (train/multimodal.py:60,232; inference/predictors.py:27).  y/out [G][M][C], M = B*H*W. */
long long mauv_bn_workspace_floats(int G, long long M, int C);
int mauv_bn_fwd_train(const float* y, int G, long long M, int C, const float* gamma,
                      const float* beta, float* run_mean, float* run_var, float momentum,
                      float eps, float* workspace, float* mean, float* invstd, float* scale,
                      float* shift, const float* res, int relu, float* out,
                      hipStream_t stream);
/* statistics from per-m-tile partials written by mauv_conv2d_fwd_f32's epilogue: Chan merge,
 * mean/invstd/scale/shift [G][C], sequential running-stat update (run_* nullable);
 * workspace: mauv_bn_stats_workspace_floats(G, nblk, C) floats (2*G*C when nblk <= 128*64;
 * larger partial counts are merged in segments).  y_shift (nullable, [C]): the centre the 16-bit
 * forward stored y with (mauv_conv2d_fwd_h16); the partials are then those of the stored values
 * and mean / shift describe them (mean = mu_stored, shift = beta - mean*scale) for every
 * consumer of that tensor, while the running mean is updated with the true mean
 * mu_stored + y_shift; y_shift may alias run_mean (it is read before the update). */
long long mauv_bn_stats_workspace_floats(int G, int nblk, int C);
int mauv_bn_stats_finalize(int G, int nblk, int C, const float* pmean, const float* pm2,
                           const float* pcnt, const float* gamma, const float* beta,
                           float* run_mean, float* run_var, float momentum, float eps,
                           float* workspace, float* mean, float* invstd, float* scale,
                           float* shift, const float* y_shift, hipStream_t stream);
/* out = [relu](y*scale + shift (+ res')); res' = res*res_scale + res_shift when res_scale is
 * non-NULL — the bottleneck's downsample BatchNorm applied inside the residual add (its output
 * is never materialised). */
int mauv_bn_apply(const float* y, const float* scale, const float* shift, const float* res,
                  const float* res_scale, const float* res_shift, int relu, float* out, int G,
                  long long M, int C, hipStream_t stream);
int mauv_bn_eval_params(int G, int C, const float* gamma, const float* beta,
                        const float* run_mean, const float* run_var, float eps, float* scale,
                        float* shift, hipStream_t stream);
/* out NULL + relu: the mask is recomputed as y*scale + shift > 0 (lazily-applied BN).
 * pre_p1/pre_p2 (nullable): partial sums already produced by a dgrad epilogue
 * ([G][pre_nblk][C]) — the partial pass over dout is skipped. */
int mauv_bn_bwd(const float* y, const float* out, const float* dout, int relu,
                const float* mean, const float* invstd, const float* scale, const float* shift,
                int G, long long M, int C, float* workspace, float* dy, float* dres,
                float* dgamma, float* dbeta, const float* pre_p1, const float* pre_p2,
                int pre_nblk, hipStream_t stream);
/* 16-bit activations (dtype 0 = bf16, 1 = f16): y/res/out/dout/dy/dres are 16-bit words;
 * statistics, scale/shift, workspace and dgamma/dbeta fp32 (same maths as above). */
int mauv_bn_apply_h16(int dtype, const void* y, const float* scale, const float* shift,
                      const void* res, const float* res_scale, const float* res_shift, int relu,
                      void* out, int G, long long M, int C, hipStream_t stream);
int mauv_bn_bwd_h16(int dtype, const void* y, const void* out, const void* dout, int relu,
                    const float* mean, const float* invstd, const float* scale,
                    const float* shift, int G, long long M, int C, float* workspace, void* dy,
                    void* dres, float* dgamma, float* dbeta, hipStream_t stream);

/* Block-output BN apply (+ReLU, +residual as mauv_bn_apply) that also writes the ReLU mask
 * bits of the stored output, mask[G][M][C/8] (bit e of byte j: out[8j+e] > 0), and the
 * BN + ReLU backward that reads them instead of the output (dres = dz as in mauv_bn_bwd).
 * dtype -1 = fp32, 0 = bf16, 1 = f16; C % 8 == 0, C <= 2048.  Same results as
 * mauv_bn_apply / mauv_bn_bwd with `out`; replaces the same torchvision Bottleneck
 * bn3 -> += identity -> relu (and its autograd) as they do. */
int mauv_bn_apply_mask(int dtype, const void* y, const float* scale, const float* shift,
                       const void* res, const float* res_scale, const float* res_shift, void* out,
                       unsigned char* mask, int G, long long M, int C, hipStream_t stream);
int mauv_bn_bwd_mask(int dtype, const void* y, const unsigned char* mask, const void* dout,
                     const float* mean, const float* invstd, const float* scale, int G,
                     long long M, int C, float* workspace, void* dy, void* dres, float* dgamma,
                     float* dbeta, hipStream_t stream);
/* Every form above in one entry (dtype -1 fp32, 0 bf16, 1 f16): ReLU mask from mask bits, else
 * out, else y*scale+shift; pre_p1/pre_p2/pre_nblk (nullable): partial sums a data-gradient
 * epilogue already wrote (mauv_conv2d_bwd_data_bn_h16 / _f32), so only the finalize and the
 * apply pass run.  dy and dres both NULL: partials / parameter gradients only. */
int mauv_bn_bwd_ex(int dtype, const void* y, const void* out, const unsigned char* mask,
                   const void* dout, int relu, const float* mean, const float* invstd,
                   const float* scale, const float* shift, int G, long long M, int C,
                   float* workspace, void* dy, void* dres, float* dgamma, float* dbeta,
                   const float* pre_p1, const float* pre_p2, int pre_nblk, hipStream_t stream);

/* ---- pooling (pool.hip): torchvision stem maxpool 3x3/2 pad 1 and adaptive avgpool ------ */
/* max-pool forward: C % 8 == 0 (the stem: 64); backward: C % 4 == 0. */
int mauv_maxpool_fwd(const float* x, int N, int H, int W, int C, float* y, unsigned char* idx,
                     hipStream_t stream);
int mauv_maxpool_bwd(const float* dy, const unsigned char* idx, int N, int H, int W, int C,
                     float* dx, hipStream_t stream);
/* The stem's pending BatchNorm + ReLU applied on load (out = maxpool(relu(y*scale[g] +
 * shift[g])), group g = image / (N/G)): the 112x112 BN output is never materialised.
 * Replaces the bn1 -> relu -> maxpool sequence of torchvision's ResNet stem
 * (models/base_models.py:15-16 builds it).  idx nullable (inference) in every maxpool entry. */
int mauv_maxpool_bn_fwd(const float* y, const float* scale, const float* shift, int G, int N,
                        int H, int W, int C, float* out, unsigned char* idx, hipStream_t stream);
int mauv_avgpool_fwd(const float* x, int N, int HW, int C, float* y, hipStream_t stream);
int mauv_avgpool_bwd(const float* dy, int N, int HW, int C, float* dx, hipStream_t stream);
/* 16-bit activations; the pooled features / their gradient stay fp32 (the head is fp32). */
int mauv_maxpool_fwd_h16(int dtype, const void* x, int N, int H, int W, int C, void* y,
                         unsigned char* idx, hipStream_t stream);
int mauv_maxpool_bwd_h16(int dtype, const void* dy, const unsigned char* idx, int N, int H,
                         int W, int C, void* dx, hipStream_t stream);
int mauv_maxpool_bn_fwd_h16(int dtype, const void* y, const float* scale, const float* shift,
                            int G, int N, int H, int W, int C, void* out, unsigned char* idx,
                            hipStream_t stream);
int mauv_avgpool_fwd_h16(int dtype, const void* x, int N, int HW, int C, float* y,
                         hipStream_t stream);
int mauv_avgpool_bwd_h16(int dtype, const float* dy, int N, int HW, int C, void* dx,
                         hipStream_t stream);
/* Stem input of the 16-bit path: fp32 NCHW [B][C][H][W] -> 16-bit NHWC [B][H][W][Cp], channels
 * C..Cp-1 zero (the caller's images are read once per trunk, shared by all MC samples). */
int mauv_pack_nchw_h16(int dtype, const float* x, int B, int C, int H, int W, int Cp, void* y,
                       hipStream_t stream);
/* Stem input of the fp32 path: NCHW -> NHWC [B][H][W][Cp] fp32, channels C..Cp-1 zero (Cp = 4:
 * the stem conv then runs the pipelined split kernel on 16-byte pixel quads). */
int mauv_pack_nchw_f32(const float* x, int B, int C, int H, int W, int Cp, float* y,
                       hipStream_t stream);

/* ---- stems over shared im2col rows (stem.hip) --------------------------------------------
 * conv1 of each trunk (7x7 / 2, models/base_models.py:18, model_utils.py:58-59) sees the same
 * images in every MC sample.  mauv_stem_im2col unrolls fp32 NCHW images once into rows
 * cols[m][k] (m = (b, oh, ow), k = c*R*S + r*S + s: the OIHW parameter order), zero for
 * k >= C*R*S up to Kp (Kp % 8 == 0); dtype -1 = fp32, 0 = bf16, 1 = f16 rows (RNE).
 * mauv_stem_fwd_{f32,h16}: y[g][m][c] = sum_k cols[m][k] w[g][c][k] as ONE GEMM with the G
 * weight sets stacked along N (w: [G][Cout][Kp], k >= C*R*S zero); per-m-tile BatchNorm
 * partials as mauv_conv2d_fwd_f32 with nblk = mauv_conv2d_fwd_stat_blocks of the stem.
 * fp32 needs Kp % 4 == 0, 16-bit Kp % 64 == 0 and Cout % 8 == 0.  The weight gradient is
 * mauv_conv2d_bwd_weight_* of a 1x1 conv over the rows (group stride 0). */
int mauv_stem_im2col(int dtype, const float* x, int B, int C, int H, int W, int R, int S,
                     int stride, int pad, int Kp, void* out, hipStream_t stream);
int mauv_stem_fwd_f32(const float* cols, const float* w, float* y, int G, int M, int Kp,
                      int Cout, float* st_mean, float* st_m2, float* st_cnt, hipStream_t stream);
int mauv_stem_fwd_h16(int dtype, const void* cols, const void* w, void* y, int G, int M, int Kp,
                      int Cout, float* st_mean, float* st_m2, float* st_cnt, const float* y_shift,
                      hipStream_t stream);

/* ---- fusion head + MC head (head.hip) ----------------------------------------------------
 * AdditiveAttention.forward (models/base_models.py:43-52) epilogues around the q|k|v and
 * score GEMMs (qkv rows [q | k | v], each hid wide; the reference's model: hid = 128):
 * t = tanh(q + k); o = v * softmax(s, dim=1) into the concat slot (:86) of ld comb_ld. */
int mauv_attn_t(const float* qkv, int rows, int hid, float* t, hipStream_t stream);
int mauv_attn_t_bwd(const float* dt, const float* t, int rows, int hid, float* dqkv,
                    hipStream_t stream);
int mauv_attn_out(const float* qkv, const float* s, int rows, int hid, float* comb, int comb_ld,
                  int comb_off, hipStream_t stream);
int mauv_attn_out_bwd(const float* dcomb, int comb_ld, int comb_off, const float* qkv,
                      const float* s, int rows, int hid, float* dqkv, float* ds,
                      hipStream_t stream);
/* bias gradients of the linear layers */
int mauv_colsum(const float* dy, int G, int rows, int N, float* out, int accumulate,
                hipStream_t stream);
/* train/multimodal.py:121 (mean over MC), :127 (CrossEntropyLoss), :151 (argmax) */
int mauv_mc_mean_ce(const float* logits, const long long* labels, int G, int B, int C,
                    float* mean, float* loss, long long* pred, hipStream_t stream);
int mauv_mc_mean_bwd(const float* dmean, const float* gloss, const float* mean,
                     const long long* labels, int G, int B, int C, float* dlogits,
                     hipStream_t stream);
/* inference/predictors.py:65-84, train/multimodal.py:305-310, train/unimodal.py:298-308:
 * sufficient statistics sums[b] = {sum_g p (C), sum_g p^2 (C), sum_g H[p_g]} (float64,
 * all-reducible across MC-sharded ranks), then mean prob, unbiased variance (mean over
 * classes), aleatoric entropy, predictive entropy, argmax. */
int mauv_mc_stats(const float* logits, int G, int B, int C, float eps_h, double* sums,
                  int accumulate, hipStream_t stream);
int mauv_mc_finalize(const double* sums, int N, int B, int C, float eps_pred, float* mean_prob,
                     float* var_unc, float* alea, float* pred_entropy, long long* pred,
                     hipStream_t stream);
/* train/multimodal.py:133,141 NaN/Inf guards as one fused scan (*out += blocks with a
 * non-finite value) */
int mauv_nonfinite_count(const float* p, long long n, int* out, hipStream_t stream);

/* ---- input staging (staging.hip) ---------------------------------------------------------
 * data/datasets.py:239-250 per-tile transforms on the device: uint8 HWC tiles [B][H][W][C] as
 * PIL decodes them -> fp32 NCHW out = x / 255 (ToTensor), then (out - mean[c]) / std[c]
 * (Normalize; mean/std nullable = ToTensor only), bit-exact with torchvision's fp32 ops.
 * uifm_bt (nullable): also apply the underwater image formation model of
 * Examples/"Example training with image noise.py":55-93 to the result:
 *   t = exp(-bt[c] * (d * depth)); out = clamp(out * t + binf[c] * (1 - t), 0, 1)
 * with bt[c] = beta_c * turbidity computed in fp32 as the reference does and d the
 * [B][1][H][W] distance map (nullable = uniform 1, what the reference passes).
 * mauv_uifm: the same degradation on fp32 NCHW tiles [B][C][H][W]. */
int mauv_stage_u8(const unsigned char* x, int B, int H, int W, int C, const float* mean,
                  const float* stdv, const float* uifm_bt, const float* uifm_binf,
                  const float* dist, float depth, float* out, hipStream_t stream);
int mauv_uifm(const float* x, int B, int C, int H, int W, const float* bt, const float* binf,
              const float* dist, float depth, float* out, hipStream_t stream);
/* data/datasets.py:240-246 transforms.Resize((256, 256)) of the decoded tiles = PIL's
 * Image.resize(size, BILINEAR) (antialiased when downscaling), bit-exact with Pillow's 8-bit
 * separable resampler (libImaging/Resample.c; the reference pins pillow 11.0.0): uint8
 * [B][H][W][C] (1 <= C <= 4) -> uint8 [B][Ho][Wo][C] (out_u8), or — out_f32 instead — the
 * resized tile through mauv_stage_u8's ToTensor / Normalize / UIFM maths into fp32 NCHW
 * [B][C][Ho][Wo] in the same pass (mean/std, uifm_bt/binf, dist [B][1][Ho][Wo] nullable as
 * there).  workspace: mauv_resize_workspace_bytes(...) device bytes (coefficient tables and
 * the 8-bit horizontal-pass image), caller-owned; -1 = bad shape. */
long long mauv_resize_workspace_bytes(int B, int H, int W, int C, int Ho, int Wo);
int mauv_resize_u8(const unsigned char* x, int B, int H, int W, int C, int Ho, int Wo,
                   void* workspace, unsigned char* out_u8, const float* mean, const float* stdv,
                   const float* uifm_bt, const float* uifm_binf, const float* dist, float depth,
                   float* out_f32, hipStream_t stream);

/* ---- evaluation metrics (metrics.hip) ----------------------------------------------------
 * train/multimodal.py:312-347 (confusion matrix) and Examples/"Example training with image
 * noise.py":530-634 (uncertainty-error AUROC, macro F1, 15-bin ECE / Emax), accumulated on the
 * device across an epoch instead of per-batch .cpu() copies:
 * mauv_confusion_update: counts[y * C + p] += 1 (int32 [C*C + 1]; out-of-range labels or
 *   predictions counted in counts[C*C]);
 * mauv_calibration_update: per MC-mean probability row, conf = max, pred = argmax (first
 *   maximum); the bin b with edges[b] < conf <= edges[b+1] (float64 edges, nbins + 1 of them)
 *   gets bins[3b] += 1, bins[3b+1] += conf, bins[3b+2] += (pred == label);
 * mauv_auroc_pairs: count2 += sum over (positive i, negative j) of 2 [s_i > s_j] + [s_i == s_j]
 *   (AUROC = count2 / (2 n_pos n_neg)). */
int mauv_confusion_update(const long long* labels, const long long* pred, int n, int C,
                          int* counts, hipStream_t stream);
int mauv_calibration_update(const float* probs, const long long* labels, int n, int C,
                            int nbins, const double* edges, double* bins, hipStream_t stream);
int mauv_auroc_pairs(const float* score, const unsigned char* positive, int n,
                     unsigned long long* count2, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MAUV_H */
