/* libfacevae — MI355X (gfx950) C-ABI for the FaceVAE training step.
 *
 * Plain C ABI: raw device pointers, sizes, a dtype enum and an explicit hipStream_t
 * (passed as void*).  No torch types.  Every entry returns an int status (FV_OK = 0;
 * >0 = FV_E_* or a hipError_t); the message of the last failure on the calling thread is
 * available from fv_last_error().  Nothing aborts, nothing allocates device memory on
 * the hot path: callers size workspaces with the *_ws_bytes / *_elems helpers.
 *
 * Activations are NHWC ("channels_last") with a channel stride `ld*` ≥ valid channels.
 * Conv weights are handed over in the reference parameter layout
 * (nn.Conv2d.weight [Cout][Cin][k][k], fp32) and re-laid out per forward by
 * fv_conv_weight_prep into the kernel layout [rows][Kpad] with k = (r*k + s)*cin + ci.
 *
 * Which reference interface each entry replaces (file:line in Luh1124/face-vae):
 *   fv_conv2d_fwd            F.conv2d inside _ConvBlock / nn.Conv2d (modules.py:32-42,
 *                            models.py:934,1096,1099) incl. nn.Upsample (modules.py:81)
 *                            folded into addressing, BN-apply+act prologue (NAC,
 *                            modules.py:13,31-39), bias/residual (modules.py:125)/sigmoid
 *                            (models.py:1110) epilogue and BN statistics partials.
 *   fv_conv2d_bwd_data       conv backward-data == transposed conv (ConvTranspose2dELR's
 *                            F.conv_transpose2d, models_utils.py:498-499, stride 1 case).
 *   fv_conv2d_bwd_weight     conv weight/bias gradient (autograd of modules.py:32).
 *   fv_spectral_norm_*       torch.nn.utils.spectral_norm as used by modules.py:14,32.
 *   fv_bn_*                  nn.SyncBatchNorm train/eval (modules.py:19; logger.py:55).
 *   fv_reparam_*             flatten_vae_nl split + reparameterisation (models.py:559-561).
 *   fv_kl_*                  KLDivergenceLoss (losses.py:385-393).
 *   fv_mse_*                 ReconLoss / nn.MSELoss (losses.py:396-403).
 *   fv_l1_*                  PerceptualLoss pixel term nn.L1Loss (losses.py:128,135).
 *   fv_conv3d_*             nn.Conv3d of ResBlock3D (modules.py:52-56,133-135; AFE models.py:935).
 *   fv_grid_sample3d_*, fv_occlusion_*, fv_sparse_motion_*, fv_heatmap_*, fv_motion_mask_*
 *                            warp path: models.py:1076-1078,1103,1106; utils.py:123-179.
 *   fv_adam_step             torch.optim.Adam(lr, betas=(0.5,0.999)) (logger.py:60-61).
 *   fv_comm_*                distributed.py:24-31 init_process_group("nccl") + DDP's
 *                            gradient all-reduce (logger.py:55,58) + SyncBN collectives.
 */
#ifndef FACEVAE_H
#define FACEVAE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FV_ABI_VERSION 2

enum fv_status {
  FV_OK = 0,
  FV_E_BADARG = 1001,
  FV_E_UNSUPPORTED = 1002,
  FV_E_COMM = 1003
};

enum fv_dtype { FV_F32 = 0, FV_BF16 = 1, FV_F64 = 2 };

int fv_abi_version(void);
const char* fv_last_error(void);

/* ---------------------------------------------------------------- convolution ---- */
typedef struct fv_conv_desc {
  int dtype;         /* FV_F32 (exact fp32 MFMA) or FV_BF16 (bf16 MFMA, fp32 accumulate) */
  int n, h, w;       /* output spatial size (== conv input size unless upsample) */
  int cin;           /* channel stride of x: power of two >= 8 (zero padded channels) */
  int cin_valid;     /* real input channels (<= cin) */
  int cout;          /* valid output channels */
  int ldy;           /* channel stride of y and res (>= cout; ignored for out_nchw_f32) */
  int ksize;         /* 1, 3 or 7; stride 1, padding ksize/2 */
  int upsample;      /* 1: x is (h/2, w/2), nearest x2 upsample folded into addressing */
  int pro_act;       /* 1: conv input is act(x*scale[c]+shift[c]) (BN-apply + act) */
  float pro_slope;   /* act slope for negatives: 0 = ReLU, 0.2 = LeakyReLU */
  int epi_sigmoid;   /* 1: y = sigmoid(conv + bias [+ res]) */
  int out_nchw_f32;  /* 1: store y as NCHW fp32 [n][cout][h][w] */
} fv_conv_desc;

/* elements of the kernel-layout weight buffers (wk for fwd, wt for bwd-data) */
size_t fv_conv_wk_elems(const fv_conv_desc* d);
size_t fv_conv_wt_elems(const fv_conv_desc* d);
/* number of BN partial records written by fv_conv2d_fwd (stats: [records][2][cout], each
 * (sum, sum of squares) over `block_pixels` consecutive output pixels, the last one short) */
int fv_conv2d_stats_blocks(const fv_conv_desc* d);
int fv_conv2d_stats_block_pixels(const fv_conv_desc* d);

/* w_param [cout][cin_valid][k][k] fp32 -> wk [rows][Kpad], wt [rows_t][Kpad_t] (either may be
 * NULL), both scaled by 1/sigma[0] when sigma != NULL (spectral norm), dtype d->dtype. */
int fv_conv_weight_prep(const fv_conv_desc* d, const float* w_param, const float* sigma,
                        void* wk, void* wt, void* stream);
/* The same for n convs in ONE launch (the generic layouts only: fv_conv_weight_prep_batchable(d)
 * != 0; all descriptors of one dtype, n <= FV_WPREP_MAX): descs is an array of n descriptors,
 * w_params / sigmas / wks / wts arrays of n pointers (sigma, wt entries may be NULL). */
#define FV_WPREP_MAX 24
int fv_conv_weight_prep_batchable(const fv_conv_desc* d);
int fv_conv_weight_prep_multi(int n, const fv_conv_desc* descs, const float* const* w_params,
                              const float* const* sigmas, void* const* wks, void* const* wts, void* stream);

/* y = epi(conv(pro(x), wk) + bias [+ res]); stats (optional) receives per-record
 * (sum, sum of squares) of the pre-sigmoid output per channel. */
int fv_conv2d_fwd(const fv_conv_desc* d, const void* x, const void* wk, const float* bias,
                  const float* pro_scale, const float* pro_shift, const void* res, void* y,
                  float* stats, void* stream);

/* dx[n][h'][w'][cin] = conv_transpose(dy, w) at the conv INPUT resolution of `d` with
 * upsample == 0 (dgrad at the upsampled resolution when d->upsample; see
 * fv_upsample2x_bwd).  dy has channel stride ldy_dy (>= cout, multiple of 8). */
int fv_conv2d_bwd_data(const fv_conv_desc* d, const void* dy, int ldy_dy, const void* wt,
                       void* dx, void* stream);
/* 1 when, for this upsample descriptor, fv_conv2d_bwd_data writes dx directly at the LOW
 * (conv input, h/2 x w/2) resolution -- the gradient of the upsample's input, computed as a
 * stride-2 4x4 conv over dy -- and wt (fv_conv_wt_elems / fv_conv_weight_prep) holds those
 * 4x4 weights; then no fv_upsample2x_bwd follows.  0 otherwise. */
int fv_conv2d_dgrad_lowres(const fv_conv_desc* d);

/* weight gradient w.r.t. the effective (post-SN) weight, split over pixels:
 * slab [nsplit][rows][Kpad] fp32 and bias slab [nsplit][rows] fp32 (sizes from the queries). */
int fv_conv2d_wgrad_nsplit(const fv_conv_desc* d);
size_t fv_conv2d_wgrad_slab_elems(const fv_conv_desc* d);
size_t fv_conv2d_wgrad_bias_slab_elems(const fv_conv_desc* d);
int fv_conv2d_bwd_weight(const fv_conv_desc* d, const void* x, const float* pro_scale,
                         const float* pro_shift, const void* dy, int ldy_dy, float* slab,
                         float* bias_slab, void* stream);
/* reduce the slabs into dw_param [cout][cin_valid][k][k] (fp32, reference layout) and
 * db [cout] (db may be NULL).  The slab contents are scratch afterwards: the reduce may use
 * them for its partial sums. */
int fv_conv2d_wgrad_reduce(const fv_conv_desc* d, const float* slab, const float* bias_slab,
                           float* dw_param, float* db, void* stream);

/* store-pass reductions of the halo-staged 3x3 kernels (fused into the bf16 store of the
 * output tile; one record per 256-pixel tile and wave, [records][2][cout] fp32):
 *   mode 1 (fv_conv2d_fwd_sr): (sum, sum of squares) of the stored output AFTER the residual
 *          add -- the statistics of the next BatchNorm (ResBlock2D's x + t feeding the next
 *          block's NAC, modules.py:125 -> 13);
 *   mode 2 (fv_conv2d_bwd_data_sr): the SyncBatchNorm backward sums (sum g, sum g * yhat) of
 *          the BN whose output gradient the data gradient produces: g = dx * act'(gamma * yhat
 *          + beta), yhat = (bn_input - mean) * invstd (replaces fv_bn_act_bwd_reduce's pass).
 * fv_conv2d_sr_records (dgrad = 1 for the data gradient of d) gives the record count, 0 when
 * the launch path of d has no store-pass records (then use the separate passes). */
typedef struct fv_store_reduce {
  int mode;                /* 1 or 2 */
  float* records;          /* [records][2][cout] */
  const void* bn_input;    /* mode 2: the BN input y, NHWC like the output */
  const float *mean, *invstd, *gamma, *beta;
  float slope;             /* act slope (0 ReLU, 0.2 LeakyReLU) */
} fv_store_reduce;
int fv_conv2d_sr_records(const fv_conv_desc* d, int dgrad, int* record_pixels);
int fv_conv2d_fwd_sr(const fv_conv_desc* d, const void* x, const void* wk, const float* bias, const void* res, void* y,
                     const fv_store_reduce* sr, void* stream);
int fv_conv2d_bwd_data_sr(const fv_conv_desc* d, const void* dy, int ldy_dy, const void* wt, void* dx,
                          const fv_store_reduce* sr, void* stream);
/* BN backward from store-pass records: dgamma / dbeta (either may be NULL) and k [2][c] over
 * `count` elements (fv_bn_bwd_finalize's outputs); red (optional, [2][c] doubles) receives the
 * rank-local sums for a SyncBN all-reduce, then k comes from fv_bn_bwd_finalize_dev. */
int fv_bn_bwd_from_records(const float* records, int nrec, int record_pixels, long pixels, int c, long count,
                           float* dgamma, float* dbeta, float* k, double* red, void* ws, void* stream);

/* ------------------------------------------- transposed conv (k4, s2, p1) ---- */
/* ConvTranspose2dELR (models_utils.py:404-516; F.conv_transpose2d at :497-498) with
 * kernel 4, stride 2, padding 1, run as the sub-pixel phases of an upsample descriptor:
 * d->upsample = 1, d->ksize = 3, d->h/w = OUTPUT size, cin/cout = the module's inch/outch.
 * Forward = fv_conv2d_fwd(d, x, wk, bias, ...); data gradient = fv_conv2d_bwd_data(d, dy,
 * ldy, wt, dx) (dx at the input resolution); weight gradient = fv_conv2d_bwd_weight(d, ...)
 * then fv_convt_wgrad_reduce.  w is the module parameter [cin][cout][4][4] fp32; the
 * effective weight is gain * w, normalised per output channel over dims [0,2,3]
 * (F.normalize, eps 1e-12: models_utils.py:461-470) when demod; inv [cout] receives
 * 1/max(norm, eps) and is read back by the weight-gradient reduce.  bf16 only. */
int fv_convt_supported(const fv_conv_desc* d);
int fv_convt_weight_prep(const fv_conv_desc* d, const float* w, int demod, float gain, float* inv,
                         void* wk, void* wt, void* stream);
/* slabs of fv_conv2d_bwd_weight(d, ...) -> dw [cin][cout][4][4] = dL/dw (through gain and
 * demod) and db [cout] (may be NULL). */
int fv_convt_wgrad_reduce(const fv_conv_desc* d, const float* slab, const float* bias_slab,
                          const float* w, int demod, float gain, const float* inv, float* dw,
                          float* db, void* stream);

/* any geometry / fp32 (convt.hip, direct kernels; NHWC, x channel stride ldx, out stride ldy):
 * W_eff = gain * W [/ max(||W[:, o, :, :]||, 1e-12) when demod] -> we [cin][cout][k][k] fp32
 * (inv [cout] receives the inverse norms); out = conv_transpose2d(x, W_eff, stride, pad) + bias;
 * the data gradient; g = dL/dW_eff (+ db); fv_convt_weight_grad turns g into dL/dW in place. */
int fv_convt_eff_weight(const float* w, int cin, int cout, int k, int demod, float gain, float* inv, float* we,
                        void* stream);
int fv_convt_weight_grad(const float* w, int cin, int cout, int k, int demod, float gain, const float* inv, float* g,
                         void* stream);
int fv_convt_direct_fwd(int dtype, const void* x, int n, int hi, int wi, int cin, int ldx, const float* we,
                        const float* bias, int cout, int ldy, int k, int stride, int pad, void* y, void* stream);
int fv_convt_direct_dgrad(int dtype, const void* dy, int n, int hi, int wi, int cin, int ldx, const float* we,
                          int cout, int ldy, int k, int stride, int pad, void* dx, void* stream);
int fv_convt_direct_wgrad(int dtype, const void* x, const void* dy, int n, int hi, int wi, int cin, int ldx, int cout,
                          int ldy, int k, int stride, int pad, float* g, float* db, void* stream);
/* per-sample channel affine y[n][p][c] = x[n][p][c] * sa[n][c] (+ sb[n][c]) (the weight
 * modulation x * (affine(w) * 0.1 + 1) and the per-sample demodulation of
 * models_utils.py:486-495, moved onto the activations) and its backward (dx may be NULL) */
int fv_chan_scale_fwd(int dtype, const void* x, int n, long hw, int c, int ld, const float* sa, const float* sb,
                      void* y, void* stream);
int fv_chan_scale_bwd(int dtype, const void* g, const void* x, int n, long hw, int c, int ld, const float* sa, void* dx,
                      float* da, float* db, void* stream);

/* ------------------------------------------------- fp8 conv path (config C5) ---- */
/* OCP e4m3 operands with per-tensor power-of-two scales: a tensor v is stored as
 * fp8(v * s), s = 2^floor(log2(448 / amax|v|)), with dq = 1 / s (a device float) beside it.
 * fv_conv2d_fwd_fp8 / fv_conv2d_bwd_data_fp8 are the forward and data gradient of a 3x3 conv
 * (fv_conv2d_fp8_supported: channel counts multiples of 128, w % 64 == 0, h % 4 == 0) on
 * v_mfma_scale_f32_16x16x128_f8f6f4 with fp32 accumulation, the epilogue multiplying by
 * dq_x * dq_w; output bf16 NHWC as fv_conv2d_fwd (bias, residual, BN partials alike).  They
 * replace the same F.conv2d calls as fv_conv2d_fwd / fv_conv2d_bwd_data (modules.py:32). */
size_t fv_fp8_ws_bytes(void);
/* y[i] = fp8(x[i] * s) for count elements (bf16 or f32 input), dq[0] = 1 / s */
int fv_quantize_fp8(int dtype_in, const void* x, long count, uint8_t* y, float* dq, void* ws,
                    void* stream);
int fv_conv2d_fp8_supported(const fv_conv_desc* d);
size_t fv_conv_fp8_wk_bytes(const fv_conv_desc* d);
size_t fv_conv_fp8_wt_bytes(const fv_conv_desc* d);
/* w_param [cout][cin][3][3] fp32 (/ sigma when given) -> wk [cout][9 cin] and/or the
 * transposed, flipped wt [cin][9 cout] (k = tap * channels + c), one scale: dq[0] */
int fv_conv_weight_prep_fp8(const fv_conv_desc* d, const float* w_param, const float* sigma,
                            uint8_t* wk, uint8_t* wt, float* dq, void* ws, void* stream);
/* fv_conv_weight_prep_fp8 for n <= FV_WPREP_MAX convs in two launches (the per-step weight
 * quantization of an fp8 model): arrays of n descriptors / pointers as fv_conv_weight_prep_multi
 * (wts[i] may be NULL), dqs[i] one float each; ws = n * fv_fp8_ws_bytes() bytes.  Bit-identical
 * to n fv_conv_weight_prep_fp8 calls. */
int fv_conv_weight_prep_fp8_multi(int n, const fv_conv_desc* descs, const float* const* w_params,
                                  const float* const* sigmas, uint8_t* const* wks, uint8_t* const* wts,
                                  float* const* dqs, void* ws, void* stream);
int fv_conv2d_fwd_fp8(const fv_conv_desc* d, const uint8_t* x8, const float* x_dq, const uint8_t* wk,
                      const float* w_dq, const float* bias, const void* res, void* y, float* stats,
                      void* stream);
/* BN partial records written by fv_conv2d_fwd_fp8 (as fv_conv2d_stats_blocks / _pixels) */
int fv_conv2d_fp8_stats_blocks(const fv_conv_desc* d);
int fv_conv2d_fp8_stats_block_pixels(const fv_conv_desc* d);
/* dx [n][h][w][cin] bf16 from dy8 [n][h][w][cout] fp8 and wt */
int fv_conv2d_bwd_data_fp8(const fv_conv_desc* d, const uint8_t* dy8, const float* dy_dq,
                           const uint8_t* wt, const float* wt_dq, void* dx, void* stream);
/* Delayed scaling (the product path): a "site" (fv_fp8_site_bytes, zero-initialised device
 * memory, one per conv operand: activation or output gradient) keeps a 16-deep amax history.
 * fv_quantize_fp8_site quantizes in ONE pass with s from max(history) (saturating at +-448)
 * and records the call's amax; seeded = 0 (the site's first call) quantizes exactly
 * (amax pass + quantize pass) and fills the history.  The *_site convs read dq from the site
 * and move the recorded amax into the history (so a site's calls must alternate quantize ->
 * conv, in stream order).  Replaces the per-call amax pass of fv_quantize_fp8. */
size_t fv_fp8_site_bytes(void);
int fv_quantize_fp8_site(int dtype_in, const void* x, long count, uint8_t* y, void* site, int seeded,
                         void* ws, void* stream);
int fv_conv2d_fwd_fp8_site(const fv_conv_desc* d, const uint8_t* x8, void* site, const uint8_t* wk,
                           const float* w_dq, const float* bias, const void* res, void* y, float* stats,
                           void* stream);
/* fv_conv2d_fwd_fp8_site + the store-pass reduction of fv_conv2d_fwd_sr (mode 1 only: the
 * (sum, sum of squares) of the stored, residual-added output, in the records
 * fv_conv2d_sr_records(d, 0, ...) sizes) */
int fv_conv2d_fwd_fp8_site_sr(const fv_conv_desc* d, const uint8_t* x8, void* site, const uint8_t* wk,
                              const float* w_dq, const float* bias, const void* res, void* y,
                              const fv_store_reduce* sr, void* stream);
int fv_conv2d_bwd_data_fp8_site(const fv_conv_desc* d, const uint8_t* dy8, void* site, const uint8_t* wt,
                                const float* wt_dq, void* dx, void* stream);
/* Data-parallel global scaling (BASELINE config C5 at N > 1; the fp8 counterpart of SyncBN's
 * global statistics, modules.py:120-121 under logger.py:54-58): with the deferred roll on, the
 * *_site convs leave each call's amax in its site; once per step the caller gathers every
 * site's in-flight amax (fv_fp8_sites_inflight, `sites` = device array of site pointers),
 * all-reduces it with MAX (fv_comm_allreduce op 2) and rolls all sites at once
 * (fv_fp8_sites_roll), so every rank quantizes with the same scales.  A site's first call
 * takes the exact amax (fv_fp8_amax), all-reduced, as its seed (fv_fp8_site_seed) and then
 * quantizes as a seeded site.  Process-wide switch. */
int fv_fp8_set_deferred_roll(int on);
int fv_fp8_amax(int dtype_in, const void* x, long count, float* amax, void* ws, void* stream);
int fv_fp8_site_seed(void* site, const float* amax, void* stream);
int fv_fp8_sites_inflight(int n, const uint64_t* sites, float* amax, void* stream);
int fv_fp8_sites_roll(int n, const uint64_t* sites, const float* amax, void* stream);
/* fp8 weight gradient of a 3x3 conv (k = (tap, ci), pixel-pair MFMA K = 128) from the e4m3 copies
 * of its input (x8, dequantisation factor x_dq) and output gradient (dy8, dy_dq) -- the operands
 * the fp8 forward and data gradient consumed: slab / bias slab sized by fv_conv2d_wgrad_slab_elems,
 * reduced by fv_conv2d_wgrad_fp8_reduce.  Supported when
 * fv_conv2d_wgrad_fp8_supported(d) (128-multiple channels, the sliding-row plan). */
int fv_conv2d_wgrad_fp8_supported(const fv_conv_desc* d);
int fv_conv2d_bwd_weight_fp8(const fv_conv_desc* d, const uint8_t* x8, const float* x_dq, const uint8_t* dy8,
                             const float* dy_dq, float* slab, float* bias_slab, void* stream);
/* reduce of fv_conv2d_bwd_weight_fp8's slabs -> dw (param layout) [+ db]: the fp8 weight
 * gradient splits a batch over fewer slabs than the bf16 plan (images per split chosen for
 * about 512 blocks), so its slabs are summed by this entry, not fv_conv2d_wgrad_reduce */
int fv_conv2d_wgrad_fp8_reduce(const fv_conv_desc* d, const float* slab, const float* bias_slab, float* dw_param,
                               float* db, void* stream);
/* layout probe: c[16][16] = a[16][128] . b[16][128]^T through one scaled fp8 MFMA tile */
int fv_fp8_mfma_probe(const uint8_t* a, const uint8_t* b, float* c, void* stream);
/* test probe: 64 lanes each read 8 bytes by ds_read_b64_tr_b8 at LDS byte offset lane_addr[lane]
 * (< 4088, 8-aligned) of a 4 KB LDS image holding byte i = i & 255; out [64][2] ints */
int fv_tr8_probe(const int* lane_addr, int* out, void* stream);

/* ------------------------------------------------ 3x3x3 conv (AFE ResBlock3D) ---- */
/* nn.Conv3d(cin, cout, 3, 1, 1) of ConvBlock3D / ResBlock3D (modules.py:52-56, 133-135) in the
 * AFE trunk (models.py:935, 943-944).  Activations NDHWC ([n][d][h][w][c], torch
 * channels_last_3d), weights in the reference layout [cout][cin][3][3][3] fp32, re-laid out
 * per forward by fv_conv3d_weight_prep (wk: forward, wt: data gradient; fv_conv3d_wk_bytes
 * each).  bf16 with cin = cout = 32 and w = 64 runs the MFMA kernels (BN partials available:
 * fv_conv3d_stats_blocks > 0); any other shape, and fp32 (parity mode), the direct kernels. */
typedef struct fv_conv3d_desc {
  int dtype;         /* FV_F32 or FV_BF16 */
  int n, d, h, w;    /* spatial size (stride 1, padding 1: output == input) */
  int cin, cout;     /* channels (dense, channel stride == count) */
} fv_conv3d_desc;
size_t fv_conv3d_wk_bytes(const fv_conv3d_desc* d);
int fv_conv3d_weight_prep(const fv_conv3d_desc* d, const float* w_param, void* wk, void* wt, void* stream);
/* fv_conv3d_weight_prep of n convs of one shape in one launch (host pointer tables; wk[i] / wt[i]
 * may be NULL) */
int fv_conv3d_weight_prep_multi(const fv_conv3d_desc* d, int n, const float* const* w_param, void* const* wk,
                                void* const* wt, void* stream);
/* BN partial records ([records][2][cout] (sum, sum of squares), block_pixels voxels each) that
 * fv_conv3d_fwd writes when stats != NULL; 0 = not available for this shape */
int fv_conv3d_stats_blocks(const fv_conv3d_desc* d);
int fv_conv3d_stats_block_pixels(const fv_conv3d_desc* d);
/* y = conv3d(x, wk) + bias [+ res] */
int fv_conv3d_fwd(const fv_conv3d_desc* d, const void* x, const void* wk, const float* bias, const void* res,
                  void* y, float* stats, void* stream);
/* dx [n][d][h][w][cin] from dy [n][d][h][w][cout] and wt */
int fv_conv3d_bwd_data(const fv_conv3d_desc* d, const void* dy, const void* wt, void* dx, void* stream);
/* dw [cout][cin][3][3][3] fp32 and db [cout] (may be NULL), deterministic; ws of
 * fv_conv3d_wgrad_ws_bytes bytes (0 = none needed) */
size_t fv_conv3d_wgrad_ws_bytes(const fv_conv3d_desc* d);
int fv_conv3d_bwd_weight(const fv_conv3d_desc* d, const void* x, const void* dy, float* dw, float* db, void* ws,
                         void* stream);
/* AFE.forward's x.view(N, C, D, H, W) of the mid_conv output (models.py:941-942) between the
 * build's layouts: src NHWC [n][hw][c*d_count] -> dst NDHWC [n][d][hw][c] (inverse = 0), or back
 * (inverse = 1: src NDHWC, dst NHWC) */
int fv_depth_split(int dtype, const void* src, int n, int hw, int c, int d_count, int inverse, void* dst,
                   void* stream);

/* ------------------------------------------------------- warp path (Generator / MFE) ---- */
/* F.grid_sample(in, grid, mode="bilinear" (trilinear), padding_mode="zeros",
 * align_corners=True) for 5-D input (models.py:1103; utils.py:175): in NDHWC [B/group][Di][Hi][Wi][C],
 * grid [B][Do][Ho][Wo][3] fp32 (x -> W, y -> H, z -> D), out NDHWC [B][Do][Ho][Wo][C]; output
 * batch b samples input batch b / group (group = K + 1 for create_deformed_source_image's
 * repeat, utils.py:168-172).  dtype FV_F32 / FV_BF16 for in / out / gout. */
int fv_grid_sample3d_fwd(int dtype, const void* in, const float* grid, int B, int Di, int Hi, int Wi, int Do,
                         int Ho, int Wo, int C, int group, void* out, void* stream);
/* gin (fp32, input layout, zeroed by the caller; float atomics) += dL/din, ggrid = dL/dgrid;
 * either may be NULL */
int fv_grid_sample3d_bwd(int dtype, const void* in, const float* grid, const void* gout, int B, int Di, int Hi,
                         int Wi, int Do, int Ho, int Wo, int C, int group, float* gin, float* ggrid, void* stream);
/* gin (dtype, input layout, every element written) = dL/din without float atomics: the output
 * voxels are bucketed by their base input cell (count, scan, fill in ws), each bucket is ordered
 * by voxel index, and each input cell sums the buckets whose corner it is (bit-reproducible).
 * ws: fv_grid_sample3d_bwd_input_ws_bytes bytes = 4 B per input cell key + 24 B per OUTPUT voxel
 * (key/rank + record): for create_deformed_source_image (group K+1, B = N (K+1) grids) at N = 8,
 * K = 15, 16x64x64 that is ~200 MB per backward. */
size_t fv_grid_sample3d_bwd_input_ws_bytes(int B, int Di, int Hi, int Wi, int Do, int Ho, int Wo, int group);
int fv_grid_sample3d_bwd_input(int dtype, const float* grid, const void* gout, int B, int Di, int Hi, int Wi, int Do,
                               int Ho, int Wo, int C, int group, void* gin, void* ws, void* stream);
int fv_f32_to(int dtype, const float* a, void* b, long n, void* stream);
/* fs * occlusion (models.py:1106): x [P][C] NHWC, occ [P] fp32; backward dx = g*occ (may be
 * NULL), docc[p] = sum_c g x (may be NULL) */
int fv_occlusion_fwd(int dtype, const void* x, const float* occ, long P, int C, void* y, void* stream);
int fv_occlusion_bwd(int dtype, const void* g, const void* x, const float* occ, long P, int C, void* dx, float* docc,
                     void* stream);
/* create_sparse_motions (utils.py:139-152) with J = Rs inv(Rd) [N][3][3]: out [N][K+1][D][H][W][3] */
int fv_sparse_motion_fwd(const float* kp_s, const float* kp_d, const float* J, int N, int K, int D, int H, int W,
                         float* out, void* stream);
/* backward sums [N][K][12] = (sum_v g_k, sum_v g_k (id - kp_d[k])^T) of the motion gradient g */
int fv_sparse_motion_bwd(const float* g, const float* kp_d, int N, int K, int D, int H, int W, float* sums,
                         void* stream);
/* create_heatmap_representations (utils.py:130-137, kp2gaussian_3d 123-129): out [N][K+1][D][H][W] */
int fv_heatmap_fwd(const float* kp_s, const float* kp_d, int N, int K, int D, int H, int W, float var, float* out,
                   void* stream);
int fv_heatmap_bwd(const float* g, const float* kp_s, const float* kp_d, int N, int K, int D, int H, int W, float var,
                   float* dkp_s, float* dkp_d, void* stream);
/* MFE mask softmax + deformation (models.py:1076-1078): prob = softmax over K1 of logits
 * [N][K1][V]; def [N][V][3] = sum_k prob_k sm[N][K1][V][3] */
int fv_motion_mask_fwd(const float* logits, const float* sm, int N, int K1, long V, float* prob, float* def,
                       void* stream);
int fv_motion_mask_bwd(const float* prob, const float* sm, const float* gdef, const float* gprob, int N, int K1,
                       long V, float* dlogits, float* dsm, void* stream);

/* ------------------------------------------------------------ perceptual loss ---- */
/* The VGG feature stacks of PerceptualLoss (losses.py:33-151) run their convs on
 * fv_conv2d_fwd / fv_conv2d_bwd_data and their per-channel normalisations
 * (apply_imagenet_normalization / apply_vggface_normalization, utils.py:182-193) and the
 * 0.5x bilinear downscale (== 2x2 average on even sizes, losses.py:148-149) on fv_bn_act_fwd
 * (slope 1 = identity, scale/shift = the affine, pool = the average).  The rest: */
int fv_relu_bwd(int dtype, const void* g, const void* y, long n, void* dx, void* stream);
int fv_maxpool2_fwd(int dtype, const void* x, int n, int h, int w, int c, void* y, void* stream);
int fv_maxpool2_bwd(int dtype, const void* x, const void* g, int n, int h, int w, int c, void* dx, void* stream);
int fv_avgpool2_bwd(int dtype, const void* g, int n, int h, int w, int c, void* dx, void* stream);
/* nn.L1Loss over bf16 / f32 operands (criterion of losses.py:127, 142-151) */
size_t fv_l1t_ws_bytes(void);
int fv_l1t_fwd(int dtype, const void* a, const void* b, long n, float* loss, void* ws, void* stream);
int fv_l1t_bwd(int dtype, const void* a, const void* b, long n, const float* gout, float scale, void* da,
               void* stream);

/* ------------------------------------------------------------- spectral norm ---- */
size_t fv_spectral_norm_ws_bytes(int rows, int cols);
/* one power iteration (u, v updated in place) when power_iter, then sigma = u.(W v) */
int fv_spectral_norm_fwd(const float* w, int rows, int cols, float* u, float* v, float* sigma,
                         int power_iter, void* ws, void* stream);
/* g_orig = g_sn/sigma - <g_sn, w>/sigma^2 * u v^T   (in place allowed: g_orig == g_sn) */
int fv_spectral_norm_bwd(const float* w, const float* g_sn, int rows, int cols, const float* u,
                         const float* v, const float* sigma, float* g_orig, void* ws,
                         void* stream);

/* batched form for all spectral-normed convs of a model (4 launches).  The caller builds
 * the table once on the host (fv_spectral_norm_batch_build writes it into table_host, which
 * the caller copies to device memory of fv_spectral_norm_batch_table_bytes) and keeps the
 * workspace (fv_spectral_norm_batch_ws_floats floats) alive.  usnap/vsnap receive the u, v
 * used for sigma (what the backward needs). */
typedef struct fv_sn_layer {
  const float* w;
  float* u;
  float* v;
  float* sigma;
  float* usnap;
  float* vsnap;
  int rows, cols;
} fv_sn_layer;
size_t fv_spectral_norm_batch_ws_floats(const fv_sn_layer* layers, int nlayers);
size_t fv_spectral_norm_batch_table_bytes(int nlayers);
int fv_spectral_norm_batch_build(const fv_sn_layer* layers, int nlayers, float* ws, void* table_host,
                                 int* nblocks3);
int fv_spectral_norm_fwd_batch(const void* table_dev, int nlayers, const int* nblocks3, int power_iter,
                               void* stream);

/* ---------------------------------------------------------------- batch norm ---- */
size_t fv_bn_ws_bytes(int c);
/* Conv-record folds (fv_bn_*_partials, fv_bn_bwd_from_records) run in ONE launch: level 1
 * chunk partials + level 2 by each 16-channel group's last-arriving block (bn.hip
 * fold16_part_kernel: sc1 stores, arrival tickets in a per-device pool; bit-reproducible). */
/* (count, sum, centred-M2) conv partials -> stats [3][c] doubles (count, sum, sumsq) */
int fv_bn_stats_from_partials(const float* partials, int nblocks, int block_pixels,
                              long total_pixels, int c, double* stats, void* ws, void* stream);
/* statistics of an NHWC tensor (pixels x c, channel stride ldc) -> stats [3][c] */
int fv_bn_stats_tensor(int dtype, const void* x, long pixels, int c, int ldc, double* stats,
                       void* ws, void* stream);
/* mean/var from stats (already all-reduced for SyncBN) -> save_mean, save_invstd and the
 * fused affine scale = gamma*invstd, shift = beta - mean*scale; running stats updated
 * with momentum and the unbiased variance when training.  In eval mode the running
 * statistics are used and stats may be NULL. */
int fv_bn_finalize(const double* stats, int c, const float* gamma, const float* beta, float eps,
                   float momentum, int training, float* running_mean, float* running_var,
                   long long* num_batches_tracked, float* save_mean, float* save_invstd, float* scale,
                   float* shift, void* stream);
/* single-process training forms (no SyncBN exchange between the statistics and finalize):
 * statistics + finalize (+ num_batches_tracked += 1) in one launch (two for a tensor) */
int fv_bn_stats_finalize_partials(const float* partials, int nblocks, int block_pixels, long total_pixels,
                                  int c, const float* gamma, const float* beta, float eps, float momentum,
                                  float* running_mean, float* running_var, long long* num_batches_tracked,
                                  float* save_mean, float* save_invstd, float* scale, float* shift,
                                  void* ws, void* stream);
int fv_bn_stats_finalize_tensor(int dtype, const void* x, long pixels, int c, int ldc, const float* gamma,
                                const float* beta, float eps, float momentum, float* running_mean,
                                float* running_var, long long* num_batches_tracked, float* save_mean,
                                float* save_invstd, float* scale, float* shift, void* ws, void* stream);
/* out = [avgpool2](act(y*scale + shift)); y [n][h][w][ldc], out [n][h/p][w/p][c] */
int fv_bn_act_fwd(int dtype, const void* y, int n, int h, int w, int c, int ldc,
                  const float* scale, const float* shift, float slope, int pool, void* out,
                  void* stream);
/* sums over pixels of g and g*yhat with g = dout_full * act'(.) -> red [2][c] doubles */
int fv_bn_act_bwd_reduce(int dtype, const void* dout, const void* y, int n, int h, int w, int c,
                         int ldc, const float* mean, const float* invstd, const float* gamma,
                         const float* beta, float slope, int pool, double* red, void* ws,
                         void* stream);
/* dgamma/dbeta and the two BN-backward coefficients k [2][c] = red / count (k may be NULL:
 * dgamma/dbeta only; dgamma/dbeta may be NULL) */
int fv_bn_bwd_finalize(const double* red, int c, long count, float* dgamma, float* dbeta,
                       float* k, void* stream);
/* the same with the element count read per channel from device memory (row 0 of the
 * all-reduced [3][c] statistics record: the global count, also for uneven per-rank batches) */
int fv_bn_bwd_finalize_dev(const double* red, int c, const double* count, float* dgamma,
                           float* dbeta, float* k, void* stream);
/* single-process form of fv_bn_act_bwd_reduce + fv_bn_bwd_finalize (two launches) */
int fv_bn_act_bwd_reduce_finalize(int dtype, const void* dout, const void* y, int n, int h, int w, int c,
                                  int ldc, const float* mean, const float* invstd, const float* gamma,
                                  const float* beta, float slope, int pool, long count, float* dgamma,
                                  float* dbeta, float* k, void* ws, void* stream);
/* dx = gamma*invstd*(g - k0 - yhat*k1) [+ addend]; dx/addend [n][h][w][ldc] */
int fv_bn_act_bwd_apply(int dtype, const void* dout, const void* y, int n, int h, int w, int c,
                        int ldc, const float* mean, const float* invstd, const float* gamma,
                        const float* beta, float slope, int pool, const float* k,
                        const void* addend, void* dx, void* stream);
/* the same two passes (no pool, ldc == c) also writing an e4m3 copy of their output for an fp8
 * conv that consumes it: out8 / dx8 [n][h][w][c] bytes = the bf16 output quantized with the
 * delayed scale of `site` (the consumer's fv_fp8_site_bytes site, already seeded), bit-identical
 * to fv_quantize_fp8_site over the output; the site's in-flight amax and dq are updated the
 * same way.  Replaces the separate quantize pass (one read of the output).  out / dx may be NULL:
 * then only the e4m3 copy is written (its values are still the bf16-rounded outputs) -- for a
 * consumer whose forward, data gradient and weight gradient all run on the e4m3 operands. */
int fv_bn_act_fwd_q8(int dtype, const void* y, int n, int h, int w, int c, const float* scale,
                     const float* shift, float slope, void* out, void* out8, void* site, void* stream);
int fv_bn_act_bwd_apply_q8(int dtype, const void* dout, const void* y, int n, int h, int w, int c,
                           const float* mean, const float* invstd, const float* gamma,
                           const float* beta, float slope, const float* k, const void* addend,
                           void* dx, void* dx8, void* site, void* stream);

/* ------------------------------------------------------ elementwise / layout ---- */
int fv_nchw_to_nhwc(int dtype_out, const float* x, int n, int c, int hw, int ldc, void* out,
                    void* stream);
int fv_nhwc_to_nchw(int dtype_in, const void* x, int n, int c, int hw, int ldc, float* out,
                    void* stream);
int fv_cast(int dtype_in, const void* x, int dtype_out, void* y, long count, void* stream);
/* g_src[n][i][j][c] = sum_{a,b} g[n][2i+a][2j+b][c]  (nearest x2 upsample backward) */
int fv_upsample2x_bwd(int dtype, const void* g, int n, int h_src, int w_src, int c, void* out,
                      void* stream);
/* dpre (NHWC, channel stride ldc, zero padded) = dy * y * (1 - y), dy/y NCHW fp32 */
int fv_sigmoid_bwd_to_nhwc(int dtype_out, const float* dy, const float* y, int n, int c, int hw,
                           int ldc, void* dpre, void* stream);

/* --------------------------------------------------------- latent and losses ---- */
size_t fv_loss_ws_bytes(void);
/* h [P][2L] (NHWC, mu = channels [0,L), logstd = [L,2L)); eps NCHW fp32 [n][L][hw];
 * mu/logstd/z [P][L] NHWC */
int fv_reparam_fwd(int dtype, const void* h, const float* eps, int n, int L, int hw, void* mu,
                   void* logstd, void* z, void* stream);
/* the same, also writing the KL mean of (mu, logstd) to kl[0] (KLDivergenceLoss forward,
 * losses.py:392) from the values it already holds; ws of fv_reparam_ws_bytes bytes */
size_t fv_reparam_ws_bytes(int n, int L, int hw);
int fv_reparam_kl_fwd(int dtype, const void* h, const float* eps, int n, int L, int hw, void* mu,
                      void* logstd, void* z, float* kl, void* ws, void* stream);
/* 1 when (L, hw) runs the tiled reparameterisation (hw % 32 == 0, L <= 496): only then may
 * fv_reparam_kl_fwd leave mu/logstd NULL (the caller reads them as channel slices of h) while
 * still reducing the KL */
int fv_reparam_tiled(int L, int hw);
/* dh = [dz + dmu | dz*exp(logstd)*eps + dlogstd]; dz/dmu/dlogstd may be NULL */
int fv_reparam_bwd(int dtype, const void* h, const float* eps, int n, int L, int hw,
                   const void* dz, const void* dmu, const void* dlogstd, void* dh, void* stream);
/* the same plus the KL gradient (KLDivergenceLoss backward, losses.py:392) folded in:
 * kl_grad = device fp32 dLoss/dKL (NULL: none); dh += kl_grad / (n L hw) *
 * [mu | exp(2 logstd) - 1] -- the separate fv_kl_bwd pass and its dmu/dlogstd tensors vanish */
int fv_reparam_kl_bwd(int dtype, const void* h, const float* eps, int n, int L, int hw,
                      const void* dz, const void* dmu, const void* dlogstd, const float* kl_grad,
                      void* dh, void* stream);
int fv_kl_fwd(int dtype, const void* mu, const void* logstd, long count, float* loss, void* ws,
              void* stream);
int fv_kl_bwd(int dtype, const void* mu, const void* logstd, long count, const float* gout,
              void* dmu, void* dlogstd, void* stream);
int fv_mse_fwd(const float* a, const float* b, long count, float* loss, void* ws, void* stream);
int fv_mse_bwd(const float* a, const float* b, long count, const float* gout, float* da,
               float* db, void* stream);
int fv_l1_fwd(const float* a, const float* b, long count, float* loss, void* ws, void* stream);
int fv_l1_bwd(const float* a, const float* b, long count, const float* gout, float* da,
              float* db, void* stream);

/* ----------------------------------------------------------------- optimiser ---- */
typedef struct fv_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  long numel;
} fv_adam_tensor;
#define FV_ADAM_CHUNK 4096
/* multi-tensor Adam (torch.optim.Adam math, no weight decay / amsgrad).  `tensors` is a
 * DEVICE array of descriptors; `blocks` a DEVICE array of nblocks (tensor, chunk) int pairs,
 * one per FV_ADAM_CHUNK elements of each tensor; `step` is the step count after increment. */
int fv_adam_step(const fv_adam_tensor* tensors, const int* blocks, int nblocks, double lr,
                 double beta1, double beta2, double eps, long step, void* stream);
/* The same update with the step count kept on the DEVICE (graph-replayable, as
 * torch.optim.Adam(capturable=True)): one launch increments *step_dev (fp64) and writes the
 * bias-correction coefficients (lr / (1 - beta1^t), sqrt(1 - beta2^t), computed in fp64 as
 * the host path does) to coef_ws (2 floats), the update kernel reads them. */
int fv_adam_step_dev(const fv_adam_tensor* tensors, const int* blocks, int nblocks, double lr,
                     double beta1, double beta2, double eps, double* step_dev, float* coef_ws,
                     void* stream);

/* ------------------------------------------------- batched spectral-norm backward ---- */
/* g <- g / sigma - (<g, w> / sigma^2) u v^T in place for n layers in two launches (the
 * per-layer fv_spectral_norm_bwd is two launches each); ws >= 256 * n floats. */
#define FV_SNB_MAX 24
typedef struct fv_sn_bwd_layer {
  const float* w;
  float* g;
  const float* u;
  const float* v;
  const float* sigma;
  int rows, cols;
} fv_sn_bwd_layer;
int fv_spectral_norm_bwd_multi(int n, const fv_sn_bwd_layer* layers, float* ws, void* stream);

/* ------------------------------------------------------------------ staging ---- */
/* stream-ordered host -> device copy of `bytes` from PINNED host memory (descriptor tables of
 * the batched spectral norm / Adam launches); captured into a HIP graph as a memcpy node. */
int fv_copy_h2d_async(void* dst, const void* src_pinned, size_t bytes, void* stream);

/* ------------------------------------------------------------ communication ---- */
typedef void* fv_comm_t;
int fv_comm_unique_id(uint8_t out[128]);
int fv_comm_init(const uint8_t id[128], int nranks, int rank, int device, fv_comm_t* comm);
/* op: 0 = sum, 1 = average, 2 = max (anything else: FV_E_BADARG); dtype: FV_F32 / FV_BF16 /
 * FV_F64 */
int fv_comm_allreduce(fv_comm_t comm, void* buf, size_t count, int dtype, int op,
                      void* stream);
int fv_comm_allgather(fv_comm_t comm, const void* send, void* recv, size_t count_per_rank,
                      int dtype, void* stream);
int fv_comm_broadcast(fv_comm_t comm, void* buf, size_t count, int dtype, int root,
                      void* stream);
int fv_comm_destroy(fv_comm_t comm);
/* Failure detection (replaces the teardown the reference gets from mp.spawn, train.py:54, and
 * NCCL_ASYNC_ERROR_HANDLING under init_process_group("nccl"), distributed.py:24-31):
 * *result = ncclCommGetAsyncError (0 = success, 7 = in progress; other values also set
 * fv_last_error), host-only, callable from a watchdog thread; fv_comm_count = ncclCommCount;
 * fv_comm_abort = ncclCommAbort (outstanding collectives abandoned, handle freed). */
int fv_comm_async_error(fv_comm_t comm, int* result);
int fv_comm_count(fv_comm_t comm, int* nranks);
int fv_comm_abort(fv_comm_t comm);

#ifdef __cplusplus
}
#endif
#endif /* FACEVAE_H */
