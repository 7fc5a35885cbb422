/*
 * rgbac.h -- C ABI of librgbac_hip.so, the MI355X (gfx950) hot path of the
 * learned RGBA codec (AutoEncoderRGB_Journal / AutoEncoderMask_Journal).
 *
 * The reference is pure Python over PyTorch + compressai and has no FFI of its
 * own: its "operator interface" is the nn.Module forward of the layers listed
 * below.  Each entry point names the reference code it replaces
 * (paths relative to the reference repo root).  The Python host side
 * (rgbac/_lib.py) binds these with ctypes; no torch types cross this boundary.
 *
 * Conventions
 *  - Activations are NHWC with a channel stride ``ldc`` (elements) that is a
 *    multiple of 8; padding channels hold zeros.  Element type is selected per
 *    call: RGBAC_F32 (parity mode) or RGBAC_BF16 (throughput mode); MFMA
 *    accumulation and all epilogue math are fp32 in both.
 *  - All launches are asynchronous on ``stream`` (a hipStream_t passed as
 *    void*).  No entry point allocates device memory, synchronises the host or
 *    keeps state between calls; callers own every buffer (scratch included).
 *  - Return 0 on success, a negative RGBAC_E* code otherwise (shape checks run
 *    before any launch); rgbac_last_error() returns a thread-local message.
 */
#ifndef RGBAC_H_
#define RGBAC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RGBAC_ABI_VERSION 2

enum rgbac_status {
  RGBAC_OK = 0,
  RGBAC_E_ARG = -1,      /* bad pointer / shape / unsupported combination */
  RGBAC_E_DTYPE = -2,    /* unsupported dtype */
  RGBAC_E_LAUNCH = -3,   /* hipLaunch / hipGetLastError failure */
};

enum rgbac_dtype { RGBAC_F32 = 0, RGBAC_BF16 = 1 };

/* Fused epilogue of rgbac_conv2d, applied per output element in fp32:
 *   v = acc + bias[n];  if (res0) v += res0;          (pre-activation add)
 *   v = act(v, res1);   if (res2) v += res2;          (post-activation add)  */
enum rgbac_act {
  RGBAC_ACT_NONE = 0,
  RGBAC_ACT_GELU = 1,      /* exact erf GELU (nn.GELU())                      */
  RGBAC_ACT_RELU = 2,
  RGBAC_ACT_LRELU = 3,     /* LeakyReLU(negative_slope = act_param)            */
  RGBAC_ACT_TANH_HALF = 4, /* res1 + 0.5*tanh(v)   (lrp update)               */
  RGBAC_ACT_GATE = 5,      /* res1 * sigmoid(v)    (then + res2)              */
  RGBAC_ACT_GDN = 6,       /* res1 / sqrt(v)       (use with square_input)     */
  RGBAC_ACT_IGDN = 7,      /* res1 * sqrt(v)                                    */
  RGBAC_ACT_MASKSEL = 8,   /* sel[p] ? v + res1 : res1   (window-drop residual) */
  RGBAC_ACT_GAUSS = 9,     /* output channels are (mu | sigma) of a latent slice:
                              GaussianConditional.forward + ste_round of res1 (= y
                              slice) -> out = round(y-mu)+mu, aux1 = likelihood,
                              partial[m-block] = sum of clamped bits; aux0 = noise
                              (training) or NULL.  One N tile, ksplit 1.          */
  RGBAC_ACT_SQBWD = 10,    /* res0 + 2*res1*acc  (GDN input gradient: dL/dx =
                              dL/dy-direct + 2 x * (gamma'^T dL/dnorm); no bias)  */
  RGBAC_ACT_DGELU = 11,    /* acc * GELU'(res0)  (input gradient of a conv whose
                              input is GELU(res0): the producer's activation
                              backward folded in; bf16: the A&S 7.1.26 derivative
                              of rgbac_act_bwd, f32: exact; no bias, res1, res2) */
  RGBAC_ACT_DLRELU = 12,   /* res0 > 0 ? acc : acc * act_param  (same, (Leaky)ReLU
                              producer: act_param = its slope, 0 for ReLU)        */
};

enum rgbac_conv_mode {
  RGBAC_CONV = 0,          /* nn.Conv2d(k, stride, pad = k/2)                  */
  RGBAC_CONVT_S2 = 1,      /* nn.ConvTranspose2d(k, s=2, p=k/2, op=1), 4 phases */
  RGBAC_SUBPEL2 = 2,       /* conv3x3 + nn.PixelShuffle(2) folded into store   */
};

/* One channel-concatenated input source (torch.cat along dim=1 is never
 * materialised: up to three sources are read in order). */
typedef struct rgbac_src {
  const void* ptr;   /* NHWC base, element type = args.dtype                */
  int64_t ldc;       /* channel stride (elements)                           */
  int32_t channels;  /* channels taken from this source (multiple of 8)     */
  int32_t _pad;
} rgbac_src;

typedef struct rgbac_conv_args {
  int32_t dtype;               /* rgbac_dtype                                     */
  int32_t mode;                /* rgbac_conv_mode                                 */
  int32_t batch, in_h, in_w;   /* input spatial size                              */
  int32_t ksize, stride;       /* kernel size (1,3,5); stride (1,2)               */
  int32_t nsrc;                /* 1..3                                            */
  rgbac_src src[3];
  int32_t cin_pad;             /* sum(src.channels) (multiple of 8)                */
  int32_t k_pad;               /* packed K per output row (mult. of 64)            */
  const void* weight;          /* packed [nphase][cout_pad][k_pad], see rgbac_conv_pack */
  const float* bias;           /* [cout_pad] fp32 (zero padded) or NULL            */
  int32_t cout;                /* real output channels (pre-shuffle for SUBPEL2)  */
  int32_t cout_pad;            /* rows of the packed weight per phase (mult. of 128) */
  int32_t out_h, out_w;        /* stored output spatial size                       */
  void* out; int64_t out_ldc; int32_t out_coff; int32_t act;
  float act_param; int32_t square_input;   /* square the input (GDN norm pool) */
  const void* res0; int64_t res0_ldc;      /* same pixel grid as out          */
  const void* res1; int64_t res1_ldc;
  const void* res2; int64_t res2_ldc;
  const uint8_t* sel;                      /* MASKSEL: per output pixel flag   */
  int32_t tile;                /* tile shape index, 0..rgbac_conv_num_tiles()-1:
                                  0:128x128 1:128x64 2:64x64 3:128x32 4:64x32
                                  5:128x16 6:64x16 (pixels x channels).
                                  Tiles with rgbac_conv_tile_weight_layout(tile) == 1
                                  (42..47, 50..53, 56..58: fragment-streamed patch
                                  tiles; 55: narrow-output patch tile) read
                                  `weight` as the FRAGMENT-MAJOR copy of the pack:
                                  bf16 [nphase][cout_pad/16][ntaps*cin32/32][64][8],
                                  cin32 = round_up(cin_pad, 32), K tap-major with each
                                  tap's channels zero-padded to cin32; lane l of a
                                  (16-row, 32-deep) block holds row l&15, k 8*(l>>4)..+7
                                  (the v_mfma_f32_16x16x32_bf16 A fragment).  The
                                  kernel cannot tell the layouts apart: passing the
                                  plain pack to these tiles gives wrong outputs.   */
  int32_t ksplit;              /* split-K factor (1 = fused epilogue in-kernel)   */
  void* workspace;             /* ksplit>1: fp32 [ksplit][nphase][M][round16(cout)] */
  const float* aux0;           /* GAUSS: fp32 noise [M][cout/2] or NULL            */
  float* aux1;                 /* GAUSS: fp32 likelihood out [M][cout/2] or NULL   */
  double* partial;             /* GAUSS: fp64 bits per M-tile block                */
  void* zout;                  /* training: pre-activation value v (after bias and
                                  res0) stored on the output grid, or NULL         */
  int64_t zout_ldc;            /* channel stride of zout (same coff as out)        */
  int32_t* tile_counters;      /* ksplit>1 on a streaming tile (0..6, 20..26): zero-
                                  initialised int32 tickets, one per (group, phase,
                                  M-tile, N-tile); the last split block of a tile sums
                                  the slabs and runs the epilogue inside the launch and
                                  resets its ticket to 0.  NULL: separate reduce kernels */
} rgbac_conv_args;

int rgbac_abi_version(void);
const char* rgbac_last_error(void);

/* Implicit-GEMM convolution on MFMA with fused epilogue.
 * Replaces nn.Conv2d / nn.ConvTranspose2d / compressai conv3x3 /
 * subpel_conv3x3 and the elementwise ops that follow them in:
 *   layers/TransformRGB.py:55-99 (x1..x4, DSE, EnhancementBlock),
 *   layers/Masked_Attention.py:150-189 (ResidualUnit, conv_a/conv_b, gate),
 *   layers/GDN.py:64-94 (norm pool as 1x1 conv on x^2 + GDN/IGDN epilogue),
 *   models/AutoEncoderRGB_Journal.py:135-198,242-264 (h_a, h_*_s, slice stacks,
 *   lrp tanh update), models/AutoEncoderMask_Journal.py:96-244. */
int rgbac_conv2d(const rgbac_conv_args* args, void* stream);
int rgbac_conv_num_tiles(void);
/* 1 if `tile` reads the fragment-major weight copy (see rgbac_conv_args.tile),
 * 0 for the plain [nphase][cout_pad][k_pad] pack, -1 if out of range. */
int rgbac_conv_tile_weight_layout(int tile);

/* ngroups (1..rgbac_conv_max_groups()) independent convs in one launch.  All
 * groups share dtype, mode, batch, input/output size, ksize, stride, tile,
 * ksplit, act/act_param and square_input; weights, sources (cin may differ),
 * cout, outputs, residuals and workspaces are per group.  Used for the
 * cc_mean/cc_scale stacks (AutoEncoderRGB_Journal.py:240-252), the conv_a /
 * conv_b residual units (Masked_Attention.py:182-189) and h_mean_s/h_scale_s
 * (AutoEncoderRGB_Journal.py:231-232). */
int rgbac_conv2d_grouped(const rgbac_conv_args* args, int ngroups, void* stream);
int rgbac_conv_max_groups(void);

/* rgbac_conv2d_grouped split into its two launches, for per-kernel timing (bench.py's
 * launch profiler): part 1 = the main conv kernel only, part 2 = the split-K reduce +
 * epilogue kernels only (a no-op when ksplit == 1), part 0 = both (== grouped). */
int rgbac_conv2d_grouped_part(const rgbac_conv_args* args, int ngroups, int part, void* stream);

/* Attention core of masked shifted-window MSA on a precomputed qkv tensor
 * (qkv = Linear(C,3C) applied per pixel by rgbac_conv2d).  For every window
 * of the cyclically shifted frame: activity = any(alpha != 0) over the
 * window; active windows compute softmax(q*scale k^T + relpos_bias + shift
 * mask(-100)) v per head and write it back at the un-shifted pixel positions;
 * inactive windows write zeros.  sel[p] receives the activity of the window
 * that pixel p belongs to (consumed by the proj conv's MASKSEL epilogue).
 * Replaces layers/masked_win_attention.py:35-47,96-131,169-251 (masked=1) and
 * layers/win_attention.py:96-115,153-207 (masked=0).
 *   qkv:   NHWC [B,H,W,ldq] (channels s*C + h*d + e)
 *   alpha: fp32 [B,H,W] (ignored when masked == 0)
 *   bias:  fp32 [heads][ws*ws][ws*ws] dense relative-position bias
 *   out:   NHWC [B,H,W,ldo], sel: uint8 [B,H,W] (may be NULL when masked==0) */
int rgbac_winattn_core(int dtype, int batch, int h, int w, int channels,
                       int heads, int ws, int shift, int masked, float scale,
                       const void* qkv, int64_t ldq, const float* alpha,
                       const float* bias, void* out, int64_t ldo, uint8_t* sel,
                       void* stream);
/* The same with (a) an explicit additive mask, fp32 [amask_nw][ws*ws][ws*ws], added to
 * the scores of window w as amask[w % amask_nw] (WindowAttention.forward(x, mask),
 * layers/masked_win_attention.py:114-122; NULL = none), and (b) the head-group size hpb
 * of the MFMA path (heads per workgroup; values that do not divide heads fall back to 1).
 * rgbac_winattn_core == rgbac_winattn_core_ex(..., NULL, 0, 1, stream). */
int rgbac_winattn_core_ex(int dtype, int batch, int h, int w, int channels,
                          int heads, int ws, int shift, int masked, float scale,
                          const void* qkv, int64_t ldq, const float* alpha,
                          const float* bias, void* out, int64_t ldo, uint8_t* sel,
                          const float* amask, int amask_nw, int hpb, void* stream);

/* compressai GaussianConditional.forward + ste_round for one channel slice
 * (models/AutoEncoderRGB_Journal.py:255-257, bits :280):
 *   out_hat = round(y - mu) + mu   (torch.round: half to even)
 *   v = |(training ? y + noise : out_hat) - mu|,  s = max(scale, 0.11)
 *   lik = max(Phi((0.5 - v)/s) - Phi((-0.5 - v)/s), 1e-9)
 *   partial[block] = sum clamp(-log(lik + 1e-10)/ln2, 0, 50)   (fp64)
 * y/mu/scale/out_hat: NHWC with their own strides (channel offset folded into
 * the pointer); noise: fp32 NHWC [npix][nch] or NULL; lik: fp32 NHWC or NULL.
 * ``partial`` must hold rgbac_reduce_blocks(npix*nch) doubles. */
int rgbac_gaussian_slice(int dtype, int64_t npix, int nch,
                         const void* y, int64_t ldy, const void* mu, int64_t ldmu,
                         const void* scale, int64_t lds, const float* noise,
                         void* out_hat, int64_t ldh, float* lik, double* partial,
                         void* stream);

/* compressai EntropyBottleneck.forward (factorized prior, filters (3,3,3,3))
 * fused with z_hat = ste_round(z - med) + med
 * (models/AutoEncoderRGB_Journal.py:225-229).  params: fp32 [C][61] packed as
 * softplus(M0..M4) (3,9,9,9,3), b0..b4 (3,3,3,3,1), tanh(f0..f3) (3x4),
 * median -- see rgbac/entropy.py.  z: NHWC [npix][ldz]; z_hat written NHWC. */
int rgbac_eb_forward(int dtype, int64_t npix, int channels, const void* z,
                     int64_t ldz, const float* params, const float* noise,
                     void* z_hat, int64_t ldh, float* lik, double* partial,
                     void* stream);

/* Number of fp64 partial sums written by a reduction over n elements. */
int rgbac_reduce_blocks(int64_t n);

/* Final scalars of AutoEncoder.forward: reconstruct_error (masked MSE,
 * models/AutoEncoderRGB_Journal.py:36-64; or plain MSE when mode==1,
 * AutoEncoderMask_Journal.py:309) and bpp = bits/(B*H*W) (:290-295).
 * x: fp32 NCHW [B,cx,H,W]; x_hat: NHWC [B,H,W,ldh]; mask: fp32 [B,H,W].
 * out[0..3] = mse, bpp, y_bpp, z_bpp.  Single-block finalize, deterministic. */
int rgbac_finalize(int dtype, int mode, int batch, int cx, int h, int w,
                   const float* x, const void* x_hat, int64_t ldh,
                   const float* mask, const double* ybits, int ny,
                   const double* zbits, int nz, double* scratch, float* out,
                   void* stream);
/* Partial-sum blocks per image of the MSE pass: ``scratch`` of rgbac_finalize /
 * rgbac_finalize_ex must hold batch * rgbac_finalize_blocks(h, w) * 2 doubles
 * (min(1024, max(64, ceil(h * w / 1024)))). */
int rgbac_finalize_blocks(int h, int w);
/* The same, also writing x_hat's fp32 NCHW copy [B,cx,H,W] (the forward's returned x_hat,
 * otherwise a separate rgbac_nhwc_to_nchw) from the reads the MSE pass makes anyway;
 * x_hat_nchw may be NULL (== rgbac_finalize). */
int rgbac_finalize_ex(int dtype, int mode, int batch, int cx, int h, int w,
                      const float* x, const void* x_hat, int64_t ldh,
                      const float* mask, const double* ybits, int ny,
                      const double* zbits, int nz, double* scratch, float* out,
                      float* x_hat_nchw, void* stream);
/* The forward's prologue in ONE launch (AutoEncoderRGB_Journal.py:209-217): the decoder mask
 * pyramid of rgbac_mask_pyramid (levels 1..4), the input's rgbac_nchw_to_nhwc (x fp32 NCHW
 * [B,c,H,W] -> xf NHWC, ldc a multiple of 8 bf16 / 4 f32, xf 16-byte aligned; alpha is
 * [B,H,W] of the same B, H, W) and a zero fill of zero[0 .. nzero) doubles (the forward's
 * bits partials).  Outputs identical to the three separate launches. */
int rgbac_forward_prologue(int dtype, int batch, int c, int h, int w, const float* x,
                           void* xf, int64_t ldc, const float* alpha, int round255,
                           float* rounded, int levels, float* const* outs,
                           double* zero, int64_t nzero, void* stream);

/* SupplyMaskToTransform (layers/SupplyMask.py:11-18): ``levels`` successive
 * AvgPool2d(3, s2, p1, count_include_pad) of fp32 [B,H,W]; if round255, the
 * input is first replaced by round(x*255)/255 (AutoEncoderRGB_Journal.py:212-214)
 * and written to ``rounded``.  outs[i] receives level i+1. */
int rgbac_mask_pyramid(int batch, int h, int w, const float* alpha, int round255,
                       float* rounded, int levels, float* const* outs,
                       void* stream);

/* Layout conversions at the model boundary: fp32 NCHW <-> NHWC (ldc >= C,
 * padding channels zeroed on the way in). */
int rgbac_nchw_to_nhwc(int dtype, int batch, int c, int h, int w,
                       const float* src, void* dst, int64_t ldc, void* stream);
int rgbac_nhwc_to_nchw(int dtype, int batch, int c, int h, int w,
                       const void* src, int64_t ldc, float* dst, void* stream);


/* Fused ResidualUnit (layers/Masked_Attention.py:150-169), bf16, C = 192:
 *   out = GELU(W3 * GELU(W2 (*)3x3 GELU(W1 * x + b1) + b2) + b3 + x)
 * W1/W2/W3 are rgbac_conv2d packed weights ([rows][k_pad], k = tap*cin + c;
 * w2_kpad >= 896 zero-padded), biases fp32.  One 8x8 output tile per
 * workgroup with both intermediates in LDS; up to 4 units of identical
 * geometry per launch.  out must not alias x.                               */
typedef struct rgbac_ru_args {
  int32_t dtype, channels, batch, h, w, _pad0;
  const void* x; int64_t x_ldc;
  const void* w1; const void* w2; const void* w3;
  int32_t w1_kpad, w2_kpad, w3_kpad, _pad1;
  const float* b1; const float* b2; const float* b3;
  void* out; int64_t out_ldc;
} rgbac_ru_args;
int rgbac_residual_unit(const rgbac_ru_args* args, int ngroups, void* stream);
/* The same with a kind and C = 80 (reference: Masked_Attention.py:150-169 ResidualUnit at
 * M = 80; models/AutoEncoderMask_Journal.py:96-110 ResBlock at 192 and 80 channels).
 * kind 0: ResidualUnit (GELU, GELU, GELU(. + x)); kind 1: ResBlock (ReLU, ReLU, . + x).
 * C = 192: packed conv weights as rgbac_residual_unit.  C = 80: w1 / w2 / w3 are the
 * fragment-major packs [3][3][64][8], [3][18][64][8], [5][2][64][8] bf16 (16-row x 32-k
 * MFMA fragments, zero padded; rgbac.layers.Masked_Attention.small_unit_packs) and b1 / b2
 * / b3 fp32 [48] / [48] / [80] (zero padded); k_pads are ignored.
 * C = 192 with every k_pad 0 (W % 16 == 0): fragment-major packs [6][6][64][8],
 * [6][27][64][8] (k = tap * 96 + ci), [12][3][64][8] bf16 and b1 / b2 / b3 fp32 [96] / [96]
 * / [192], 16-byte aligned (rgbac.layers.Masked_Attention.wide_unit_packs): the barrier-free
 * weight-streaming kernel, one 8x16 output tile per workgroup. */
int rgbac_residual_unit_ex(const rgbac_ru_args* args, int ngroups, int kind, void* stream);
/* The LAST unit pair of a C = 192 Win_noShift_Attention block and its gate in ONE launch
 * (layers/Masked_Attention.py:177-189): args[0] = conv_a[2] on a, args[1] = conv_b[2] on b (both
 * fragment-major, as rgbac_residual_unit_ex's streamed form); gate_w = conv_b[3] (1x1,
 * 192 -> 192) fragment-major [12][6][64][8] bf16, gate_b fp32 [192]; ident = the block input.
 * args[1].out receives the block output a3 * sigmoid(conv_b[3](b3)) + ident; args[0].out
 * receives a3 (the in-launch hand-off buffer).  flags: nflags >= B*(H/8)*(W/16) + 1 uint32,
 * zero on entry and left zero; the last word, flags[nflags - 1], turns 1 if a hand-off wait
 * ever gave up (never expected: the waited-on workgroups are dispatched first). */
int rgbac_residual_unit_gate(const rgbac_ru_args* args, const void* gate_w,
                             const float* gate_b, const void* ident, int64_t ident_ldc,
                             uint32_t* flags, int64_t nflags, void* stream);

/* ====================================================================== *
 * Training step (trainRGB.py:178-198): backward kernels, optimizer.       *
 * The input gradient of a conv is rgbac_conv2d over a repacked weight      *
 * (transposed + flipped taps; a stride-2 conv's is the CONVT_S2 mode and   *
 * vice versa); the forward saves its pre-activation through args.zout.    *
 * ====================================================================== */

/* dL/dv of a fused epilogue y = act(v [, res1]) (v = the saved zout), and
 * dL/dres1 for the activations res1 enters (GATE, GDN, IGDN); channels
 * [channels, ldd*) of the outputs are zeroed.  NONE/MASKSEL need no z.
 * Replaces autograd of nn.GELU/ReLU/LeakyReLU, torch.sigmoid gate
 * (Masked_Attention.py:189), 0.5*tanh (AutoEncoderRGB_Journal.py:263),
 * GDN/IGDN (GDN.py:88-94) and the window scatter (masked_win_attention.py:235). */
int rgbac_act_bwd(int dtype, int act, float act_param, int64_t npix, int channels,
                  const void* dy, int64_t ldy, const void* z, int64_t ldz, const void* res1,
                  int64_t ld1, const uint8_t* sel, void* dz, int64_t lddz, void* dres1,
                  int64_t lddr1, void* stream);

/* Weight gradient of a conv as an MFMA GEMM reducing over pixels:
 *   D[n][k] = sum_m G[m][n] * Col(S)[m][k],  k = tap * cin_pad + cin,
 * m over the (batch, grid_h, grid_w) grid of G; S sampled at
 * (y*stride + ty - pad, x*stride + tx - pad) of the in_h x in_w sources.
 * Conv layers: G = dL/dv (output grid), S = the forward input.
 * ConvTranspose layers: G = the forward input, S = dL/dv (k5, s2, p2).
 * Output: fp32 slabs partial[nsplit][n_pad][k_pad] (+ column sums of G in
 * bias_partial[nsplit][n_pad] if non-NULL), summed by rgbac_wgrad_reduce.   */
typedef struct rgbac_wgrad_args {
  int32_t dtype;
  int32_t batch, grid_h, grid_w;
  const void* g; int64_t g_ldc; int32_t g_channels;   /* multiple of 8          */
  int32_t in_h, in_w, ksize, stride, pad;
  int32_t nsrc; int32_t cin_pad;
  rgbac_src src[3];
  int32_t square_input;        /* S = x^2 (GDN gamma gradient)                 */
  int32_t n_pad, k_pad;        /* slab dims: multiples of 64                   */
  int32_t nsplit;              /* pixel splits (deterministic fixed-order sum) */
  float* partial;
  float* bias_partial;
} rgbac_wgrad_args;
int rgbac_conv_wgrad(const rgbac_wgrad_args* args, void* stream);

/* Fixed-order sum of the slabs, scattered into the PyTorch parameter layout:
 * dw[fmap[e]] = sum_s partial[s*slab + e] for slab slots e < nslot with
 * fmap[e] >= 0 (fmap = the packed layout's slot -> parameter element map);
 * db[j] = sum_s bias_partial[s*n_pad + j], j < nbias.  accumulate != 0: add
 * the sums into dw / db (gradients accumulated straight into param.grad).    */
int rgbac_wgrad_reduce(int64_t nslot, const int32_t* fmap, const float* partial, int nsplit,
                       int64_t slab, float* dw, int nbias, const float* bias_partial, int n_pad,
                       float* db, int accumulate, void* stream);

/* Up to 8 rgbac_wgrad_reduce calls in one launch: tasks[11*t ..] = {nslot, fmap, partial,
 * nsplit, slab, dw, nbias, bias_partial, n_pad, db, accumulate} as int64 (pointers as
 * integers), each task the same fixed-order sum as rgbac_wgrad_reduce.  The training step
 * queues the weight-gradient reductions that add straight into param.grad and issues them in
 * batches (~195 reduce launches per step otherwise, each a few microseconds of fixed cost). */
int rgbac_wgrad_reduce_multi(int ntasks, const int64_t* tasks, void* stream);

/* Backward of rgbac_winattn_core: dqkv [B,H,W,>=3C] (dq, dk, dv; zero for
 * dropped windows) and per-block dense bias gradients bias_partial
 * [nblk][heads][N][N] (N = ws*ws), reduced by rgbac_relpos_bwd into the
 * relative_position_bias_table gradient [(2ws-1)^2][heads]
 * (masked_win_attention.py:96-131 autograd).                               */
int rgbac_winattn_core_bwd(int dtype, int batch, int h, int w, int channels, int heads, int ws,
                           int shift, int masked, float scale, const void* qkv, int64_t ldq,
                           const float* alpha, const float* bias, const void* dout, int64_t ldo,
                           void* dqkv, int64_t lddq, int nblk, float* bias_partial,
                           void* stream);
/* ... with the explicit additive mask of rgbac_winattn_core_ex (NULL = none). */
int rgbac_winattn_core_bwd_ex(int dtype, int batch, int h, int w, int channels, int heads,
                              int ws, int shift, int masked, float scale, const void* qkv,
                              int64_t ldq, const float* alpha, const float* bias,
                              const void* dout, int64_t ldo, void* dqkv, int64_t lddq, int nblk,
                              float* bias_partial, const float* amask, int amask_nw,
                              void* stream);
/* csr_off[(2ws-1)^2 + 1] / csr_ij[N*N]: for table row t, the flattened (i, j)
 * positions with relative_position_index[i][j] == t (fixed order).          */
int rgbac_relpos_bwd(int nblk, int heads, int ws, const float* bias_partial,
                     const int32_t* csr_off, const int32_t* csr_ij, float* dense, float* dtable,
                     void* stream);

/* GaussianConditional + bits + ste_round backward of one latent slice
 * (AutoEncoderRGB_Journal.py:255-257,280): gbits = device dL/d(sum bits),
 * dhat = dL/d y_hat (STE: passes to y), noise = training noise or NULL.     */
int rgbac_gaussian_bwd(int dtype, int64_t npix, int nch, const void* y, int64_t ldy,
                       const void* mu, int64_t ldmu, const void* scale, int64_t lds,
                       const float* noise, const float* gbits, const void* dhat, int64_t lddh,
                       void* dy, int64_t lddy, void* dmu, int64_t lddmu, void* dscale,
                       int64_t lddsc, void* stream);

/* EntropyBottleneck likelihood/bits backward (compressai >= 1.2, :225-229):
 * dz (plus dL/dz_hat through the STE), dparams [C][64] w.r.t. the packed
 * values of rgbac_eb_forward's block (softplus(M), b, tanh(f), median).     */
int rgbac_eb_bwd(int dtype, int64_t npix, int channels, const void* z, int64_t ldz,
                 const float* params, const float* noise, const float* gbits, const void* dzhat,
                 int64_t lddh, void* dz, int64_t lddz, float* dparams, void* stream);

/* reconstruct_error backward (AutoEncoderRGB_Journal.py:36-64 / mask :309);
 * scratch = the forward rgbac_finalize's scratch (per-image counts).        */
int rgbac_mse_bwd(int dtype, int mode, int batch, int cx, int h, int w, const float* x,
                  const void* x_hat, int64_t ldh, const float* mask, const double* scratch,
                  const float* gmse, void* dx_hat, int64_t lddx, void* stream);

/* grad = clamp(grad * grad_scale, -clip, clip) (clip <= 0: no clamp; the
 * result is written back like grad.clamp_) + torch.optim.Adam step over a flat
 * fp32 parameter buffer (trainRGB.py:190-198).  grad_scale = 1/world after a
 * data-parallel all-reduce sum.                                             */
int rgbac_adam_clamp(int64_t n, float* param, float* grad, float* exp_avg, float* exp_avg_sq,
                     double lr, double beta1, double beta2, double eps, int64_t step,
                     float clip, float grad_scale, void* stream);

/* rgbac_adam_clamp with the step count in device memory (a CUDA/HIP-graph
 * replayable training step): uses step = *step_dev + 1, then stores it.     */
int rgbac_adam_clamp_dstep(int64_t n, float* param, float* grad, float* exp_avg,
                           float* exp_avg_sq, double lr, double beta1, double beta2, double eps,
                           int64_t* step_dev, float clip, float grad_scale, void* stream);

/* PixelShuffle(2) (dir 0) / PixelUnshuffle(2) (dir 1) on NHWC; c = channels
 * after shuffling.  Channel copy for concatenation / split.                 */
int rgbac_pixel_shuffle(int dtype, int dir, int batch, int h, int w, int c, const void* in,
                        int64_t ldi, void* out, int64_t ldo, void* stream);
int rgbac_channel_copy(int dtype, int64_t npix, int channels, const void* src, int64_t lds,
                       int scoff, void* dst, int64_t ldd, int dcoff, void* stream);
/* Up to 16 channel copies over the same npix in one launch: desc = ntasks x 7 int64
 * {src, lds, scoff, channels, dst, ldd, dcoff} (host memory, read at the call; pointers as
 * integers).  Replaces the per-part rgbac_channel_copy launches of a concatenation
 * (torch.cat(..., dim=1) of the slice supports, AutoEncoderRGB_Journal.py:249-262) and of
 * its backward split.                                                      */
int rgbac_channel_copy_multi(int dtype, int64_t npix, int ntasks, const int64_t* desc,
                             void* stream);

/* rgbac_channel_copy_multi with an 8th descriptor field per task: accumulate (0 = copy,
 * 1 = dst += src, rounded once to the element type).  The backward split of a concatenation
 * adds each part's gradient slice straight into the gradient buffer its producer reads (the
 * training step's activation-gradient sinks, rgbac/autograd.py), in place of a copy plus an
 * autograd add (trainRGB.py:187 rd_loss.backward(): the slice supports of
 * AutoEncoderRGB_Journal.py:249-262 are each used by up to 11 later concatenations).   */
int rgbac_channel_copy_multi_ex(int dtype, int64_t npix, int ntasks, const int64_t* desc,
                                void* stream);

/* Weight repack through a cached index map: dst[i] = idx[i] >= 0 ? src[idx[i]] : 0
 * (src = fp32 PyTorch parameter, dst = packed [nphase][cout_pad][k_pad]).   */
int rgbac_weight_gather(int dtype, int64_t n, const float* src, const int32_t* idx, void* dst,
                        void* stream);

/* Many rgbac_weight_gather calls in one launch: tasks[5*t ..] = {src (const
 * float*), idx (const int32_t*), dst, n, dtype} as int64 in DEVICE memory;
 * task t owns blocks [blk0[t], blk0[t+1]) of 2048 elements (blk0 in device
 * memory, ntask + 1 entries, blk0[ntask] = nblk).  dtype 16: a 16-byte chunk
 * copy -- src / dst are arrays of 16-byte chunks, n counts chunks, idx[i] is
 * the source chunk (< 0: zeros); a block owns 2048 chunks.                  */
int rgbac_weight_gather_multi(int ntask, const int64_t* tasks, const int64_t* blk0, int64_t nblk,
                              void* stream);
/* The bf16 training packs' per-step repack as strided 8-element chunks (replaces the
 * element gather + 16-byte chunk copy pair of rgbac_weight_gather_multi for maps of that
 * form): tasks[8*t ..] = {src (const float*), cmap (const int32_t*), dst (16-byte chunks),
 * nchunk, stride, fmap (const int32_t* or 0), fdst (16-byte chunks or 0), 0} as int64 in
 * DEVICE memory; cmap[c] < 0: dst[c] = 0, else with base = cmap[c] & 0x0FFFFFFF and
 * nv = ((cmap[c] >> 28) & 7) + 1, element j of dst[c] = j < nv ? bf16(src[base + j*stride])
 * : 0; fmap[c] >= 0: fdst[fmap[c]] = dst[c].  Task t owns blocks [blk0[t], blk0[t+1]) of 256
 * chunks (blk0 as for rgbac_weight_gather_multi).                              */
int rgbac_weight_repack_multi(int ntask, const int64_t* tasks, const int64_t* blk0, int64_t nblk,
                              void* stream);
/* Per-channel sums over pixels into partial[nsplit][channels] (bias grads). */
int rgbac_colsum(int dtype, int64_t npix, int channels, const void* x, int64_t ldx, int nsplit,
                 float* partial, void* stream);
/* out[r] = (float) sum_j partial[r][j]  (fixed order; bits sums -> loss scalars). */
int rgbac_sum_partials(int rows, int n, const double* partial, float* out, void* stream);

/* Fused analysis stem (bf16): conv5x5/s2/p2 of an NHWC input with 8 (zero-padded) channels
 * to 192 channels, then GDN (inverse=0) or IGDN (1), writing only the GDN output.
 * Replaces layers/TransformRGB.py:55-56,66 (self.x1 -> self.gdn1) with layers/GDN.py:64-94.
 * w1: packed conv weights [>=192 rows][w1_kpad], k = tap*8 + c (rgbac_conv2d's layout),
 * b1: its bias (or NULL); w2: gamma' packed [>=192][w2_kpad]; beta: beta' [192];
 * out: NHWC bf16 [batch][ceil(h/2)][ceil(w/2)][out_ldc]. */
int rgbac_stem_gdn(int batch, int in_h, int in_w, const void* x, int64_t x_ldc, const void* w1,
                   int w1_kpad, const float* b1, const void* w2, int w2_kpad, const float* beta,
                   int inverse, void* out, int64_t out_ldc, void* stream);

/* Training-data augmentation for a batch (reference: my_datasets/MYdataset.py:55-115,
 * COCOP3MDataset.__getitem__ after the PNG decode): ToTensor (/255) -> RandomResizedCrop to
 * out_h x out_w (crop + bilinear resize, antialiased like torchvision >= 0.17 when antialias
 * != 0) -> horizontal / vertical flip -> alpha fill (alpha := 1) -> masked_image =
 * where(alpha > 0, img, alpha).  descs: device array of `batch` descriptors
 *   struct { const uint8_t* src; int32 h, w, crop_top, crop_left, crop_h, crop_w, flags, pad; }
 * (src = h x w x 4 RGBA uint8; flags bit 0 hflip, 1 vflip, 2 alpha fill; the random draws are
 * the host's, mirroring the reference's RNG calls: rgbac/data.py).  Outputs NCHW fp32:
 * masked (B,3,H,W), alpha (B,1,H,W), img (B,3,H,W), rgba (B,4,H,W) -- the reference's tuple
 * (masked_image, alpha, img, alpha, images_with_alpha). */
int rgbac_rgba_augment(int batch, const void* descs, int out_h, int out_w, int antialias,
                       float* masked, float* alpha, float* img, float* rgba, void* stream);

/* GDN / IGDN parameter reparametrisation (reference: layers/GDN.py:9-23 LowerBound, :71-78),
 * fp32, nb beta and ng gamma elements in one launch:
 *   beta_out = max(beta, beta_bound)^2 - pedestal,  gamma_out = max(gamma, gamma_bound)^2 - pedestal
 * and its backward: g2 = d_out * (2 max(p, bound)), passed where p >= bound or g2 < 0,
 * stored to dbeta / dgamma (accumulate == 0) or added into them (accumulate == 1; a null
 * d_out is a zero gradient).  Uncontracted, op for op torch's arithmetic. */
int rgbac_gdn_reparam(int nb, int ng, const float* beta, const float* gamma, float beta_bound,
                      float gamma_bound, float pedestal, float* beta_out, float* gamma_out,
                      void* stream);
int rgbac_gdn_reparam_bwd(int nb, int ng, const float* beta, const float* gamma,
                          float beta_bound, float gamma_bound, const float* dbeta_out,
                          const float* dgamma_out, float* dbeta, float* dgamma, int accumulate,
                          void* stream);

/* EntropyBottleneck parameter block (compressai EntropyBottleneck, filters (3, 3, 3, 3)):
 * params = the 15 fp32 parameters _matrix0..4, _bias0..4, _factor0..3, quantiles ([C][1][3]);
 * out [channels][64] = softplus(_matrix0..4) (33) | _bias0..4 (13) | tanh(_factor0..3) (12) |
 * quantiles[c][0][1] | 0 x 5 -- the block rgbac_eb_forward / rgbac_eb_bwd read.  The
 * backward maps dout to the 15 gradients (softplus / tanh derivatives; quantiles: the median
 * entry only), stored (accumulate == 0; quantiles' other entries untouched) or added. */
int rgbac_eb_params(int channels, const float* const* params, float* out, void* stream);
int rgbac_eb_params_bwd(int channels, const float* const* params, const float* dout,
                        float* const* grads, int accumulate, void* stream);

/* Fused masked shifted-window attention block, bf16, window 8, C = 192, 8 heads
 * (reference: layers/masked_win_attention.py:96-131 WindowAttention.forward, :169-251
 * WinBasedAttention.forward).  out = x + proj(attn(x)) on windows whose alpha is non-zero
 * anywhere (all windows when masked == 0), out = x elsewhere; the cyclic shift, window
 * partition / drop / reverse, the shifted-frame region mask and the relative position bias
 * are index math inside the kernels.  x, out: NHWC bf16 [batch][h][w][ld] (h, w multiples of
 * 8, out != x, 16-byte aligned); alpha: fp32 [batch][h][w] (masked only); wq_packed /
 * wp_packed: the fragment-major qkv / proj packs of WindowAttention.block_packs() (wq
 * [4][54][64][8]; wp [2][12][3][64][8] in the kernel's accumulator-operand k order: element e
 * of lane l in k-step s of pair-pair u is input channel 96u + 32s + 4(l >> 4) + (e & 3) +
 * 16(e >> 2)); bias_pack: fp32 [5][256] = bproj (192) | per head pair p: qkv.bias rows
 * 48p.., 192 + 48p.., 384 + 48p.. (48 each), zero padded; table_pad: fp32 [4][1024], per head
 * pair p [var 2][head 2][225] = (relative_position_bias_table[:, 2p + head] (- 100 for var 1))
 * * log2(e) in fp32, zero padded.  work: device workspace of at least
 * rgbac_winattn_block_workspace(batch, h, w) bytes, 256-byte aligned (no initial contents
 * needed).  Two bit-identical forms, chosen by the window count: below 2,048 windows one
 * launch of the round-3 kernel (one workgroup per window pair, all four head pairs' weights
 * streamed through its LDS); from 2,048 on, per 8,192 windows: one flag pass (masked only),
 * the persistent head-pair kernel (qkv + attention of one head pair over a share of the
 * active windows, O to the workspace, inactive windows copied) and the proj kernel over the
 * compacted active windows (env RGBAC_WINBLOCK_FORM=2|3 forces a form).  Replaces the qkv
 * GEMM, rgbac_winattn_core_ex and the MASKSEL proj GEMM of one WinBasedAttention call. */
int64_t rgbac_winattn_block_workspace(int batch, int h, int w);
int rgbac_winattn_block(int batch, int h, int w, int shift, int masked, float scale,
                        const void* x, int64_t ldx, const float* alpha, const void* wq_packed,
                        const float* bias_pack, const void* wp_packed, const float* table_pad,
                        void* out, int64_t ldo, void* work, int64_t work_bytes, void* stream);

/* The same block at window 4, C = 80, 8 heads of 10 (the 1/16-resolution attention blocks,
 * layers/TransformRGB.py:63,80): one wave per window, every product after the qkv GEMM in
 * registers.  h, w multiples of 4, shift < 4; x, out NHWC bf16 (ld >= 80, multiple of 8,
 * 16-byte aligned); wq_packed [45][64][8] bf16 (15 16-row tiles of the qkv weight (q | k |
 * v) x 3 32-deep k-steps, k >= 80 zero); wp_packed [5][5][64][4] bf16 (16x16x16 fragments of
 * the proj weight: lane l holds row 16m + (l & 15), input channels 16kt + 4(l >> 4) .. +3),
 * allocated to 13 KiB (zero tail); bqkv [240], bproj [80] fp32 (16-byte aligned); table
 * [49][8] fp32. */
int rgbac_winattn_block_ws4(int batch, int h, int w, int shift, int masked, float scale,
                            const void* x, int64_t ldx, const float* alpha, const void* wq_packed,
                            const float* bqkv, const void* wp_packed, const float* bproj,
                            const float* table, void* out, int64_t ldo, void* stream);

/* Fused DSE EnhancementBlock, bf16 NHWC (reference: layers/TransformRGB.py:16-49 --
 * EnhancementBlock.forward :23-28 and DSE.forward :39-49; the alpha codec's DSE,
 * models/AutoEncoderMask_Journal.py:39-48).  One launch computes
 *   out = conv2(act(conv1(t))) + t         (3x3 32->32, zero padding; the act map stays on chip;
 *                                           act = ReLU (slope 0) or LeakyReLU(slope))
 * mode 0 (first block): t = in_conv(x) is evaluated on the fly from the DSE input x;
 * mode 1 (middle block): t is read from `t` [batch][h][w][ldt], out is 32 channels;
 * mode 2 (last block):  out = out_conv(bf16(block(t) + in_conv(x))) + x, cin channels.
 * x: DSE input [batch][h][w][ldx] (cin <= 7 used channels, ldx % 8 == 0); w_in / w1 / w2 /
 * w_out: rgbac_conv2d-packed bf16 weights ([rows][kp], k = tap*32 + c for the 3x3 packs,
 * so kp1, kp2 >= 288), biases fp32.  Replaces the 8 launches of DSE.forward. */
int rgbac_dse_block(int mode, int batch, int h, int w, int cin, float slope, const void* x,
                    int64_t ldx,
                    const void* t, int64_t ldt, const void* w_in, int kp_in, const float* b_in,
                    const void* w1, int kp1, const float* b1, const void* w2, int kp2,
                    const float* b2, const void* w_out, int kp_out, const float* b_out,
                    void* out, int64_t ldo, void* stream);

/* Kernel timing (bench.py's launch profiler; no reference counterpart).  Events are created
 * with hipEventDisableSystemFence (no cache writeback/invalidate per record); recorded on a
 * capturing stream they become external event nodes of the HIP graph, so per-launch times
 * can be read from a graph replay.  rgbac_timer_elapsed_ms needs both events completed. */
int rgbac_timer_create(void** event);
int rgbac_timer_record(void* event, void* stream);
int rgbac_timer_elapsed_ms(void* start, void* stop, float* ms);
int rgbac_timer_destroy(void* event);

/* ---------------------------------------------------------------- bitstream (§8f rank 1)
 * GPU side of AutoEncoder.compress / decompress (AutoEncoderRGB_Journal.py:312-416).
 * Symbols and CDF indexes are int32 in NCHW order of each slice: o = ((b*cs + c)*h + y)*w + x,
 * the order of the reference's y_q_slice.reshape(-1).tolist() (:354-355) / index (:401).
 *
 * rgbac_gauss_code: one latent slice, NHWC activations.  ms holds (mu | sigma): mu in
 * channels [0, cs), sigma in [cs, 2cs) (the cc_mean / cc_scale outputs, :343-348).
 *   mode 0 (compress):   sym = int(round(y - mu)) (quantize "symbols", half-to-even),
 *                        idx = build_indexes(sigma), pre = sym + mu           (:350-352)
 *   mode 1 (indexes):    idx = build_indexes(sigma)                            (:400)
 *   mode 2 (dequantize): pre = sym + mu                                        (:403)
 * build_indexes: s' = max(sigma, scale_bound); idx = n_scales-1 - #{t < n_scales-1 :
 * s' <= table[t]} (compressai GaussianConditional.build_indexes).  y is read at channel
 * offset 0 of its pointer (pass y + slice offset). */
int rgbac_gauss_code(int dtype, int mode, int batch, int h, int w, int cs, const void* y,
                     int64_t ldy, const void* ms, int64_t ldm, const float* scale_table,
                     int n_scales, float scale_bound, int32_t* sym, int32_t* idx, void* pre,
                     int64_t ldp, void* stream);
/* rgbac_eb_code: EntropyBottleneck.compress / decompress element work (:319-320,:374),
 * z / z_hat NHWC (batch, h, w, channels), sym NCHW int32, medians fp32 [channels].
 *   mode 0: sym = int(round(z - med)), z_hat = sym + med;   mode 1: z_hat = sym + med. */
int rgbac_eb_code(int dtype, int mode, int batch, int h, int w, int channels, const void* z,
                  int64_t ldz, const float* medians, int32_t* sym, void* z_hat, int64_t ldh,
                  void* stream);

/* RGBA evaluation pipeline (csrc/rgba.hip), replaces trainRGB.py:284-304 between the alpha
 * codec and the RGB codec.  All tensors fp32 NCHW, single channel for the alpha planes.
 * rgbac_alpha_recon: recon = constraint(quantise ? round(clamp(x,0,1)*255)/255 : x)
 *   (trainRGB.py:285-287 and constraint() :98-111; recon must not alias x).  When
 *   true_mask is given, *not_all_ones is reset and set to 1 if any true_mask != 1
 *   (the `torch.all(mask == 1.0)` test of :300, on the device).
 * rgbac_rgba_finish: x_out = clamp(x_hat, 0, 1) (:290; may alias x_hat); optional scalars
 *   bpp_total = bpp + (*not_all_ones ? *bpp_mask : 0) (:300-303) and
 *   psnr = 10*log(1/mse)/log(10) (:306). */
int rgbac_alpha_recon(int batch, int h, int w, int quantise, const float* x_hat_mask,
                      float* recon_mask, const float* true_mask, int32_t* not_all_ones,
                      void* stream);
int rgbac_rgba_finish(int64_t n, const float* x_hat, float* x_out, const float* bpp,
                      const float* bpp_mask, const int32_t* not_all_ones, const float* mse,
                      float* bpp_total, float* psnr, void* stream);

/* MS-SSIM / SSIM metric (csrc/msssim.hip), replaces metrics/ms_ssim_torch.py:5-194.
 * fp32 NCHW planes.  rgbac_ssim_level: one scale of _ssim (:36-83) with the VALID 1-D gaussian
 *   win[win_size] (W pass then H pass, :21-33), C1 = (K1*range)^2, C2 = (K2*range)^2;
 *   partials: caller scratch of batch*channels*ceil((h-ws+1)/16)*ceil((w-ws+1)/16)*2 floats;
 *   ssim_out[b], cs_out[b] = CHW means of ssim_map / cs_map.  win_size odd, <= 15.
 * rgbac_avgpool2: F.avg_pool2d(kernel 2, padding (h%2, w%2)) of planes x (h, w) (:183-185).
 * rgbac_msssim_combine: per_image[b] = prod_{l<L-1} mcs[l][b]^w[l] * ssim_last[b]^w[L-1]
 *   (the broadcast of :189-190), mean = batch mean (:192-193); either output may be NULL. */
int rgbac_ssim_level(int batch, int channels, int h, int w, int win_size, const float* x,
                     const float* y, const float* win, float c1, float c2, float* partials,
                     float* ssim_out, float* cs_out, void* stream);
int rgbac_avgpool2(int planes, int h, int w, const float* x, float* y, void* stream);
int rgbac_msssim_combine(int levels, int batch, const float* mcs, const float* ssim_last,
                         const float* weights, float* per_image, float* mean, void* stream);

/* Masked MS-SSIM / SSIM (csrc/msssim.hip), replaces metrics/masked_ms_ssim_torch.py:56-265.
 * fp32 NCHW planes; the mask has 1 (broadcast over the channels) or C channels.
 * rgbac_masked_apply: one level's start (:246-248): mask_out = (mask > 0), x_out = x * it,
 *   y_out = y * it (mask_out shaped like mask).
 * rgbac_masked_ssim_level: _ssim (:56-118) on x, y with the binary level mask: VALID ssim / cs
 *   maps, kept where mask NEAREST-resized to (h-ws+1, w-ws+1) is nonzero (:103-105);
 *   ssim_out[b*C+c], cs_out[b*C+c] = masked sums / (count + 1e-10) (:115-116);
 *   partials: caller scratch of batch*channels*ceil((h-ws+1)/16)*ceil((w-ws+1)/16)*3 floats.
 * rgbac_masked_msssim_combine: v[b,c] = prod_{l<L-1} relu(mcs[l][b,c])^w[l] *
 *   relu(ssim_last[b,c])^w[L-1] (:252-260); per_image[b] = mean_c v, mean = mean_{b,c} v
 *   (:262-265); either output may be NULL; mcs may be NULL when levels == 1. */
int rgbac_masked_apply(int batch, int channels, int mask_channels, int h, int w, const float* x,
                       const float* y, const float* mask, float* x_out, float* y_out,
                       float* mask_out, void* stream);
int rgbac_masked_ssim_level(int batch, int channels, int mask_channels, int h, int w,
                            int win_size, const float* x, const float* y, const float* mask,
                            const float* win, float c1, float c2, float* partials,
                            float* ssim_out, float* cs_out, void* stream);
int rgbac_masked_msssim_combine(int levels, int batch, int channels, const float* mcs,
                                const float* ssim_last, const float* weights, float* per_image,
                                float* mean, void* stream);

/* Data-parallel gradient exchange (csrc/comm.cpp; BASELINE config 5 -- the reference trains
 * on one GPU, DataParallel is commented out at trainRGB.py:374, so no reference interface is
 * replaced: this is the all-reduce of rgbac/parallel.py's gradient buckets).  RCCL is called
 * directly on the caller's stream (capturable in a HIP graph); the library is the librccl.so
 * PyTorch loaded, dlopen'ed by rgbac_comm_load.  The unique id is 128 bytes (rank 0 makes it,
 * the host side broadcasts it).  rgbac_comm_allreduce_sum: in place, sum, fp32 or bf16. */
int rgbac_comm_load(const char* librccl_path);
int rgbac_comm_unique_id(void* id_out);
int rgbac_comm_init(const void* id, int world, int rank, int device, void** comm);
int rgbac_comm_allreduce_sum(void* comm, int dtype, void* buf, int64_t count, void* stream);
int rgbac_comm_destroy(void* comm);
/* Health and size of a communicator: rgbac_comm_count -> ranks RCCL itself spans
 * (ncclCommCount); rgbac_comm_async_error -> *err = 0 healthy, else the ncclResult_t of an
 * asynchronous failure (ncclCommGetAsyncError); rgbac_comm_abort releases pending collectives
 * and frees the handle (ncclCommAbort) -- the host then exits non-zero
 * (rgbac.parallel.CommWatchdog), it never restarts a process that touched the GPU. */
int rgbac_comm_count(void* comm, int* count);
int rgbac_comm_async_error(void* comm, int* err);
int rgbac_comm_abort(void* comm);

/* Host-side range-ANS coder (csrc/rans.cpp), byte-compatible with compressai.ans:
 * replaces BufferedRansEncoder.encode_with_indexes/flush (:334,:367-368), RansDecoder
 * set_stream/decode_stream (:387-388,:401) and the EntropyModel compress/decompress coders.
 * CDF tables: cdfs[ncdf][cdf_stride] int32, row i valid up to cdf_sizes[i]; offsets[ncdf]
 * (compressai's _quantized_cdf / _cdf_length / _offset buffers). */
int rgbac_pmf_to_quantized_cdf(const float* pmf, int n, int precision, uint32_t* cdf);
int rgbac_rans_encoder_create(void** handle);
int rgbac_rans_encoder_destroy(void* handle);
int rgbac_rans_encoder_put(void* handle, const int32_t* symbols, const int32_t* indexes,
                           int64_t n, const int32_t* cdfs, int cdf_stride,
                           const int32_t* cdf_sizes, const int32_t* offsets, int ncdf);
/* upper bound of the flushed stream size in bytes (-1 for a NULL handle) */
int64_t rgbac_rans_encoder_bound(void* handle);
int rgbac_rans_encoder_flush(void* handle, uint8_t* out, int64_t capacity, int64_t* nbytes);
/* caller-owned decoder state over a caller-owned byte stream */
typedef struct rgbac_rans_decoder {
  uint64_t state;
  const uint8_t* data;
  int64_t size;
  int64_t pos;
} rgbac_rans_decoder_t;
int rgbac_rans_decoder_init(rgbac_rans_decoder_t* dec, const uint8_t* data, int64_t nbytes);
int rgbac_rans_decode(rgbac_rans_decoder_t* dec, const int32_t* indexes, int64_t n,
                      const int32_t* cdfs, int cdf_stride, const int32_t* cdf_sizes,
                      const int32_t* offsets, int ncdf, int32_t* out);

#ifdef __cplusplus
}
#endif
#endif /* RGBAC_H_ */
