// Slice-chain convs with the chain's narrow tail conv folded in (rgbac_conv_fold) and the
// deferred bits of the folded quantisation (rgbac_gauss_bits); bf16 inference only.
//
// Reference: models/AutoEncoderRGB_Journal.py:240-264.  Per latent slice the chain is
//   cc1 -> cc2 -> (mu | sigma) + quantise -> lrp1 -> lrp2 -> lrp3 (tanh update)
// on a 32 x 32 latent at batch 8: 8192 pixels, launch-latency bound (a workgroup's staging,
// K loop and epilogue are one dependent chain of a few microseconds and the next launch waits
// for the last workgroup).  The narrow convs (128 -> 8 channels) produce the LAST 8 input
// channels of the next wide conv, so here the wide conv's workgroup recomputes them for its
// own (4+2) x (16+2) input patch as a prologue -- a few hundred MFMAs per workgroup instead of
// one more launch on the critical path:
//   * mu_i = cc_mean_transforms[i][4](t2_mean_i) folds into lrp_transforms[i][0], whose last
//     input channels are y_hat_i^pre = rint(y_i - mu_i) + mu_i (:255-262);
//   * lrp_transforms[i][4] (y_hat_i = pre_i + 0.5 tanh(.), :263-264) folds into
//     cc_*_transforms[i+1][0], whose last input channels are y_hat_i (:241-252).
// The bits of the folded quantisation need sigma_i as well; they are computed for all slices
// by one rgbac_gauss_bits launch after the chain (off its critical path), from the fp32 mu
// the fold stored.
//
// Workgroup: 4 waves, a 4 x 16-pixel output tile and 64 * TN output channels.
//   1. LDS-DMA: the wide conv's (4+2) x 18 patch (channels [0, c0), rows of 4 * CPT + 2
//      chunks of 16 bytes as conv_fpatch_kernel) and the narrow conv's (4+4) x 20 halo of its
//      128-channel input (rows of 17 chunks: the 16 consecutive rows of a fragment read fall
//      on distinct banks); the narrow conv's 9 k-steps of this wave and the aux operands are
//      requested behind them, the wide conv's weight ring behind those (left in flight).
//   2. Narrow conv over the 6 x 18 = 108 patch pixels (7 groups of 16) with K split over the
//      4 waves (9 of its 36 k-steps each); partials summed through LDS in a fixed order;
//      waves finalize groups wave, wave + 4 and write the 8 values into the patch chunk c0/8.
//   3. Wide conv: the unrolled K loop of conv_fpatch_kernel (9 taps x CPT k-steps, fragment-
//      major weights streamed through an RC-deep register ring) and the bias + GELU epilogue.
#include "common.h"
#include "conv_common.h"

namespace rgbac {

constexpr int kFoldMaxGroups = 12;
constexpr int kNarrowPS = 17;          // halo row stride (16-byte chunks): 16 data + 1 pad
constexpr int kNarrowKPW = 9;          // narrow-conv k-steps per wave (36 = 9 taps x 4 / 4 waves)

struct FoldDev {
  int batch, h, w, mode, ngroups, _pad[3];
  rgbac_fold_group g[kFoldMaxGroups];
};
struct BitsDev {
  int batch, h, w, ngroups;
  rgbac_bits_group g[kFoldMaxGroups];
};

// LDS-DMA of a rows x cols pixel window (top-left iy0, ix0; zero page outside the image) of a
// 128-channel NHWC source into LDS rows of kNarrowPS chunks, the pieces spread over nwave waves.
__device__ __forceinline__ void stage_halo(const bf16_t* src, long long ld, int b, int H, int W,
                                           int iy0, int ix0, int rows, int cols, uint32_t lbase,
                                           int wave, int nwave, int lane) {
  const int n = rows * cols;
  const int npiece = (n * kNarrowPS + 63) >> 6;
  for (int pc = wave; pc < npiece; pc += nwave) {
    const int f = (pc << 6) + lane;
    const int row = f / kNarrowPS, c = f - (f / kNarrowPS) * kNarrowPS;
    const int py = row / cols, px = row - (row / cols) * cols;
    const int iy = iy0 + py, ix = ix0 + px;
    const bool ok = row < n && c < 16 && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    const bf16_t* p = src + ((long long)(b * H + iy) * W + ix) * ld + c * 8;
    dma16_l(ok ? (const void*)p : (const void*)g_zero_page, lbase + (pc << 10));
  }
}

// This wave's share (k-steps [9 wave, 9 wave + 9)) of the narrow 3x3 conv over NG 16-pixel
// groups of an OW-wide output region (flat pixel p = r * OW + c, p < npx; lanes past npx
// repeat the last pixel), its (. + 2) x (OW + 2) input halo at P.
template <int NG, int OW>
__device__ __forceinline__ void narrow_part(const uint4* P, const uint4 (&wr)[kNarrowKPW],
                                            int wave, int lane, int npx, f32x4 (&acc)[NG]) {
  const int fr = lane & 15, fq = lane >> 4;
  int base[NG];
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    int p = 16 * g + fr;
    p = p < npx ? p : npx - 1;
    const int r = p / OW, c = p - (p / OW) * OW;
    base[g] = (r * (OW + 2) + c) * kNarrowPS + fq;
    acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int u = 0; u < kNarrowKPW; ++u) {
    const int ks = kNarrowKPW * wave + u;             // k-step = tap * 4 + 32-channel chunk
    const int tap = ks >> 2, cc = ks & 3;
    const int dy = tap / 3, dx = tap - 3 * (tap / 3);
    const int off = (dy * (OW + 2) + dx) * kNarrowPS + cc * 4;
#pragma unroll
    for (int g = 0; g < NG; ++g) mma_step<bf16_t>(acc[g], wr[u], P[base[g] + off]);
  }
}

template <int TN, int CPT>
__global__ void __launch_bounds__(256) conv_fold_kernel(const FoldDev args) {
  using T = bf16_t;
  constexpr int TW = 16, PW = TW + 2, PR = 6 * PW, NW = 4, BN = 64 * TN, TM = 4;
  constexpr int RS = 4 * CPT + 2;                       // wide patch row stride (chunks)
  constexpr int NKS = 9 * CPT;
  constexpr int RC0 = TN == 1 ? 24 : 12;                // weight ring depth (conv_fpatch_kernel)
  constexpr int RC = RC0 < NKS ? RC0 : NKS;
  constexpr int NG = 7;                                 // 16-pixel groups of the 108 patch pixels
  constexpr int MAIN_U4 = ((PR * RS + 63) >> 6) * 64;   // wide patch, whole 1-KiB DMA pieces
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  uint4* const patch = lds;
  uint4* const halo = lds + MAIN_U4;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int H = args.h, W = args.w;
  const int txn = W / TW, tyn = H / 4;
  int t = blockIdx.x;
  const int txi = t % txn; t /= txn;
  const int tyi = t % tyn;
  const int b = t / tyn;
  const int nblk = blockIdx.y;
  const rgbac_fold_group& g = args.g[blockIdx.z];
  const int n0 = nblk * BN;
  if (n0 >= g.cout) return;
  const int y0 = tyi * 4, x0 = txi * TW;
  const int c0 = g.c0, cout = g.cout;
  const bool gauss = args.mode == RGBAC_FOLD_GAUSS;

  // ---- wide-conv biases (the epilogue's), narrow-conv biases
  const int ntile0 = (n0 >> 4) + wave * TN;
  float pbias[TN][4];
  {
    const int nb0 = n0 + wave * TN * 16 + fq * 4;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pbias[j][r] = (g.bias && nb0 + j * 16 + r < cout) ? g.bias[nb0 + j * 16 + r] : 0.0f;
  }
  float nbias[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) nbias[r] = fq < 2 ? g.pbias[4 * fq + r] : 0.0f;

  // ---- 1. staging: wide patch (channels < c0), narrow halo, then the register operands
  {
    const char* const sp0 = reinterpret_cast<const char*>(g.src[0].ptr);
    const char* const sp1 = reinterpret_cast<const char*>(g.src[1].ptr);
    const int send0 = g.src[0].channels;
    const long long sld0 = g.src[0].ldc, sld1 = g.src[1].ldc;
    const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)patch);
    constexpr int npiece = MAIN_U4 >> 6;
    for (int pc = wave; pc < npiece; pc += NW) {
      const int f = (pc << 6) + lane;
      const int row = f / RS, c = f - (f / RS) * RS;
      const int py = row / PW, px = row - (row / PW) * PW;
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const int ch = c << 3;
      const bool in0 = ch < send0;
      const bool ok = row < PR && c < 4 * CPT && ch < c0 && (unsigned)iy < (unsigned)H &&
                      (unsigned)ix < (unsigned)W;
      const long long pix = (long long)(b * H + iy) * W + ix;
      const char* p = in0 ? sp0 + (pix * sld0 + ch) * 2 : sp1 + (pix * sld1 + (ch - send0)) * 2;
      dma16_l(ok ? (const void*)p : (const void*)g_zero_page, lbase + (pc << 10));
    }
    const uint32_t hbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)halo);
    stage_halo(reinterpret_cast<const T*>(g.pin), g.pin_ldc, b, H, W, y0 - 2, x0 - 2, 8, 20,
               hbase, wave, NW, lane);
  }
  uint4 wr[kNarrowKPW];
  {
    const uint4* pw = reinterpret_cast<const uint4*>(g.pweight) + kNarrowKPW * wave * 64 + lane;
#pragma unroll
    for (int u = 0; u < kNarrowKPW; ++u) wr[u] = pw[u * 64];
  }
  // aux operands of the (up to two) groups this wave finalizes: lanes fq < 2, 4 channels
  uint2 ax[2] = {uint2{0u, 0u}, uint2{0u, 0u}};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int p = 16 * (wave + 4 * k) + fr;
    const int r = p / PW, c = p - (p / PW) * PW;
    const int iy = y0 - 1 + r, ix = x0 - 1 + c;
    if (fq < 2 && p < PR && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W)
      ax[k] = *reinterpret_cast<const uint2*>(reinterpret_cast<const T*>(g.aux) +
                                              ((long long)(b * H + iy) * W + ix) * g.aux_ldc +
                                              4 * fq);
  }
  const uint4* wj[TN];
  uint4 cring[RC][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j)
    wj[j] = reinterpret_cast<const uint4*>(g.weight) + (size_t)(ntile0 + j) * NKS * 64 + lane;
#pragma unroll
  for (int u = 0; u < RC; ++u)
#pragma unroll
    for (int j = 0; j < TN; ++j) cring[u][j] = wj[j][u * 64];
  wait_vm<RC * TN>();                    // in-order returns: everything but the ring
  __syncthreads();

  // ---- 2. narrow conv -> the folded channels of the wide patch
  {
    f32x4 pacc[NG];
    narrow_part<NG, PW>(halo, wr, wave, lane, PR, pacc);
    __syncthreads();                                   // every wave is done with the halo
    f32x4* const red = reinterpret_cast<f32x4*>(halo);
#pragma unroll
    for (int q = 0; q < NG; ++q) red[(wave * NG + q) * 64 + lane] = pacc[q];
    __syncthreads();
    const bool writer = g.writer && nblk == 0;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = wave + 4 * k;
      if (q >= NG) break;
      const int p = 16 * q + fr;
      if (fq >= 2 || p >= PR) continue;
      f32x4 v = red[(0 * NG + q) * 64 + lane];
#pragma unroll
      for (int w = 1; w < NW; ++w) {
        const f32x4 s = red[(w * NG + q) * 64 + lane];
        v = f32x4{v[0] + s[0], v[1] + s[1], v[2] + s[2], v[3] + s[3]};
      }
      const int r = p / PW, c = p - (p / PW) * PW;
      const int iy = y0 - 1 + r, ix = x0 - 1 + c;
      float val[4] = {0.f, 0.f, 0.f, 0.f};
      if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
        const float a[4] = {bf2f(ax[k].x & 0xFFFF), bf2f(ax[k].x >> 16), bf2f(ax[k].y & 0xFFFF),
                            bf2f(ax[k].y >> 16)};
        float mu[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          mu[e] = v[e] + nbias[e];
          val[e] = gauss ? rintf(a[e] - mu[e]) + mu[e] : a[e] + 0.5f * tanhf(mu[e]);
        }
        if (writer && r >= 1 && r <= 4 && c >= 1 && c <= TW) {
          const long long pix = (long long)(b * H + iy) * W + ix;
          Elem<T>::st4(reinterpret_cast<T*>(g.put) + pix * g.put_ldc + 4 * fq, val);
          if (gauss)
            *reinterpret_cast<float4*>(g.mu + pix * g.mu_ldc + 4 * fq) =
                make_float4(mu[0], mu[1], mu[2], mu[3]);
        }
      }
      uint2 pk;
      pk.x = pack_bf16x2(val[0], val[1]);
      pk.y = pack_bf16x2(val[2], val[3]);
      *reinterpret_cast<uint2*>(reinterpret_cast<char*>(patch) + (p * RS + (c0 >> 3)) * 16 +
                                8 * fq) = pk;
    }
    __syncthreads();
  }

  // ---- 3. wide conv, unrolled K (conv_fpatch_kernel's CPT loop), bias + GELU epilogue
  int lb[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) lb[i] = (i * PW + fr) * RS + fq;
  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    const int tap = ks / CPT, cc = ks - (ks / CPT) * CPT;
    const int off = ((tap / 3) * PW + tap % 3) * RS + cc * 4;
    uint4 bb[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) bb[i] = patch[lb[i] + off];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], cring[ks % RC][j], bb[i]);
    if (ks + RC < NKS) {
#pragma unroll
      for (int j = 0; j < TN; ++j) cring[ks % RC][j] = wj[j][(ks + RC) * 64];
    }
  }
  T* const out = reinterpret_cast<T*>(g.out) + g.out_coff;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const long long opix = (long long)(b * H + y0 + i) * W + x0 + fr;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wave * TN * 16 + j * 16 + fq * 4;
      if (n < cout) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_t<T>(acc[j][i][r] + pbias[j][r]);
        Elem<T>::st4(out + opix * g.out_ldc + n, v);
      }
    }
  }
}

// Deferred bits of the folded quantisation: sigma conv over the tile's (4+2) x 18 halo (K
// split over the 4 waves as above), wave w finalizes pixel row w with the stored mu.
__global__ void __launch_bounds__(256) gauss_bits_kernel(const BitsDev args) {
  using T = bf16_t;
  constexpr int TW = 16, NW = 4;
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  __shared__ double wsum[NW];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int H = args.h, W = args.w;
  const int txn = W / TW, tyn = H / 4;
  int t = blockIdx.x;
  const int txi = t % txn; t /= txn;
  const int tyi = t % tyn;
  const int b = t / tyn;
  const rgbac_bits_group& g = args.g[blockIdx.y];
  const int y0 = tyi * 4, x0 = txi * TW;
  const long long pix = (long long)(b * H + y0 + wave) * W + x0 + fr;

  const uint32_t hbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)lds);
  stage_halo(reinterpret_cast<const T*>(g.pin), g.pin_ldc, b, H, W, y0 - 1, x0 - 1, 6, 18, hbase,
             wave, NW, lane);
  uint4 wr[kNarrowKPW];
  {
    const uint4* pw = reinterpret_cast<const uint4*>(g.pweight) + kNarrowKPW * wave * 64 + lane;
#pragma unroll
    for (int u = 0; u < kNarrowKPW; ++u) wr[u] = pw[u * 64];
  }
  float sb[4] = {0.f, 0.f, 0.f, 0.f}, yv[4] = {0.f, 0.f, 0.f, 0.f}, mu[4] = {0.f, 0.f, 0.f, 0.f};
  if (fq < 2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) sb[r] = g.pbias[4 * fq + r];
    Elem<T>::ld4(reinterpret_cast<const T*>(g.y) + pix * g.y_ldc + 4 * fq, yv);
    const float4 m = *reinterpret_cast<const float4*>(g.mu + pix * g.mu_ldc + 4 * fq);
    mu[0] = m.x; mu[1] = m.y; mu[2] = m.z; mu[3] = m.w;
  }
  wait_vm<0>();
  __syncthreads();

  f32x4 pacc[4];
  narrow_part<4, TW>(lds, wr, wave, lane, 64, pacc);
  __syncthreads();
  f32x4* const red = reinterpret_cast<f32x4*>(lds);
#pragma unroll
  for (int q = 0; q < 4; ++q) red[(wave * 4 + q) * 64 + lane] = pacc[q];
  __syncthreads();
  double bits = 0.0;
  if (fq < 2) {
    f32x4 v = red[wave * 64 + lane];                     // (wave 0, row `wave`)
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const f32x4 s = red[(w * 4 + wave) * 64 + lane];
      v = f32x4{v[0] + s[0], v[1] + s[1], v[2] + s[2], v[3] + s[3]};
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      // compressai GaussianConditional._likelihood + the bits of AutoEncoderRGB_Journal.py:280
      // (as gauss_elem_y, eval mode: the quantised value's distance to mu)
      const float hat = rintf(yv[r] - mu[r]) + mu[r];
      const float d = fabsf(hat - mu[r]);
      const float sc = fmaxf(v[r] + sb[r], 0.11f);
      const float lik = fmaxf(std_cum_f((0.5f - d) / sc) - std_cum_f((-0.5f - d) / sc), 1e-9f);
      const float bt = (-1.0f * logf(lik + 1e-10f)) / 0.69314718055994530942f;
      bits += (double)fminf(fmaxf(bt, 0.0f), 50.0f);
    }
  }
  for (int o = 32; o > 0; o >>= 1) bits += __shfl_xor(bits, o);
  if (lane == 0) wsum[wave] = bits;
  __syncthreads();
  if (tid == 0) g.partial[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

static int check_narrow(const void* pin, long long pin_ldc, const void* pw, const float* pb) {
  if (!pin || !pw || !pb || !aligned16(pin) || !aligned16(pw) || pin_ldc < 128 || pin_ldc % 8)
    return -1;
  return 0;
}

template <int TN, int CPT>
static void launch_fold_k(const FoldDev& d, dim3 grid, size_t lds, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_fold_kernel<TN, CPT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 128 * 1024);
    (void)hipGetLastError();
    attr = true;
  }
  hipLaunchKernelGGL((conv_fold_kernel<TN, CPT>), grid, dim3(256), lds, st, d);
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_conv_fold(const rgbac_fold_group* groups, int ngroups, int batch, int h,
                               int w, int mode, int bn, void* stream) {
  RGBAC_REQUIRE(groups && ngroups >= 1 && ngroups <= kFoldMaxGroups, "ngroups must be 1..12");
  RGBAC_REQUIRE(batch >= 1 && h >= 4 && w >= 16 && h % 4 == 0 && w % 16 == 0,
              "h must be a multiple of 4 and w of 16");
  RGBAC_REQUIRE(mode == RGBAC_FOLD_GAUSS || mode == RGBAC_FOLD_TANH, "unknown fold mode");
  RGBAC_REQUIRE(bn == 64 || bn == 128, "bn must be 64 or 128");
  FoldDev d{};
  d.batch = batch; d.h = h; d.w = w; d.mode = mode; d.ngroups = ngroups;
  int cpt = 0, cmax = 0;
  for (int i = 0; i < ngroups; ++i) {
    const rgbac_fold_group& g = groups[i];
    const int s0 = g.src[0].channels, s1 = g.src[1].channels;
    RGBAC_REQUIRE(s0 > 0 && s0 % 8 == 0 && s1 >= 0 && s1 % 8 == 0 && s0 + s1 == g.c0,
                "source channels must be multiples of 8 summing to c0");
    RGBAC_REQUIRE(g.src[0].ptr && aligned16(g.src[0].ptr) && g.src[0].ldc % 8 == 0 &&
                g.src[0].ldc >= s0, "src[0]: 16-byte aligned NHWC with ldc % 8 == 0");
    RGBAC_REQUIRE(s1 == 0 || (g.src[1].ptr && aligned16(g.src[1].ptr) && g.src[1].ldc % 8 == 0 &&
                            g.src[1].ldc >= s1), "src[1]: 16-byte aligned NHWC with ldc % 8 == 0");
    const int c = (g.c0 + 8 + 31) / 32;
    RGBAC_REQUIRE(c == 3 || c == 4, "the folded conv's input must have 72..128 channels");
    RGBAC_REQUIRE(cpt == 0 || c == cpt, "all groups must round to the same 32-channel k-steps");
    cpt = c;
    RGBAC_REQUIRE(g.cout >= 4 && g.cout % 4 == 0 && g.out && g.out_ldc % 4 == 0 &&
                g.out_coff % 4 == 0 && g.out_coff + g.cout <= g.out_ldc && g.weight &&
                aligned16(g.weight), "wide-conv output / weights");
    RGBAC_REQUIRE(check_narrow(g.pin, g.pin_ldc, g.pweight, g.pbias) == 0,
                "narrow conv: 16-byte aligned 128-channel input (ldc % 8 == 0), weights, bias");
    RGBAC_REQUIRE(g.aux && g.aux_ldc >= 8 && g.aux_ldc % 4 == 0 && ((uintptr_t)g.aux & 7) == 0,
                "aux: 8 channels, 8-byte aligned rows");
    if (g.writer) {
      RGBAC_REQUIRE(g.put && g.put_ldc >= 8 && g.put_ldc % 4 == 0 && ((uintptr_t)g.put & 7) == 0,
                  "writer: put must hold 8 channels, 8-byte aligned rows");
      RGBAC_REQUIRE(mode != RGBAC_FOLD_GAUSS ||
                  (g.mu && g.mu_ldc >= 8 && g.mu_ldc % 4 == 0 && aligned16(g.mu)),
                  "GAUSS writer: fp32 mu with 16-byte aligned rows");
    }
    cmax = g.cout > cmax ? g.cout : cmax;
    d.g[i] = g;
  }
  const int tn = bn / 64;
  const int rs = 4 * cpt + 2;
  const size_t main_b = (size_t)((6 * 18 * rs + 63) / 64) * 1024;
  const size_t halo_b = (size_t)((8 * 20 * kNarrowPS + 63) / 64) * 1024;
  const size_t lds = main_b + halo_b;                  // the partials (7 KiB per wave) reuse the halo
  const dim3 grid((unsigned)(batch * (h / 4) * (w / 16)), (unsigned)((cmax + bn - 1) / bn),
                  (unsigned)ngroups);
  hipStream_t st = (hipStream_t)stream;
  if (tn == 1) {
    if (cpt == 3) launch_fold_k<1, 3>(d, grid, lds, st);
    else launch_fold_k<1, 4>(d, grid, lds, st);
  } else {
    if (cpt == 3) launch_fold_k<2, 3>(d, grid, lds, st);
    else launch_fold_k<2, 4>(d, grid, lds, st);
  }
  return check_launch("conv_fold_kernel");
}

extern "C" int rgbac_gauss_bits(const rgbac_bits_group* groups, int ngroups, int batch, int h,
                                int w, void* stream) {
  RGBAC_REQUIRE(groups && ngroups >= 1 && ngroups <= kFoldMaxGroups, "ngroups must be 1..12");
  RGBAC_REQUIRE(batch >= 1 && h >= 4 && w >= 16 && h % 4 == 0 && w % 16 == 0,
              "h must be a multiple of 4 and w of 16");
  BitsDev d{};
  d.batch = batch; d.h = h; d.w = w; d.ngroups = ngroups;
  for (int i = 0; i < ngroups; ++i) {
    const rgbac_bits_group& g = groups[i];
    RGBAC_REQUIRE(check_narrow(g.pin, g.pin_ldc, g.pweight, g.pbias) == 0,
                "sigma conv: 16-byte aligned 128-channel input (ldc % 8 == 0), weights, bias");
    RGBAC_REQUIRE(g.y && g.y_ldc >= 8 && g.y_ldc % 4 == 0 && ((uintptr_t)g.y & 7) == 0 && g.mu &&
                g.mu_ldc >= 8 && g.mu_ldc % 4 == 0 && aligned16(g.mu) && g.partial,
                "y (8 channels, 8-byte aligned rows), fp32 mu (16-byte aligned rows), partial");
    d.g[i] = g;
  }
  const size_t lds = (size_t)((6 * 18 * kNarrowPS + 63) / 64) * 1024;   // >= 16 KiB partials
  const dim3 grid((unsigned)(batch * (h / 4) * (w / 16)), (unsigned)ngroups, 1);
  hipLaunchKernelGGL(gauss_bits_kernel, grid, dim3(256), lds, (hipStream_t)stream, d);
  return check_launch("gauss_bits_kernel");
}
