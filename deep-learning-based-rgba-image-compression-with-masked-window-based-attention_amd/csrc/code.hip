// GPU side of the bitstream path (AutoEncoder.compress / decompress,
// models/AutoEncoderRGB_Journal.py:312-416): the per-element work between the slice convs
// and the host rANS coder (csrc/rans.cpp).
//   * gauss_code_kernel: quantize(y, "symbols", mu), build_indexes(sigma), y_q + mu and
//     dequantize(sym, mu) for one latent slice (compressai GaussianConditional semantics);
//   * eb_code_kernel: EntropyBottleneck quantize / dequantize around its medians.
// One thread per latent pixel: the NHWC reads of a pixel's channels are contiguous, and the
// int32 symbol / index planes are written in the reference's NCHW order (consecutive
// threads -> consecutive x), so every store is coalesced.  Both are HBM/latency bound
// (config 2: 65 k symbols per slice); the integer outputs are exact, no floating-point
// reduction is involved.
#include "common.h"

namespace rgbac {

template <typename T>
__global__ void __launch_bounds__(256)
gauss_code_kernel(int mode, int HW, long long npix, int cs, const T* __restrict__ y,
                  long long ldy, const T* __restrict__ ms, long long ldm,
                  const float* __restrict__ table, int ntab, float bound,
                  int* __restrict__ sym, int* __restrict__ idx, T* __restrict__ pre,
                  long long ldp) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  const long long b = p / HW;
  const long long s = p - b * HW;
  for (int c = 0; c < cs; ++c) {
    const long long o = (b * cs + c) * HW + s;
    const float mu = Elem<T>::ld(ms + p * ldm + c);
    if (mode != 2) {
      // GaussianConditional.build_indexes: lower_bound_scale, then count the table entries
      // the scale does not exceed (the last entry never counts)
      const float sc = fmaxf(Elem<T>::ld(ms + p * ldm + cs + c), bound);
      int k = ntab - 1;
      for (int t = 0; t < ntab - 1; ++t) k -= (sc <= table[t]) ? 1 : 0;
      idx[o] = k;
    }
    if (mode == 0) {
      const float q = rintf(Elem<T>::ld(y + p * ldy + c) - mu);  // torch.round: half-to-even
      sym[o] = (int)q;
      Elem<T>::st(pre + p * ldp + c, q + mu);
    } else if (mode == 2) {
      Elem<T>::st(pre + p * ldp + c, (float)sym[o] + mu);
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
eb_code_kernel(int mode, int HW, long long npix, int C, const T* __restrict__ z, long long ldz,
               const float* __restrict__ med, int* __restrict__ sym, T* __restrict__ zhat,
               long long ldh) {
  const long long p = (long long)blockIdx.x * 256 + threadIdx.x;
  if (p >= npix) return;
  const long long b = p / HW;
  const long long s = p - b * HW;
  for (int c = 0; c < C; ++c) {
    const long long o = (b * C + c) * HW + s;
    const float m = med[c];
    float q;
    if (mode == 0) {
      q = rintf(Elem<T>::ld(z + p * ldz + c) - m);
      sym[o] = (int)q;
    } else {
      q = (float)sym[o];
    }
    Elem<T>::st(zhat + p * ldh + c, q + m);
  }
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_gauss_code(int dtype, int mode, int batch, int h, int w, int cs,
                                const void* y, int64_t ldy, const void* ms, int64_t ldm,
                                const float* scale_table, int n_scales, float scale_bound,
                                int32_t* sym, int32_t* idx, void* pre, int64_t ldp,
                                void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(mode >= 0 && mode <= 2, "mode");
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && cs > 0, "shape");
  RGBAC_REQUIRE(ms && ldm >= 2 * cs, "mu|sigma source");
  RGBAC_REQUIRE(mode == 2 || (scale_table && n_scales > 0 && idx), "scale table / indexes");
  RGBAC_REQUIRE(mode != 0 || (y && ldy >= cs), "y");
  RGBAC_REQUIRE(mode == 1 || (sym && pre && ldp >= cs), "symbols / output");
  const long long npix = (long long)batch * h * w;
  const int g = (int)((npix + 255) / 256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(gauss_code_kernel<float>, dim3(g), dim3(256), 0, st, mode, h * w, npix,
                       cs, (const float*)y, ldy, (const float*)ms, ldm, scale_table, n_scales,
                       scale_bound, sym, idx, (float*)pre, ldp);
  else
    hipLaunchKernelGGL(gauss_code_kernel<bf16_t>, dim3(g), dim3(256), 0, st, mode, h * w, npix,
                       cs, (const bf16_t*)y, ldy, (const bf16_t*)ms, ldm, scale_table, n_scales,
                       scale_bound, sym, idx, (bf16_t*)pre, ldp);
  return check_launch("gauss_code_kernel");
}

extern "C" int rgbac_eb_code(int dtype, int mode, int batch, int h, int w, int channels,
                             const void* z, int64_t ldz, const float* medians, int32_t* sym,
                             void* z_hat, int64_t ldh, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(mode == 0 || mode == 1, "mode");
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && channels > 0, "shape");
  RGBAC_REQUIRE(medians && sym && z_hat && ldh >= channels, "null pointer");
  RGBAC_REQUIRE(mode == 1 || (z && ldz >= channels), "z");
  const long long npix = (long long)batch * h * w;
  const int g = (int)((npix + 255) / 256);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(eb_code_kernel<float>, dim3(g), dim3(256), 0, st, mode, h * w, npix,
                       channels, (const float*)z, ldz, medians, sym, (float*)z_hat, ldh);
  else
    hipLaunchKernelGGL(eb_code_kernel<bf16_t>, dim3(g), dim3(256), 0, st, mode, h * w, npix,
                       channels, (const bf16_t*)z, ldz, medians, sym, (bf16_t*)z_hat, ldh);
  return check_launch("eb_code_kernel");
}
