// Training-data augmentation on the GPU (reference: my_datasets/MYdataset.py:55-115,
// COCOP3MDataset.__getitem__): decoded RGBA uint8 images -> ToTensor (/255) ->
// RandomResizedCrop to out_h x out_w (torchvision resized_crop = crop + bilinear resize,
// antialiased when downscaling: torch's separable "aa" triangle filter) -> random h/v flips ->
// alpha "fill" (alpha := 1 with probability fill_mix_ratio) -> masked_image =
// where(alpha > 0, img, alpha).  The random parameters are drawn on the host exactly as the
// reference draws them (rgbac/data.py); this kernel does the pixel work for a whole batch in
// one launch and writes the reference's 5-tuple tensors (NCHW fp32) directly.
//
// One thread per output pixel: for each of the (at most kAugMaxTaps) source rows of its vertical
// filter window it sums the horizontal window (weights computed once per thread), then
// combines the rows -- horizontal pass then vertical pass, as ATen's separable upsample.
// HBM-bound: 4 B read per covered source pixel (cached: neighbouring threads share rows),
// 44 B written per output pixel (masked 12 + alpha 4 + img 12 + rgba 16).
#include "common.h"

namespace rgbac {

struct AugDesc {                 // one image of the batch
  const uint8_t* src;            // H x W x 4 (RGBA, row-major, contiguous)
  int h, w;                      // source size
  int ci, cj, ch, cw;            // crop box (top, left, height, width)
  int flags;                     // bit 0: hflip, bit 1: vflip, bit 2: alpha fill
  int pad;
};

constexpr int kAugMaxTaps = 64;  // filter window cap (downscale factor <= 32)

// torch's antialiased-bilinear weights for output index o (ATen UpSampleKernel
// _compute_indices_weights_aa, interp_size 2): center = scale (o + 0.5), support = scale
// (>= 1) or 1, window [xmin, xmin + xsize), w_k = max(0, 1 - |(k + xmin - center + 0.5) /
// max(scale, 1)|), normalised.  With antialias off: the plain align_corners=False bilinear.
__device__ __forceinline__ int aa_window(int o, int in_size, float scale, int antialias,
                                          float (&wt)[kAugMaxTaps], int& xmin) {
  if (!antialias) {
    float src = scale * (o + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    int x0 = (int)src;
    if (x0 > in_size - 1) x0 = in_size - 1;
    const int x1 = x0 + (x0 < in_size - 1 ? 1 : 0);
    const float l1 = src - (float)x0, l0 = 1.f - l1;
    xmin = x0;
    wt[0] = l0;
    wt[1] = x1 > x0 ? l1 : 0.f;
    if (x1 == x0) wt[0] = 1.f;
    return x1 > x0 ? 2 : 1;
  }
  const float support = scale >= 1.0f ? scale : 1.0f;
  const float center = scale * (o + 0.5f);
  const float invscale = scale >= 1.0f ? 1.0f / scale : 1.0f;
  // ATen forms these with a double 0.5 (float center/support/invscale): same here, so the
  // window bounds and weights round identically
  xmin = (int)((double)center - (double)support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)((double)center + (double)support + 0.5);
  if (xmax > in_size) xmax = in_size;
  int n = xmax - xmin;
  if (n > kAugMaxTaps) n = kAugMaxTaps;
  float total = 0.f;
  for (int k = 0; k < n; ++k) {
    float t = (float)(((double)((float)(k + xmin) - center) + 0.5) * (double)invscale);
    t = t < 0.f ? -t : t;
    const float v = t < 1.0f ? 1.0f - t : 0.0f;
    wt[k] = v;
    total += v;
  }
  if (total != 0.f)
    for (int k = 0; k < n; ++k) wt[k] /= total;
  return n;
}

__global__ void __launch_bounds__(256) rgba_augment_kernel(const AugDesc* __restrict__ descs,
                                                           int out_h, int out_w, int antialias,
                                                           float* __restrict__ masked,
                                                           float* __restrict__ alpha,
                                                           float* __restrict__ img,
                                                           float* __restrict__ rgba) {
  const int b = blockIdx.y;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= out_h * out_w) return;
  const AugDesc d = descs[b];
  // a malformed descriptor (crop outside the image) writes nothing rather than reading out
  // of bounds (the host builds them checked: rgbac/data.py)
  if (d.ci < 0 || d.cj < 0 || d.ch < 1 || d.cw < 1 || d.ci + d.ch > d.h || d.cj + d.cw > d.w)
    return;
  const int oy = p / out_w, ox = p - (p / out_w) * out_w;
  // flips act on the resized crop: output (oy, ox) shows resized (ry, rx)
  const int rx = (d.flags & 1) ? out_w - 1 - ox : ox;
  const int ry = (d.flags & 2) ? out_h - 1 - oy : oy;
  float wx[kAugMaxTaps], wy[kAugMaxTaps];
  int x0, y0;
  const int nx = aa_window(rx, d.cw, (float)d.cw / (float)out_w, antialias, wx, x0);
  const int ny = aa_window(ry, d.ch, (float)d.ch / (float)out_h, antialias, wy, y0);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int ky = 0; ky < ny; ++ky) {
    const uint8_t* row = d.src + ((size_t)(d.ci + y0 + ky) * d.w + d.cj + x0) * 4;
    float r[4] = {0.f, 0.f, 0.f, 0.f};
    for (int kx = 0; kx < nx; ++kx) {
      const uchar4 v = *reinterpret_cast<const uchar4*>(row + 4 * kx);
      const float w = wx[kx];
      r[0] += w * ((float)v.x / 255.0f);
      r[1] += w * ((float)v.y / 255.0f);
      r[2] += w * ((float)v.z / 255.0f);
      r[3] += w * ((float)v.w / 255.0f);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] += wy[ky] * r[c];
  }
  const float a = (d.flags & 4) ? 1.0f : acc[3];
  const size_t plane = (size_t)out_h * out_w;
  const size_t o3 = (size_t)b * 3 * plane + p, o4 = (size_t)b * 4 * plane + p;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    img[o3 + c * plane] = acc[c];
    masked[o3 + c * plane] = a > 0.f ? acc[c] : a;
    rgba[o4 + c * plane] = acc[c];
  }
  rgba[o4 + 3 * plane] = a;
  alpha[(size_t)b * plane + p] = a;
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_rgba_augment(int batch, const void* descs, int out_h, int out_w,
                                  int antialias, float* masked, float* alpha, float* img,
                                  float* rgba, void* stream) {
  RGBAC_REQUIRE(batch > 0 && batch < 65536 && out_h > 0 && out_w > 0, "shape");
  RGBAC_REQUIRE(descs && masked && alpha && img && rgba, "null pointer");
  RGBAC_REQUIRE((long long)out_h * out_w < (1LL << 31), "output too large");
  const int blocks = (int)(((long long)out_h * out_w + 255) / 256);
  hipLaunchKernelGGL(rgba_augment_kernel, dim3(blocks, batch), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const AugDesc*>(descs), out_h, out_w, antialias, masked,
                     alpha, img, rgba);
  return check_launch("rgba_augment_kernel");
}
