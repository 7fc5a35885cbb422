// MS-SSIM / SSIM evaluation metric (reference: metrics/ms_ssim_torch.py:5-194), used by the
// eval loop on the reconstruction (trainRGB.py:308-311).
//   * ssim_tile_kernel: one 16x16 tile of the VALID ssim / cs maps of one (image, channel)
//     plane (:59-71).  The (T+ws-1)^2 input patch of X and Y is staged in LDS, the 1-D
//     gaussian runs along W first and then along H (gaussian_filter :30-33), on the five
//     planes X, Y, X*X, Y*Y, X*Y; each workgroup leaves one (sum ssim, sum cs) partial pair
//     (fixed-order tree in the workgroup), so the result does not depend on scheduling.
//   * ssim_reduce_kernel: per image, the partials in a fixed order (double accumulation) ->
//     the CHW means of ssim_map and cs_map (:77-78).
//   * avgpool2_kernel: F.avg_pool2d(kernel 2, padding (H%2, W%2), count_include_pad) (:183-185).
//   * msssim_combine_kernel: prod_l (mcs_l ** w_l) * (ssim_last ** w_last) over the first
//     L-1 levels, broadcast exactly as :189-190 writes it, then the optional batch mean.
// The metric reads each level once (HBM-bound, ~8 B/pixel/level); it is not on the codec path.
#include "common.h"

namespace rgbac {

constexpr int SS_T = 16;         // output tile edge
constexpr int SS_MAXWS = 15;     // largest odd window the LDS patch holds
constexpr int SS_R = SS_T + SS_MAXWS - 1;

__global__ void __launch_bounds__(256)
ssim_tile_kernel(int H, int W, int ws, const float* __restrict__ X, const float* __restrict__ Y,
                 const float* __restrict__ win, float C1, float C2, int tiles_x, int ntiles,
                 float* __restrict__ partials) {
  __shared__ float sx[SS_R][SS_R + 1];
  __shared__ float sy[SS_R][SS_R + 1];
  __shared__ float sh[5][SS_R][SS_T + 1];
  __shared__ float red[2][4];
  const int tile = blockIdx.x;
  const long long plane = blockIdx.y;                 // b * C + c
  const int ty0 = (tile / tiles_x) * SS_T, tx0 = (tile % tiles_x) * SS_T;
  const int R = SS_T + ws - 1;
  const int Ho = H - ws + 1, Wo = W - ws + 1;
  const float* xp = X + plane * H * W;
  const float* yp = Y + plane * H * W;
  const int tid = threadIdx.x;
  for (int i = tid; i < R * R; i += 256) {
    const int r = i / R, c = i - r * R;
    const int gy = ty0 + r, gx = tx0 + c;
    const bool in = gy < H && gx < W;
    sx[r][c] = in ? xp[(long long)gy * W + gx] : 0.f;
    sy[r][c] = in ? yp[(long long)gy * W + gx] : 0.f;
  }
  __syncthreads();
  // horizontal pass (conv with win of shape (1, ws)): rows 0..R-1, output columns 0..T-1
  for (int i = tid; i < R * SS_T; i += 256) {
    const int r = i / SS_T, c = i - r * SS_T;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
    for (int k = 0; k < ws; ++k) {
      const float w = win[k];
      const float xv = sx[r][c + k], yv = sy[r][c + k];
      a0 += w * xv;
      a1 += w * yv;
      a2 += w * (xv * xv);
      a3 += w * (yv * yv);
      a4 += w * (xv * yv);
    }
    sh[0][r][c] = a0; sh[1][r][c] = a1; sh[2][r][c] = a2; sh[3][r][c] = a3; sh[4][r][c] = a4;
  }
  __syncthreads();
  const int ty = tid / SS_T, tx = tid - (tid / SS_T) * SS_T;
  float ssim_v = 0.f, cs_v = 0.f;
  if (ty0 + ty < Ho && tx0 + tx < Wo) {
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
    for (int k = 0; k < ws; ++k) {
      const float w = win[k];
      m1 += w * sh[0][ty + k][tx];
      m2 += w * sh[1][ty + k][tx];
      e11 += w * sh[2][ty + k][tx];
      e22 += w * sh[3][ty + k][tx];
      e12 += w * sh[4][ty + k][tx];
    }
    const float mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu1_mu2 = m1 * m2;
    const float s11 = e11 - mu1_sq, s22 = e22 - mu2_sq, s12 = e12 - mu1_mu2;
    cs_v = (2.f * s12 + C2) / (s11 + s22 + C2);
    ssim_v = ((2.f * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * cs_v;
  }
  for (int o = 32; o > 0; o >>= 1) {
    ssim_v += __shfl_xor(ssim_v, o);
    cs_v += __shfl_xor(cs_v, o);
  }
  if ((tid & 63) == 0) { red[0][tid >> 6] = ssim_v; red[1][tid >> 6] = cs_v; }
  __syncthreads();
  if (tid == 0) {
    float* out = partials + (plane * ntiles + tile) * 2;
    out[0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    out[1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
}

__global__ void __launch_bounds__(64)
ssim_reduce_kernel(int B, int C, int ntiles, long long npix, const float* __restrict__ partials,
                   float* __restrict__ ssim_out, float* __restrict__ cs_out) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  double s = 0.0, c = 0.0;
  const float* p = partials + (long long)b * C * ntiles * 2;
  for (long long i = 0; i < (long long)C * ntiles; ++i) {
    s += p[2 * i];
    c += p[2 * i + 1];
  }
  const double n = (double)C * (double)npix;
  ssim_out[b] = (float)(s / n);
  cs_out[b] = (float)(c / n);
}

__global__ void __launch_bounds__(256)
avgpool2_kernel(long long nout, int H, int W, int Ho, int Wo, int ph, int pw,
                const float* __restrict__ x, float* __restrict__ y) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nout) return;
  const long long plane = i / ((long long)Ho * Wo);
  const int s = (int)(i - plane * Ho * Wo);
  const int oy = s / Wo, ox = s - (s / Wo) * Wo;
  const float* xp = x + plane * H * W;
  float acc = 0.f;
  for (int dy = 0; dy < 2; ++dy) {
    const int iy = oy * 2 - ph + dy;
    for (int dx = 0; dx < 2; ++dx) {
      const int ix = ox * 2 - pw + dx;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) acc += xp[(long long)iy * W + ix];
    }
  }
  y[i] = acc / 4.f;  // count_include_pad: the 2x2 window always lies inside the padded plane
}

__global__ void __launch_bounds__(64)
msssim_combine_kernel(int levels, int B, const float* __restrict__ mcs,
                      const float* __restrict__ ssim_last, const float* __restrict__ weights,
                      float* __restrict__ per_image, float* __restrict__ mean) {
  __shared__ float vals[64];
  float total = 0.f;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int b = b0 + threadIdx.x;
    float v = 0.f;
    if (b < B) {
      const float tail = powf(ssim_last[b], weights[levels - 1]);
      v = 1.f;
      for (int l = 0; l < levels - 1; ++l) v *= powf(mcs[(long long)l * B + b], weights[l]) * tail;
      if (per_image) per_image[b] = v;
    }
    vals[threadIdx.x] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int j = 0; j < 64 && b0 + j < B; ++j) total += vals[j];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && mean) mean[0] = total / (float)B;
}

// ---- masked variant (reference: metrics/masked_ms_ssim_torch.py:56-265) ----
//   * masked_apply_kernel: the start of one ms_ssim level (:246-248): mask -> (mask > 0), and
//     X, Y multiplied by it (mask planes: 1, broadcast over the channels, or one per channel).
//   * masked_ssim_tile_kernel: the same VALID ssim / cs tile as above on the masked planes;
//     each output pixel is kept when the level mask, NEAREST-resized from (H, W) to
//     (H-ws+1, W-ws+1) (:103-105, torchvision resize = F.interpolate 'nearest': source index
//     min(floor(dst * (float)in / out), in - 1)), is nonzero.  Per tile: (sum ssim*keep,
//     sum cs*keep, count) (:107-116).
//   * masked_ssim_reduce_kernel: per (image, channel) plane, fixed-order double sums ->
//     sum / (count + 1e-10) (:115-116).
//   * masked_msssim_combine_kernel: prod_{l<L-1} relu(cs_l)^w_l * relu(ssim_last)^w_{L-1} per
//     (image, channel) (:252-260), then the channel mean per image and the (image, channel)
//     mean (:262-265).
__global__ void __launch_bounds__(256)
masked_apply_kernel(long long n, int C, int Cm, long long HW, const float* __restrict__ x,
                    const float* __restrict__ y, const float* __restrict__ mask,
                    float* __restrict__ xo, float* __restrict__ yo, float* __restrict__ mo) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const long long p = i % HW;
  const long long bc = i / HW;
  const long long b = bc / C;
  const int c = (int)(bc - b * C);
  const long long mi = (b * Cm + (Cm == 1 ? 0 : c)) * HW + p;
  const float m = mask[mi] > 0.f ? 1.f : 0.f;
  xo[i] = x[i] * m;
  yo[i] = y[i] * m;
  if (c < Cm) mo[mi] = m;
}

__global__ void __launch_bounds__(256)
masked_ssim_tile_kernel(int C, int Cm, int H, int W, int ws, const float* __restrict__ X,
                        const float* __restrict__ Y, const float* __restrict__ M,
                        const float* __restrict__ win, float C1, float C2, float scale_h,
                        float scale_w, int tiles_x, int ntiles, float* __restrict__ partials) {
  __shared__ float sx[SS_R][SS_R + 1];
  __shared__ float sy[SS_R][SS_R + 1];
  __shared__ float sh[5][SS_R][SS_T + 1];
  __shared__ float red[3][4];
  const int tile = blockIdx.x;
  const long long plane = blockIdx.y;                 // b * C + c
  const long long b = plane / C;
  const int c = (int)(plane - b * C);
  const int ty0 = (tile / tiles_x) * SS_T, tx0 = (tile % tiles_x) * SS_T;
  const int R = SS_T + ws - 1;
  const int Ho = H - ws + 1, Wo = W - ws + 1;
  const float* xp = X + plane * H * W;
  const float* yp = Y + plane * H * W;
  const float* mp = M + (b * Cm + (Cm == 1 ? 0 : c)) * (long long)H * W;
  const int tid = threadIdx.x;
  for (int i = tid; i < R * R; i += 256) {
    const int r = i / R, cc = i - r * R;
    const int gy = ty0 + r, gx = tx0 + cc;
    const bool in = gy < H && gx < W;
    sx[r][cc] = in ? xp[(long long)gy * W + gx] : 0.f;
    sy[r][cc] = in ? yp[(long long)gy * W + gx] : 0.f;
  }
  __syncthreads();
  for (int i = tid; i < R * SS_T; i += 256) {
    const int r = i / SS_T, cc = i - r * SS_T;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f, a4 = 0.f;
    for (int k = 0; k < ws; ++k) {
      const float w = win[k];
      const float xv = sx[r][cc + k], yv = sy[r][cc + k];
      a0 += w * xv;
      a1 += w * yv;
      a2 += w * (xv * xv);
      a3 += w * (yv * yv);
      a4 += w * (xv * yv);
    }
    sh[0][r][cc] = a0; sh[1][r][cc] = a1; sh[2][r][cc] = a2; sh[3][r][cc] = a3; sh[4][r][cc] = a4;
  }
  __syncthreads();
  const int ty = tid / SS_T, tx = tid - (tid / SS_T) * SS_T;
  float ssim_v = 0.f, cs_v = 0.f, keep = 0.f;
  const int oy = ty0 + ty, ox = tx0 + tx;
  if (oy < Ho && ox < Wo) {
    float m1 = 0.f, m2 = 0.f, e11 = 0.f, e22 = 0.f, e12 = 0.f;
    for (int k = 0; k < ws; ++k) {
      const float w = win[k];
      m1 += w * sh[0][ty + k][tx];
      m2 += w * sh[1][ty + k][tx];
      e11 += w * sh[2][ty + k][tx];
      e22 += w * sh[3][ty + k][tx];
      e12 += w * sh[4][ty + k][tx];
    }
    const float mu1_sq = m1 * m1, mu2_sq = m2 * m2, mu1_mu2 = m1 * m2;
    const float s11 = e11 - mu1_sq, s22 = e22 - mu2_sq, s12 = e12 - mu1_mu2;
    const float csm = (2.f * s12 + C2) / (s11 + s22 + C2);
    const float ssm = ((2.f * mu1_mu2 + C1) / (mu1_sq + mu2_sq + C1)) * csm;
    const int sy_ = min((int)floorf((float)oy * scale_h), H - 1);
    const int sx_ = min((int)floorf((float)ox * scale_w), W - 1);
    keep = mp[(long long)sy_ * W + sx_] != 0.f ? 1.f : 0.f;
    ssim_v = ssm * keep;
    cs_v = csm * keep;
  }
  for (int o = 32; o > 0; o >>= 1) {
    ssim_v += __shfl_xor(ssim_v, o);
    cs_v += __shfl_xor(cs_v, o);
    keep += __shfl_xor(keep, o);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = ssim_v; red[1][tid >> 6] = cs_v; red[2][tid >> 6] = keep;
  }
  __syncthreads();
  if (tid == 0) {
    float* out = partials + (plane * ntiles + tile) * 3;
    out[0] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    out[1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    out[2] = (red[2][0] + red[2][1]) + (red[2][2] + red[2][3]);   // exact: <= 256 ones
  }
}

__global__ void __launch_bounds__(64)
masked_ssim_reduce_kernel(long long planes, int ntiles, const float* __restrict__ partials,
                          float* __restrict__ ssim_out, float* __restrict__ cs_out) {
  const long long pl = (long long)blockIdx.x * 64 + threadIdx.x;
  if (pl >= planes) return;
  double s = 0.0, c = 0.0, n = 0.0;
  const float* p = partials + pl * ntiles * 3;
  for (int i = 0; i < ntiles; ++i) {
    s += p[3 * i];
    c += p[3 * i + 1];
    n += p[3 * i + 2];
  }
  const float den = (float)n + 1e-10f;
  ssim_out[pl] = (float)s / den;
  cs_out[pl] = (float)c / den;
}

__global__ void __launch_bounds__(64)
masked_msssim_combine_kernel(int levels, int B, int C, const float* __restrict__ mcs,
                             const float* __restrict__ ssim_last,
                             const float* __restrict__ weights, float* __restrict__ per_image,
                             float* __restrict__ mean) {
  __shared__ float vals[64];
  const long long BC = (long long)B * C;
  double total = 0.0;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int b = b0 + threadIdx.x;
    double img = 0.0;
    if (b < B) {
      for (int c = 0; c < C; ++c) {
        const long long k = (long long)b * C + c;
        float v = powf(fmaxf(ssim_last[k], 0.f), weights[levels - 1]);
        for (int l = 0; l < levels - 1; ++l) v *= powf(fmaxf(mcs[l * BC + k], 0.f), weights[l]);
        img += v;
      }
      if (per_image) per_image[b] = (float)(img / C);
    }
    vals[threadIdx.x] = (float)img;
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int j = 0; j < 64 && b0 + j < B; ++j) total += vals[j];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && mean) mean[0] = (float)(total / (double)BC);
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_ssim_level(int batch, int channels, int h, int w, int win_size,
                                const float* x, const float* y, const float* win, float c1,
                                float c2, float* partials, float* ssim_out, float* cs_out,
                                void* stream) {
  RGBAC_REQUIRE(batch > 0 && channels > 0, "shape");
  RGBAC_REQUIRE(win_size >= 1 && win_size <= SS_MAXWS && (win_size & 1), "window size");
  RGBAC_REQUIRE(h >= win_size && w >= win_size, "image smaller than the window");
  RGBAC_REQUIRE(x && y && win && partials && ssim_out && cs_out, "null pointer");
  const int ho = h - win_size + 1, wo = w - win_size + 1;
  const int tiles_x = (wo + SS_T - 1) / SS_T, tiles_y = (ho + SS_T - 1) / SS_T;
  const int ntiles = tiles_x * tiles_y;
  RGBAC_REQUIRE((long long)batch * channels <= 65535, "too many planes for one launch");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(ssim_tile_kernel, dim3(ntiles, batch * channels), dim3(256), 0, st, h, w,
                     win_size, x, y, win, c1, c2, tiles_x, ntiles, partials);
  int rc = check_launch("ssim_tile_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(ssim_reduce_kernel, dim3((batch + 63) / 64), dim3(64), 0, st, batch,
                     channels, ntiles, (long long)ho * wo, partials, ssim_out, cs_out);
  return check_launch("ssim_reduce_kernel");
}

extern "C" int rgbac_avgpool2(int planes, int h, int w, const float* x, float* y, void* stream) {
  RGBAC_REQUIRE(planes > 0 && h > 0 && w > 0 && x && y, "shape / pointer");
  const int ph = h % 2, pw = w % 2;
  const int ho = (h + 2 * ph - 2) / 2 + 1, wo = (w + 2 * pw - 2) / 2 + 1;
  const long long n = (long long)planes * ho * wo;
  hipLaunchKernelGGL(avgpool2_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), n, h, w, ho, wo, ph, pw, x, y);
  return check_launch("avgpool2_kernel");
}

extern "C" int rgbac_msssim_combine(int levels, int batch, const float* mcs,
                                    const float* ssim_last, const float* weights,
                                    float* per_image, float* mean, void* stream) {
  RGBAC_REQUIRE(levels >= 1 && batch > 0 && mcs && ssim_last && weights, "arguments");
  RGBAC_REQUIRE(per_image || mean, "no output");
  hipLaunchKernelGGL(msssim_combine_kernel, dim3(1), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), levels, batch, mcs, ssim_last,
                     weights, per_image, mean);
  return check_launch("msssim_combine_kernel");
}

extern "C" int rgbac_masked_apply(int batch, int channels, int mask_channels, int h, int w,
                                  const float* x, const float* y, const float* mask, float* x_out,
                                  float* y_out, float* mask_out, void* stream) {
  RGBAC_REQUIRE(batch > 0 && channels > 0 && h > 0 && w > 0, "shape");
  RGBAC_REQUIRE(mask_channels == 1 || mask_channels == channels, "mask channels: 1 or C");
  RGBAC_REQUIRE(x && y && mask && x_out && y_out && mask_out, "null pointer");
  const long long n = (long long)batch * channels * h * w;
  hipLaunchKernelGGL(masked_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), n, channels, mask_channels,
                     (long long)h * w, x, y, mask, x_out, y_out, mask_out);
  return check_launch("masked_apply_kernel");
}

extern "C" int rgbac_masked_ssim_level(int batch, int channels, int mask_channels, int h, int w,
                                       int win_size, const float* x, const float* y,
                                       const float* mask, const float* win, float c1, float c2,
                                       float* partials, float* ssim_out, float* cs_out,
                                       void* stream) {
  RGBAC_REQUIRE(batch > 0 && channels > 0, "shape");
  RGBAC_REQUIRE(mask_channels == 1 || mask_channels == channels, "mask channels: 1 or C");
  RGBAC_REQUIRE(win_size >= 1 && win_size <= SS_MAXWS && (win_size & 1), "window size");
  RGBAC_REQUIRE(h >= win_size && w >= win_size, "image smaller than the window");
  RGBAC_REQUIRE(x && y && mask && win && partials && ssim_out && cs_out, "null pointer");
  const int ho = h - win_size + 1, wo = w - win_size + 1;
  const int tiles_x = (wo + SS_T - 1) / SS_T, tiles_y = (ho + SS_T - 1) / SS_T;
  const int ntiles = tiles_x * tiles_y;
  RGBAC_REQUIRE((long long)batch * channels <= 65535, "too many planes for one launch");
  // torch's nearest scale: (float)input_size / output_size (no scale_factor given)
  const float scale_h = (float)h / (float)ho, scale_w = (float)w / (float)wo;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(masked_ssim_tile_kernel, dim3(ntiles, batch * channels), dim3(256), 0, st,
                     channels, mask_channels, h, w, win_size, x, y, mask, win, c1, c2, scale_h,
                     scale_w, tiles_x, ntiles, partials);
  int rc = check_launch("masked_ssim_tile_kernel");
  if (rc) return rc;
  const long long planes = (long long)batch * channels;
  hipLaunchKernelGGL(masked_ssim_reduce_kernel, dim3((unsigned)((planes + 63) / 64)), dim3(64), 0,
                     st, planes, ntiles, partials, ssim_out, cs_out);
  return check_launch("masked_ssim_reduce_kernel");
}

extern "C" int rgbac_masked_msssim_combine(int levels, int batch, int channels, const float* mcs,
                                           const float* ssim_last, const float* weights,
                                           float* per_image, float* mean, void* stream) {
  RGBAC_REQUIRE(levels >= 1 && batch > 0 && channels > 0, "arguments");
  RGBAC_REQUIRE((levels == 1 || mcs) && ssim_last && weights, "null pointer");
  RGBAC_REQUIRE(per_image || mean, "no output");
  hipLaunchKernelGGL(masked_msssim_combine_kernel, dim3(1), dim3(64), 0,
                     reinterpret_cast<hipStream_t>(stream), levels, batch, channels, mcs,
                     ssim_last, weights, per_image, mean);
  return check_launch("masked_msssim_combine_kernel");
}
