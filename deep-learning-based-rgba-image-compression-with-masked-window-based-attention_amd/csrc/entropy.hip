// Coalesced HBM-bound kernels around the conv/attention engine:
//   * Gaussian conditional likelihood + quantise + bits (per channel slice),
//   * factorized-prior (EntropyBottleneck) likelihood + z quantise,
//   * masked MSE / bpp finalisation (deterministic two-level fp64 sums),
//   * SupplyMaskToTransform pyramid (+ reconmask round to 1/255),
//   * NCHW <-> NHWC conversion at the model boundary,
//   * the library's error plumbing.
#include <cmath>
#include <cstdio>

#include "common.h"

namespace rgbac {

static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(e));
    return RGBAC_E_LAUNCH;
  }
  return RGBAC_OK;
}

// compressai GaussianConditional._standardized_cumulative: 0.5*erfc(-(2^-0.5) * t)
__device__ __forceinline__ float std_cum(float t) {
  return 0.5f * erfcf(-0.70710678118654752440f * t);
}
__device__ __forceinline__ float bits_of(float lik) {
  // clamp(-1.0 * log(lik + 1e-10) / log(2.0), 0, 50)   (AutoEncoderRGB_Journal.py:280)
  float b = (-1.0f * logf(lik + 1e-10f)) / 0.69314718055994530942f;
  return fminf(fmaxf(b, 0.0f), 50.0f);
}

template <typename T>
__global__ void __launch_bounds__(256)
gaussian_slice_kernel(long long n, int nch, const T* __restrict__ y, long long ldy,
                      const T* __restrict__ mu, long long ldmu, const T* __restrict__ sc,
                      long long lds, const float* __restrict__ noise, T* __restrict__ hat,
                      long long ldh, float* __restrict__ likout, double* __restrict__ partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const long long pix = e / nch;
    const int ch = (int)(e - pix * nch);
    const float yv = Elem<T>::ld(y + pix * ldy + ch);
    const float mv = Elem<T>::ld(mu + pix * ldmu + ch);
    const float sv = Elem<T>::ld(sc + pix * lds + ch);
    const float qh = rintf(yv - mv) + mv;              // ste_round(y - mu) + mu (forward value)
    Elem<T>::st(hat + pix * ldh + ch, qh);
    const float xin = noise ? yv + noise[e] : qh;      // quantize("noise" | "dequantize")
    const float v = fabsf(xin - mv);
    const float s = fmaxf(sv, 0.11f);                  // lower_bound_scale
    const float up = std_cum((0.5f - v) / s);
    const float lo = std_cum((-0.5f - v) / s);
    const float lik = fmaxf(up - lo, 1e-9f);           // likelihood_lower_bound
    if (likout) likout[e] = lik;
    acc += (double)bits_of(lik);
  }
  const double s = block_sum_f64(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// EntropyBottleneck param block per channel (fp32, 64 floats):
//  [0:3) sp(M0) [3:12) sp(M1) [12:21) sp(M2) [21:30) sp(M3) [30:33) sp(M4)
//  [33:36) b0 [36:39) b1 [39:42) b2 [42:45) b3 [45] b4
//  [46:49) tanh(f0) [49:52) tanh(f1) [52:55) tanh(f2) [55:58) tanh(f3) [58] median
constexpr int kEbStride = 64;

__device__ __forceinline__ float eb_logits(const float* P, float x) {
  float t[3], u[3];
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    float a = P[0 + o] * x;
    a = a + P[33 + o];
    t[o] = a + P[46 + o] * tanhf(a);
  }
#pragma unroll
  for (int layer = 0; layer < 3; ++layer) {
    const float* Mx = P + 3 + 9 * layer;
    const float* bx = P + 36 + 3 * layer;
    const float* fx = P + 49 + 3 * layer;
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      float a = Mx[o * 3 + 0] * t[0];
      a = fmaf(Mx[o * 3 + 1], t[1], a);
      a = fmaf(Mx[o * 3 + 2], t[2], a);
      a = a + bx[o];
      u[o] = a + fx[o] * tanhf(a);
    }
#pragma unroll
    for (int o = 0; o < 3; ++o) t[o] = u[o];
  }
  float a = P[30] * t[0];
  a = fmaf(P[31], t[1], a);
  a = fmaf(P[32], t[2], a);
  return a + P[45];
}
__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }

template <typename T>
__global__ void __launch_bounds__(256)
eb_forward_kernel(long long n, int C, const T* __restrict__ z, long long ldz,
                  const float* __restrict__ params, const float* __restrict__ noise,
                  T* __restrict__ zhat, long long ldh, float* __restrict__ likout,
                  double* __restrict__ partial) {
  __shared__ double red[4];
  double acc = 0.0;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const long long pix = e / C;
    const int ch = (int)(e - pix * C);
    const float* P = params + (size_t)ch * kEbStride;
    const float med = P[58];
    const float zv = Elem<T>::ld(z + pix * ldz + ch);
    const float q = rintf(zv - med) + med;
    Elem<T>::st(zhat + pix * ldh + ch, q);
    const float xin = noise ? zv + noise[e] : q;
    const float lo = eb_logits(P, xin - 0.5f);
    const float up = eb_logits(P, xin + 0.5f);
    const float lik = fmaxf(sigm(up) - sigm(lo), 1e-9f);
    if (likout) likout[e] = lik;
    acc += (double)bits_of(lik);
  }
  const double s = block_sum_f64(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// Per-(image, block) partial sums of the reconstruction error.
//   mode 0: masked (AutoEncoderRGB_Journal.py:36-64): se = sum m*(x-xh)^2 over 3 channels,
//           cnt = 3 * #(mask > 0)
//   mode 1: plain (AutoEncoderMask_Journal.py:309): se = sum (xh - x)^2, cnt = #elements
template <typename T>
__device__ __forceinline__ void mse_block(int mode, int cx, int HW, const float* __restrict__ x,
                                          const T* __restrict__ xh, long long ldh,
                                          const float* __restrict__ mask, double* __restrict__ part,
                                          float* __restrict__ xo, int vec, double* red) {
  // xo (or null): x_hat's fp32 NCHW copy, written from the same reads (rgbac_finalize_ex).
  // vec (cx <= 4, vector-aligned rows): the pixel's channels arrive in one vector load.
  const int b = blockIdx.y;
  double se = 0.0, cnt = 0.0;
  if (vec) {
    // the thread's (<= 4, rgbac_finalize_blocks) pixels: every load issued before the first
    // use, then the same per-pixel, per-channel order as the loop below (bit-identical sums;
    // the loop's dependent load -> add chain was ~3x the HBM time of the pass)
    constexpr int U = 4;
    const int stride = gridDim.x * 256;
    for (int p0 = blockIdx.x * 256 + threadIdx.x; p0 < HW; p0 += U * stride) {
      float mv[U], hq[U][4], xv[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * stride;
        mv[u] = 0.0f;
        if (p < HW) {
          const long long pix = (long long)b * HW + p;
          mv[u] = mode == 0 ? (mask[pix] > 0.0f ? 1.0f : 0.0f) : 1.0f;
          Elem<T>::ld4(xh + pix * ldh, hq[u]);
#pragma unroll
          for (int c = 0; c < 4; ++c)
            xv[u][c] = c < cx ? x[((long long)b * cx + c) * HW + p] : 0.0f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int p = p0 + u * stride;
        if (p >= HW) break;
        const float m = mv[u];
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if (c >= cx) break;
          const float hv = hq[u][c], xc = xv[u][c];
          if (xo) xo[((long long)b * cx + c) * HW + p] = hv;
          const float dlt = mode == 0 ? (xc * m - hv * m) : (hv - xc);
          se += (double)(dlt * dlt);
        }
        cnt += (double)(m * cx);
      }
    }
  } else
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
    const long long pix = (long long)b * HW + p;
    float m = 1.0f;
    if (mode == 0) m = mask[pix] > 0.0f ? 1.0f : 0.0f;
    auto term = [&](int c, float hv) {
      const float xv = x[((long long)b * cx + c) * HW + p];
      if (xo) xo[((long long)b * cx + c) * HW + p] = hv;
      const float dlt = mode == 0 ? (xv * m - hv * m) : (hv - xv);
      se += (double)(dlt * dlt);
    };
    if (vec) {
      float hq[4];
      Elem<T>::ld4(xh + pix * ldh, hq);
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (c < cx) term(c, hq[c]);
    } else {
      for (int c = 0; c < cx; ++c) term(c, Elem<T>::ld(xh + pix * ldh + c));
    }
    cnt += (double)(m * cx);
  }
  const double s0 = block_sum_f64(se, red);
  const double s1 = block_sum_f64(cnt, red);
  if (threadIdx.x == 0) {
    part[((size_t)b * gridDim.x + blockIdx.x) * 2 + 0] = s0;
    part[((size_t)b * gridDim.x + blockIdx.x) * 2 + 1] = s1;
  }
}

template <typename T>
__global__ void __launch_bounds__(256)
mse_partial_kernel(int mode, int cx, int HW, const float* __restrict__ x, const T* __restrict__ xh,
                   long long ldh, const float* __restrict__ mask, double* __restrict__ part,
                   float* __restrict__ xo, int vec) {
  __shared__ double red[4];
  mse_block<T>(mode, cx, HW, x, xh, ldh, mask, part, xo, vec, red);
}

constexpr int kFinWaves = 16;   // finalize_kernel: one 1024-thread block

// The finalisation of one forward by the NW waves of one block: every reduction is a wave
// reduction (shuffles, no barrier) and the waves' results meet once in LDS, combined in wave
// order (fixed order: deterministic).  Wave w owns images w, w + NW, ...  The bits partials are
// summed four independent chains per thread (their loads in flight together: a single dependent
// chain over the 1024^2 frame's 20k partials was 37 us of load latencies), the chains then added
// in a fixed order.
template <int NW>
__device__ __forceinline__ void finalize_body(int mode, int batch, int nblk, double npix,
                                              const double* __restrict__ part,
                                              const double* __restrict__ yb, int ny,
                                              const double* __restrict__ zb, int nz,
                                              float* __restrict__ out, double (*wred)[5]) {
  constexpr int NT = 64 * NW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double ya[4] = {0.0, 0.0, 0.0, 0.0}, za[4] = {0.0, 0.0, 0.0, 0.0};
  for (int i0 = threadIdx.x; i0 < ny; i0 += 4 * NT) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * NT;
      ya[u] += i < ny ? yb[i] : 0.0;
    }
  }
  for (int i0 = threadIdx.x; i0 < nz; i0 += 4 * NT) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * NT;
      za[u] += i < nz ? zb[i] : 0.0;
    }
  }
  double ys = (ya[0] + ya[1]) + (ya[2] + ya[3]);
  double zs = (za[0] + za[1]) + (za[2] + za[3]);
  for (int o = 32; o > 0; o >>= 1) {
    ys += __shfl_xor(ys, o);
    zs += __shfl_xor(zs, o);
  }
  double mse_acc = 0.0, se_all = 0.0, cnt_all = 0.0;
  for (int b = wave; b < batch; b += NW) {
    double se = 0.0, cnt = 0.0;
    for (int i = lane; i < nblk; i += 64) {
      se += part[((size_t)b * nblk + i) * 2 + 0];
      cnt += part[((size_t)b * nblk + i) * 2 + 1];
    }
    for (int o = 32; o > 0; o >>= 1) {
      se += __shfl_xor(se, o);
      cnt += __shfl_xor(cnt, o);
    }
    // per-image mean: torch.div(mse, clamp(num_unmasked, min=1)) in fp32
    const float sef = (float)se, cf = fmaxf((float)cnt, 1.0f);
    mse_acc += (double)(sef / cf);
    se_all += se;
    cnt_all += cnt;
  }
  if (lane == 0) {
    wred[wave][0] = ys; wred[wave][1] = zs; wred[wave][2] = mse_acc;
    wred[wave][3] = se_all; wred[wave][4] = cnt_all;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      t[k] = 0.0;
      for (int w = 0; w < NW; ++w) t[k] += wred[w][k];
    }
    float mse;
    if (mode == 0)
      mse = (float)(t[2] / batch);
    else
      mse = (float)(t[3] / t[4]);
    const float ybits = (float)t[0], zbits = (float)t[1];
    const float yb_pp = ybits / (float)npix, zb_pp = zbits / (float)npix;
    out[0] = mse;
    out[1] = yb_pp + zb_pp;
    out[2] = yb_pp;
    out[3] = zb_pp;
  }
}

__global__ void __launch_bounds__(64 * kFinWaves)
finalize_kernel(int mode, int batch, int nblk, double npix, const double* __restrict__ part,
                const double* __restrict__ yb, int ny, const double* __restrict__ zb, int nz,
                float* __restrict__ out) {
  __shared__ double wred[kFinWaves][5];
  finalize_body<kFinWaves>(mode, batch, nblk, npix, part, yb, ny, zb, nz, out, wred);
}

__global__ void round255_kernel(long long n, const float* __restrict__ in, float* __restrict__ out) {
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    out[i] = rintf(in[i] * 255.0f) / 255.0f;
  }
}

// AvgPool2d(3, stride=2, padding=1, count_include_pad=True) on [B,H,W]
__global__ void avgpool3s2_kernel(int batch, int H, int W, int Ho, int Wo,
                                  const float* __restrict__ in, float* __restrict__ out) {
  const long long n = (long long)batch * Ho * Wo;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int ox = (int)(i % Wo);
    const long long t = i / Wo;
    const int oy = (int)(t % Ho);
    const int b = (int)(t / Ho);
    float s = 0.f;
    for (int dy = -1; dy <= 1; ++dy) {
      const int iy = 2 * oy + dy;
      if (iy < 0 || iy >= H) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int ix = 2 * ox + dx;
        if (ix < 0 || ix >= W) continue;
        s += in[((long long)b * H + iy) * W + ix];
      }
    }
    out[i] = s / 9.0f;
  }
}

// The whole mask pyramid of rgbac_mask_pyramid (optional round(255 a) / 255, then L levels of
// AvgPool2d(3, 2, 1, count_include_pad)) in ONE launch instead of 1 + L: a workgroup owns a
// TP x TP tile of the last level and recomputes, in LDS, every level's region that tile
// depends on (region of level l = 2 x that of level l + 1, plus one), writing the core rows
// of every level it owns.  Each value is the same float sum in the same tap order as
// avgpool3s2_kernel (out-of-image taps there are skipped, here added as +0): bit-identical.
struct PyrOuts { float* p[4]; };

template <int L>
__device__ __forceinline__ void pyramid_tile(int blk, int batch, int H, int W,
                                             const float* __restrict__ alpha, int round255,
                                             float* __restrict__ rounded, const PyrOuts& outs,
                                             float* pyr) {
  constexpr int TP = 32 >> L;                          // last-level tile: 16 / 8 / 4 / 2
  constexpr int N0 = (TP + 1) * (1 << L) - 1;          // level-0 region side (33 .. 47)
  constexpr int NL0 = (N0 * N0 + 255) / 256;           // level-0 elements per thread
  float* bufA = pyr;
  float* bufB = pyr + N0 * N0;
  int sh[L + 1], sw[L + 1];
  sh[0] = H; sw[0] = W;
#pragma unroll
  for (int l = 1; l <= L; ++l) { sh[l] = (sh[l - 1] - 1) / 2 + 1; sw[l] = (sw[l - 1] - 1) / 2 + 1; }
  const int ntx = (sw[L] + TP - 1) / TP, nty = (sh[L] + TP - 1) / TP;
  int t = blk;
  const int tx = t % ntx; t /= ntx;
  const int ty = t % nty;
  const int b = t / nty;
  // level-0 region origin and side
  const int s0 = 1 << L;
  const int ry = ty * TP * s0 - (s0 - 1), rx = tx * TP * s0 - (s0 - 1);
  const float* ab = alpha + (long long)b * H * W;
  // every load of the thread first (one memory round trip, not NL0 dependent ones), then the
  // rounding, the owned-core stores and the LDS image
  float v0[NL0];
#pragma unroll
  for (int k = 0; k < NL0; ++k) {
    const int e = threadIdx.x + 256 * k;
    const int i = e / N0, j = e - (e / N0) * N0;
    const int y = ry + i, x = rx + j;
    const bool in = e < N0 * N0 && y >= 0 && y < H && x >= 0 && x < W;
    v0[k] = in ? ab[(long long)y * W + x] : 0.0f;
  }
#pragma unroll
  for (int k = 0; k < NL0; ++k) {
    const int e = threadIdx.x + 256 * k;
    if (e >= N0 * N0) break;
    const int i = e / N0, j = e - (e / N0) * N0;
    const int y = ry + i, x = rx + j;
    float v = v0[k];
    if (round255 && y >= 0 && y < H && x >= 0 && x < W) {
      v = rintf(v * 255.0f) / 255.0f;
      // core rows / cols of level 0 owned by this tile
      if (i >= s0 - 1 && i < s0 - 1 + TP * s0 && j >= s0 - 1 && j < s0 - 1 + TP * s0)
        rounded[((long long)b * H + y) * W + x] = v;
    }
    bufA[e] = v;
  }
  __syncthreads();
  int n = N0;                                          // side of the previous level's region
#pragma unroll
  for (int l = 1; l <= L; ++l) {
    const int m = (n - 1) / 2;                         // this level's region side
    const int sc = 1 << (L - l);
    const int oy = ty * TP * sc - (sc - 1), ox = tx * TP * sc - (sc - 1);   // region origin
    float* const o = outs.p[l - 1];
    for (int e = threadIdx.x; e < m * m; e += 256) {
      const int i = e / m, j = e - (e / m) * m;
      const int y = oy + i, x = ox + j;
      float v = 0.0f;
      if (y >= 0 && y < sh[l] && x >= 0 && x < sw[l]) {
        float s = 0.f;
#pragma unroll
        for (int dy = 0; dy < 3; ++dy)
#pragma unroll
          for (int dx = 0; dx < 3; ++dx) s += bufA[(2 * i + dy) * n + 2 * j + dx];
        v = s / 9.0f;
        if (i >= sc - 1 && i < sc - 1 + TP * sc && j >= sc - 1 && j < sc - 1 + TP * sc)
          o[((long long)b * sh[l] + y) * sw[l] + x] = v;
      }
      bufB[e] = v;
    }
    __syncthreads();
    float* tmp = bufA; bufA = bufB; bufB = tmp;
    n = m;
  }
}

template <int L>
__global__ void __launch_bounds__(256) pyramid_kernel(int batch, int H, int W,
                                                      const float* __restrict__ alpha,
                                                      int round255, float* __restrict__ rounded,
                                                      PyrOuts outs) {
  extern __shared__ float pyr[];
  pyramid_tile<L>(blockIdx.x, batch, H, W, alpha, round255, rounded, outs, pyr);
}

template <typename T>
__global__ void nchw_to_nhwc_kernel(int batch, int C, int HW, const float* __restrict__ src,
                                    T* __restrict__ dst, long long ldc) {
  const long long n = (long long)batch * HW * ldc;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long pix = i / ldc;
    const int c = (int)(i - pix * ldc);
    const int b = (int)(pix / HW);
    const int p = (int)(pix - (long long)b * HW);
    const float v = c < C ? src[((long long)b * C + c) * HW + p] : 0.0f;
    Elem<T>::st(dst + i, v);
  }
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(int batch, int C, int HW, const T* __restrict__ src,
                                    long long ldc, float* __restrict__ dst) {
  const long long n = (long long)batch * C * HW;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int p = (int)(i % HW);
    const long long t = i / HW;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    dst[i] = Elem<T>::ld(src + ((long long)b * HW + p) * ldc + c);
  }
}

// One thread per (pixel, 16-byte chunk of the NHWC row): the reads of a channel plane are
// coalesced over consecutive pixels, the row chunk goes out as one 16-byte store, and the
// indices are 32-bit (the grid-stride form above divides 64-bit indices per element).
template <typename T>
__device__ __forceinline__ void nchw_chunk(int i, int nck, int C, int HW,
                                           const float* __restrict__ src, T* __restrict__ dst,
                                           int ldc) {
  constexpr int E = Elem<T>::EPV;
  const int pix = i / nck, ck = i - (i / nck) * nck;
  const int b = pix / HW, p = pix - (pix / HW) * HW;
  float v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int c = ck * E + e;
    v[e] = c < C ? src[((long long)b * C + c) * HW + p] : 0.0f;
  }
  T* o = dst + (long long)pix * ldc + ck * E;
  if constexpr (E == 8) {
    uint4 q;
    q.x = pack_bf16x2(v[0], v[1]); q.y = pack_bf16x2(v[2], v[3]);
    q.z = pack_bf16x2(v[4], v[5]); q.w = pack_bf16x2(v[6], v[7]);
    *reinterpret_cast<uint4*>(o) = q;
  } else {
    *reinterpret_cast<float4*>(o) = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) nchw_to_nhwc_chunk_kernel(int n, int nck, int C, int HW,
                                                                 const float* __restrict__ src,
                                                                 T* __restrict__ dst, int ldc) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) nchw_chunk<T>(i, nck, C, HW, src, dst, ldc);
}

// The forward's prologue in ONE launch (rgbac_forward_prologue): three independent jobs that
// each took a launch of their own at the head of the forward graph --
//   blocks [0, npyr):  the decoder's mask pyramid (pyramid_tile, round(255 a) / 255 first),
//   blocks [npyr, ..): the input's NCHW -> NHWC conversion (one 16-byte row chunk per thread),
//                      and, grid-strided over the same blocks, the zero fill of the forward's
//                      bits partials.
// Every job writes exactly what its own kernel writes: the outputs are bit-identical.
template <int L, typename T>
__global__ void __launch_bounds__(256) prologue_kernel(int npyr, int batch, int H, int W,
                                                       const float* __restrict__ alpha,
                                                       int round255, float* __restrict__ rounded,
                                                       PyrOuts outs, int n, int nck, int C,
                                                       const float* __restrict__ src,
                                                       T* __restrict__ dst, int ldc,
                                                       double* __restrict__ zero, int nzero) {
  extern __shared__ float pyr[];
  if ((int)blockIdx.x < npyr) {
    pyramid_tile<L>(blockIdx.x, batch, H, W, alpha, round255, rounded, outs, pyr);
    return;
  }
  const int bx = (int)blockIdx.x - npyr, ncv = (int)gridDim.x - npyr;
  for (int e = bx * 256 + threadIdx.x; e < nzero; e += ncv * 256) zero[e] = 0.0;
  const int i = bx * 256 + threadIdx.x;
  if (i < n) nchw_chunk<T>(i, nck, C, H * W, src, dst, ldc);
}

// One thread per pixel: its NHWC row read in 16-byte chunks, each channel written to its plane
// (coalesced over consecutive pixels).
template <typename T>
__global__ void __launch_bounds__(256) nhwc_to_nchw_px_kernel(int npix, int C, int HW,
                                                              const T* __restrict__ src, int ldc,
                                                              float* __restrict__ dst) {
  constexpr int E = Elem<T>::EPV;
  const int pix = blockIdx.x * 256 + threadIdx.x;
  if (pix >= npix) return;
  const int b = pix / HW, p = pix - (pix / HW) * HW;
  const T* row = src + (long long)pix * ldc;
  for (int c0 = 0; c0 < C; c0 += E) {
    const uint4 q = *reinterpret_cast<const uint4*>(row + c0);
    float v[E];
    if constexpr (E == 8) {
      const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) { v[2 * k] = bf2f(w[k] & 0xFFFF); v[2 * k + 1] = bf2f(w[k] >> 16); }
    } else {
      v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y);
      v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
    }
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (c0 + e < C) dst[((long long)b * C + c0 + e) * HW + p] = v[e];
  }
}

static int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_abi_version(void) { return RGBAC_ABI_VERSION; }
extern "C" const char* rgbac_last_error(void) { return g_last_error.c_str(); }
extern "C" int rgbac_reduce_blocks(int64_t n) { return reduce_blocks(n); }

extern "C" int rgbac_gaussian_slice(int dtype, int64_t npix, int nch, const void* y, int64_t ldy,
                                    const void* mu, int64_t ldmu, const void* scale, int64_t lds,
                                    const float* noise, void* out_hat, int64_t ldh, float* lik,
                                    double* partial, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(npix > 0 && nch > 0, "empty slice");
  RGBAC_REQUIRE(y && mu && scale && out_hat && partial, "null pointer");
  const long long n = npix * (long long)nch;
  const int g = reduce_blocks(n);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(gaussian_slice_kernel<float>, dim3(g), dim3(256), 0, st, n, nch,
                       (const float*)y, ldy, (const float*)mu, ldmu, (const float*)scale, lds,
                       noise, (float*)out_hat, ldh, lik, partial);
  else
    hipLaunchKernelGGL(gaussian_slice_kernel<bf16_t>, dim3(g), dim3(256), 0, st, n, nch,
                       (const bf16_t*)y, ldy, (const bf16_t*)mu, ldmu, (const bf16_t*)scale, lds,
                       noise, (bf16_t*)out_hat, ldh, lik, partial);
  return check_launch("gaussian_slice_kernel");
}

extern "C" int rgbac_eb_forward(int dtype, int64_t npix, int channels, const void* z, int64_t ldz,
                                const float* params, const float* noise, void* z_hat, int64_t ldh,
                                float* lik, double* partial, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(npix > 0 && channels > 0, "empty tensor");
  RGBAC_REQUIRE(z && params && z_hat && partial, "null pointer");
  const long long n = npix * (long long)channels;
  const int g = reduce_blocks(n);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(eb_forward_kernel<float>, dim3(g), dim3(256), 0, st, n, channels,
                       (const float*)z, ldz, params, noise, (float*)z_hat, ldh, lik, partial);
  else
    hipLaunchKernelGGL(eb_forward_kernel<bf16_t>, dim3(g), dim3(256), 0, st, n, channels,
                       (const bf16_t*)z, ldz, params, noise, (bf16_t*)z_hat, ldh, lik, partial);
  return check_launch("eb_forward_kernel");
}

extern "C" int rgbac_finalize_blocks(int h, int w) {
  const long long hw = (long long)h * w;
  long long n = (hw + 1023) / 1024;
  return (int)(n < 64 ? 64 : (n > 1024 ? 1024 : n));
}

extern "C" int rgbac_finalize(int dtype, int mode, int batch, int cx, int h, int w, const float* x,
                              const void* x_hat, int64_t ldh, const float* mask,
                              const double* ybits, int ny, const double* zbits, int nz,
                              double* scratch, float* out, void* stream) {
  return rgbac_finalize_ex(dtype, mode, batch, cx, h, w, x, x_hat, ldh, mask, ybits, ny, zbits,
                           nz, scratch, out, nullptr, stream);
}

extern "C" int rgbac_finalize_ex(int dtype, int mode, int batch, int cx, int h, int w,
                                 const float* x, const void* x_hat, int64_t ldh,
                                 const float* mask, const double* ybits, int ny,
                                 const double* zbits, int nz, double* scratch, float* out,
                                 float* x_hat_nchw, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(mode == 0 || mode == 1, "mode");
  RGBAC_REQUIRE(batch > 0 && cx > 0 && h > 0 && w > 0, "shape");
  RGBAC_REQUIRE(x && x_hat && scratch && out && ybits && zbits, "null pointer");
  RGBAC_REQUIRE(mode == 1 || mask, "masked mse needs the mask");
  RGBAC_REQUIRE(ldh >= cx, "ldh");
  const int vec = cx <= 4 && ldh % 4 == 0 &&
                  ((uintptr_t)x_hat % (dtype == RGBAC_F32 ? 16 : 8)) == 0;
  const int HW = h * w;
  // scratch holds batch * nblk * 2 doubles (rgbac_finalize_blocks): <= 4 pixels per thread, so
  // the large frames' MSE pass is not a long dependent loop per thread (1024^2: 64 -> 1024
  // blocks per image)
  const int nblk = rgbac_finalize_blocks(h, w);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(mse_partial_kernel<float>, dim3(nblk, batch), dim3(256), 0, st, mode, cx,
                       HW, x, (const float*)x_hat, ldh, mask, scratch, x_hat_nchw, vec);
  else
    hipLaunchKernelGGL(mse_partial_kernel<bf16_t>, dim3(nblk, batch), dim3(256), 0, st, mode, cx,
                       HW, x, (const bf16_t*)x_hat, ldh, mask, scratch, x_hat_nchw, vec);
  int rc = check_launch("mse_partial_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(finalize_kernel, dim3(1), dim3(64 * kFinWaves), 0, st, mode, batch, nblk,
                     (double)batch * HW, scratch, ybits, ny, zbits, nz, out);
  return check_launch("finalize_kernel");
}

extern "C" int rgbac_forward_prologue(int dtype, int batch, int c, int h, int w, const float* x,
                                      void* xf, int64_t ldc, const float* alpha, int round255,
                                      float* rounded, int levels, float* const* outs,
                                      double* zero, int64_t nzero, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(batch > 0 && c > 0 && h > 0 && w > 0 && ldc >= c && x && xf && alpha, "shape");
  RGBAC_REQUIRE(levels >= 1 && levels <= 4, "levels: 1..4");
  RGBAC_REQUIRE(!round255 || rounded, "round255 needs an output buffer");
  RGBAC_REQUIRE(nzero >= 0 && (nzero == 0 || zero) && nzero < (1ll << 30), "zero range");
  for (int l = 0; l < levels; ++l) RGBAC_REQUIRE(outs && outs[l], "null pyramid output");
  const int E = dtype == RGBAC_F32 ? 4 : 8;
  const long long n = (long long)batch * h * w * ldc;
  RGBAC_REQUIRE(ldc % E == 0 && ((uintptr_t)xf & 15) == 0 && n / E < (1ll << 31) - 256,
                "the fused prologue needs 16-byte NHWC row chunks (ldc % 8 bf16 / % 4 f32)");
  PyrOuts po{};
  for (int l = 0; l < levels; ++l) po.p[l] = outs[l];
  int hl = h, wl = w;
  for (int l = 0; l < levels; ++l) { hl = (hl - 1) / 2 + 1; wl = (wl - 1) / 2 + 1; }
  const int tp = 32 >> levels;
  const long long npyr = (long long)batch * ((hl + tp - 1) / tp) * ((wl + tp - 1) / tp);
  const int nck = (int)(ldc / E), nn = (int)(n / E);
  const long long ncv = (nn + 255) / 256;
  RGBAC_REQUIRE(npyr + ncv < (1ll << 31), "too many prologue blocks");
  const int n0 = (tp + 1) * (1 << levels) - 1;
  const size_t lds = (size_t)2 * n0 * n0 * sizeof(float);
  const dim3 grid((unsigned)(npyr + ncv));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define PRO_LAUNCH(L_, T_)                                                                      \
  hipLaunchKernelGGL((prologue_kernel<L_, T_>), grid, dim3(256), lds, st, (int)npyr, batch, h, w, \
                     alpha, round255, rounded, po, nn, nck, c, x, (T_*)xf, (int)ldc, zero,      \
                     (int)nzero)
  if (dtype == RGBAC_F32) {
    switch (levels) {
      case 1: PRO_LAUNCH(1, float); break;
      case 2: PRO_LAUNCH(2, float); break;
      case 3: PRO_LAUNCH(3, float); break;
      default: PRO_LAUNCH(4, float); break;
    }
  } else {
    switch (levels) {
      case 1: PRO_LAUNCH(1, bf16_t); break;
      case 2: PRO_LAUNCH(2, bf16_t); break;
      case 3: PRO_LAUNCH(3, bf16_t); break;
      default: PRO_LAUNCH(4, bf16_t); break;
    }
  }
#undef PRO_LAUNCH
  return check_launch("prologue_kernel");
}

extern "C" int rgbac_mask_pyramid(int batch, int h, int w, const float* alpha, int round255,
                                  float* rounded, int levels, float* const* outs, void* stream) {
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && alpha, "shape");
  RGBAC_REQUIRE(levels >= 0 && levels <= 8, "levels");
  RGBAC_REQUIRE(!round255 || rounded, "round255 needs an output buffer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  static const bool fused = [] {
    const char* e = getenv("RGBAC_PYRAMID_FUSED");
    return !(e && e[0] == '0');
  }();
  if (fused && levels >= 1 && levels <= 4) {           // the forward's 4-level pyramids: 1 launch
    for (int l = 0; l < levels; ++l) RGBAC_REQUIRE(outs && outs[l], "null pyramid output");
    PyrOuts po{};
    for (int l = 0; l < levels; ++l) po.p[l] = outs[l];
    int hl = h, wl = w;
    for (int l = 0; l < levels; ++l) { hl = (hl - 1) / 2 + 1; wl = (wl - 1) / 2 + 1; }
    const int tp = 32 >> levels;
    const long long nblk = (long long)batch * ((hl + tp - 1) / tp) * ((wl + tp - 1) / tp);
    RGBAC_REQUIRE(nblk < (1ll << 31), "too many pyramid tiles");
    const int n0 = (tp + 1) * (1 << levels) - 1;
    const size_t lds = (size_t)2 * n0 * n0 * sizeof(float);
    switch (levels) {
      case 1: hipLaunchKernelGGL(pyramid_kernel<1>, dim3((unsigned)nblk), dim3(256), lds, st, batch, h, w, alpha, round255, rounded, po); break;
      case 2: hipLaunchKernelGGL(pyramid_kernel<2>, dim3((unsigned)nblk), dim3(256), lds, st, batch, h, w, alpha, round255, rounded, po); break;
      case 3: hipLaunchKernelGGL(pyramid_kernel<3>, dim3((unsigned)nblk), dim3(256), lds, st, batch, h, w, alpha, round255, rounded, po); break;
      default: hipLaunchKernelGGL(pyramid_kernel<4>, dim3((unsigned)nblk), dim3(256), lds, st, batch, h, w, alpha, round255, rounded, po); break;
    }
    return check_launch("pyramid_kernel");
  }
  const float* cur = alpha;
  if (round255) {
    const long long n = (long long)batch * h * w;
    hipLaunchKernelGGL(round255_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, alpha, rounded);
    int rc = check_launch("round255_kernel");
    if (rc) return rc;
    cur = rounded;
  }
  int H = h, W = w;
  for (int l = 0; l < levels; ++l) {
    RGBAC_REQUIRE(outs && outs[l], "null pyramid output");
    const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
    const long long n = (long long)batch * Ho * Wo;
    hipLaunchKernelGGL(avgpool3s2_kernel, dim3(grid_for(n)), dim3(256), 0, st, batch, H, W, Ho,
                       Wo, cur, outs[l]);
    int rc = check_launch("avgpool3s2_kernel");
    if (rc) return rc;
    cur = outs[l];
    H = Ho;
    W = Wo;
  }
  return RGBAC_OK;
}

extern "C" int rgbac_nchw_to_nhwc(int dtype, int batch, int c, int h, int w, const float* src,
                                  void* dst, int64_t ldc, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(batch > 0 && c > 0 && h > 0 && w > 0 && ldc >= c && src && dst, "shape");
  const long long n = (long long)batch * h * w * ldc;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int E = dtype == RGBAC_F32 ? 4 : 8;
  if (ldc % E == 0 && ((uintptr_t)dst & 15) == 0 && n / E < (1ll << 31) - 256) {
    const int nck = (int)(ldc / E), nn = (int)(n / E);
    const dim3 grid((unsigned)((nn + 255) / 256));
    if (dtype == RGBAC_F32)
      hipLaunchKernelGGL(nchw_to_nhwc_chunk_kernel<float>, grid, dim3(256), 0, st, nn, nck, c,
                         h * w, src, (float*)dst, (int)ldc);
    else
      hipLaunchKernelGGL(nchw_to_nhwc_chunk_kernel<bf16_t>, grid, dim3(256), 0, st, nn, nck, c,
                         h * w, src, (bf16_t*)dst, (int)ldc);
    return check_launch("nchw_to_nhwc_chunk_kernel");
  }
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, batch, c,
                       h * w, src, (float*)dst, ldc);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, batch, c,
                       h * w, src, (bf16_t*)dst, ldc);
  return check_launch("nchw_to_nhwc_kernel");
}

extern "C" int rgbac_nhwc_to_nchw(int dtype, int batch, int c, int h, int w, const void* src,
                                  int64_t ldc, float* dst, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(batch > 0 && c > 0 && h > 0 && w > 0 && ldc >= c && src && dst, "shape");
  const long long n = (long long)batch * h * w * c;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int E = dtype == RGBAC_F32 ? 4 : 8;
  const long long npix = (long long)batch * h * w;
  if (ldc % E == 0 && ((uintptr_t)src & 15) == 0 && npix < (1ll << 31) - 256 &&
      npix * ldc < (1ll << 40)) {
    const dim3 grid((unsigned)((npix + 255) / 256));
    if (dtype == RGBAC_F32)
      hipLaunchKernelGGL(nhwc_to_nchw_px_kernel<float>, grid, dim3(256), 0, st, (int)npix, c,
                         h * w, (const float*)src, (int)ldc, dst);
    else
      hipLaunchKernelGGL(nhwc_to_nchw_px_kernel<bf16_t>, grid, dim3(256), 0, st, (int)npix, c,
                         h * w, (const bf16_t*)src, (int)ldc, dst);
    return check_launch("nhwc_to_nchw_px_kernel");
  }
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, batch, c,
                       h * w, (const float*)src, ldc, dst);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, batch, c,
                       h * w, (const bf16_t*)src, ldc, dst);
  return check_launch("nhwc_to_nchw_kernel");
}
