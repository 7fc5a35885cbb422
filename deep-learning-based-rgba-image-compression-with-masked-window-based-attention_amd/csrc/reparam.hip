// GDN / IGDN parameter reparametrisation of the training step (reference: layers/GDN.py:9-23
// LowerBound, :71-78), one launch per layer instead of ~9 elementwise torch launches each way:
//   forward   beta'  = max(beta, beta_bound)^2 - pedestal,
//             gamma' = max(gamma, gamma_bound)^2 - pedestal
//   backward  g2 = g * (2 m)  (m = max(p, bound): pow's backward), passed where p >= bound or
//             g2 < 0 (LowerBound's rule), then added into the parameter's .grad (or stored).
// The arithmetic is torch's, op for op and uncontracted (m * m, then - pedestal; 2 m, then
// g * (2 m); 1 or 0 times that), so values and gradients are bit-identical to the autograd
// graph of GDN.py's LowerBound / ** 2 / - pedestal.
#include "common.h"

namespace rgbac {

__global__ void __launch_bounds__(256) gdn_reparam_kernel(int nb, int ng, const float* beta,
                                                          const float* gamma, float bb, float gb,
                                                          float ped, float* bo, float* go) {
#pragma clang fp contract(off)
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nb + ng; i += gridDim.x * 256) {
    const bool isb = i < nb;
    const float p = isb ? beta[i] : gamma[i - nb];
    const float m = fmaxf(p, isb ? bb : gb);
    const float sq = m * m;
    const float v = sq - ped;
    if (isb) bo[i] = v;
    else go[i - nb] = v;
  }
}

__global__ void __launch_bounds__(256) gdn_reparam_bwd_kernel(
    int nb, int ng, const float* beta, const float* gamma, float bb, float gb, const float* dbo,
    const float* dgo, float* dbeta, float* dgamma, int accumulate) {
#pragma clang fp contract(off)
  for (int i = blockIdx.x * 256 + threadIdx.x; i < nb + ng; i += gridDim.x * 256) {
    const bool isb = i < nb;
    const int j = isb ? i : i - nb;
    const float p = isb ? beta[j] : gamma[j];
    const float bound = isb ? bb : gb;
    const float m = fmaxf(p, bound);
    const float g = isb ? (dbo ? dbo[j] : 0.0f) : (dgo ? dgo[j] : 0.0f);
    const float two_m = 2.0f * m;
    const float g2 = g * two_m;
    const bool pass = p >= bound || g2 < 0.0f;
    const float gin = (pass ? 1.0f : 0.0f) * g2;
    float* d = isb ? dbeta : dgamma;
    if (accumulate) {
      const float prev = d[j];
      d[j] = prev + gin;
    } else {
      d[j] = gin;
    }
  }
}

// EntropyBottleneck parameter block of the training step (compressai EntropyBottleneck,
// filters (3, 3, 3, 3); rgbac.train_forward.eb_params_t): per channel c the 64-float row
//   [softplus(_matrix0..4) 33 | _bias0..4 13 | tanh(_factor0..3) 12 | median 1 | 0 x 5]
// that rgbac_eb_forward / rgbac_eb_bwd read, in one launch each way instead of the softplus /
// tanh / cat / pad chain and its backward (+ one .grad accumulate per parameter).
struct EbParamSet {
  const float* p[15];          // _matrix0..4, _bias0..4, _factor0..3, quantiles
  float* g[15];                // their gradients (backward)
};
__device__ __forceinline__ void eb_col(int j, int& k, int& cnt, int& off, int& op) {
  // op 0 softplus, 1 identity, 2 tanh, 3 median (quantiles[c][0][1]), 4 zero pad
  constexpr int CNT[15] = {3, 9, 9, 9, 3, 3, 3, 3, 3, 1, 3, 3, 3, 3, 1};
  int start = 0;
  k = 15; cnt = 1; off = 0; op = 4;
#pragma unroll
  for (int i = 0; i < 15; ++i) {
    if (k == 15 && j < start + CNT[i]) {
      k = i; cnt = CNT[i]; off = j - start;
      op = i < 5 ? 0 : (i < 10 ? 1 : (i < 14 ? 2 : 3));
    }
    start += CNT[i];
  }
}

__global__ void __launch_bounds__(256) eb_params_kernel(int C, EbParamSet s, float* out) {
#pragma clang fp contract(off)
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= C * 64) return;
  const int c = e >> 6, j = e & 63;
  int k, cnt, off, op;
  eb_col(j, k, cnt, off, op);
  float v = 0.0f;
  if (op == 3) v = s.p[14][c * 3 + 1];
  else if (op != 4) {
    const float x = s.p[k][c * cnt + off];
    v = op == 0 ? (x > 20.0f ? x : log1pf(expf(x))) : (op == 2 ? tanhf(x) : x);
  }
  out[e] = v;
}

__global__ void __launch_bounds__(256) eb_params_bwd_kernel(int C, EbParamSet s, const float* dout,
                                                            int accumulate) {
#pragma clang fp contract(off)
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= C * 64) return;
  const int c = e >> 6, j = e & 63;
  int k, cnt, off, op;
  eb_col(j, k, cnt, off, op);
  if (op == 4) return;
  const float g = dout[e];
  int idx;
  float gin;
  if (op == 3) {
    idx = c * 3 + 1;
    gin = g;
  } else {
    idx = c * cnt + off;
    const float x = s.p[k][idx];
    if (op == 0) {                                     // softplus_backward (beta 1, threshold 20)
      const float z = expf(x);
      gin = x > 20.0f ? g : (g * z) / (z + 1.0f);
    } else if (op == 2) {                              // tanh_backward on the output
      const float y = tanhf(x);
      const float yy = y * y;
      gin = g * (1.0f - yy);
    } else {
      gin = g;
    }
  }
  float* d = s.g[k];
  if (accumulate) {
    const float prev = d[idx];
    d[idx] = prev + gin;
  } else {
    d[idx] = gin;
  }
}

}  // namespace rgbac

using namespace rgbac;

static int reparam_grid(long long n) {
  long long b = (n + 255) / 256;
  if (b > 1024) b = 1024;
  return (int)(b < 1 ? 1 : b);
}

extern "C" int rgbac_gdn_reparam(int nb, int ng, const float* beta, const float* gamma,
                                 float beta_bound, float gamma_bound, float pedestal,
                                 float* beta_out, float* gamma_out, void* stream) {
  RGBAC_REQUIRE(nb > 0 && ng > 0 && beta && gamma && beta_out && gamma_out, "args");
  hipLaunchKernelGGL(gdn_reparam_kernel, dim3(reparam_grid((long long)nb + ng)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), nb, ng, beta, gamma, beta_bound,
                     gamma_bound, pedestal, beta_out, gamma_out);
  return check_launch("gdn_reparam_kernel");
}

extern "C" int rgbac_gdn_reparam_bwd(int nb, int ng, const float* beta, const float* gamma,
                                     float beta_bound, float gamma_bound,
                                     const float* dbeta_out, const float* dgamma_out,
                                     float* dbeta, float* dgamma, int accumulate, void* stream) {
  RGBAC_REQUIRE(nb > 0 && ng > 0 && beta && gamma && dbeta && dgamma, "args");
  hipLaunchKernelGGL(gdn_reparam_bwd_kernel, dim3(reparam_grid((long long)nb + ng)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), nb, ng, beta, gamma, beta_bound,
                     gamma_bound, dbeta_out, dgamma_out, dbeta, dgamma, accumulate);
  return check_launch("gdn_reparam_bwd_kernel");
}

extern "C" int rgbac_eb_params(int channels, const float* const* params, float* out, void* stream) {
  RGBAC_REQUIRE(channels > 0 && params && out, "args");
  EbParamSet s;
  for (int i = 0; i < 15; ++i) {
    RGBAC_REQUIRE(params[i], "null parameter");
    s.p[i] = params[i];
    s.g[i] = nullptr;
  }
  hipLaunchKernelGGL(eb_params_kernel, dim3((channels * 64 + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), channels, s, out);
  return check_launch("eb_params_kernel");
}

extern "C" int rgbac_eb_params_bwd(int channels, const float* const* params, const float* dout,
                                   float* const* grads, int accumulate, void* stream) {
  RGBAC_REQUIRE(channels > 0 && params && dout && grads, "args");
  EbParamSet s;
  for (int i = 0; i < 15; ++i) {
    RGBAC_REQUIRE(params[i] && grads[i], "null parameter or gradient");
    s.p[i] = params[i];
    s.g[i] = grads[i];
  }
  hipLaunchKernelGGL(eb_params_bwd_kernel, dim3((channels * 64 + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), channels, s, dout, accumulate);
  return check_launch("eb_params_bwd_kernel");
}
