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
