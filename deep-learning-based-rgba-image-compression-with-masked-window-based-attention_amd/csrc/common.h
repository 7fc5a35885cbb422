// Shared device/host helpers for librgbac_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/rgbac.h"

namespace rgbac {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

// bf16 storage is carried as raw 16-bit words.
struct bf16_t { uint16_t u; };

__device__ __forceinline__ float bf2f(uint16_t u) {
  return __uint_as_float(((uint32_t)u) << 16);
}
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_hw;
// round to nearest even by the hardware conversion (v_cvt_pk_bf16_f32): for finite inputs the
// same bits as (u + 0x7FFF + ((u >> 16) & 1)) >> 16, in one instruction per pair, and a NaN
// stays a NaN (MI355X_MICROARCH.md, correctness boundaries)
__device__ __forceinline__ uint16_t f2bf(float f) {
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const bf16x2_hw v = {(__bf16)a, (__bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// Element access for the two storage types.
template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int EPV = 4;  // elements per 16-byte chunk
  __device__ static float ld(const float* p) { return *p; }
  __device__ static void st(float* p, float v) { *p = v; }
  __device__ static void ld4(const float* p, float (&v)[4]) {
    float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  __device__ static void st4(float* p, const float (&v)[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
};
template <> struct Elem<bf16_t> {
  static constexpr int EPV = 8;
  __device__ static float ld(const bf16_t* p) { return bf2f(p->u); }
  __device__ static void st(bf16_t* p, float v) { p->u = f2bf(v); }
  __device__ static void ld4(const bf16_t* p, float (&v)[4]) {
    uint2 t = *reinterpret_cast<const uint2*>(p);
    v[0] = bf2f(t.x & 0xFFFF); v[1] = bf2f(t.x >> 16);
    v[2] = bf2f(t.y & 0xFFFF); v[3] = bf2f(t.y >> 16);
  }
  __device__ static void st4(bf16_t* p, const float (&v)[4]) {
    uint2 t;
    t.x = pack_bf16x2(v[0], v[1]);
    t.y = pack_bf16x2(v[2], v[3]);
    *reinterpret_cast<uint2*>(p) = t;
  }
};

// One MFMA k-step on 16-byte operand chunks held per lane (lane l: row l&15,
// chunk l>>4 of the 64-byte k-step):  acc[n][m] += sum_k A[n][k] * B[m][k].
//   bf16: v_mfma_f32_16x16x32_bf16 (k-step = 32 elements)
//   f32 : v_mfma_f32_16x16x4_f32 x4 (k-step = 16 elements; element e of every
//         lane's chunk feeds MFMA e, a permutation of k applied to both operands)
template <typename T>
__device__ __forceinline__ void mma_step(f32x4& acc, uint4 a, uint4 b);
template <>
__device__ __forceinline__ void mma_step<bf16_t>(f32x4& acc, uint4 a, uint4 b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mma_step<float>(f32x4& acc, uint4 a, uint4 b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}

// GELU(x) = 0.5 x (1 + erf(x / sqrt 2)) with a branch-free erf (Abramowitz &
// Stegun 7.1.26, |erf error| <= 1.5e-7; 1 + erf is formed as q = 1 - erf(|z|)
// for x < 0, so no cancellation): ~16 instructions instead of erff's ~40
// divergent ones.  Used where results are stored as bf16 (3 significant
// digits); the fp32 parity mode keeps erff.
// Written as max(x, 0) - |x|/2 * q (q = 1 - erf(|x|/sqrt 2)): the same value for both signs
// with no compare/select, and exp(-x^2/2) as one v_exp_f32 of a scaled x^2.
__device__ __forceinline__ float gelu_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752440f, ax, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170368f);   // exp(-x^2/2)
  const float q = p * t * e;                      // 1 - erf(|x| / sqrt 2)
  return fmaf(-0.5f * ax, q, fmaxf(x, 0.0f));
}


// gelu_fast on two values with packed FP32 math (v_pk_fma_f32 / v_pk_mul_f32 do both halves in
// one instruction; the rcp / exp stay per element): the same operations in the same order as
// gelu_fast, so bit-identical to it, in 21 instructions per pair instead of 32.  The GELU
// epilogues are VALU-bound (the residual unit's three epilogues were ~2/3 of its SIMD cycles).
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 gelu2_fast(f32x2 x) {
  const f32x2 ax = {fabsf(x.x), fabsf(x.y)};
  constexpr float c1 = 0.3275911f * 0.70710678118654752440f;
  const f32x2 den = __builtin_elementwise_fma((f32x2){c1, c1}, ax, (f32x2){1.0f, 1.0f});
  const f32x2 t = {__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 p = __builtin_elementwise_fma((f32x2){1.061405429f, 1.061405429f}, t,
                                      (f32x2){-1.453152027f, -1.453152027f});
  p = __builtin_elementwise_fma(p, t, (f32x2){1.421413741f, 1.421413741f});
  p = __builtin_elementwise_fma(p, t, (f32x2){-0.284496736f, -0.284496736f});
  p = __builtin_elementwise_fma(p, t, (f32x2){0.254829592f, 0.254829592f});
  const f32x2 arg = (x * x) * (f32x2){-0.72134752044448170368f, -0.72134752044448170368f};
  const f32x2 e = {__builtin_amdgcn_exp2f(arg.x), __builtin_amdgcn_exp2f(arg.y)};
  const f32x2 q = (p * t) * e;
  const f32x2 h = (f32x2){-0.5f, -0.5f} * ax;
  const f32x2 m = {fmaxf(x.x, 0.0f), fmaxf(x.y, 0.0f)};
  return __builtin_elementwise_fma(h, q, m);
}
// v[r] = gelu_fast(v[r]) for a quad, as two packed pairs
__device__ __forceinline__ void gelu4_fast(float (&v)[4]) {
#ifdef RGBAC_GELU_SCALAR
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = gelu_fast(v[r]);
  return;
#endif
  const f32x2 a = gelu2_fast((f32x2){v[0], v[1]}), b = gelu2_fast((f32x2){v[2], v[3]});
  v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
}

// GELU'(v) = Phi(v) + v phi(v) with the Abramowitz & Stegun 7.1.26 erfc of the forward's
// gelu_fast (|erf error| <= 1.5e-7; exp(-v^2/2) shared by both terms): ~15 instructions
// instead of erfcf + expf.  bf16 only (the f32 parity path keeps erfcf).
__device__ __forceinline__ float gelu_grad_fast(float v) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * 0.70710678118654752440f, fabsf(v), 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float e = __builtin_amdgcn_exp2f(v * v * -0.72134752044448170368f);   // exp(-v^2/2)
  const float q = p * t * e;                     // erfc(|v| / sqrt 2)
  const float cdf = v >= 0.0f ? fmaf(-0.5f, q, 1.0f) : 0.5f * q;
  return fmaf(0.39894228040143267794f * v, e, cdf);
}

// exact GELU'(v) = Phi(v) + v phi(v) (erfcf + expf; the same expression as train.hip's
// t_cdf(v) + v * t_phi(v)): the f32 parity path
__device__ __forceinline__ float gelu_grad_exact(float v) {
  return 0.5f * erfcf(-0.70710678118654752440f * v) +
         v * (0.39894228040143267794f * expf(-0.5f * v * v));
}


// Lane exchanges without an LDS round trip (gfx950 v_permlane16_swap / v_permlane32_swap;
// __shfl_xor is a ds_bpermute).  With the same value in both operands the swap returns
// {the lower row's / half's value, the upper one's} on both lanes of a pair.
__device__ __forceinline__ uint32_t xor32_u(uint32_t v) {        // value of lane ^ 32
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return (threadIdx.x & 32) ? r[0] : r[1];
}
__device__ __forceinline__ float xor32_f(float v) { return __uint_as_float(xor32_u(__float_as_uint(v))); }
__device__ __forceinline__ float sum32_f(float v) {             // v + v(lane ^ 32), same on both
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float sum16_f(float v) {             // v + v(lane ^ 16), same on both
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ---------------------------------------------------------------- host side
void set_error(const std::string& msg);
int check_launch(const char* what);

#define RGBAC_REQUIRE(cond, msg)                                   \
  do {                                                             \
    if (!(cond)) {                                                 \
      ::rgbac::set_error(std::string(__func__) + ": " + (msg));    \
      return RGBAC_E_ARG;                                          \
    }                                                              \
  } while (0)

// Per-device launch facts, cached per device id (a process may drive several GPUs):
// the CU count, and the dynamic-LDS opt-in of a kernel above 64 KiB (one call per device).
inline int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (cus[dev] == 0) {
    int n = 0;
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    cus[dev] = n > 0 ? n : 256;
  }
  return cus[dev];
}
inline void lds_optin(const void* kern, int bytes, unsigned long long* done_mask) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const unsigned long long bit = 1ull << (dev & 63);
  if (*done_mask & bit) return;
  (void)hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  *done_mask |= bit;
}

constexpr int kReduceThreads = 256;
constexpr int kReduceMaxBlocks = 1024;
inline int reduce_blocks(int64_t n) {
  // one element per thread up to the block cap: the per-element entropy math (factorized
  // density MLP, erfc) is latency-bound, so spreading it wide beats per-thread loops
  int64_t b = (n + kReduceThreads - 1) / kReduceThreads;
  if (b < 1) b = 1;
  if (b > kReduceMaxBlocks) b = kReduceMaxBlocks;
  return (int)b;
}

// fp64 block reduction of one value per thread (blockDim == kReduceThreads).
__device__ __forceinline__ double block_sum_f64(double v, double* smem) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) smem[wave] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r += smem[i];
  }
  __syncthreads();
  return r;  // valid on thread 0
}

}  // namespace rgbac
