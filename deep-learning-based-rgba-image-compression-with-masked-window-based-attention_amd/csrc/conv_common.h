// Shared by the implicit-GEMM convolution translation units (conv.hip): the
// device-side launch descriptors (ConvArgsDev), the fused-epilogue helpers and the LDS-DMA /
// wait primitives.  Everything here is inline or has internal linkage (each TU holds its own
// zero page), so the TUs compile independently.
#pragma once
#include "common.h"

namespace rgbac {

constexpr int kMaxGroups = 10;

struct ConvGroup {                  // per-group operands
  const void* sp0; const void* sp1; const void* sp2;
  long long sld0, sld1, sld2;
  const void* w;
  const float* bias;
  void* out;
  const void* res0; const void* res1; const void* res2;
  long long ld0, ld1, ld2, out_ldc;
  const uint8_t* sel;
  float* ws;                        // split-K slabs [ksplit][nphase][M][cout16]
  const float* aux0;                // GAUSS: noise [M][cout/2] or NULL
  float* aux1;                      // GAUSS: likelihood out [M][cout/2] or NULL
  double* partial;                  // GAUSS: bits per M-tile block
  void* zout;                       // training: pre-activation store (or NULL)
  long long zld;
  int* cnt;                         // split-K tickets (in-launch reduction) or NULL
  int send0, send1, send2;          // cumulative channel ends
  int cin_pad, k_pad, cout, rows, cout16, out_coff;
};

struct ConvShared {
  double rWm, rHm;                  // 1/Wm, 1/Hm for divide-free pixel decode
  int mode, batch, in_h, in_w, Hm, Wm, out_h, out_w, M, sy;
  int ksize, pad;
  int act; float act_param; int square;
  int ksplit, nphase, ngroups;
  int remap;                        // XCD-aware block order: 1 contiguous runs (env
                                    // RGBAC_XCD_REMAP=0: plain order)
};

struct ConvArgsDev {
  ConvShared s;
  ConvGroup g[kMaxGroups];
};

static __device__ uint4 g_zero_page[64];
   // zero source for padding taps (static, never written)

// n / d for 0 <= n < 2^31 via a double reciprocal and one correction step
// (|n*rd - n/d| < 2^-21, so the truncated quotient is off by at most one).
__device__ __forceinline__ int udiv(int n, int d, double rd) {
  int q = (int)((double)n * rd);
  const int r = n - q * d;
  if (r < 0) --q;
  else if (r >= d) ++q;
  return q;
}

__device__ __forceinline__ float gelu_f(float v) {
  return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
}
// exact erf GELU for fp32 (parity mode), the branch-free form for bf16 outputs
template <typename T> __device__ __forceinline__ float gelu_t(float v);
template <> __device__ __forceinline__ float gelu_t<float>(float v) { return gelu_f(v); }
template <> __device__ __forceinline__ float gelu_t<bf16_t>(float v) { return gelu_fast(v); }
__device__ __forceinline__ float sigmoid_f(float v) { return 1.0f / (1.0f + expf(-v)); }
// GDN / IGDN output x / sqrt(n), x * sqrt(n): IEEE sqrt + divide in the fp32 parity mode,
// the hardware rsq / sqrt (~1 ulp fp32) where the result is stored as bf16
template <typename T> __device__ __forceinline__ float gdn_t(float x, float n);
template <> __device__ __forceinline__ float gdn_t<float>(float x, float n) { return x / sqrtf(n); }
template <> __device__ __forceinline__ float gdn_t<bf16_t>(float x, float n) {
  return x * __builtin_amdgcn_rsqf(n);
}
template <typename T> __device__ __forceinline__ float igdn_t(float x, float n);
template <> __device__ __forceinline__ float igdn_t<float>(float x, float n) { return x * sqrtf(n); }
template <> __device__ __forceinline__ float igdn_t<bf16_t>(float x, float n) {
  return x * __builtin_amdgcn_sqrtf(n);
}
__device__ __forceinline__ float std_cum_f(float t) {
  return 0.5f * erfcf(-0.70710678118654752440f * t);
}

template <typename T>
__device__ __forceinline__ uint4 square_chunk(uint4 v);
template <>
__device__ __forceinline__ uint4 square_chunk<float>(uint4 v) {
  float a = __uint_as_float(v.x), b = __uint_as_float(v.y);
  float c = __uint_as_float(v.z), d = __uint_as_float(v.w);
  return make_uint4(__float_as_uint(a * a), __float_as_uint(b * b),
                    __float_as_uint(c * c), __float_as_uint(d * d));
}
__device__ __forceinline__ uint32_t sq_pair(uint32_t w) {
  float lo = bf2f(w & 0xFFFF), hi = bf2f(w >> 16);
  return (uint32_t)f2bf(lo * lo) | ((uint32_t)f2bf(hi * hi) << 16);
}
template <>
__device__ __forceinline__ uint4 square_chunk<bf16_t>(uint4 v) {
  return make_uint4(sq_pair(v.x), sq_pair(v.y), sq_pair(v.z), sq_pair(v.w));
}

template <typename T>
__device__ __forceinline__ void load_res(const void* ptr, long long ld, long long opix, int n,
                                         int cout, float (&v)[4]) {
  const T* r = reinterpret_cast<const T*>(ptr) + opix * ld + n;
  if (n + 3 < cout) {
    Elem<T>::ld4(r, v);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = (n + q < cout) ? Elem<T>::ld(r + q) : 0.0f;
  }
}

// Input gradient through the producer's activation (ACT_DGELU / ACT_DLRELU, res0 = the
// producer's pre-activation z): acc * act'(z), the activation backward folded into the
// consumer's input-gradient conv (rgbac.autograd deferred activations).  Same arithmetic as
// train.hip's act_bwd on dy = acc: the fast derivative for bf16, the exact one for f32.
template <typename T>
__device__ __forceinline__ float dact_apply(int act, float p, float acc, float z) {
  if (act == RGBAC_ACT_DGELU)
    return acc * (sizeof(T) == 4 ? gelu_grad_exact(z) : gelu_grad_fast(z));
  return z > 0.0f ? acc : acc * p;
}
__host__ __device__ __forceinline__ bool is_dact(int act) {
  return act == RGBAC_ACT_DGELU || act == RGBAC_ACT_DLRELU;
}

template <typename T, bool DACT = true>
__device__ __forceinline__ void epilogue4_body(const ConvShared& s, const ConvGroup& g,
                                               long long opix, int n, float (&v)[4]);

// Bias + fused epilogue + store of channels n..n+3 of M-grid pixel m (phase ph).
template <typename T, bool DACT = true>
__device__ __forceinline__ void epilogue4(const ConvShared& s, const ConvGroup& g, int ph, int m,
                                          int n, float (&v)[4]) {
  const int t = udiv(m, s.Wm, s.rWm);
  const int mx = m - t * s.Wm;
  const int b = udiv(t, s.Hm, s.rHm);
  const int my = t - b * s.Hm;
  T* out = reinterpret_cast<T*>(g.out);
  if (s.mode == RGBAC_SUBPEL2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += (g.bias ? g.bias[n + r] : 0.0f);
    // conv channel n+r = 4*cc + 2*ii + jj -> pixel (2my+ii, 2mx+jj), channel cc
    const int cc = n >> 2;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = v[r];
      const int oy = 2 * my + (r >> 1), ox = 2 * mx + (r & 1);
      const long long op = (long long)(b * s.out_h + oy) * s.out_w + ox;
      if (g.zout) Elem<T>::st(reinterpret_cast<T*>(g.zout) + op * g.zld + g.out_coff + cc, x);
      if (s.act == RGBAC_ACT_GELU) x = gelu_t<T>(x);
      Elem<T>::st(out + op * g.out_ldc + g.out_coff + cc, x);
    }
    return;
  }
  long long opix;
  if (s.mode == RGBAC_CONVT_S2)
    opix = (long long)(b * s.out_h + 2 * my + (ph >> 1)) * s.out_w + 2 * mx + (ph & 1);
  else
    opix = (long long)(b * s.out_h + my) * s.out_w + mx;
  epilogue4_body<T, DACT>(s, g, opix, n, v);
}

// Same for a stride-1 CONV whose output grid is the M grid (output pixel = m).
template <typename T>
__device__ __forceinline__ void epilogue4_at(const ConvShared& s, const ConvGroup& g, int m, int n,
                                             float (&v)[4]) {
  epilogue4_body<T>(s, g, (long long)m, n, v);
}

// Operands the epilogue reads from memory, loaded ahead of the math so several quads'
// loads can be in flight together (EpiIn::load, then epilogue4_fin).
struct EpiIn {
  float r0[4], r1[4], r2[4];
  bool on;
  template <typename T>
  __device__ __forceinline__ void load(const ConvGroup& g, int act, long long opix, int n) {
#pragma unroll
    for (int r = 0; r < 4; ++r) { r0[r] = 0.f; r1[r] = 0.f; r2[r] = 0.f; }
    if (g.res0) load_res<T>(g.res0, g.ld0, opix, n, g.cout, r0);
    if (g.res1) load_res<T>(g.res1, g.ld1, opix, n, g.cout, r1);
    if (g.res2) load_res<T>(g.res2, g.ld2, opix, n, g.cout, r2);
    on = act == RGBAC_ACT_MASKSEL ? g.sel[opix] != 0 : true;
  }
};

// DACT = false: an instantiation without the folded activation backward (ACT_DGELU /
// ACT_DLRELU), for kernels at their register limit that run it in a separate instance
template <typename T, bool DACT = true>
__device__ __forceinline__ void epilogue4_fin(const ConvShared& s, const ConvGroup& g,
                                              long long opix, int n, float (&v)[4],
                                              const float (&bias)[4], const EpiIn& in);

template <typename T, bool DACT>
__device__ __forceinline__ void epilogue4_body(const ConvShared& s, const ConvGroup& g,
                                               long long opix, int n, float (&v)[4]) {
  EpiIn in;
  in.template load<T>(g, s.act, opix, n);
  float bias[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) bias[r] = g.bias ? g.bias[n + r] : 0.0f;
  epilogue4_fin<T, DACT>(s, g, opix, n, v, bias, in);
}

template <typename T, bool DACT>
__device__ __forceinline__ void epilogue4_fin(const ConvShared& s, const ConvGroup& g,
                                              long long opix, int n, float (&v)[4],
                                              const float (&bias)[4], const EpiIn& in) {
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] += bias[r];
  T* out = reinterpret_cast<T*>(g.out);
  const float (&r0)[4] = in.r0;
  const float (&r1)[4] = in.r1;
  if (DACT && is_dact(s.act)) {              // uniform branch: keeps the derivative out of the
#pragma unroll                        // other epilogues (no if-converted select per element)
    for (int r = 0; r < 4; ++r) v[r] = dact_apply<T>(s.act, s.act_param, v[r], r0[r]);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      v[r] = s.act == RGBAC_ACT_SQBWD ? r0[r] + 2.0f * r1[r] * v[r] : v[r] + r0[r];
  }
  if (g.zout) {
    T* z = reinterpret_cast<T*>(g.zout) + opix * g.zld + g.out_coff + n;
    if (n + 3 < g.cout) {
      Elem<T>::st4(z, v);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (n + r < g.cout) Elem<T>::st(z + r, v[r]);
    }
  }
  switch (s.act) {
    case RGBAC_ACT_GELU:
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gelu_t<T>(v[r]);
      break;
    case RGBAC_ACT_RELU:
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
      break;
    case RGBAC_ACT_LRELU:
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * s.act_param;
      break;
    case RGBAC_ACT_TANH_HALF:
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = r1[r] + 0.5f * tanhf(v[r]);
      break;
    case RGBAC_ACT_GATE:
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = r1[r] * sigmoid_f(v[r]);
      break;
    case RGBAC_ACT_GDN:
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = gdn_t<T>(r1[r], v[r]);
      break;
    case RGBAC_ACT_IGDN:
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = igdn_t<T>(r1[r], v[r]);
      break;
    case RGBAC_ACT_MASKSEL: {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = in.on ? r1[r] + v[r] : r1[r];
      break;
    }
    default:
      break;
  }
  if (g.res2) {
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += in.r2[r];
  }
  const long long base = opix * g.out_ldc + g.out_coff + n;
  if (n + 3 < g.cout) {
    Elem<T>::st4(out + base, v);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < g.cout) Elem<T>::st(out + base + r, v[r]);
  }
}

// conv_kernel epilogue of accumulator row i (pixel m, channels nn[j]..+3 for j < TN):
// every residual load of the row is issued before any math/store.
template <typename T, int TN, int TM, bool DACT = true>
__device__ __forceinline__ void epilogue_tile_row(const ConvShared& s, const ConvGroup& g, int ph,
                                                  int m, const int (&nn)[TN],
                                                  const f32x4 (&acc)[TN][TM], int i) {
  if (s.mode == RGBAC_SUBPEL2) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (nn[j] >= g.cout) continue;
      float v[4] = {acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]};
      epilogue4<T, DACT>(s, g, ph, m, nn[j], v);
    }
    return;
  }
  const int t = udiv(m, s.Wm, s.rWm);
  const int mx = m - t * s.Wm;
  const int b = udiv(t, s.Hm, s.rHm);
  const int my = t - b * s.Hm;
  long long opix;
  if (s.mode == RGBAC_CONVT_S2)
    opix = (long long)(b * s.out_h + 2 * my + (ph >> 1)) * s.out_w + 2 * mx + (ph & 1);
  else
    opix = (long long)(b * s.out_h + my) * s.out_w + mx;
  EpiIn in[TN];
  float bias[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    if (nn[j] < g.cout) in[j].template load<T>(g, s.act, opix, nn[j]);
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = (g.bias && nn[j] < g.cout) ? g.bias[nn[j] + r] : 0.0f;
  }
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    if (nn[j] >= g.cout) continue;
    float v[4] = {acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]};
    epilogue4_fin<T, DACT>(s, g, opix, nn[j], v, bias[j], in[j]);
  }
}

// Epilogue of one pixel row held by a lane: channels nn[j]..nn[j]+3 for j < TN.
// The pixel index is decoded once and every residual load of the row is issued
// before any store (stores could alias later loads in program order otherwise,
// which serialises one memory latency per 16x16 tile).
template <typename T, int TN>
__device__ __forceinline__ void epilogue_row(const ConvShared& s, const ConvGroup& g, int ph, int m,
                                             const int (&nn)[TN], float (&v)[TN][4]) {
  const int t = udiv(m, s.Wm, s.rWm);
  const int mx = m - t * s.Wm;
  const int b = udiv(t, s.Hm, s.rHm);
  const int my = t - b * s.Hm;
#pragma unroll
  for (int j = 0; j < TN; ++j)
    if (nn[j] < g.cout)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] += (g.bias ? g.bias[nn[j] + r] : 0.0f);
  T* out = reinterpret_cast<T*>(g.out);
  if (s.mode == RGBAC_SUBPEL2) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (nn[j] >= g.cout) continue;
      const int cc = nn[j] >> 2;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float x = v[j][r];
        const int oy = 2 * my + (r >> 1), ox = 2 * mx + (r & 1);
        const long long op = (long long)(b * s.out_h + oy) * s.out_w + ox;
        if (g.zout) Elem<T>::st(reinterpret_cast<T*>(g.zout) + op * g.zld + g.out_coff + cc, x);
        if (s.act == RGBAC_ACT_GELU) x = gelu_t<T>(x);
        Elem<T>::st(out + op * g.out_ldc + g.out_coff + cc, x);
      }
    }
    return;
  }
  long long opix;
  if (s.mode == RGBAC_CONVT_S2)
    opix = (long long)(b * s.out_h + 2 * my + (ph >> 1)) * s.out_w + 2 * mx + (ph & 1);
  else
    opix = (long long)(b * s.out_h + my) * s.out_w + mx;
  float r0[TN][4], r1[TN][4], r2[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
#pragma unroll
    for (int r = 0; r < 4; ++r) r0[j][r] = r1[j][r] = r2[j][r] = 0.0f;
    if (nn[j] >= g.cout) continue;
    if (g.res0) load_res<T>(g.res0, g.ld0, opix, nn[j], g.cout, r0[j]);
    if (g.res1) load_res<T>(g.res1, g.ld1, opix, nn[j], g.cout, r1[j]);
    if (g.res2) load_res<T>(g.res2, g.ld2, opix, nn[j], g.cout, r2[j]);
  }
  const bool on = s.act != RGBAC_ACT_MASKSEL || g.sel[opix] != 0;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    if (nn[j] >= g.cout) continue;
    float* vv = v[j];
    if (is_dact(s.act)) {             // uniform: the folded activation backward, no zout
#pragma unroll
      for (int r = 0; r < 4; ++r) vv[r] = dact_apply<T>(s.act, s.act_param, vv[r], r0[j][r]);
      const long long base = opix * g.out_ldc + g.out_coff + nn[j];
      if (nn[j] + 3 < g.cout) {
        Elem<T>::st4(out + base, v[j]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nn[j] + r < g.cout) Elem<T>::st(out + base + r, vv[r]);
      }
      continue;
    }
    if (g.zout) {
      float zv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        zv[r] = s.act == RGBAC_ACT_SQBWD ? r0[j][r] + 2.0f * r1[j][r] * vv[r] : vv[r] + r0[j][r];
      T* z = reinterpret_cast<T*>(g.zout) + opix * g.zld + g.out_coff + nn[j];
      if (nn[j] + 3 < g.cout) {
        Elem<T>::st4(z, zv);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (nn[j] + r < g.cout) Elem<T>::st(z + r, zv[r]);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = s.act == RGBAC_ACT_SQBWD ? r0[j][r] + 2.0f * r1[j][r] * vv[r] : vv[r] + r0[j][r];
      switch (s.act) {
        case RGBAC_ACT_GELU: x = gelu_t<T>(x); break;
        case RGBAC_ACT_RELU: x = x > 0.f ? x : 0.f; break;
        case RGBAC_ACT_LRELU: x = x > 0.f ? x : x * s.act_param; break;
        case RGBAC_ACT_TANH_HALF: x = r1[j][r] + 0.5f * tanhf(x); break;
        case RGBAC_ACT_GATE: x = r1[j][r] * sigmoid_f(x); break;
        case RGBAC_ACT_GDN: x = gdn_t<T>(r1[j][r], x); break;
        case RGBAC_ACT_IGDN: x = igdn_t<T>(r1[j][r], x); break;
        case RGBAC_ACT_MASKSEL: x = on ? r1[j][r] + x : r1[j][r]; break;
        default: break;
      }
      vv[r] = x + r2[j][r];
    }
    const long long base = opix * g.out_ldc + g.out_coff + nn[j];
    if (nn[j] + 3 < g.cout) {
      Elem<T>::st4(out + base, v[j]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (nn[j] + r < g.cout) Elem<T>::st(out + base + r, vv[r]);
    }
  }
}

// GaussianConditional + ste_round on a (mu | sigma) conv output (ACT_GAUSS):
//   hat = round(y - mu) + mu -> out;  v = |(train ? y + noise : hat) - mu|;
//   lik = max(Phi((.5-v)/s) - Phi((-.5-v)/s), 1e-9), s = max(sigma, .11);
//   returns clamp(-log(lik + 1e-10)/ln2, 0, 50)   (AutoEncoderRGB_Journal.py:255-257,280)
template <typename T>
__device__ __forceinline__ float gauss_elem(const ConvGroup& g, int m, int c, int nch, float mu,
                                            float sg) {
  const float yv = Elem<T>::ld(reinterpret_cast<const T*>(g.res1) + (long long)m * g.ld1 + c);
  const float hat = rintf(yv - mu) + mu;
  Elem<T>::st(reinterpret_cast<T*>(g.out) + (long long)m * g.out_ldc + g.out_coff + c, hat);
  const float xin = g.aux0 ? yv + g.aux0[(long long)m * nch + c] : hat;
  const float v = fabsf(xin - mu);
  const float sc = fmaxf(sg, 0.11f);
  const float lik = fmaxf(std_cum_f((0.5f - v) / sc) - std_cum_f((-0.5f - v) / sc), 1e-9f);
  if (g.aux1) g.aux1[(long long)m * nch + c] = lik;
  const float bits = (-1.0f * logf(lik + 1e-10f)) / 0.69314718055994530942f;
  return fminf(fmaxf(bits, 0.0f), 50.0f);
}

// gauss_elem with y (res1) already loaded by the caller
template <typename T>
__device__ __forceinline__ float gauss_elem_y(const ConvGroup& g, int m, int c, int nch, float mu,
                                              float sg, float yv) {
  const float hat = rintf(yv - mu) + mu;
  Elem<T>::st(reinterpret_cast<T*>(g.out) + (long long)m * g.out_ldc + g.out_coff + c, hat);
  const float xin = g.aux0 ? yv + g.aux0[(long long)m * nch + c] : hat;
  const float v = fabsf(xin - mu);
  const float sc = fmaxf(sg, 0.11f);
  const float lik = fmaxf(std_cum_f((0.5f - v) / sc) - std_cum_f((-0.5f - v) / sc), 1e-9f);
  if (g.aux1) g.aux1[(long long)m * nch + c] = lik;
  const float bits = (-1.0f * logf(lik + 1e-10f)) / 0.69314718055994530942f;
  return fminf(fmaxf(bits, 0.0f), 50.0f);
}

// the two-deep pointwise GDN / IGDN forward (pw3.hip), dispatched by conv.hip's launch_pw
bool pw3_ok(const ConvArgsDev& d, int cin_max);
void launch_pw3(const ConvArgsDev& d, hipStream_t st);

typedef __attribute__((address_space(3))) void* lptr_t;

// One LDS-DMA piece: each lane moves 16 bytes from its own global address to
// lds_block + 16*lane.  Issued from inline asm so hipcc neither counts it nor
// inserts its own vmcnt(0) before later ds_reads; every wait on it is the
// kernel's explicit counted s_waitcnt (M0 saved/restored inside the statement).
__device__ __forceinline__ void dma16(const void* src, uint4* lds_block) {
  const uint32_t lds = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)lds_block);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

// The same with a wave-uniform base address and a per-lane 32-bit byte offset (the SADDR
// form: no per-lane 64-bit address arithmetic).
__device__ __forceinline__ void dma16_s(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %3\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %2\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(sbase), "s"(lds)
      : "memory");
}
// dma16 with a precomputed wave-uniform LDS byte address (no per-call generic->LDS cast).
__device__ __forceinline__ void dma16_l(const void* src, uint32_t lds) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(src), "s"(lds)
      : "memory");
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct KDec { int ci, tap, ty, tx; };      // a lane's (channel, tap) position in K

// Retire the oldest ring stage when `after` stages (LW DMA pieces each) were issued
// behind it: vmcnt(LW * min(after, D)), D = the ring's steady-state look-ahead.
template <int LW, int D>
__device__ __forceinline__ void wait_ring(int after) {
  if constexpr (D <= 0) {
    wait_vm<0>();
  } else {
    if (after >= D) wait_vm<LW * D>();
    else wait_ring<LW, D - 1>(after);
  }
}


// rgbac_conv_args -> the device-side group descriptor (validates the group; conv.hip)
int fill_group(const rgbac_conv_args* a, int ntaps_max, ConvGroup& g);

}  // namespace rgbac
