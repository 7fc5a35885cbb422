// Backward kernels of the training step (reference: trainRGB.py:178-198 --
// rd_loss.backward(), grad.clamp_(-5, 5), Adam).  The forward convs save their
// pre-activation value through rgbac_conv_args.zout; the input gradient of a
// conv is the same MFMA conv engine run over a repacked (transposed / flipped /
// phase-split) weight; this file holds what has no forward twin:
//
//   act_bwd_kernel       dL/dv of every fused epilogue (GELU, ReLU, LeakyReLU,
//                        tanh-half, sigmoid gate, GDN/IGDN, window-drop select)
//   wgrad_kernel         dW[n][k] = sum_m G[m][n] * Col(S)[m][k] on MFMA: the
//                        reduction runs over PIXELS, so both operands are read
//                        from pixel-major LDS tiles with ds_read_b64_tr_b16
//                        (bf16) -- split over M with deterministic fp32 slabs
//   wgrad_reduce_kernel  slab sum + scatter into the PyTorch weight layout, bias
//   winattn_bwd_kernel   softmax(QK^T+B+M)V backward per (window group, head),
//                        relative-position-bias gradient as per-block partials
//   gaussian_bwd_kernel  GaussianConditional likelihood + bits + STE backward
//   eb_bwd_kernel        EntropyBottleneck factorized density backward (per channel)
//   mse_bwd_kernel       reconstruct_error backward
//   adam_clamp_kernel    grad.clamp_(-c, c) + torch.optim.Adam step (fp32)
//   pixel_shuffle_kernel / channel_copy_kernel   layout helpers (subpel, concat)
#include <algorithm>
#include <cmath>
#include <type_traits>

#include "common.h"

namespace rgbac {

__device__ __forceinline__ float t_sigmoid(float v) { return 1.0f / (1.0f + expf(-v)); }
__device__ __forceinline__ float t_phi(float t) {       // standard normal pdf
  return 0.39894228040143267794f * expf(-0.5f * t * t);
}
__device__ __forceinline__ float t_cdf(float t) {       // 0.5 * erfc(-t / sqrt 2)
  return 0.5f * erfcf(-0.70710678118654752440f * t);
}

// e / d and e % d for 0 <= e < 2^50, d > 0, from a double reciprocal and one correction step
// (the elementwise backward kernels' 64-bit integer division compiled to a ~100-instruction
// software routine per element)
__device__ __forceinline__ long long ediv(long long e, int d, double rd, int& rem) {
  long long q = (long long)((double)e * rd);
  long long r = e - q * d;
  if (r < 0) { --q; r += d; }
  else if (r >= d) { ++q; r -= d; }
  rem = (int)r;
  return q;
}

// ------------------------------------------------------------------ act_bwd
// dz = dL/dv for y = act(v [, r1]); dr1 = dL/dr1 where r1 enters the activation
// (GATE: y = r1*sigmoid(v); GDN: y = r1/sqrt(v); IGDN: y = r1*sqrt(v)).
// Channels [C, ld) of the outputs are written as zeros.  One thread per group of
// 4 channels of a pixel (vector loads/stores; all leading dims are multiples of 4).
template <bool FAST>
__device__ __forceinline__ void act_bwd1(int act, float slope, float g, float v, float a,
                                         bool on, float& gz, float& gr) {
  gz = g;
  gr = 0.0f;
  switch (act) {
    case RGBAC_ACT_GELU:
      gz = FAST ? g * gelu_grad_fast(v) : g * (t_cdf(v) + v * t_phi(v));
      break;
    case RGBAC_ACT_RELU:
      gz = v > 0.0f ? g : 0.0f;
      break;
    case RGBAC_ACT_LRELU:
      gz = v > 0.0f ? g : g * slope;
      break;
    case RGBAC_ACT_TANH_HALF: {
      const float t = tanhf(v);
      gz = g * 0.5f * (1.0f - t * t);
      gr = g;
      break;
    }
    case RGBAC_ACT_GATE: {
      const float s = t_sigmoid(v);
      gz = g * a * (s * (1.0f - s));
      gr = g * s;
      break;
    }
    case RGBAC_ACT_GDN: {
      const float rs = 1.0f / sqrtf(v);
      gz = g * a * (-0.5f) * rs / v;
      gr = g * rs;
      break;
    }
    case RGBAC_ACT_IGDN: {
      const float sq = sqrtf(v);
      gz = g * a * 0.5f / sq;
      gr = g * sq;
      break;
    }
    case RGBAC_ACT_MASKSEL:
      gz = on ? g : 0.0f;
      gr = g;
      break;
    default:
      break;
  }
}

template <typename T, bool FAST>
__global__ void __launch_bounds__(256)
act_bwd_kernel(int act, float slope, long long npix, int C, const T* __restrict__ dy, long long ldy,
               const T* __restrict__ z, long long ldz, const T* __restrict__ r1, long long ld1,
               const uint8_t* __restrict__ sel, T* __restrict__ dz, long long lddz,
               T* __restrict__ dr1, long long lddr1) {
  const int q4 = (int)(lddz / 4);
  const double rq4 = 1.0 / q4;
  const long long n = npix * q4;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    int cq;
    const long long p = ediv(e, q4, rq4, cq);
    const int c0 = cq * 4;
    float gz[4] = {0.f, 0.f, 0.f, 0.f}, gr[4] = {0.f, 0.f, 0.f, 0.f};
    if (c0 + 3 < C) {
      float g[4], v[4] = {0.f, 0.f, 0.f, 0.f}, a[4] = {0.f, 0.f, 0.f, 0.f};
      Elem<T>::ld4(dy + p * ldy + c0, g);
      if (z) Elem<T>::ld4(z + p * ldz + c0, v);
      if (r1 && (act == RGBAC_ACT_GATE || act == RGBAC_ACT_GDN || act == RGBAC_ACT_IGDN))
        Elem<T>::ld4(r1 + p * ld1 + c0, a);
      const bool on = sel ? sel[p] != 0 : true;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        act_bwd1<FAST>(act, slope, g[r], v[r], a[r], on, gz[r], gr[r]);
    } else {
      const bool on = sel ? sel[p] != 0 : true;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + r;
        if (c < C) {
          const float g = Elem<T>::ld(dy + p * ldy + c);
          const float v = z ? Elem<T>::ld(z + p * ldz + c) : 0.0f;
          const float a = (r1 && (act == RGBAC_ACT_GATE || act == RGBAC_ACT_GDN ||
                                  act == RGBAC_ACT_IGDN)) ? Elem<T>::ld(r1 + p * ld1 + c) : 0.0f;
          act_bwd1<FAST>(act, slope, g, v, a, on, gz[r], gr[r]);
        }
      }
    }
    Elem<T>::st4(dz + p * lddz + c0, gz);
    if (dr1 && c0 < lddr1) Elem<T>::st4(dr1 + p * lddr1 + c0, gr);
  }
}

// bf16 act_bwd over unpadded, equally strided operands (C == every leading dim, no select):
// a flat elementwise pass, 8 channels per thread with 16-byte loads and no pixel/channel
// division.
template <bool FAST>
__global__ void __launch_bounds__(256)
act_bwd_flat_kernel(int act, float slope, long long n8, const uint4* __restrict__ dy,
                    const uint4* __restrict__ z, const uint4* __restrict__ r1,
                    uint4* __restrict__ dz, uint4* __restrict__ dr1) {
  const bool use_r1 = r1 && (act == RGBAC_ACT_GATE || act == RGBAC_ACT_GDN || act == RGBAC_ACT_IGDN);
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n8; e += (long long)gridDim.x * 256) {
    const uint4 gq = dy[e], zq = z[e];
    const uint4 aq = use_r1 ? r1[e] : make_uint4(0, 0, 0, 0);
    const uint32_t gw[4] = {gq.x, gq.y, gq.z, gq.w}, zw[4] = {zq.x, zq.y, zq.z, zq.w},
                   aw[4] = {aq.x, aq.y, aq.z, aq.w};
    uint32_t ow[4], rw[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float gz0, gr0, gz1, gr1;
      act_bwd1<FAST>(act, slope, bf2f(gw[i] & 0xFFFF), bf2f(zw[i] & 0xFFFF), bf2f(aw[i] & 0xFFFF),
                     true, gz0, gr0);
      act_bwd1<FAST>(act, slope, bf2f(gw[i] >> 16), bf2f(zw[i] >> 16), bf2f(aw[i] >> 16), true,
                     gz1, gr1);
      ow[i] = pack_bf16x2(gz0, gz1);
      rw[i] = pack_bf16x2(gr0, gr1);
    }
    dz[e] = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    if (dr1) dr1[e] = make_uint4(rw[0], rw[1], rw[2], rw[3]);
  }
}

// ------------------------------------------------------------------ wgrad
struct WgradDev {
  const void* g; long long ldg; int gch;
  const void* sp0; const void* sp1; const void* sp2;
  long long sld0, sld1, sld2;
  int send0, send1, send2;
  int cin_pad, K, k_pad, n_pad;
  int M, Hg, Wg;
  double rWg, rHg;
  int in_h, in_w, ksize, stride, pad, square;
  int m_chunk;
  float* part;
  float* bpart;
};

typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s* lds_v4s_ptr;

__device__ __forceinline__ int wdiv(int n, int d, double rd) {   // n / d, 0 <= n < 2^31
  int q = (int)((double)n * rd);
  const int r = n - q * d;
  if (r < 0) --q;
  else if (r >= d) ++q;
  return q;
}

// D[n][k] = sum_m G[m][n] * Col(S)[m][k]; a 64(n) x BK(k) tile per workgroup
// (BK = 32*KT), 4 waves as 2(n) x 2(k), each 32 x 16*KT; 64 pixels per stage,
// register-staged, double-buffered LDS tiles whose rows are pixels.
//   bf16: the 16-B chunk c of LDS row r lives at slot c ^ swz(r) so that the
//         ds_read_b64_tr_b16 reads of a 32-lane half (rows 8q..8q+3 of two
//         16-lane groups, 32 B each) hit 64 distinct banks:
//           128-B rows (64 elements): swz = 2*((r>>1)&1) + 4*((r>>3)&1)
//           256-B rows (128 elements): swz = 2*((r&3) + 4*((r>>3)&1))
//         The MFMA operand of lane l (row l&15 of a 16-row tile, pixels
//         8q..8q+7 of the 32-deep k-step, q = l>>4) = two transposed reads.
//   f32 : KT = 2, rows padded to 272 B, operands are 4 scalar LDS reads per lane.
template <typename T, int KT>
__global__ void __launch_bounds__(256) wgrad_kernel(const WgradDev a) {
  constexpr int EPV = Elem<T>::EPV;
  constexpr int BK = 32 * KT;
  constexpr int CPRG = 64 / EPV;                  // 16-B chunks per G row (64 channels)
  constexpr int CPRS = BK / EPV;                  // chunks per S row
  constexpr int NLG = 64 * CPRG / 256;            // chunks per thread per tile
  constexpr int NLS = 64 * CPRS / 256;
  constexpr int RSG = sizeof(T) == 2 ? 128 : 272; // LDS row strides (bytes)
  constexpr int RSS = sizeof(T) == 2 ? BK * 2 : BK * 4 + 16;
  static_assert(sizeof(T) == 2 || KT == 2, "f32 wgrad uses KT = 2");
  __shared__ __attribute__((aligned(16))) unsigned char ldsG[2][64 * RSG];
  __shared__ __attribute__((aligned(16))) unsigned char ldsS[2][64 * RSS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int k0 = blockIdx.x * BK, n0 = blockIdx.y * 64, split = blockIdx.z;
  const int mbeg = split * a.m_chunk;
  int mend = mbeg + a.m_chunk;
  if (mend > a.M) mend = a.M;
  const bool do_bias = a.bpart && blockIdx.x == 0;

  auto slotG = [&](int r, int c) -> int {
    if constexpr (sizeof(T) == 2) return r * RSG + 16 * (c ^ (2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1)));
    else return r * RSG + 16 * c;
  };
  auto slotS = [&](int r, int c) -> int {
    if constexpr (sizeof(T) == 2) {
      if constexpr (BK == 64) return r * RSS + 16 * (c ^ (2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1)));
      else return r * RSS + 16 * (c ^ (2 * ((r & 3) + 4 * ((r >> 3) & 1))));
    } else {
      return r * RSS + 16 * c;
    }
  };

  // per-thread chunk geometry (fixed over stages)
  int grow[NLG], gcol[NLG];
  bool g_ok[NLG];
#pragma unroll
  for (int j = 0; j < NLG; ++j) {
    const int c = tid + 256 * j;
    grow[j] = c / CPRG;
    gcol[j] = c % CPRG;
    g_ok[j] = n0 + gcol[j] * EPV < a.gch;
  }
  int srow[NLS], scol[NLS], s_src[NLS], s_cs[NLS], s_dy[NLS], s_dx[NLS];
  bool s_ok[NLS];
#pragma unroll
  for (int j = 0; j < NLS; ++j) {
    const int c = tid + 256 * j;
    srow[j] = c / CPRS;
    scol[j] = c % CPRS;
    const int k = k0 + scol[j] * EPV;
    const int tap = k / a.cin_pad;
    const int ci = k - tap * a.cin_pad;
    s_ok[j] = k < a.K;
    s_dy[j] = tap / a.ksize - a.pad;
    s_dx[j] = tap % a.ksize - a.pad;
    if (ci < a.send0) { s_src[j] = 0; s_cs[j] = ci; }
    else if (ci < a.send1) { s_src[j] = 1; s_cs[j] = ci - a.send0; }
    else { s_src[j] = 2; s_cs[j] = ci - a.send1; s_ok[j] = s_ok[j] && ci < a.send2; }
  }

  uint4 rg[NLG], rs[NLS];
  auto load_stage = [&](int mb) {
#pragma unroll
    for (int j = 0; j < NLG; ++j) {
      const int m = mb + grow[j];
      rg[j] = make_uint4(0, 0, 0, 0);
      if (m < mend && g_ok[j])
        rg[j] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(a.g) +
                                                (long long)m * a.ldg + n0 + gcol[j] * EPV);
    }
#pragma unroll
    for (int j = 0; j < NLS; ++j) {
      const int m = mb + srow[j];
      rs[j] = make_uint4(0, 0, 0, 0);
      if (m < mend && s_ok[j]) {
        const int t = wdiv(m, a.Wg, a.rWg);
        const int x = m - t * a.Wg;
        const int b = wdiv(t, a.Hg, a.rHg);
        const int y = t - b * a.Hg;
        const int iy = y * a.stride + s_dy[j], ix = x * a.stride + s_dx[j];
        if (iy >= 0 && iy < a.in_h && ix >= 0 && ix < a.in_w) {
          const int sj = s_src[j];
          const T* base = reinterpret_cast<const T*>(sj == 0 ? a.sp0 : (sj == 1 ? a.sp1 : a.sp2));
          const long long ld = sj == 0 ? a.sld0 : (sj == 1 ? a.sld1 : a.sld2);
          rs[j] = *reinterpret_cast<const uint4*>(
              base + ((long long)(b * a.in_h + iy) * a.in_w + ix) * ld + s_cs[j]);
        }
      }
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int j = 0; j < NLG; ++j)
      *reinterpret_cast<uint4*>(&ldsG[buf][slotG(grow[j], gcol[j])]) = rg[j];
#pragma unroll
    for (int j = 0; j < NLS; ++j) {
      uint4 sv = rs[j];
      if (a.square) {
        if constexpr (sizeof(T) == 2) {
          uint32_t w[4] = {sv.x, sv.y, sv.z, sv.w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float lo = bf2f(w[q] & 0xFFFF), hi = bf2f(w[q] >> 16);
            w[q] = (uint32_t)f2bf(lo * lo) | ((uint32_t)f2bf(hi * hi) << 16);
          }
          sv = make_uint4(w[0], w[1], w[2], w[3]);
        } else {
          const float p0 = __uint_as_float(sv.x), p1 = __uint_as_float(sv.y);
          const float p2 = __uint_as_float(sv.z), p3 = __uint_as_float(sv.w);
          sv = make_uint4(__float_as_uint(p0 * p0), __float_as_uint(p1 * p1),
                          __float_as_uint(p2 * p2), __float_as_uint(p3 * p3));
        }
      }
      *reinterpret_cast<uint4*>(&ldsS[buf][slotS(srow[j], scol[j])]) = sv;
    }
  };

  f32x4 acc[2][KT];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < KT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.0f;

  const int wn = wave >> 1, wk = wave & 1;
  const int fi = lane & 15, fq = lane >> 4;
  const int nst = mend > mbeg ? (mend - mbeg + 63) / 64 : 0;
  if (nst > 0) {
    load_stage(mbeg);
    store_stage(0);
  }
  __syncthreads();
  for (int it = 0; it < nst; ++it) {
    const int buf = it & 1;
    if (it + 1 < nst) load_stage(mbeg + (it + 1) * 64);
    const unsigned char* Gs = ldsG[buf];
    const unsigned char* Ss = ldsS[buf];
    if (do_bias && tid < 64) {
      // column sums of G (bias gradient) over this stage's 64 pixels
#pragma unroll 4
      for (int r = 0; r < 64; ++r) {
        const int off = slotG(r, tid / EPV) + (tid % EPV) * (int)sizeof(T);
        if constexpr (sizeof(T) == 2) bacc += bf2f(*reinterpret_cast<const uint16_t*>(Gs + off));
        else bacc += *reinterpret_cast<const float*>(Gs + off);
      }
    }
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        uint4 A[2], B[KT];
        const int ra = kk * 32 + 8 * fq + (fi >> 2);     // block row of this lane's address
        const int cq = (fi & 3);                         // 4-column quad within 16 columns
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int ncol = wn * 32 + t * 16 + 4 * cq;
          const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4s_ptr)(Gs + slotG(ra, ncol >> 3) + (ncol & 7) * 2));
          const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4s_ptr)(Gs + slotG(ra + 4, ncol >> 3) + (ncol & 7) * 2));
          const uint2 ua0 = __builtin_bit_cast(uint2, a0), ua1 = __builtin_bit_cast(uint2, a1);
          A[t] = make_uint4(ua0.x, ua0.y, ua1.x, ua1.y);
        }
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const int kcol = wk * 16 * KT + t * 16 + 4 * cq;
          const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4s_ptr)(Ss + slotS(ra, kcol >> 3) + (kcol & 7) * 2));
          const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
              (lds_v4s_ptr)(Ss + slotS(ra + 4, kcol >> 3) + (kcol & 7) * 2));
          const uint2 ub0 = __builtin_bit_cast(uint2, b0), ub1 = __builtin_bit_cast(uint2, b1);
          B[t] = make_uint4(ub0.x, ub0.y, ub1.x, ub1.y);
        }
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
#pragma unroll
          for (int tk = 0; tk < KT; ++tk) mma_step<bf16_t>(acc[tn][tk], A[tn], B[tk]);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        uint4 A[2], B[KT];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int ncol = wn * 32 + t * 16 + fi;
          uint32_t av[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            av[e] = *reinterpret_cast<const uint32_t*>(Gs + (ks * 16 + 4 * fq + e) * RSG + ncol * 4);
          A[t] = make_uint4(av[0], av[1], av[2], av[3]);
        }
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const int kcol = wk * 16 * KT + t * 16 + fi;
          uint32_t bv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e)
            bv[e] = *reinterpret_cast<const uint32_t*>(Ss + (ks * 16 + 4 * fq + e) * RSS + kcol * 4);
          B[t] = make_uint4(bv[0], bv[1], bv[2], bv[3]);
        }
#pragma unroll
        for (int tn = 0; tn < 2; ++tn)
#pragma unroll
          for (int tk = 0; tk < KT; ++tk) mma_step<float>(acc[tn][tk], A[tn], B[tk]);
      }
    }
    if (it + 1 < nst) store_stage(buf ^ 1);
    __syncthreads();
  }
  // partial slab [split][n_pad][k_pad]: lane holds D[n = 4*fq + r][k = fi] per 16x16 tile
  float* P = a.part + (size_t)split * a.n_pad * a.k_pad;
#pragma unroll
  for (int tn = 0; tn < 2; ++tn)
#pragma unroll
    for (int tk = 0; tk < KT; ++tk)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 32 + tn * 16 + 4 * fq + r;
        const int k = k0 + wk * 16 * KT + tk * 16 + fi;
        if (k < a.k_pad) P[(size_t)n * a.k_pad + k] = acc[tn][tk][r];
      }
  if (do_bias && tid < 64) a.bpart[(size_t)split * a.n_pad + n0 + tid] = bacc;
}

// ---------------------------------------------------------------------------------------
// Ring-pipelined weight gradient (bf16, no squared input): the same 64(n) x BK(k) tiles, wave
// layout, LDS images (pixel rows, XOR-swizzled 16-B chunks) and transposed fragment reads as
// wgrad_kernel, but every stage is moved global -> LDS by LDS-DMA (global_load_lds_dwordx4,
// 1 KiB per wave instruction, no register staging) into a WR-deep ring, so the loads of the
// next WR-1 stages are in flight while a stage's MFMAs run.  wgrad_kernel stages through
// registers one stage ahead: each 64-pixel stage (256 MFMA cycles per wave) waited for a full
// global-memory round trip (~2k cycles under load) -- 4-6 % of the MFMA peak.
//   A DMA piece is 1 KiB of one stage image: lane l writes image byte 16 l of the piece, i.e.
//   row r = (piece rows) + l / chunks-per-row, slot l % chunks-per-row, which holds chunk
//   c = slot ^ swz(r) (the swizzle is an involution) -- so each lane fetches the global
//   16-byte chunk c of its row directly; out-of-range pixels / channels / taps read a zero page.
//   The per-lane (tap, channel, source) of every S piece is fixed over the stages; the pixel of
//   a piece row is decoded per stage.
__device__ uint4 g_wgrad_zero[64];

typedef __attribute__((address_space(3))) void* wg_lptr_t;

__device__ __forceinline__ void wg_dma16(const void* src, uint32_t lds) {
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
__device__ __forceinline__ void wg_wait_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// retire the oldest ring stage with `after` later stages (PW pieces each) in flight
template <int PW, int D>
__device__ __forceinline__ void wg_wait_ring(int after) {
  if constexpr (D <= 0) {
    wg_wait_vm<0>();
  } else {
    if (after >= D) wg_wait_vm<PW * D>();
    else wg_wait_ring<PW, D - 1>(after);
  }
}

// WGN x WGK waves (2 x 2: 256 threads, the original layout; 2 x 4: 512 threads), each owning a
// (16 TN) x (16 KT) block of the BN x BK tile.  The 512-thread 128 x 256 tile (TN = KT = 4)
// moves 48 KiB per 64-pixel stage for 4.2 MFLOP -- twice the MFMAs per DMA piece and per L2
// byte of the 64 x 128 tile, whose per-stage DMA issue and address VALU (8.4 VALU + 7.6 SALU
// per MFMA, 45 % of wave cycles issuing: PMC on the slice-stack shape) bounded it.
template <int TN, int KT, int WR, int WGN = 2, int WGK = 2>
__global__ void __launch_bounds__(64 * WGN * WGK) wgrad_ring_kernel(const WgradDev a) {
  constexpr int NW = WGN * WGK, NTH = 64 * NW;
  constexpr int BN = 16 * TN * WGN, BK = 16 * KT * WGK;
  constexpr int RSG = BN * 2, RSS = BK * 2;       // LDS row bytes (G: BN channels, S: BK k)
  static_assert(RSG == 128 || RSG % 256 == 0, "G rows: 128 B or multiples of 256 B (swizzle)");
  static_assert(RSS == 128 || RSS % 256 == 0, "S rows: 128 B or multiples of 256 B (swizzle)");
  constexpr int GB = 64 * RSG, SB = 64 * RSS;     // stage image bytes
  constexpr int CRS = RSS / 16;                   // 16-B chunks per S row (8, 16 or 32)
  constexpr int RPS = 64 / CRS;                   // S rows per 1-KiB piece (8, 4 or 2)
  constexpr int CRG = RSG / 16, RPG = 64 / CRG;   // the same for G rows
  constexpr int PG = GB / 1024 / NW, PS = SB / 1024 / NW;   // pieces per wave per stage
  static_assert(PG * NW * 1024 == GB && PS * NW * 1024 == SB, "whole pieces per wave");
  constexpr int PW = PG + PS;
  __shared__ __attribute__((aligned(16))) unsigned char ring[WR * (GB + SB)];
  __shared__ float bred[NTH / BN][BN];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-aware tile order: the hardware deals workgroup i to XCD i mod 8, so consecutive ids
  // (the k tiles of one pixel split, which read the same G / S pixels) would land on 8
  // different L2s and each fetch the pixels from HBM.  Remapped, an XCD runs a contiguous run
  // of (k tile fastest, n tile, split) and its L2 serves the other k tiles' re-reads.
  int kt, nt, split;
  {
    const int nwg = gridDim.x * gridDim.y * gridDim.z;
    int t = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    const int xcd = t & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (t >> 3);
    kt = t % gridDim.x; t /= gridDim.x;
    nt = t % gridDim.y;
    split = t / gridDim.y;
  }
  const int k0 = kt * BK, n0 = nt * BN;
  const int mbeg = split * a.m_chunk;
  const int mend = min(mbeg + a.m_chunk, a.M);
  const bool do_bias = a.bpart && kt == 0;
  // 128-B rows: chunk c of row r at c ^ (2 r1 + 4 r3); 256-B rows: c ^ 2 (r&3 + 4 r3)
  // (r_i = bit i of r): conflict-free transposed reads, and rows r + 4 h + 32 kk keep r's
  // swizzle (only row bits 0, 1, 3 enter it)
  // (rows of >= 256 B: a row is a multiple of 64 banks, so the 256-B-row swizzle -- chunk XORs
  // below 16 -- spreads the 8 rows of a transposed read over all banks for any such length)
  auto swzG = [](int r) {
    if constexpr (RSG == 128) return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1);
    else return 2 * ((r & 3) + 4 * ((r >> 3) & 1));
  };
  auto swzS = [](int r) {
    if constexpr (RSS == 128) return 2 * ((r >> 1) & 1) + 4 * ((r >> 3) & 1);
    else return 2 * ((r & 3) + 4 * ((r >> 3) & 1));
  };

  // ---- per-lane DMA geometry, fixed over the stages
  int grow[PG];
  const char* gsrc[PG];
  bool gok[PG];
#pragma unroll
  for (int j = 0; j < PG; ++j) {
    const int q = wave + NW * j;                  // G piece = rows RPG q .. RPG q + RPG - 1
    grow[j] = RPG * q + lane / CRG;
    const int c = (lane % CRG) ^ swzG(grow[j]);
    const int n = n0 + 8 * c;
    gok[j] = n < a.gch;
    gsrc[j] = reinterpret_cast<const char*>(a.g) + (size_t)(gok[j] ? n : 0) * 2;
  }
  int srow[PS], sdy[PS], sdx[PS], sld[PS];
  const char* ssrc[PS];
  bool sok[PS];
#pragma unroll
  for (int j = 0; j < PS; ++j) {
    const int q = wave + NW * j;                  // S piece = rows RPS q .. RPS q + RPS - 1
    srow[j] = RPS * q + lane / CRS;
    const int c = (lane % CRS) ^ swzS(srow[j]);
    const int k = k0 + 8 * c;
    const int tap = k / a.cin_pad, ci = k - (k / a.cin_pad) * a.cin_pad;
    sdy[j] = tap / a.ksize - a.pad;
    sdx[j] = tap % a.ksize - a.pad;
    const char* base;
    int ld, cs;
    if (ci < a.send0) { base = (const char*)a.sp0; ld = (int)a.sld0; cs = ci; }
    else if (ci < a.send1) { base = (const char*)a.sp1; ld = (int)a.sld1; cs = ci - a.send0; }
    else { base = (const char*)a.sp2; ld = (int)a.sld2; cs = ci - a.send1; }
    sok[j] = k < a.K && ci < a.send2;
    ssrc[j] = base + (size_t)(sok[j] ? cs : 0) * 2;
    sld[j] = ld * 2;                              // bytes per source pixel
  }
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(wg_lptr_t)ring);
  const int ldg2 = (int)a.ldg * 2;
  // pixel (b, y, x) of every S piece row for the next stage to issue: decoded once, then
  // advanced by 64 pixels per stage (no per-stage division); 1x1 stride-1: the M index is the
  // source pixel index
  const bool pdirect = a.ksize == 1 && a.stride == 1;
  const int adx = 64 % a.Wg, ady = 64 / a.Wg;
  int pb[PS], py[PS], px[PS];
#pragma unroll
  for (int j = 0; j < PS; ++j) {
    const int m = mbeg + srow[j];
    const int t = wdiv(m, a.Wg, a.rWg);
    px[j] = m - t * a.Wg;
    pb[j] = wdiv(t, a.Hg, a.rHg);
    py[j] = t - pb[j] * a.Hg;
  }

  // G piece addresses advance by 64 pixel rows per stage; stride-1 S piece addresses too
  // (source pixel = M pixel + dy * W + dx on the same grid), only their bounds test needs the
  // (y, x) state.  Stride 2 recomputes the source pixel from (b, y, x).
  const bool s1 = a.stride == 1;
  const char* gp[PG];
  const char* sp[PS];
  const void* const zp = (const void*)g_wgrad_zero;
#pragma unroll
  for (int j = 0; j < PG; ++j) gp[j] = gsrc[j] + (size_t)(mbeg + grow[j]) * ldg2;
#pragma unroll
  for (int j = 0; j < PS; ++j)
    sp[j] = ssrc[j] + (long long)(mbeg + srow[j] + sdy[j] * a.in_w + sdx[j]) * sld[j];
  const size_t gstep = (size_t)64 * ldg2;
  auto issue = [&](int st) {                      // DMA stage st into ring slot st % WR
    const int mb = mbeg + st * 64;
    const uint32_t lg = lbase + (uint32_t)((st % WR) * (GB + SB));
    const uint32_t ls = lg + GB;
#pragma unroll
    for (int j = 0; j < PG; ++j) {
      const bool ok = gok[j] && mb + grow[j] < mend;
      wg_dma16(ok ? (const void*)gp[j] : zp, lg + (uint32_t)((wave + NW * j) * 1024));
      gp[j] += gstep;
    }
#pragma unroll
    for (int j = 0; j < PS; ++j) {
      const int iy = py[j] * a.stride + sdy[j], ix = px[j] * a.stride + sdx[j];
      const bool ok = sok[j] && mb + srow[j] < mend && (unsigned)iy < (unsigned)a.in_h &&
                      (unsigned)ix < (unsigned)a.in_w;
      const void* src;
      if (s1) {
        src = ok ? (const void*)sp[j] : zp;
        sp[j] += (size_t)64 * sld[j];
      } else {
        src = ok ? (const void*)(ssrc[j] + (size_t)((pb[j] * a.in_h + iy) * a.in_w + ix) * sld[j])
                 : zp;
      }
      wg_dma16(src, ls + (uint32_t)((wave + NW * j) * 1024));
      if (!pdirect) {                             // advance to the next stage's pixel
        px[j] += adx;
        py[j] += ady;
        if (px[j] >= a.Wg) { px[j] -= a.Wg; ++py[j]; }
        while (py[j] >= a.Hg) { py[j] -= a.Hg; ++pb[j]; }
      }
    }
  };

  f32x4 acc[TN][KT];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < KT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.0f;
  const int wn = wave / WGK, wk = wave % WGK;
  const int fi = lane & 15, fq = lane >> 4;
  int aoff[TN], boff[KT];                         // per-lane fragment read offsets (bytes)
  {
    const int ra0 = 8 * fq + (fi >> 2), cq = fi & 3;
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      const int ncol = wn * 16 * TN + t * 16 + 4 * cq;
      aoff[t] = ra0 * RSG + 16 * ((ncol >> 3) ^ swzG(ra0)) + (ncol & 7) * 2;
    }
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int kcol = wk * 16 * KT + t * 16 + 4 * cq;
      boff[t] = ra0 * RSS + 16 * ((kcol >> 3) ^ swzS(ra0)) + (kcol & 7) * 2;
    }
  }
  const int nst = mend > mbeg ? (mend - mbeg + 63) / 64 : 0;
  for (int st = 0; st < WR - 1; ++st)
    if (st < nst) issue(st);
  for (int it = 0; it < nst; ++it) {
    wg_wait_ring<PW, WR - 2>(min(WR - 2, nst - 1 - it));
    __syncthreads();                              // stage it landed for every wave; slot
                                                  // (it - 1) % WR is free again
    if (it + WR - 1 < nst) issue(it + WR - 1);
    const unsigned char* Gs = ring + (it % WR) * (GB + SB);
    const unsigned char* Ss = Gs + GB;
    if (do_bias) {                                // G column sums: row groups x BN channels
      constexpr int NRG = NTH / BN, RPR = 64 / NRG;
      const int c = tid % BN, rg = tid / BN;
#pragma unroll 4
      for (int r = RPR * rg; r < RPR * rg + RPR; ++r)
        bacc += bf2f(*reinterpret_cast<const uint16_t*>(
            Gs + r * RSG + 16 * ((c >> 3) ^ swzG(r)) + (c & 7) * 2));
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 A[TN], B[KT];
      // rows ra0 + 32 kk + 4 h share ra0's swizzle (it reads row bits 0, 1, 3 only): one
      // per-lane offset per fragment column, the row step a compile-time immediate
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const unsigned char* q = Gs + aoff[t] + kk * 32 * RSG;
        const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)q);
        const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)(q + 4 * RSG));
        const uint2 ua0 = __builtin_bit_cast(uint2, a0), ua1 = __builtin_bit_cast(uint2, a1);
        A[t] = make_uint4(ua0.x, ua0.y, ua1.x, ua1.y);
      }
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const unsigned char* q = Ss + boff[t] + kk * 32 * RSS;
        const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)q);
        const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)(q + 4 * RSS));
        const uint2 ub0 = __builtin_bit_cast(uint2, b0), ub1 = __builtin_bit_cast(uint2, b1);
        B[t] = make_uint4(ub0.x, ub0.y, ub1.x, ub1.y);
      }
#pragma unroll
      for (int tn = 0; tn < TN; ++tn)
#pragma unroll
        for (int tk = 0; tk < KT; ++tk) mma_step<bf16_t>(acc[tn][tk], A[tn], B[tk]);
    }
  }
  float* P = a.part + (size_t)split * a.n_pad * a.k_pad;
#pragma unroll
  for (int tn = 0; tn < TN; ++tn)
#pragma unroll
    for (int tk = 0; tk < KT; ++tk)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + wn * 16 * TN + tn * 16 + 4 * fq + r;
        const int k = k0 + wk * 16 * KT + tk * 16 + fi;
        if (k < a.k_pad && n < a.n_pad) P[(size_t)n * a.k_pad + k] = acc[tn][tk][r];
      }
  if (do_bias) {
    constexpr int NRG = NTH / BN;
    bred[tid / BN][tid % BN] = bacc;
    __syncthreads();
    if (tid < BN && n0 + tid < a.n_pad) {
      float sum = bred[0][tid];
#pragma unroll
      for (int g2 = 1; g2 < NRG; ++g2) sum += bred[g2][tid];
      a.bpart[(size_t)split * a.n_pad + n0 + tid] = sum;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Patch weight gradient for the narrow-output 3x3 convs (bf16, stride 1, pad 1, one source,
// <= 32 output channels: the DSE's 32 -> 32 convs at full resolution, the slice stacks'
// 128 -> 8 / 16 tails).  The ring kernel's im2col stages re-read each source pixel once per
// tap (9x the source bytes through L2 -> LDS) and pads N to a 64-wide tile (2-8x the MFMAs);
// here a workgroup stages one 8 x 32-pixel output patch of G and its 10 x 34 source halo
// (one 32-channel block) ONCE per patch by LDS-DMA, and every tap reads the halo at a shifted
// row: the 32 pixels of one output row segment are 32 consecutive halo rows.
//   LDS rows are pixels of 64 B (32 channels).  G rows: 16-B chunk c of row r at c ^ 2*bit3(r)
//   (conflict-free transposed reads).  Halo rows are unswizzled: a (tap, half) pair's fragment
//   address is then a per-lane register plus the row's immediate offset (a swizzled, shifted
//   row cost ~5 VALU of address math per MFMA), for 2-way bank conflicts on those reads.
//   The 18 (tap, 16-channel half) pairs of the block are dealt to the 4 waves (5/5/4/4); each
//   wave runs all 8 row segments of the patch for its pairs and both 16-channel n tiles, so the
//   accumulators never cross waves: each lane stores its own slab elements.
//   Double-buffered over the workgroup's run of patches (m_chunk = patches per split); the
//   slab layout [split][n_pad][k_pad], k = tap * cin_pad + channel, is the ring kernel's, so
//   wgrad_reduce is unchanged.
constexpr int kWpTH = 8, kWpTW = 32, kWpPW = kWpTW + 2;
constexpr int kWpSRows = (kWpTH + 2) * kWpPW;          // 340 staged source pixels
constexpr int kWpSPieces = (kWpSRows + 15) / 16;       // 22 one-KiB pieces of 16 rows
constexpr int kWpGPieces = kWpTH * kWpTW / 16;         // 16
constexpr int kWpBuf = (kWpSPieces + kWpGPieces) * 1024;

__device__ __forceinline__ int wp_swz(int r) { return 2 * ((r >> 3) & 1); }

template <int NT>
__global__ void __launch_bounds__(256) wgrad_patch_kernel(const WgradDev a) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[2 * kWpBuf];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // XCD-contiguous (channel block fastest, split): the channel blocks of one split read the
  // same G patches from one L2
  int cb, split;
  {
    const int nwg = gridDim.x * gridDim.y;
    int t = blockIdx.x + gridDim.x * blockIdx.y;
    const int xcd = t & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (t >> 3);
    cb = t % gridDim.x;
    split = t / gridDim.x;
  }
  const int H = a.Hg, W = a.Wg;
  const int pw = W / kWpTW, ppi = pw * (H / kWpTH);
  const int P = a.M / (kWpTH * kWpTW);
  const int pbeg = split * a.m_chunk;
  const int pend = min(pbeg + a.m_chunk, P);
  const bool do_bias = a.bpart && cb == 0;
  const void* const zp = (const void*)g_wgrad_zero;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(wg_lptr_t)ring);

  // ---- per-lane DMA geometry (fixed over the patches)
  constexpr int PSW = (kWpSPieces + 3) / 4, PGW = kWpGPieces / 4;
  const int nps = (kWpSPieces - wave + 3) / 4;          // this wave's S pieces (6 or 5)
  int s_rel[PSW], s_i[PSW], s_j[PSW], s_c[PSW];
  bool s_on[PSW];
  const int choff = (cb * 32) * 2;
#pragma unroll
  for (int j = 0; j < PSW; ++j) {
    const int q = wave + 4 * j;                         // S piece = halo rows 16 q .. 16 q + 15
    const int R = 16 * q + (lane >> 2);
    s_c[j] = (lane & 3) * 16;                           // halo rows unswizzled (see below)
    s_i[j] = R / kWpPW;
    s_j[j] = R - s_i[j] * kWpPW;
    s_on[j] = q < kWpSPieces && R < kWpSRows;
    s_rel[j] = (s_i[j] - 1) * W + (s_j[j] - 1);         // pixel offset from the patch origin
  }
  int g_rel[PGW], g_c[PGW];
  bool g_on[PGW];
#pragma unroll
  for (int j = 0; j < PGW; ++j) {
    const int R = 16 * (wave + 4 * j) + (lane >> 2);
    const int c = (lane & 3) ^ wp_swz(R);
    g_rel[j] = (R >> 5) * W + (R & 31);
    g_on[j] = 8 * c < a.gch;
    g_c[j] = c * 16;
  }
  const char* const sbase = reinterpret_cast<const char*>(a.sp0) + choff;
  const long long sld2 = a.sld0 * 2, ldg2 = a.ldg * 2;
  const char* const gbase = reinterpret_cast<const char*>(a.g);

  auto issue = [&](int p, int buf) {
    const int b = p / ppi, rem = p - b * ppi;
    const int y0 = (rem / pw) * kWpTH, x0 = (rem - (rem / pw) * pw) * kWpTW;
    const long long pix0 = ((long long)b * H + y0) * W + x0;
    const uint32_t ls = lbase + (uint32_t)(buf * kWpBuf);
    const uint32_t lg = ls + kWpSPieces * 1024;
#pragma unroll
    for (int j = 0; j < PSW; ++j) {
      if (j < nps) {
        const int y = y0 + s_i[j] - 1, x = x0 + s_j[j] - 1;
        const bool ok = s_on[j] && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
        wg_dma16(ok ? (const void*)(sbase + (pix0 + s_rel[j]) * sld2 + s_c[j]) : zp,
                 ls + (uint32_t)((wave + 4 * j) * 1024));
      }
    }
#pragma unroll
    for (int j = 0; j < PGW; ++j)
      wg_dma16(g_on[j] ? (const void*)(gbase + (pix0 + g_rel[j]) * ldg2 + g_c[j]) : zp,
               lg + (uint32_t)((wave + 4 * j) * 1024));
  };

  // ---- this wave's (tap, channel half) pairs: e = wave + 4 i < 18
  f32x4 acc[5][NT];
#pragma unroll
  for (int i = 0; i < 5; ++i)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.0f;
  const int fi = lane & 15, fq = lane >> 4, cq = fi & 3;
  const int ra0 = 8 * fq + (fi >> 2);
  int aoff[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) aoff[t] = ra0 * 64 + 16 * ((2 * t + (cq >> 1)) ^ wp_swz(ra0)) + 8 * (cq & 1);
  // per-lane fragment offsets of this wave's pairs (unswizzled halo rows: the address is this
  // register plus the row's immediate, no per-read arithmetic)
  const int npr = (18 - wave + 3) / 4;                  // 5 or 4 (wave-uniform)
  int boff[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int e = min(wave + 4 * i, 17);
    const int tap = e >> 1, u = e & 1;
    const int ky = tap / 3, kx = tap - 3 * (tap / 3);
    boff[i] = (ky * kWpPW + kx + ra0) * 64 + 16 * (2 * u + (cq >> 1)) + 8 * (cq & 1);
  }
  const uint32_t rbase = (uint32_t)(size_t)(wg_lptr_t)ring;

  if (pbeg < pend) issue(pbeg, 0);
  for (int p = pbeg, it = 0; p < pend; ++p, ++it) {
    const int buf = it & 1;
    if (p + 1 < pend) {
      issue(p + 1, buf ^ 1);
      if (nps == PSW) wg_wait_vm<PSW + PGW>();
      else wg_wait_vm<PSW - 1 + PGW>();
    } else {
      wg_wait_vm<0>();
    }
    __syncthreads();                                     // patch p landed for every wave
    const unsigned char* Ss = ring + buf * kWpBuf;
    const unsigned char* Gs = Ss + kWpSPieces * 1024;
    if (do_bias) {                                       // G column sums: 8 row groups x 32
      const int c = tid & 31, rg = tid >> 5;
#pragma unroll 4
      for (int r = 32 * rg; r < 32 * rg + 32; ++r)
        bacc += bf2f(*reinterpret_cast<const uint16_t*>(
            Gs + r * 64 + 16 * ((c >> 3) ^ wp_swz(r)) + (c & 7) * 2));
    }
    uint32_t bp[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) bp[i] = rbase + (uint32_t)(buf * kWpBuf) + (uint32_t)boff[i];
    const uint32_t gp = rbase + (uint32_t)(buf * kWpBuf + kWpSPieces * 1024);
#pragma unroll 2
    for (int yy = 0; yy < kWpTH; ++yy) {
      uint4 A[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const lds_v4s_ptr q = (lds_v4s_ptr)(size_t)(gp + aoff[t] + yy * 32 * 64);
        const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q);
        const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q + 4 * 64 / 8);
        const uint2 u0 = __builtin_bit_cast(uint2, a0), u1 = __builtin_bit_cast(uint2, a1);
        A[t] = make_uint4(u0.x, u0.y, u1.x, u1.y);
      }
#pragma unroll
      for (int i = 0; i < 5; ++i) {
        if (i < npr) {                                   // wave-uniform
          const lds_v4s_ptr q = (lds_v4s_ptr)(size_t)(bp[i] + yy * kWpPW * 64);
          const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q);
          const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q + 4 * 64 / 8);
          const uint2 u0 = __builtin_bit_cast(uint2, b0), u1 = __builtin_bit_cast(uint2, b1);
          const uint4 B = make_uint4(u0.x, u0.y, u1.x, u1.y);
#pragma unroll
          for (int t = 0; t < NT; ++t) mma_step<bf16_t>(acc[i][t], A[t], B);
        }
      }
    }
    __syncthreads();                                     // buf free for patch p + 2
  }
  // slab: lane holds D[n = 16 t + 4 fq + r][channel = 16 u + fi] of pair (tap, u)
  float* Pp = a.part + (size_t)split * a.n_pad * a.k_pad;
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int e = wave + 4 * i;
    if (e < 18) {
      const int tap = e >> 1, u = e & 1;
      const int k = tap * a.cin_pad + cb * 32 + 16 * u + fi;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = 16 * t + 4 * fq + r;
          if (n < a.gch) Pp[(size_t)n * a.k_pad + k] = acc[i][t][r];
        }
    }
  }
  if (do_bias) {
    float* bred = reinterpret_cast<float*>(ring);        // [8][32], the buffers are free
    bred[tid] = bacc;
    __syncthreads();
    if (tid < 32 && tid < a.gch) {
      float s = bred[tid];
#pragma unroll
      for (int g2 = 1; g2 < 8; ++g2) s += bred[32 * g2 + tid];
      a.bpart[(size_t)split * a.n_pad + tid] = s;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Halo-staged weight gradients (bf16, 32-channel source blocks x 64-channel output blocks, up
// to three concatenated sources):
//   STRIDE 2: the 5x5 stride-2 pad-2 convs and ConvTransposes (Analysis x2 / x3, their
//     Synthesis mirrors; 120 GFLOP per step at 64^2).  Through im2col the ring kernel re-reads
//     every source pixel ~6x per k tile and once per n tile (1.3 GB of L2 -> LDS traffic per
//     launch at 64^2 B16); here, as in the forward's polyphase patch conv, the source splits
//     into its 4 stride phases S_q[i][j] = S[2i + qy][2j + qx], and kernel tap (ky, kx) =
//     (2 ty + qy, 2 tx + qx) is a stride-1 tap (ty, tx) of phase q:
//       dW[n][ky][kx][c] = sum_o G[o][n] * S_q[oy + ty - 1][ox + tx - 1][c];
//   STRIDE 1: the 3x3 pad-1 convs with more than 32 outputs (slice stacks, residual units,
//     hyper convs): one phase, tap (ky, kx) at shift (ky, kx) of the halo.
// A workgroup (8 waves) stages a 4 x 32-pixel G patch (64 channels) and the phase halos
// (6 x 34 pixels, 32 channels) once per patch by LDS-DMA (double-buffered: 136 KiB for stride
// 2, one workgroup per CU; 58 KiB for stride 1, two); the (tap, 16-channel half) pairs are
// dealt to the waves, every wave covering the block's 4 n tiles, so accumulators stay in the
// wave.  LDS rows: halo pixels of 64 B, unswizzled (a pair's fragment address is then a
// per-lane constant plus an immediate -- the address arithmetic of a swizzled, shifted row cost
// ~5 VALU per MFMA, PMC -- at the price of 2-way bank conflicts on those reads), and G pixels
// of 128 B (swizzle 2 bit1(r) ^ 4 bit3(r), conflict-free).  Slab layout as the ring kernel's.
constexpr int kWsTH = 4, kWsTW = 32, kWsPW = kWsTW + 2;
constexpr int kWsPRows = (kWsTH + 2) * kWsPW;          // 204 halo pixels per phase
constexpr int kWsPPieces = (kWsPRows + 15) / 16;       // 13 one-KiB pieces per phase
constexpr int kWsGPieces = kWsTH * kWsTW * 128 / 1024; // 16 (128-B G rows)

__device__ __forceinline__ int ws_swz128(int r) { return 2 * ((r >> 1) & 1) ^ 4 * ((r >> 3) & 1); }

template <int STRIDE>
__global__ void __launch_bounds__(512) wgrad_halo_kernel(const WgradDev a) {
  constexpr bool S2 = STRIDE == 2;
  constexpr int NPH = S2 ? 4 : 1, KS = S2 ? 5 : 3, NTAP = KS * KS, NPAIR = 2 * NTAP;
  constexpr int SPIECES = NPH * kWsPPieces;             // 52 | 13
  constexpr int BUF = (SPIECES + kWsGPieces) * 1024;
  __shared__ __attribute__((aligned(16))) unsigned char ring[2 * BUF];
  constexpr int NW = 8;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ncb = (a.cin_pad + 31) / 32;
  int cb, nb, split;
  {
    const int nwg = gridDim.x * gridDim.y;
    int t = blockIdx.x + gridDim.x * blockIdx.y;
    const int xcd = t & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (t >> 3);
    const int blk = t % gridDim.x;
    split = t / gridDim.x;
    cb = blk % ncb;
    nb = blk / ncb;
  }
  const int H = a.Hg, W = a.Wg, IH = a.in_h, IW = a.in_w;
  const int pw = W / kWsTW, ppi = pw * (H / kWsTH);
  const int P = a.M / (kWsTH * kWsTW);
  const int pbeg = split * a.m_chunk;
  const int pend = min(pbeg + a.m_chunk, P);
  const bool do_bias = a.bpart && cb == 0;
  const void* const zp = (const void*)g_wgrad_zero;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(wg_lptr_t)ring);

  // ---- DMA: S pieces q = wave + 8 j, G pieces q = wave + 8 j (< 16); the halo geometry is
  // recomputed at each issue (a few VALU per patch) rather than held in registers.  This lane's
  // 8-channel chunk of the block: its source (up to three concatenated) and channel offset.
  constexpr int PSW = (SPIECES + NW - 1) / NW, PGW = kWsGPieces / NW;
  const int nps = (SPIECES - wave + NW - 1) / NW;
  const char* sbase;
  long long sld2;
  bool schan;
  {
    const int ch = cb * 32 + 8 * (lane & 3);
    const void* sp;
    long long ld;
    int cs;
    if (ch < a.send0) { sp = a.sp0; ld = a.sld0; cs = ch; }
    else if (ch < a.send1) { sp = a.sp1; ld = a.sld1; cs = ch - a.send0; }
    else { sp = a.sp2; ld = a.sld2; cs = ch - a.send1; }
    schan = ch < a.send2;
    sbase = reinterpret_cast<const char*>(sp) + (schan ? cs : 0) * 2;
    sld2 = ld * 2;
  }
  const long long ldg2 = a.ldg * 2;
  const char* const gbase = reinterpret_cast<const char*>(a.g);

  auto issue = [&](int p, int buf) {
    const int b = p / ppi, rem = p - b * ppi;
    const int oy0 = (rem / pw) * kWsTH, ox0 = (rem - (rem / pw) * pw) * kWsTW;
    const long long gpix0 = ((long long)b * H + oy0) * W + ox0;
    const long long spix0 = ((long long)b * IH + STRIDE * oy0) * IW + STRIDE * ox0;
    const uint32_t ls = lbase + (uint32_t)(buf * BUF);
    const uint32_t lg = ls + SPIECES * 1024;
#pragma unroll
    for (int j = 0; j < PSW; ++j) {
      if (j < nps) {
        const int q = wave + NW * j;
        const int ph = q / kWsPPieces, pp = q - ph * kWsPPieces;
        const int R = 16 * pp + (lane >> 2);            // row within the phase halo
        const int i = R / kWsPW, jj = R - (R / kWsPW) * kWsPW;
        // source pixel offset from (STRIDE oy0, STRIDE ox0): rows STRIDE (i - 1) + qy, ...
        const int dy = STRIDE * (i - 1) + (ph >> 1), dx = STRIDE * (jj - 1) + (ph & 1);
        const int sy = STRIDE * oy0 + dy, sx = STRIDE * ox0 + dx;
        const bool ok = schan && R < kWsPRows && (unsigned)sy < (unsigned)IH &&
                        (unsigned)sx < (unsigned)IW;
        wg_dma16(ok ? (const void*)(sbase + (spix0 + (long long)dy * IW + dx) * sld2) : zp,
                 ls + (uint32_t)(q * 1024));
      }
    }
#pragma unroll
    for (int j = 0; j < PGW; ++j) {
      const int R = 8 * (wave + NW * j) + (lane >> 3);  // G pixel row of the patch
      const int cg = nb * 64 + 8 * ((lane & 7) ^ ws_swz128(R));
      const bool ok = cg < a.gch;
      wg_dma16(ok ? (const void*)(gbase + (gpix0 + (R >> 5) * W + (R & 31)) * ldg2 + cg * 2) : zp,
               lg + (uint32_t)((wave + NW * j) * 1024));
    }
  };

  // ---- this wave's (tap, channel half) pairs e = wave + 8 i < NPAIR, all 4 n tiles
  constexpr int NPR = (NPAIR + NW - 1) / NW;            // 7 | 3
  const int npr = (NPAIR - wave + NW - 1) / NW;         // wave-uniform
  f32x4 acc[NPR][4];
#pragma unroll
  for (int i = 0; i < NPR; ++i)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc = 0.0f;
  const int fi = lane & 15, fq = lane >> 4, cq = fi & 3;
  const int ra0 = 8 * fq + (fi >> 2);
  int aoff[4];
#pragma unroll
  for (int t = 0; t < 4; ++t)
    aoff[t] = ra0 * 128 + 16 * ((2 * t + (cq >> 1)) ^ ws_swz128(ra0)) + 8 * (cq & 1);
  int boff[NPR];                                         // relative to the S region of buffer 0
#pragma unroll
  for (int i = 0; i < NPR; ++i) {
    const int e = min(wave + NW * i, NPAIR - 1);
    const int tap = e >> 1, u = e & 1;
    const int ky = tap / KS, kx = tap - KS * (tap / KS);
    const int ph = S2 ? 2 * (ky & 1) + (kx & 1) : 0;
    const int sy = S2 ? ky >> 1 : ky, sx = S2 ? kx >> 1 : kx;
    boff[i] = ph * (kWsPPieces * 1024) + (sy * kWsPW + sx + ra0) * 64 +
              16 * (2 * u + (cq >> 1)) + 8 * (cq & 1);
  }
  const uint32_t rbase = (uint32_t)(size_t)(wg_lptr_t)ring;

  if (pbeg < pend) issue(pbeg, 0);
  for (int p = pbeg, it = 0; p < pend; ++p, ++it) {
    const int buf = it & 1;
    if (p + 1 < pend) {
      issue(p + 1, buf ^ 1);
      if (nps == PSW) wg_wait_vm<PSW + PGW>();
      else wg_wait_vm<PSW - 1 + PGW>();
    } else {
      wg_wait_vm<0>();
    }
    __syncthreads();                                     // patch p landed for every wave
    const unsigned char* Gs = ring + buf * BUF + SPIECES * 1024;
    if (do_bias) {                                       // G column sums: 8 row groups x 64
      const int c = tid & 63, rg = tid >> 6;
#pragma unroll 4
      for (int r = 16 * rg; r < 16 * rg + 16; ++r)
        bacc += bf2f(*reinterpret_cast<const uint16_t*>(
            Gs + r * 128 + 16 * ((c >> 3) ^ ws_swz128(r)) + (c & 7) * 2));
    }
    uint32_t bp[NPR];
#pragma unroll
    for (int i = 0; i < NPR; ++i) bp[i] = rbase + (uint32_t)(buf * BUF) + (uint32_t)boff[i];
    const uint32_t gp = rbase + (uint32_t)(buf * BUF + SPIECES * 1024);
#pragma unroll
    for (int yy = 0; yy < kWsTH; ++yy) {
      uint4 A[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const lds_v4s_ptr q = (lds_v4s_ptr)(size_t)(gp + aoff[t] + yy * 32 * 128);
        const v4s a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q);
        const v4s a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q + 4 * 128 / 8);
        const uint2 u0 = __builtin_bit_cast(uint2, a0), u1 = __builtin_bit_cast(uint2, a1);
        A[t] = make_uint4(u0.x, u0.y, u1.x, u1.y);
      }
#pragma unroll
      for (int i = 0; i < NPR; ++i) {
        if (i < npr) {                                   // wave-uniform
          const lds_v4s_ptr q = (lds_v4s_ptr)(size_t)(bp[i] + yy * kWsPW * 64);
          const v4s b0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q);
          const v4s b1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(q + 4 * 64 / 8);
          const uint2 u0 = __builtin_bit_cast(uint2, b0), u1 = __builtin_bit_cast(uint2, b1);
          const uint4 B = make_uint4(u0.x, u0.y, u1.x, u1.y);
#pragma unroll
          for (int t = 0; t < 4; ++t) mma_step<bf16_t>(acc[i][t], A[t], B);
        }
      }
    }
    __syncthreads();                                     // buf free for patch p + 2
  }
  float* Pp = a.part + (size_t)split * a.n_pad * a.k_pad;
#pragma unroll
  for (int i = 0; i < NPR; ++i) {
    const int e = wave + NW * i;
    const int ch = cb * 32 + 16 * (e & 1) + fi;
    if (e < NPAIR && ch < a.cin_pad) {
      const int k = (e >> 1) * a.cin_pad + ch;
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb * 64 + 16 * t + 4 * fq + r;
          if (n < a.gch) Pp[(size_t)n * a.k_pad + k] = acc[i][t][r];
        }
    }
  }
  if (do_bias) {
    float* bred = reinterpret_cast<float*>(ring);        // [8][64], the buffers are free
    bred[tid] = bacc;
    __syncthreads();
    if (tid < 64 && nb * 64 + tid < a.gch) {
      float s = bred[tid];
#pragma unroll
      for (int g2 = 1; g2 < 8; ++g2) s += bred[64 * g2 + tid];
      a.bpart[(size_t)split * a.n_pad + nb * 64 + tid] = s;
    }
  }
}

// Slab reduction in the slab's own (coalesced) order: for slab position e (row n,
// column k of the packed layout), dw[fmap[e]] = sum_s part[s][e] (fmap < 0: a pad
// slot, skipped; every parameter element owns exactly one slot);
// db[j] = sum_s bpart[s][j].  Fixed summation order: deterministic.
__global__ void __launch_bounds__(256)
wgrad_reduce_kernel(long long nslot, const int* __restrict__ fmap, const float* __restrict__ part,
                    int nsplit, long long slab, float* __restrict__ dw, int nbias,
                    const float* __restrict__ bpart, int n_pad, float* __restrict__ db, int acc) {
  const long long total = nslot + nbias;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    if (e < nslot) {
      const int i = fmap[e];
      if (i < 0) continue;
      float s = 0.0f;
      for (int q = 0; q < nsplit; ++q) s += part[q * slab + e];
      dw[i] = acc ? dw[i] + s : s;
    } else {
      const int j = (int)(e - nslot);
      float s = 0.0f;
      for (int q = 0; q < nsplit; ++q) s += bpart[(size_t)q * n_pad + j];
      db[j] = acc ? db[j] + s : s;
    }
  }
}

// Many-split variant (nsplit >= 16: the full-resolution layers split over up to ~200 pixel
// chunks): a block covers 32 slots x 8 split groups; thread (g, slot) sums splits g, g+8, ..
// in order, then thread (0, slot) adds the 8 group sums in order -- still a fixed order
// (deterministic), but 8x the parallelism and 32 coalesced slots per load.
__global__ void __launch_bounds__(256)
wgrad_reduce_wide_kernel(long long nslot, const int* __restrict__ fmap,
                         const float* __restrict__ part, int nsplit, long long slab,
                         float* __restrict__ dw, int nbias, const float* __restrict__ bpart,
                         int n_pad, float* __restrict__ db, int accum) {
  __shared__ float red[8][32];
  const int sl = threadIdx.x & 31, sg = threadIdx.x >> 5;
  const long long e = blockIdx.x * 32ll + sl;
  const long long total = nslot + nbias;
  float acc = 0.0f;
  if (e < total) {
    const bool wslot = e < nslot;
    if (!wslot || fmap[e] >= 0) {
      const float* src = wslot ? part + e : bpart + (e - nslot);
      const long long stride = wslot ? slab : (long long)n_pad;
      // four independent loads in flight per iteration
      int q = sg;
      for (; q + 24 < nsplit; q += 32) {
        const float v0 = src[q * stride], v1 = src[(q + 8) * stride];
        const float v2 = src[(q + 16) * stride], v3 = src[(q + 24) * stride];
        acc += v0; acc += v1; acc += v2; acc += v3;
      }
      for (; q < nsplit; q += 8) acc += src[q * stride];
    }
  }
  red[sg][sl] = acc;
  __syncthreads();
  if (sg == 0 && e < total) {
    float s = red[0][sl];
#pragma unroll
    for (int g = 1; g < 8; ++g) s += red[g][sl];
    if (e < nslot) {
      const int i = fmap[e];
      if (i >= 0) dw[i] = accum ? dw[i] + s : s;
    } else {
      db[e - nslot] = accum ? db[e - nslot] + s : s;
    }
  }
}

// Up to 8 reductions in one launch (rgbac_wgrad_reduce_multi): task t owns blocks
// [blk0[t], blk0[t + 1]); each block is wgrad_reduce_wide_kernel's 32 slots x 8 split groups.
struct ReduceTask {
  long long nslot, slab;
  const int* fmap;
  const float* part;
  float* dw;
  const float* bpart;
  float* db;
  int nsplit, nbias, n_pad, acc;
};
struct ReduceTasks {
  ReduceTask t[8];
  int blk0[9];
  int ntask;
};

__global__ void __launch_bounds__(256) wgrad_reduce_multi_kernel(const ReduceTasks tasks) {
  __shared__ float red[8][32];
  int ti = 0;
  while (ti + 1 < tasks.ntask && (int)blockIdx.x >= tasks.blk0[ti + 1]) ++ti;
  const ReduceTask& k = tasks.t[ti];
  const int sl = threadIdx.x & 31, sg = threadIdx.x >> 5;
  const long long e = (long long)(blockIdx.x - tasks.blk0[ti]) * 32 + sl;
  const long long total = k.nslot + k.nbias;
  float acc = 0.0f;
  if (e < total) {
    const bool wslot = e < k.nslot;
    if (!wslot || k.fmap[e] >= 0) {
      const float* src = wslot ? k.part + e : k.bpart + (e - k.nslot);
      const long long stride = wslot ? k.slab : (long long)k.n_pad;
      int q = sg;
      for (; q + 24 < k.nsplit; q += 32) {
        const float v0 = src[q * stride], v1 = src[(q + 8) * stride];
        const float v2 = src[(q + 16) * stride], v3 = src[(q + 24) * stride];
        acc += v0; acc += v1; acc += v2; acc += v3;
      }
      for (; q < k.nsplit; q += 8) acc += src[q * stride];
    }
  }
  red[sg][sl] = acc;
  __syncthreads();
  if (sg == 0 && e < total) {
    float s = red[0][sl];
#pragma unroll
    for (int g = 1; g < 8; ++g) s += red[g][sl];
    if (e < k.nslot) {
      const int i = k.fmap[e];
      if (i >= 0) k.dw[i] = k.acc ? k.dw[i] + s : s;
    } else {
      k.db[e - k.nslot] = k.acc ? k.db[e - k.nslot] + s : s;
    }
  }
}

// ------------------------------------------------------------------ attention core backward
// Recomputes P = softmax(q k^T * scale + B + M) per window (fp32, same op order
// as the VALU forward), then dV = P^T dO, dP = dO V^T, dS = P (dP - rowsum(P dP)),
// dQ = scale dS K, dK = dS^T (scale Q).  Grid (blocks, heads): block b, head h
// walks window groups g = b, b + gridDim.x, ... accumulating its dS sum (the
// dense bias gradient of head h) in registers -> bpart[b][h][N][N].
template <typename T, int WS>
__global__ void __launch_bounds__(256)
winattn_bwd_kernel(int batch, int H, int W, int C, int heads, int shift, int masked, float scale,
                   const T* __restrict__ qkv, long long ldq, const float* __restrict__ alpha,
                   const float* __restrict__ bias, const T* __restrict__ dout, long long ldo,
                   T* __restrict__ dqkv, long long lddq, float* __restrict__ bpart,
                   const float* __restrict__ amask, int amask_nw) {
  constexpr int N = WS * WS;
  constexpr int NWIN = 64 / N;
  constexpr int DP = 25;
  constexpr int NR = (N == 64) ? 16 : 1;        // dense-bias entries per thread
  __shared__ float qs[64 * DP], ks[64 * DP], vs[64 * DP], gs[64 * DP];
  __shared__ float P[64 * (N + 1)], G[64 * (N + 1)];
  __shared__ float Dsum[64];
  __shared__ int pix_s[64];
  __shared__ int act_s[NWIN];

  const int tid = threadIdx.x;
  const int h = blockIdx.y;
  const int nwx = W / WS, nwy = H / WS;
  const int total = batch * nwx * nwy;
  const int ngroups = (total + NWIN - 1) / NWIN;
  const int d = C / heads;
  float bacc[NR];
#pragma unroll
  for (int r = 0; r < NR; ++r) bacc[r] = 0.0f;

  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    if (tid < NWIN) act_s[tid] = masked ? 0 : 1;
    __syncthreads();
    if (tid < 64) {
      const int wi = tid / N, lt = tid % N;
      const int gw = grp * NWIN + wi;
      int pix = -1;
      if (gw < total) {
        const int b = gw / (nwx * nwy);
        const int rem = gw - b * nwx * nwy;
        const int wy = rem / nwx, wx = rem - (rem / nwx) * nwx;
        const int r = wy * WS + lt / WS, c = wx * WS + lt % WS;
        int oy = r + shift; if (oy >= H) oy -= H;
        int ox = c + shift; if (ox >= W) ox -= W;
        pix = (b * H + oy) * W + ox;
        if (masked && alpha[pix] != 0.0f) act_s[wi] = 1;
      }
      pix_s[tid] = pix;
    }
    __syncthreads();
    // ---- stage q*scale, k, v, dO of head h (zeros for inactive windows / padding)
    for (int e = tid; e < 64 * d; e += 256) {
      const int t = e / d, j = e - t * d;
      const int pix = pix_s[t];
      float q = 0.f, k = 0.f, v = 0.f, g = 0.f;
      if (pix >= 0 && act_s[t / N]) {
        const T* row = qkv + (long long)pix * ldq + h * d + j;
        q = Elem<T>::ld(row) * scale;
        k = Elem<T>::ld(row + C);
        v = Elem<T>::ld(row + 2 * C);
        g = Elem<T>::ld(dout + (long long)pix * ldo + h * d + j);
      }
      qs[t * DP + j] = q;
      ks[t * DP + j] = k;
      vs[t * DP + j] = v;
      gs[t * DP + j] = g;
    }
    __syncthreads();
    // ---- scores (same arithmetic as the forward) and dP = dO V^T: each thread a CB x CB
    // block of (token, key) pairs of one window, so a q-step's 2 CB row / column values feed
    // 2 CB^2 FMAs from registers (one LDS read per FMA in the 1 x 1 form)
    const float* bh = bias + (size_t)h * N * N;
    constexpr int CB = (N == 64) ? 4 : 2;          // 64 x N pairs = 256 threads x CB^2
    constexpr int TPR = N / CB;
    {
      const int i0 = (tid / TPR) * CB, j0 = (tid % TPR) * CB;
      const int wb0 = (i0 / N) * N;
      float sb[CB][CB], db[CB][CB];
#pragma unroll
      for (int r = 0; r < CB; ++r)
#pragma unroll
        for (int c = 0; c < CB; ++c) { sb[r][c] = 0.f; db[r][c] = 0.f; }
      for (int q = 0; q < d; ++q) {
        float qv[CB], gv[CB], kv[CB], vv[CB];
#pragma unroll
        for (int r = 0; r < CB; ++r) {
          qv[r] = qs[(i0 + r) * DP + q];
          gv[r] = gs[(i0 + r) * DP + q];
          kv[r] = ks[(wb0 + j0 + r) * DP + q];
          vv[r] = vs[(wb0 + j0 + r) * DP + q];
        }
#pragma unroll
        for (int r = 0; r < CB; ++r)
#pragma unroll
          for (int c = 0; c < CB; ++c) {
            sb[r][c] = fmaf(qv[r], kv[c], sb[r][c]);
            db[r][c] = fmaf(gv[r], vv[c], db[r][c]);
          }
      }
#pragma unroll
      for (int r = 0; r < CB; ++r)
#pragma unroll
        for (int c = 0; c < CB; ++c) {
      const int i = i0 + r, j = j0 + c;
      const int wbase = wb0;
      const int li = i - wbase;
      float s = sb[r][c];
      const float dp = db[r][c];
      s += bh[li * N + j];
      if (shift > 0) {
        const int wi = i / N;
        const int gw = grp * NWIN + wi;
        const int rem = gw % (nwx * nwy);
        const int wy = rem / nwx, wx = rem % nwx;
        const int ri = wy * WS + li / WS, ci = wx * WS + li % WS;
        const int rj = wy * WS + j / WS, cj = wx * WS + j % WS;
        const int gi = 3 * (ri < H - WS ? 0 : (ri < H - shift ? 1 : 2)) +
                       (ci < W - WS ? 0 : (ci < W - shift ? 1 : 2));
        const int gj = 3 * (rj < H - WS ? 0 : (rj < H - shift ? 1 : 2)) +
                       (cj < W - WS ? 0 : (cj < W - shift ? 1 : 2));
        if (gi != gj) s += -100.0f;
      }
      if (amask) s += amask[((size_t)((grp * NWIN + i / N) % amask_nw) * N + li) * N + j];
      P[i * (N + 1) + j] = s;
      G[i * (N + 1) + j] = dp;
        }
    }
    __syncthreads();
    // ---- softmax rows and D_i = sum_j P dP (4 lanes per row)
    {
      const int i = tid >> 2, part = tid & 3;
      float mx = -INFINITY;
      for (int j = part; j < N; j += 4) mx = fmaxf(mx, P[i * (N + 1) + j]);
      mx = fmaxf(mx, __shfl_xor(mx, 1));
      mx = fmaxf(mx, __shfl_xor(mx, 2));
      float sum = 0.f;
      for (int j = part; j < N; j += 4) {
        const float ex = expf(P[i * (N + 1) + j] - mx);
        P[i * (N + 1) + j] = ex;
        sum += ex;
      }
      sum += __shfl_xor(sum, 1);
      sum += __shfl_xor(sum, 2);
      const float inv = 1.0f / sum;
      float dd = 0.f;
      for (int j = part; j < N; j += 4) {
        const float pv = P[i * (N + 1) + j] * inv;
        P[i * (N + 1) + j] = pv;
        dd = fmaf(pv, G[i * (N + 1) + j], dd);
      }
      dd += __shfl_xor(dd, 1);
      dd += __shfl_xor(dd, 2);
      if (part == 0) Dsum[i] = dd;
    }
    __syncthreads();
    // ---- dS = P (dP - D) in place of dP; dense-bias gradient accumulation
    for (int e = tid; e < 64 * N; e += 256) {
      const int i = e / N, j = e - i * N;
      const float ds = P[i * (N + 1) + j] * (G[i * (N + 1) + j] - Dsum[i]);
      G[i * (N + 1) + j] = act_s[i / N] ? ds : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      if (N == 64) {
        const int e = tid + 256 * r;               // (i, j), one window of 64 tokens
        bacc[r] += G[(e / N) * (N + 1) + (e % N)];
      } else {
        // ws 4: entry (li, j) = tid, summed over the group's NWIN windows
        const int li = tid / N, j = tid % N;
#pragma unroll
        for (int w = 0; w < NWIN; ++w) bacc[r] += G[(w * N + li) * (N + 1) + j];
      }
    }
    // ---- dq, dk, dv at the tokens' original pixels: thread = (token i, a quarter of the head
    // channels); per key j the three dS / P scalars are read once for up to 6 channels
    {
      constexpr int MAXC = 6;                      // d <= 24 (host-checked)
      const int i = tid >> 2, cpt = (d + 3) >> 2, c0 = (tid & 3) * cpt;
      const int wbase = (i / N) * N;
      const int li = i - wbase;
      float dq[MAXC], dk[MAXC], dv[MAXC];
#pragma unroll
      for (int k = 0; k < MAXC; ++k) { dq[k] = 0.f; dk[k] = 0.f; dv[k] = 0.f; }
      for (int j = 0; j < N; ++j) {
        const float gij = G[i * (N + 1) + j];
        const float gji = G[(wbase + j) * (N + 1) + li];
        const float pji = P[(wbase + j) * (N + 1) + li];
        const float* kr = ks + (wbase + j) * DP + c0;
        const float* qr = qs + (wbase + j) * DP + c0;
        const float* gr = gs + (wbase + j) * DP + c0;
#pragma unroll
        for (int k = 0; k < MAXC; ++k)
          if (k < cpt) {
            dq[k] = fmaf(gij, kr[k], dq[k]);
            dk[k] = fmaf(gji, qr[k], dk[k]);
            dv[k] = fmaf(pji, gr[k], dv[k]);
          }
      }
      const int pix = pix_s[i];
      if (pix >= 0) {
        const bool on = act_s[i / N] != 0;
#pragma unroll
        for (int k = 0; k < MAXC; ++k) {
          const int c = c0 + k;
          if (k < cpt && c < d) {
            T* row = dqkv + (long long)pix * lddq + h * d + c;
            Elem<T>::st(row, on ? dq[k] * scale : 0.0f);
            Elem<T>::st(row + C, on ? dk[k] : 0.0f);
            Elem<T>::st(row + 2 * C, on ? dv[k] : 0.0f);
          }
        }
      }
    }
    __syncthreads();
  }
  float* bp = bpart + ((size_t)blockIdx.x * heads + h) * N * N;
#pragma unroll
  for (int r = 0; r < NR; ++r) bp[N == 64 ? tid + 256 * r : tid] = bacc[r];
}

// ------------------------------------------------------------------ attention core backward, MFMA
// The model's two shapes, (ws 8, head dim 24) and (ws 4, head dim 10), with the grid and the
// bias-partial contract of winattn_bwd_kernel.  Per (window group, head h), in LDS:
//   Qs Ks Vs Gs [64][DP]     q*scale, k, v, dO with the token on rows (DP: head dim padded to a
//                            k-step, zeros)
//   QT KT GT    [16 CT][64]  q*scale, k, dO transposed (token index contiguous)
//   PT DT       [64][64]     P and dS with the KEY on rows;  DQ [64][64]: dS, query on rows
// Wave w: S^T = K Q^T and dP^T = V dO^T over query tile w (keys on the MFMA rows, one query per
// lane column -- the softmax and D_i = sum_j P dP row reductions are two lane swaps, as in the
// forward winattn_mfma_kernel); then over token tile w, dQ^T = K^T dS^T, dK^T = (scale Q)^T dS
// and dV^T = dO^T P leave 4 consecutive channels of one token per lane (vector stores).  The
// next group's q/k/v/dO rows are loaded into registers while the current one computes.
// bf16: P and dS enter the last three products rounded to bf16 (fp32 accumulation), like the
// bf16 P of the forward; f32: v_mfma_f32_16x16x4_f32 throughout.
namespace wbwd {
template <typename T, int DH>
struct Lay {
  static constexpr int EPV = Elem<T>::EPV, KSTEP = 4 * EPV;
  static constexpr int DP = (DH + KSTEP - 1) / KSTEP * KSTEP;
  static constexpr int QRS = DP / EPV + 1;      // token-major row stride, 16-B chunks (+1 pad)
  static constexpr int PRS = 64 / EPV + 1;      // 64-column row stride, chunks
  static constexpr int CT = (DH + 15) / 16;     // 16-channel output tiles
  static constexpr int ROWS = 64 * QRS, TRS = CT * 16 * PRS, PS = 64 * PRS;
  static constexpr int QS = 0, KS = ROWS, VS = 2 * ROWS, GS = 3 * ROWS;
  static constexpr int QT = 4 * ROWS, KT = QT + TRS, GT = KT + TRS;
  static constexpr int PT = GT + TRS, DT = PT + PS, DQ = DT + PS;
  static constexpr int CHUNKS = DQ + PS;
  static constexpr int BYTES = CHUNKS * 16 + (64 + 64 + 4) * 4;   // + pix_s, rid_s, act_s
};
template <int V> struct Raw;
template <> struct Raw<16> { using type = uint4; };
template <> struct Raw<8> { using type = uint2; };
template <> struct Raw<4> { using type = uint32_t; };
__device__ __forceinline__ float max16_f(float v) {             // max(v, v(lane ^ 16))
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float max32_f(float v) {             // max(v, v(lane ^ 32))
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
}  // namespace wbwd

template <typename T, int WS, int DH>
__global__ void __launch_bounds__(256)
winattn_bwd_mfma_kernel(int batch, int H, int W, int C, int heads, int shift, int masked,
                        float scale, const T* __restrict__ qkv, long long ldq,
                        const float* __restrict__ alpha, const float* __restrict__ bias,
                        const T* __restrict__ dout, long long ldo, T* __restrict__ dqkv,
                        long long lddq, float* __restrict__ bpart,
                        const float* __restrict__ amask, int amask_nw) {
  using Ly = wbwd::Lay<T, DH>;
  constexpr int N = WS * WS, NWIN = 64 / N;
  constexpr int EPV = Ly::EPV, KSTEP = Ly::KSTEP, DP = Ly::DP, QRS = Ly::QRS, PRS = Ly::PRS;
  constexpr int CT = Ly::CT;
  constexpr int ROWB = DH * (int)sizeof(T);
  constexpr int VEC = (ROWB % 16 == 0) ? 16 : (ROWB % 8 == 0 ? 8 : 4);
  constexpr int NP = ROWB / VEC, EV = VEC / (int)sizeof(T);
  constexpr int NPIECE = 4 * 64 * NP;           // q, k, v, dO rows of 64 tokens
  constexpr int PPT = (NPIECE + 255) / 256;
  constexpr int KT = (WS == 8) ? 4 : 1;         // key tiles per query tile
  using RawT = typename wbwd::Raw<VEC>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  uint4* const c16 = reinterpret_cast<uint4*>(sm);
  T* const el = reinterpret_cast<T*>(sm);       // element view (chunk c = el + c * EPV)
  int* const pix_s = reinterpret_cast<int*>(sm + Ly::CHUNKS * 16);
  int* const rid_s = pix_s + 64;
  int* const act_s = rid_s + 64;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int h = blockIdx.y;
  const int nwx = W / WS, nwy = H / WS;
  const int total = batch * nwx * nwy;
  const int ngroups = (total + NWIN - 1) / NWIN;

  // token t of window group grp -> pixel (-1 past the last window), shifted-frame region id
  auto tok_pix = [&](int grp, int t, int& rid) -> int {
    const int gw = grp * NWIN + t / N, lt = t % N;
    rid = 0;
    if (gw >= total) return -1;
    const int b = gw / (nwx * nwy);
    const int rem = gw - b * nwx * nwy;
    const int wy = rem / nwx, wx = rem - wy * nwx;
    const int r = wy * WS + lt / WS, c = wx * WS + lt % WS;
    rid = 3 * (r < H - WS ? 0 : (r < H - shift ? 1 : 2)) + (c < W - WS ? 0 : (c < W - shift ? 1 : 2));
    int oy = r + shift; if (oy >= H) oy -= H;
    int ox = c + shift; if (ox >= W) ox -= W;
    return (b * H + oy) * W + ox;
  };
  RawT raw[PPT];
  auto load_group = [&](int grp) {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + 256 * i;
      raw[i] = RawT{};
      if (NPIECE % 256 == 0 || e < NPIECE) {
        const int which = e / (64 * NP), rem = e - which * 64 * NP;
        const int t = rem / NP, pc = rem - t * NP;
        int rid;
        const int pix = tok_pix(grp, t, rid);
        if (pix >= 0) {
          const T* src = which < 3 ? qkv + (long long)pix * ldq + which * C + h * DH + pc * EV
                                   : dout + (long long)pix * ldo + h * DH + pc * EV;
          raw[i] = *reinterpret_cast<const RawT*>(src);
        }
      }
    }
  };

  // zero what the staging never writes but the MFMAs read: chunks past the head dim, the
  // transposed rows past it, and for ws 4 the off-window entries of PT / DT / DQ
  {
    constexpr int C0 = DH / EPV, C1 = DP / EPV;
    for (int e = tid; e < 4 * 64 * (C1 - C0); e += 256) {
      const int a = e / (64 * (C1 - C0)), r = e - a * 64 * (C1 - C0);
      c16[a * Ly::ROWS + (r / (C1 - C0)) * QRS + C0 + r % (C1 - C0)] = make_uint4(0, 0, 0, 0);
    }
    constexpr int TZ = (CT * 16 - DH) * PRS;
    for (int e = tid; e < 3 * TZ; e += 256)
      c16[Ly::QT + (e / TZ) * Ly::TRS + DH * PRS + e % TZ] = make_uint4(0, 0, 0, 0);
    if constexpr (WS == 4)
      for (int e = tid; e < 3 * Ly::PS; e += 256) c16[Ly::PT + e] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  const int qi = wave * 16 + fr;                // this lane's query (S^T column) / output token
  const int qloc = qi % N;
  float bias_r[KT][4], bacc[KT][4];
  {
    const float* bh = bias + (size_t)h * N * N;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int ktile = (WS == 8) ? kt : wave;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bias_r[kt][r] = bh[qloc * N + (ktile * 16 + fq * 4 + r) % N];
        bacc[kt][r] = 0.0f;
      }
    }
  }
  if (blockIdx.x < ngroups) load_group(blockIdx.x);

  for (int grp = blockIdx.x; grp < ngroups; grp += gridDim.x) {
    // ---- window bookkeeping (wave 0): pixels, region ids, active windows by ballot
    if (tid < 64) {
      int rid;
      const int pix = tok_pix(grp, tid, rid);
      const bool a = pix >= 0 && (!masked || alpha[pix] != 0.0f);
      const unsigned long long bal = __ballot(a);
      pix_s[tid] = pix;
      rid_s[tid] = rid;
      const unsigned long long wmask = (N == 64) ? ~0ull : (((1ull << N) - 1) << (tid / N * N));
      if (tid % N == 0) act_s[tid / N] = (bal & wmask) != 0;
    }
    // ---- stage this group's rows (q scaled) and the transposed copies
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + 256 * i;
      if (NPIECE % 256 == 0 || e < NPIECE) {
        const int which = e / (64 * NP), rem = e - which * 64 * NP;
        const int t = rem / NP, pc = rem - t * NP;
        const T* v = reinterpret_cast<const T*>(&raw[i]);
        T* row = el + (which * Ly::ROWS + t * QRS) * EPV + pc * EV;
        if (which == 0) {
#pragma unroll
          for (int q = 0; q < EV; ++q) Elem<T>::st(row + q, Elem<T>::ld(v + q) * scale);
        } else {
          *reinterpret_cast<RawT*>(row) = raw[i];
        }
        if (which != 2) {
          const int tb = which == 0 ? Ly::QT : (which == 1 ? Ly::KT : Ly::GT);
          T* tr = el + (tb + (pc * EV) * PRS) * EPV + t;
#pragma unroll
          for (int q = 0; q < EV; ++q)
            Elem<T>::st(tr + q * PRS * EPV, which == 0 ? Elem<T>::ld(v + q) * scale : Elem<T>::ld(v + q));
        }
      }
    }
    __syncthreads();
    if (grp + (int)gridDim.x < ngroups) load_group(grp + gridDim.x);

    // ---- S^T, dP^T over this wave's query tile; softmax; D_i; dS
    const int qwin = qi / N;
    const bool qact = act_s[qwin] != 0;
    const int qrid = rid_s[qi];
    const float* qmask = amask ? amask + ((size_t)((grp * NWIN + qwin) % amask_nw) * N + qloc) * N
                               : nullptr;
    f32x4 s[KT], g[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int ktile = (WS == 8) ? kt : wave;
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
      g[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < DP / KSTEP; ++ks) {
        const int kr = (ktile * 16 + fr) * QRS + 4 * ks + fq, qr = qi * QRS + 4 * ks + fq;
        mma_step<T>(s[kt], c16[Ly::KS + kr], c16[Ly::QS + qr]);
        mma_step<T>(g[kt], c16[Ly::VS + kr], c16[Ly::GS + qr]);
      }
    }
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int ktile = (WS == 8) ? kt : wave;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kj = ktile * 16 + fq * 4 + r;
        float v = s[kt][r] + bias_r[kt][r];
        if (shift > 0 && rid_s[kj] != qrid) v += -100.0f;
        if (qmask) v += qmask[kj % N];
        s[kt][r] = v;
        mx = fmaxf(mx, v);
      }
    }
    mx = wbwd::max32_f(wbwd::max16_f(mx));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ex = expf(s[kt][r] - mx);
        s[kt][r] = ex;
        sum += ex;
      }
    sum = sum32_f(sum16_f(sum));
    const float inv = 1.0f / sum;
    float dd = 0.f;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s[kt][r] *= inv;
        dd = fmaf(s[kt][r], g[kt][r], dd);
      }
    dd = sum32_f(sum16_f(dd));
    T* const pt = el + Ly::PT * EPV;
    T* const dt = el + Ly::DT * EPV;
    T* const dq = el + Ly::DQ * EPV;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int ktile = (WS == 8) ? kt : wave;
      float ds[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        ds[r] = qact ? s[kt][r] * (g[kt][r] - dd) : 0.0f;
        bacc[kt][r] += ds[r];
        const int kj = ktile * 16 + fq * 4 + r;
        Elem<T>::st(pt + kj * PRS * EPV + qi, s[kt][r]);
        Elem<T>::st(dt + kj * PRS * EPV + qi, ds[r]);
      }
      Elem<T>::st4(dq + qi * PRS * EPV + ktile * 16 + fq * 4, ds);
    }
    __syncthreads();

    // ---- dQ^T, dK^T, dV^T over token tile `wave` (= this lane's qi)
    const int pix = pix_s[qi];
    const bool on = act_s[qwin] != 0;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      f32x4 oq = f32x4{0.f, 0.f, 0.f, 0.f}, ok = oq, ov = oq;
#pragma unroll
      for (int ks = 0; ks < 64 / KSTEP; ++ks) {
        const int tr = (ct * 16 + fr) * PRS + 4 * ks + fq, pr = qi * PRS + 4 * ks + fq;
        mma_step<T>(oq, c16[Ly::KT + tr], c16[Ly::DQ + pr]);
        mma_step<T>(ok, c16[Ly::QT + tr], c16[Ly::DT + pr]);
        mma_step<T>(ov, c16[Ly::GT + tr], c16[Ly::PT + pr]);
      }
      const int c0 = ct * 16 + fq * 4;
      if (pix >= 0 && c0 < DH) {
        float vq[4], vk[4], vv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          vq[r] = on ? oq[r] * scale : 0.0f;
          vk[r] = on ? ok[r] : 0.0f;
          vv[r] = on ? ov[r] : 0.0f;
        }
        T* dst = dqkv + (long long)pix * lddq + h * DH + c0;
        if constexpr (DH % 4 == 0) {
          Elem<T>::st4(dst, vq);
          Elem<T>::st4(dst + C, vk);
          Elem<T>::st4(dst + 2 * C, vv);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c0 + r < DH) {
              Elem<T>::st(dst + r, vq[r]);
              Elem<T>::st(dst + C + r, vk[r]);
              Elem<T>::st(dst + 2 * C + r, vv[r]);
            }
        }
      }
    }
    __syncthreads();
  }

  // ---- dense-bias gradient partial of (block, head): entry (query-local i, key-local j)
  float* bp = bpart + ((size_t)blockIdx.x * heads + h) * N * N;
  if constexpr (WS == 8) {
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
      *reinterpret_cast<float4*>(bp + qi * N + kt * 16 + fq * 4) =
          make_float4(bacc[kt][0], bacc[kt][1], bacc[kt][2], bacc[kt][3]);
  } else {
    // ws 4: wave w held window w of each group; sum the four waves' (i, j) entries
    float* red = reinterpret_cast<float*>(sm);
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave * 256 + fr * N + fq * 4 + r] = bacc[0][r];
    __syncthreads();
    bp[tid] = red[tid] + red[256 + tid] + red[512 + tid] + red[768 + tid];
  }
}

// dtable[e][h] = sum over blocks and (i, j) with index[i][j] == e of bpart[blk][h][i][j]
__global__ void __launch_bounds__(256)
relpos_reduce_kernel(int nblk, int heads, int N, const float* __restrict__ bpart,
                     float* __restrict__ dense) {
  const int total = heads * N * N;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    float s = 0.0f;
    for (int b = 0; b < nblk; ++b) s += bpart[(size_t)b * total + e];
    dense[e] = s;
  }
}
__global__ void __launch_bounds__(256)
relpos_scatter_kernel(int ntab, int heads, int N, const int* __restrict__ csr_off,
                      const int* __restrict__ csr_ij, const float* __restrict__ dense,
                      float* __restrict__ dtable) {
  const int total = ntab * heads;
  for (int e = blockIdx.x * 256 + threadIdx.x; e < total; e += gridDim.x * 256) {
    const int t = e / heads, h = e - t * heads;
    float s = 0.0f;
    for (int q = csr_off[t]; q < csr_off[t + 1]; ++q) s += dense[(size_t)h * N * N + csr_ij[q]];
    dtable[e] = s;
  }
}

// ------------------------------------------------------------------ Gaussian conditional
// Forward (per element): x = y + noise (training) | round(y-mu)+mu; v = |x - mu|;
// s = LB(sigma, .11); lik = LB(Phi((.5-v)/s) - Phi((-.5-v)/s), 1e-9);
// bits = clamp(-log(lik+1e-10)/ln2, 0, 50); hat = ste_round(y - mu) + mu.
// Backward with g = dL/dbits (device scalar) and dhat = dL/dhat:
//   dy = dhat + g * dbits/dy (training only), dmu = -g * dbits/dv sign(x-mu)
//   (training only; dhat/dmu = 0), dsigma through compressai's LowerBound rule.
template <typename T>
__global__ void __launch_bounds__(256)
gaussian_bwd_kernel(long long n, int nch, const T* __restrict__ y, long long ldy,
                    const T* __restrict__ mu, long long ldmu, const T* __restrict__ sc,
                    long long lds, const float* __restrict__ noise, const float* __restrict__ gbits,
                    const T* __restrict__ dhat, long long lddh, T* __restrict__ dy, long long lddy,
                    T* __restrict__ dmu, long long lddmu, T* __restrict__ dsc, long long lddsc) {
  const float gb = *gbits;
  const double rn = 1.0 / nch;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    int ch;
    const long long pix = ediv(e, nch, rn, ch);
    const float yv = Elem<T>::ld(y + pix * ldy + ch);
    const float mv = Elem<T>::ld(mu + pix * ldmu + ch);
    const float sv = Elem<T>::ld(sc + pix * lds + ch);
    const float xin = noise ? yv + noise[e] : rintf(yv - mv) + mv;
    const float val = xin - mv;
    const float v = fabsf(val);
    const float s = fmaxf(sv, 0.11f);
    const float ta = (0.5f - v) / s, tb = (-0.5f - v) / s;
    const float lraw = t_cdf(ta) - t_cdf(tb);
    const float lik = fmaxf(lraw, 1e-9f);
    const float braw = (-1.0f * logf(lik + 1e-10f)) / 0.69314718055994530942f;
    float gl = (braw >= 0.0f && braw <= 50.0f) ? gb * (-1.0f / ((lik + 1e-10f) * 0.69314718055994530942f)) : 0.0f;
    if (!(lraw >= 1e-9f || gl < 0.0f)) gl = 0.0f;                // likelihood LowerBound
    const float pa = t_phi(ta), pb = t_phi(tb);
    const float gv = gl * (pb - pa) / s;
    float gs = gl * (tb * pb - ta * pa) / s;
    if (!(sv >= 0.11f || gs < 0.0f)) gs = 0.0f;                  // scale LowerBound
    const float sg = val > 0.0f ? 1.0f : (val < 0.0f ? -1.0f : 0.0f);
    const float gval = noise ? gv * sg : 0.0f;
    const float dh = dhat ? Elem<T>::ld(dhat + pix * lddh + ch) : 0.0f;
    Elem<T>::st(dy + pix * lddy + ch, gval + dh);
    Elem<T>::st(dmu + pix * lddmu + ch, -gval);
    Elem<T>::st(dsc + pix * lddsc + ch, gs);
  }
}

// ------------------------------------------------------------------ EntropyBottleneck
// One block per channel.  Per element: x = z + noise (training) | round(z-med)+med;
// lik = LB(sigmoid(l(x+.5)) - sigmoid(l(x-.5)), 1e-9), l = the factorized MLP
// over the packed param block (entropy.hip layout); bits as above.  Gradients are
// w.r.t. the PACKED values (softplus(matrix), bias, tanh(factor)) in the same
// [C][64] positions (the host chains them to the raw parameters); [58] = median
// (quantiles[:, 0, 1]) in eval mode.
struct EbCache { float x; float a[4][3]; float t[4][3]; };

__device__ __forceinline__ float eb_fwd_cache(const float* P, float x, EbCache& c) {
  c.x = x;
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    float a = P[0 + o] * x;
    a = a + P[33 + o];
    c.a[0][o] = a;
    c.t[0][o] = a + P[46 + o] * tanhf(a);
  }
#pragma unroll
  for (int layer = 1; layer < 4; ++layer) {
    const float* Mx = P + 3 + 9 * (layer - 1);
    const float* bx = P + 36 + 3 * (layer - 1);
    const float* fx = P + 49 + 3 * (layer - 1);
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      float a = Mx[o * 3 + 0] * c.t[layer - 1][0];
      a = fmaf(Mx[o * 3 + 1], c.t[layer - 1][1], a);
      a = fmaf(Mx[o * 3 + 2], c.t[layer - 1][2], a);
      a = a + bx[o];
      c.a[layer][o] = a;
      c.t[layer][o] = a + fx[o] * tanhf(a);
    }
  }
  float a = P[30] * c.t[3][0];
  a = fmaf(P[31], c.t[3][1], a);
  a = fmaf(P[32], c.t[3][2], a);
  return a + P[45];
}

// accumulate d(params) (packed positions, w.r.t. sp(M), b, tanh(f)) for dL/dlogit = g; returns dL/dx
__device__ __forceinline__ float eb_bwd_acc(const float* P, const EbCache& c, float g, float* gp) {
  float dt[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    gp[30 + i] += g * c.t[3][i];
    dt[i] = g * P[30 + i];
  }
  gp[45] += g;
#pragma unroll
  for (int layer = 3; layer >= 1; --layer) {
    const float* Mx = P + 3 + 9 * (layer - 1);
    const float* fx = P + 49 + 3 * (layer - 1);
    float da[3];
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      const float th = tanhf(c.a[layer][o]);
      gp[49 + 3 * (layer - 1) + o] += dt[o] * th;
      da[o] = dt[o] * (1.0f + fx[o] * (1.0f - th * th));
      gp[36 + 3 * (layer - 1) + o] += da[o];
#pragma unroll
      for (int i = 0; i < 3; ++i) gp[3 + 9 * (layer - 1) + o * 3 + i] += da[o] * c.t[layer - 1][i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) dt[i] = da[0] * Mx[0 * 3 + i] + da[1] * Mx[1 * 3 + i] + da[2] * Mx[2 * 3 + i];
  }
  float dx = 0.0f;
#pragma unroll
  for (int o = 0; o < 3; ++o) {
    const float th = tanhf(c.a[0][o]);
    gp[46 + o] += dt[o] * th;
    const float da = dt[o] * (1.0f + P[46 + o] * (1.0f - th * th));
    gp[33 + o] += da;
    gp[0 + o] += da * c.x;
    dx += da * P[0 + o];
  }
  return dx;
}

template <typename T>
__global__ void __launch_bounds__(256)
eb_bwd_kernel(long long npix, int C, const T* __restrict__ z, long long ldz,
              const float* __restrict__ params, const float* __restrict__ noise,
              const float* __restrict__ gbits, const T* __restrict__ dzhat, long long lddh,
              T* __restrict__ dz, long long lddz, float* __restrict__ dparams) {
  __shared__ float red[4][60];
  const int ch = blockIdx.x;
  const float* P = params + (size_t)ch * 64;
  const float gb = *gbits;
  float gp[59];
#pragma unroll
  for (int i = 0; i < 59; ++i) gp[i] = 0.0f;
  for (long long pix = threadIdx.x; pix < npix; pix += 256) {
    const long long e = pix * C + ch;
    const float med = P[58];
    const float zv = Elem<T>::ld(z + pix * ldz + ch);
    const float xin = noise ? zv + noise[e] : rintf(zv - med) + med;
    EbCache cl, cu;
    const float lo = eb_fwd_cache(P, xin - 0.5f, cl);
    const float up = eb_fwd_cache(P, xin + 0.5f, cu);
    const float su = t_sigmoid(up), sl = t_sigmoid(lo);
    const float lraw = su - sl;
    const float lik = fmaxf(lraw, 1e-9f);
    const float braw = (-1.0f * logf(lik + 1e-10f)) / 0.69314718055994530942f;
    float gl = (braw >= 0.0f && braw <= 50.0f) ? gb * (-1.0f / ((lik + 1e-10f) * 0.69314718055994530942f)) : 0.0f;
    if (!(lraw >= 1e-9f || gl < 0.0f)) gl = 0.0f;
    const float gu = gl * su * (1.0f - su);
    const float glo = -gl * sl * (1.0f - sl);
    float dx = eb_bwd_acc(P, cu, gu, gp);
    dx += eb_bwd_acc(P, cl, glo, gp);
    float dzv = dzhat ? Elem<T>::ld(dzhat + pix * lddh + ch) : 0.0f;
    if (noise) dzv += dx;
    else gp[58] += dx;                        // dequantize: d x / d median = 1
    Elem<T>::st(dz + pix * lddz + ch, dzv);
  }
  // block reduction of the 59 parameter gradients
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 59; ++i) {
    float v = gp[i];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[wave][i] = v;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    float v = 0.0f;
    if (i < 59) v = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    dparams[(size_t)ch * 64 + i] = v;
  }
}

// ------------------------------------------------------------------ reconstruct_error backward
// mode 0 (AutoEncoderRGB_Journal.py:36-64): mse = mean_b sum_c,p (m x - m xh)^2 / max(cnt_b, 1)
//   -> dxh = g * 2 m (m xh - m x) / (B max(cnt_b, 1)); cnt_b from the forward's partials.
// mode 1 (AutoEncoderMask_Journal.py:309): mse = mean (xh - x)^2 -> dxh = g * 2 (xh - x) / count.
template <typename T>
__global__ void __launch_bounds__(256)
mse_bwd_kernel(int mode, int batch, int cx, int HW, int nblk, const float* __restrict__ x,
               const T* __restrict__ xh, long long ldh, const float* __restrict__ mask,
               const double* __restrict__ part, const float* __restrict__ gmse, T* __restrict__ dxh,
               long long lddx) {
  const int b = blockIdx.y;
  __shared__ float scale_s;
  if (threadIdx.x == 0) {
    double cnt = 0.0;
    if (mode == 0) {
      for (int i = 0; i < nblk; ++i) cnt += part[((size_t)b * nblk + i) * 2 + 1];
      scale_s = *gmse * 2.0f / ((float)batch * fmaxf((float)cnt, 1.0f));
    } else {
      scale_s = *gmse * 2.0f / ((float)batch * (float)cx * (float)HW);
    }
  }
  __syncthreads();
  const float sc = scale_s;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
    const long long pix = (long long)b * HW + p;
    const float m = mode == 0 ? (mask[pix] > 0.0f ? 1.0f : 0.0f) : 1.0f;
    for (int c = 0; c < (int)lddx; ++c) {
      float g = 0.0f;
      if (c < cx) {
        const float xv = x[((long long)b * cx + c) * HW + p];
        const float hv = Elem<T>::ld(xh + pix * ldh + c);
        g = mode == 0 ? sc * m * (hv * m - xv * m) : sc * (hv - xv);
      }
      Elem<T>::st(dxh + pix * lddx + c, g);
    }
  }
}

// ------------------------------------------------------------------ optimizer
// trainRGB.py:190-198: grad.clamp_(-clip, clip) then torch.optim.Adam (no weight
// decay, no amsgrad): m = lerp(m, g, 1-b1); v = b2 v + (1-b2) g^2;
// p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps), step_size = lr / bc1.
__global__ void __launch_bounds__(256)
adam_clamp_kernel(long long n, float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                  float* __restrict__ v, float w1, float b2, float w2, float bc2_sqrt, float eps,
                  float step_size, float clip, float gscale) {
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    float gv = g[e];
    if (gscale != 1.0f) gv *= gscale;             // data-parallel mean (after the all-reduce sum)
    if (clip > 0.0f) gv = fminf(fmaxf(gv, -clip), clip);
    g[e] = gv;
    const float mv = m[e] + w1 * (gv - m[e]);
    const float vv = v[e] * b2 + w2 * (gv * gv);
    m[e] = mv;
    v[e] = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    p[e] = p[e] + (-step_size) * (mv / denom);
  }
}

// The same with the step count in device memory (graph-replayable training step): every
// thread forms torch.optim.Adam's scalars from step = *step_dev + 1 in double exactly as the
// host entry does; step_advance_kernel then stores the new count.
__global__ void __launch_bounds__(256)
adam_clamp_dstep_kernel(long long n, float* __restrict__ p, float* __restrict__ g,
                        float* __restrict__ m, float* __restrict__ v, const long long* step_dev,
                        double lr, double beta1, double beta2, double eps, float clip,
                        float gscale) {
  const double step = (double)(*step_dev + 1);
  const double bc1 = 1.0 - pow(beta1, step);
  const double bc2 = 1.0 - pow(beta2, step);
  const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, w2 = (float)(1.0 - beta2);
  const float bc2_sqrt = (float)sqrt(bc2), epsf = (float)eps, step_size = (float)(lr / bc1);
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    float gv = g[e];
    if (gscale != 1.0f) gv *= gscale;
    if (clip > 0.0f) gv = fminf(fmaxf(gv, -clip), clip);
    g[e] = gv;
    const float mv = m[e] + w1 * (gv - m[e]);
    const float vv = v[e] * b2 + w2 * (gv * gv);
    m[e] = mv;
    v[e] = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + epsf;
    p[e] = p[e] + (-step_size) * (mv / denom);
  }
}

__global__ void step_advance_kernel(long long* step_dev) {
  if (threadIdx.x == 0) *step_dev += 1;
}

// ------------------------------------------------------------------ layout helpers
// dir 0: shuffle   in (B,H,W,4C) -> out (B,2H,2W,C), out[2y+i][2x+j][c] = in[y][x][4c+2i+j]
// dir 1: unshuffle in (B,2H,2W,C) -> out (B,H,W,4C)
template <typename T>
__global__ void __launch_bounds__(256)
pixel_shuffle_kernel(int dir, int batch, int H, int W, int C, const T* __restrict__ in,
                     long long ldi, T* __restrict__ out, long long ldo) {
  const long long n = (long long)batch * H * W * 4 * C;
  const double r4c = 1.0 / (4 * C), rw = 1.0 / W, rh = 1.0 / H;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    int cc, x, y;
    const long long pix = ediv(e, 4 * C, r4c, cc);
    const long long t = ediv(pix, W, rw, x);
    const int b = (int)ediv(t, H, rh, y);
    const int c = cc >> 2, i = (cc >> 1) & 1, j = cc & 1;
    const long long lo = pix * (dir == 0 ? ldi : ldo) + cc;
    const long long hi = ((long long)(b * 2 * H + 2 * y + i) * (2 * W) + 2 * x + j) * (dir == 0 ? ldo : ldi) + c;
    if (dir == 0) Elem<T>::st(out + hi, Elem<T>::ld(in + lo));
    else Elem<T>::st(out + lo, Elem<T>::ld(in + hi));
  }
}

// dst[p][dcoff + c] = src[p][scoff + c] for c < C   (channel concat / split)
template <typename T>
__global__ void __launch_bounds__(256)
channel_copy_kernel(long long npix, int C, const T* __restrict__ src, long long lds, int scoff,
                    T* __restrict__ dst, long long ldd, int dcoff) {
  const long long n = npix * C;
  const double rc = 1.0 / C;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    int c;
    const long long p = ediv(e, C, rc, c);
    dst[p * ldd + dcoff + c] = src[p * lds + scoff + c];
  }
}

// Up to 16 channel copies over the same pixel count in one launch (a concatenation's parts,
// or a split's gradient pieces; 5 us of launch each when issued one by one, ~236 per training
// step).  Task t = blockIdx.y; 16-byte vectors when every channel count, offset and row
// stride of the task is a multiple of 16 bytes.
struct CopyTask {
  const void* src;
  void* dst;
  long long lds, ldd;                           // row strides, elements
  int scoff, dcoff, C, vec, acc;                // acc: dst += src (one rounding)
};
struct CopyTasks { CopyTask t[16]; };

template <typename T>
__global__ void __launch_bounds__(256)
channel_copy_multi_kernel(long long npix, CopyTasks tasks) {
  const CopyTask k = tasks.t[blockIdx.y];
  if (k.vec) {
    constexpr int E = 16 / (int)sizeof(T);
    const int cv = k.C / E;
    const long long n = npix * cv;
    const double rc = 1.0 / cv;
    for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
      int c;
      const long long p = ediv(e, cv, rc, c);
      uint4* d = reinterpret_cast<uint4*>(static_cast<T*>(k.dst) + p * k.ldd + k.dcoff + c * E);
      uint4 v = *reinterpret_cast<const uint4*>(static_cast<const T*>(k.src) + p * k.lds + k.scoff + c * E);
      if (k.acc) {
        const uint4 o = *d;
        if constexpr (sizeof(T) == 2) {
          const uint32_t a[4] = {o.x, o.y, o.z, o.w}, b[4] = {v.x, v.y, v.z, v.w};
          uint32_t r[4];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            r[q] = pack_bf16x2(bf2f(a[q] & 0xFFFF) + bf2f(b[q] & 0xFFFF),
                               bf2f(a[q] >> 16) + bf2f(b[q] >> 16));
          v = make_uint4(r[0], r[1], r[2], r[3]);
        } else {
          v = make_uint4(__float_as_uint(__uint_as_float(o.x) + __uint_as_float(v.x)),
                         __float_as_uint(__uint_as_float(o.y) + __uint_as_float(v.y)),
                         __float_as_uint(__uint_as_float(o.z) + __uint_as_float(v.z)),
                         __float_as_uint(__uint_as_float(o.w) + __uint_as_float(v.w)));
        }
      }
      *d = v;
    }
  } else {
    const long long n = npix * k.C;
    const double rc = 1.0 / k.C;
    for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
      int c;
      const long long p = ediv(e, k.C, rc, c);
      T* d = static_cast<T*>(k.dst) + p * k.ldd + k.dcoff + c;
      const T s = static_cast<const T*>(k.src)[p * k.lds + k.scoff + c];
      if (k.acc) {
        if constexpr (sizeof(T) == 2)
          *d = (T)f2bf(bf2f(*d) + bf2f(s));
        else
          *d = *d + s;
      } else {
        *d = s;
      }
    }
  }
}

// ------------------------------------------------------------------ small helpers
// packed[i] = idx[i] >= 0 ? (T) src[idx[i]] : 0   (weight repack through a cached map)
template <typename T>
__global__ void __launch_bounds__(256)
gather_kernel(long long n, const float* __restrict__ src, const int* __restrict__ idx,
              T* __restrict__ dst) {
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
    const int j = idx[e];
    Elem<T>::st(dst + e, j >= 0 ? src[j] : 0.0f);
  }
}

// Many gathers in one launch (the per-step repack of every layer's forward and
// input-gradient weights): task t = {src, idx, dst, n, dtype} as 5 int64 in device memory,
// blocks [blk0[t], blk0[t+1]) cover its elements, 2048 per block; a block finds its task by
// binary search over blk0.
constexpr int kGatherChunk = 2048;
constexpr long long kGatherCopy16 = 16;   // task dtype: 16-byte chunk copy (rgbac.h)
// the bf16 path covers a block's chunk as 256 threads x 8 elements
static_assert(kGatherChunk == 256 * 8, "gather_multi_kernel: bf16 chunk = 256 threads x 8");
__global__ void __launch_bounds__(256)
gather_multi_kernel(int ntask, const long long* __restrict__ tasks,
                    const long long* __restrict__ blk0) {
  const long long b = blockIdx.x;
  int lo = 0, hi = ntask - 1;
  while (lo < hi) {                       // last t with blk0[t] <= b
    const int mid = (lo + hi + 1) >> 1;
    if (blk0[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const long long* tk = tasks + 5 * lo;
  const float* src = reinterpret_cast<const float*>(tk[0]);
  const int* idx = reinterpret_cast<const int*>(tk[1]);
  const long long n = tk[3];
  const long long e0 = (b - blk0[lo]) * kGatherChunk;
  if (tk[4] == kGatherCopy16) {
    // 16-byte chunk copy through a chunk map: the fragment-major training packs are a
    // permutation of 8-element runs of the plain pack written by the previous launch (L2 /
    // MALL-hot bf16 rows), not a second element gather from the fp32 parameter
    const uint4* s4 = reinterpret_cast<const uint4*>(tk[0]);
    uint4* d4 = reinterpret_cast<uint4*>(tk[2]);
#pragma unroll
    for (int r = 0; r < kGatherChunk / 256; ++r) {
      const long long e = e0 + r * 256 + threadIdx.x;
      if (e < n) { const int j = idx[e]; d4[e] = j >= 0 ? s4[j] : make_uint4(0, 0, 0, 0); }
    }
    return;
  }
  if (tk[4] == RGBAC_F32) {
    float* dst = reinterpret_cast<float*>(tk[2]);
#pragma unroll
    for (int r = 0; r < kGatherChunk / 256; ++r) {
      const long long e = e0 + r * 256 + threadIdx.x;
      if (e < n) { const int j = idx[e]; dst[e] = j >= 0 ? src[j] : 0.0f; }
    }
  } else {
    bf16_t* dst = reinterpret_cast<bf16_t*>(tk[2]);
    // 8 consecutive elements per thread: two 16-byte index loads, 8 gathers, one 16-byte
    // store (the element-per-lane form issued 3 memory instructions per element); the
    // task's tail chunk (or a misaligned buffer) takes the per-element path
    const long long e = e0 + threadIdx.x * 8;
    const bool vec = ((reinterpret_cast<uintptr_t>(idx) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
    if (vec && e + 8 <= n) {
      const int4 i0 = *reinterpret_cast<const int4*>(idx + e);
      const int4 i1 = *reinterpret_cast<const int4*>(idx + e + 4);
      const int j[8] = {i0.x, i0.y, i0.z, i0.w, i1.x, i1.y, i1.z, i1.w};
      float v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) v[r] = j[r] >= 0 ? src[j[r]] : 0.0f;
      *reinterpret_cast<uint4*>(dst + e) = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                                                      pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        if (e + r < n) {
          const int jj = idx[e + r];
          Elem<bf16_t>::st(dst + e + r, jj >= 0 ? src[jj] : 0.0f);
        }
    }
  }
}

// The per-step repack of the bf16 training packs as strided 8-element chunks: every 16-byte
// chunk of a pack is 1..8 consecutive elements of ONE run of the fp32 parameter with a fixed
// per-pack stride (a tap's input channels of a conv row, a tap's output channels of an
// input-gradient row, ...), so the map holds one int32 per chunk instead of one per element
// (index traffic / 8), and the chunk also goes straight to its slot of the fragment-major copy
// (no second launch re-reading the plain pack).  Task t = 8 int64 {src, cmap, dst, nchunk,
// stride, fmap, fdst, 0}; cmap[c] < 0: a zero chunk, else base = bits 0..27, valid elements - 1
// = bits 28..30; fmap[c] >= 0: the fragment-major chunk it also fills.  A block owns 256
// chunks, one per thread: every chunk's map load -> gathers -> stores chain in its own lane
// (eight chunks per thread in a loop serialised eight such chains: 1.5x slower).
constexpr int kRepackChunks = 256;
__global__ void __launch_bounds__(256)
repack_multi_kernel(int ntask, const long long* __restrict__ tasks,
                    const long long* __restrict__ blk0) {
  const long long b = blockIdx.x;
  int lo = 0, hi = ntask - 1;
  while (lo < hi) {                       // last t with blk0[t] <= b
    const int mid = (lo + hi + 1) >> 1;
    if (blk0[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const long long* tk = tasks + 8 * lo;
  const float* src = reinterpret_cast<const float*>(tk[0]);
  const int* cmap = reinterpret_cast<const int*>(tk[1]);
  uint4* dst = reinterpret_cast<uint4*>(tk[2]);
  const long long n = tk[3];
  const long long stride = tk[4];
  const int* fmap = reinterpret_cast<const int*>(tk[5]);
  uint4* fdst = reinterpret_cast<uint4*>(tk[6]);
  const long long c = (b - blk0[lo]) * kRepackChunks + threadIdx.x;
  if (c < n) {
    const int m = cmap[c];
    const int f = fmap ? fmap[c] : -1;               // (issued with the map load)
    float v[8];
    if (m >= 0) {
      const long long base = m & 0x0FFFFFFF;
      const int nv = ((m >> 28) & 7) + 1;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = j < nv ? src[base + j * stride] : 0.0f;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = 0.0f;
    }
    const uint4 q = make_uint4(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]),
                               pack_bf16x2(v[4], v[5]), pack_bf16x2(v[6], v[7]));
    dst[c] = q;
    if (f >= 0) fdst[f] = q;
  }
}

// partial[blk][c] = sum over the block's pixels of x[p][c]   (bias gradients)
template <typename T>
__global__ void __launch_bounds__(256)
colsum_kernel(long long npix, int C, const T* __restrict__ x, long long ldx, long long chunk,
              float* __restrict__ partial) {
  const long long p0 = blockIdx.x * chunk;
  long long p1 = p0 + chunk;
  if (p1 > npix) p1 = npix;
  for (int c = threadIdx.x; c < C; c += 256) {
    float s = 0.0f;
    for (long long p = p0; p < p1; ++p) s += Elem<T>::ld(x + p * ldx + c);
    partial[(size_t)blockIdx.x * C + c] = s;
  }
}

// out[i] = (float) sum_j part[i][j] over n fp64 partials per row (fixed order)
__global__ void __launch_bounds__(256)
sum_rows_kernel(int rows, int n, const double* __restrict__ part, float* __restrict__ out) {
  __shared__ double red[4];
  for (int r = 0; r < rows; ++r) {
    double s = 0.0;
    for (int j = threadIdx.x; j < n; j += 256) s += part[(size_t)r * n + j];
    s = block_sum_f64(s, red);
    if (threadIdx.x == 0) out[r] = (float)s;
  }
}

static int grid_for(long long n) {
  long long g = (n + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace rgbac

using namespace rgbac;

#define RGBAC_DT_DISPATCH(dtype, KERNEL, ...)                                    \
  do {                                                                           \
    if ((dtype) == RGBAC_F32) { KERNEL(float, __VA_ARGS__); }                    \
    else { KERNEL(bf16_t, __VA_ARGS__); }                                        \
  } while (0)

extern "C" int rgbac_act_bwd(int dtype, int act, float act_param, int64_t npix, int channels,
                             const void* dy, int64_t ldy, const void* z, int64_t ldz,
                             const void* res1, int64_t ld1, const uint8_t* sel, void* dz,
                             int64_t lddz, void* dres1, int64_t lddr1, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(act >= RGBAC_ACT_NONE && act <= RGBAC_ACT_MASKSEL, "act has no backward here");
  RGBAC_REQUIRE(npix >= 0 && channels > 0 && lddz >= channels && ldy >= channels, "shape");
  RGBAC_REQUIRE(lddz % 4 == 0 && ldy % 4 == 0 && (!z || ldz % 4 == 0) && (!res1 || ld1 % 4 == 0) &&
                    (!dres1 || (lddr1 % 4 == 0 && lddr1 == lddz)), "leading dims must be multiples of 4");
  RGBAC_REQUIRE(dy && dz, "null pointer");
  RGBAC_REQUIRE(act == RGBAC_ACT_NONE || act == RGBAC_ACT_MASKSEL || z, "act needs z");
  RGBAC_REQUIRE(!(act == RGBAC_ACT_GATE || act == RGBAC_ACT_GDN || act == RGBAC_ACT_IGDN) || res1,
                "act needs res1");
  RGBAC_REQUIRE(act != RGBAC_ACT_MASKSEL || sel, "MASKSEL needs sel");
  if (npix == 0) return RGBAC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int g = grid_for(npix * lddz / 4);
  // bf16: the fast GELU derivative (RGBAC_GELU_BWD_EXACT=1 keeps erfcf, A/B)
  static const bool exact = [] {
    const char* e = getenv("RGBAC_GELU_BWD_EXACT");
    return e && e[0] == '1';
  }();
#define K_(T, F)                                                                              \
  hipLaunchKernelGGL((act_bwd_kernel<T, F>), dim3(g), dim3(256), 0, st, act, act_param, npix,   \
                     channels, (const T*)dy, ldy, (const T*)z, ldz, (const T*)res1, ld1, sel,   \
                     (T*)dz, lddz, (T*)dres1, lddr1)
  static const bool no_flat = [] {
    const char* e = getenv("RGBAC_ACT_BWD_FLAT");
    return e && e[0] == '0';
  }();
  auto al16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
  const bool flat = !no_flat && dtype == RGBAC_BF16 && !sel && z && channels == lddz &&
                    ldy == lddz && ldz == lddz && (!res1 || ld1 == lddz) &&
                    (npix * lddz) % 8 == 0 && al16(dy) && al16(z) && al16(dz) &&
                    (!res1 || al16(res1)) && (!dres1 || al16(dres1));
  if (flat) {
    const long long n8 = npix * lddz / 8;
#define F_(F)                                                                                  \
  hipLaunchKernelGGL((act_bwd_flat_kernel<F>), dim3(grid_for(n8)), dim3(256), 0, st, act,       \
                     act_param, n8, (const uint4*)dy, (const uint4*)z, (const uint4*)res1,      \
                     (uint4*)dz, (uint4*)dres1)
    if (exact) F_(false); else F_(true);
#undef F_
    return check_launch("act_bwd_flat_kernel");
  }
  if (dtype == RGBAC_F32) K_(float, false);
  else if (exact) K_(bf16_t, false);
  else K_(bf16_t, true);
#undef K_
  return check_launch("act_bwd_kernel");
}

// RGBAC_WGRAD_BIG=0: keep the 64 x 128 tile on the wide shapes (A/B switch)
static bool wgrad_big_enabled() {
  static const bool on = [] {
    const char* e = getenv("RGBAC_WGRAD_BIG");
    return !(e && e[0] == '0');
  }();
  return on;
}

// The patch kernel's shapes (rgbac.autograd.wgrad_tile mirrors this rule to size the split):
// bf16, 3x3 stride 1 pad 1, one source of whole 32-channel blocks, <= 32 output channels,
// the grid 8-row x 32-column patches of the input grid.  RGBAC_WGRAD_PATCH=0 turns it off.
static bool wgrad_patch_ok(const rgbac_wgrad_args* a) {
  static const bool on = [] {
    const char* e = getenv("RGBAC_WGRAD_PATCH");
    return !(e && e[0] == '0');
  }();
  return on && a->dtype == RGBAC_BF16 && !a->square_input && a->ksize == 3 && a->stride == 1 &&
         a->pad == 1 && a->nsrc == 1 && a->g_channels <= 32 && a->cin_pad % 32 == 0 &&
         a->grid_w % kWpTW == 0 && a->grid_h % kWpTH == 0 && a->in_h == a->grid_h &&
         a->in_w == a->grid_w;
}

// The halo kernel's shapes (mirrored by rgbac.autograd.wgrad_halo_ok): bf16, no squared input,
// 5x5 stride 2 pad 2, or 3x3 stride 1 pad 1 with more than 32 outputs; the output grid 4-row x
// 32-column patches of the input grid (of half of it, stride 2).  RGBAC_WGRAD_HALO=0 turns
// it off (RGBAC_WGRAD_S2=0: the stride-2 shapes only).  Returns the stride, 0 = not eligible.
static int wgrad_halo_ok(const rgbac_wgrad_args* a) {
  static const bool on = [] {
    const char* e = getenv("RGBAC_WGRAD_HALO");
    return !(e && e[0] == '0');
  }();
  static const bool on2 = [] {
    const char* e = getenv("RGBAC_WGRAD_S2");
    return !(e && e[0] == '0');
  }();
  if (!on || a->dtype != RGBAC_BF16 || a->square_input || a->grid_w % kWsTW != 0 ||
      a->grid_h % kWsTH != 0)
    return 0;
  if (on2 && a->ksize == 5 && a->stride == 2 && a->pad == 2 && a->in_h == 2 * a->grid_h &&
      a->in_w == 2 * a->grid_w)
    return 2;
  if (a->ksize == 3 && a->stride == 1 && a->pad == 1 && a->g_channels > 32 &&
      a->in_h == a->grid_h && a->in_w == a->grid_w)
    return 1;
  return 0;
}

extern "C" int rgbac_conv_wgrad(const rgbac_wgrad_args* a, void* stream) {
  RGBAC_REQUIRE(a != nullptr, "null args");
  RGBAC_REQUIRE(a->dtype == RGBAC_F32 || a->dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(a->batch > 0 && a->grid_h > 0 && a->grid_w > 0, "grid");
  RGBAC_REQUIRE(a->g && a->partial, "null pointer");
  RGBAC_REQUIRE(a->g_ldc % 8 == 0 && a->g_channels > 0 && a->g_channels <= a->g_ldc &&
                    a->g_channels % 8 == 0, "g channels must be a multiple of 8 within g_ldc");
  RGBAC_REQUIRE(a->ksize >= 1 && a->ksize <= 5 && a->stride >= 1 && a->stride <= 2 &&
                    a->pad >= 0 && a->pad < a->ksize, "kernel geometry");
  RGBAC_REQUIRE(a->nsrc >= 1 && a->nsrc <= 3, "nsrc must be 1..3");
  RGBAC_REQUIRE(a->n_pad % 64 == 0 && a->n_pad >= a->g_channels, "n_pad");
  int csum = 0;
  for (int i = 0; i < a->nsrc; ++i) {
    RGBAC_REQUIRE(a->src[i].ptr && a->src[i].channels % 8 == 0 && a->src[i].channels > 0 &&
                      a->src[i].ldc % 8 == 0 && a->src[i].ldc >= a->src[i].channels,
                  "bad source");
    RGBAC_REQUIRE(((uintptr_t)a->src[i].ptr) % 16 == 0, "source pointers must be 16-byte aligned");
    csum += a->src[i].channels;
  }
  RGBAC_REQUIRE(csum == a->cin_pad, "sum of source channels must equal cin_pad");
  const int K = a->ksize * a->ksize * a->cin_pad;
  RGBAC_REQUIRE(a->k_pad % 64 == 0 && a->k_pad >= K, "k_pad");
  RGBAC_REQUIRE(a->nsplit >= 1 && a->nsplit <= 4096, "nsplit");
  const long long M = (long long)a->batch * a->grid_h * a->grid_w;
  RGBAC_REQUIRE(M < (1ll << 31), "too many pixels");
  WgradDev d{};
  d.g = a->g; d.ldg = a->g_ldc; d.gch = a->g_channels;
  d.sp0 = a->src[0].ptr; d.sld0 = a->src[0].ldc; d.send0 = a->src[0].channels;
  d.sp1 = a->nsrc > 1 ? a->src[1].ptr : d.sp0;
  d.sld1 = a->nsrc > 1 ? a->src[1].ldc : d.sld0;
  d.send1 = d.send0 + (a->nsrc > 1 ? a->src[1].channels : 0);
  d.sp2 = a->nsrc > 2 ? a->src[2].ptr : d.sp1;
  d.sld2 = a->nsrc > 2 ? a->src[2].ldc : d.sld1;
  d.send2 = d.send1 + (a->nsrc > 2 ? a->src[2].channels : 0);
  d.cin_pad = a->cin_pad; d.K = K; d.k_pad = a->k_pad; d.n_pad = a->n_pad;
  d.M = (int)M; d.Hg = a->grid_h; d.Wg = a->grid_w;
  d.in_h = a->in_h; d.in_w = a->in_w; d.ksize = a->ksize; d.stride = a->stride; d.pad = a->pad;
  d.square = a->square_input;
  d.m_chunk = (int)(((M + a->nsplit - 1) / a->nsplit + 63) / 64 * 64);
  d.rWg = 1.0 / a->grid_w;
  d.rHg = 1.0 / a->grid_h;
  d.part = a->partial;
  d.bpart = a->bias_partial;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // 64 x 128 tiles when K is wide (8 MFMAs per k-step per wave on 12 transposed reads);
  // 128 x 256 tiles (512 threads) when N and K are both wide (rgbac.autograd.wgrad_tile mirrors
  // this rule to size the pixel split)
  const bool wide = a->dtype == RGBAC_BF16 && a->k_pad >= 512;
  const bool big = wide && !a->square_input && a->n_pad >= 128 && wgrad_big_enabled();
  dim3 grid(wide ? (a->k_pad + 127) / 128 : a->k_pad / 64, a->n_pad / 64, a->nsplit);
  if (big) grid = dim3((a->k_pad + 255) / 256, (a->n_pad + 127) / 128, a->nsplit);
  // bf16 without the squared input: the LDS-DMA ring kernel (RGBAC_WGRAD_RING=0: the
  // register-staged kernel, A/B switch)
  static const bool ring_env = [] {
    const char* e = getenv("RGBAC_WGRAD_RING");
    return !(e && e[0] == '0');
  }();
  if (const int hs = wgrad_halo_ok(a)) {
    // 4 x 32-pixel patches of the output grid; nsplit workgroups per (32-channel source block,
    // 64-channel output block)
    const long long P = M / (kWsTH * kWsTW);
    d.m_chunk = (int)((P + a->nsplit - 1) / a->nsplit);
    const dim3 sgrid(((a->cin_pad + 31) / 32) * ((a->g_channels + 63) / 64), a->nsplit);
    if (hs == 2) hipLaunchKernelGGL(wgrad_halo_kernel<2>, sgrid, dim3(512), 0, st, d);
    else hipLaunchKernelGGL(wgrad_halo_kernel<1>, sgrid, dim3(512), 0, st, d);
    return check_launch("wgrad_halo_kernel");
  }
  if (wgrad_patch_ok(a)) {
    // patches of 8 x 32 output pixels; nsplit workgroups per 32-channel source block
    const long long P = M / (kWpTH * kWpTW);
    d.m_chunk = (int)((P + a->nsplit - 1) / a->nsplit);
    const dim3 pgrid(a->cin_pad / 32, a->nsplit);
    if (a->g_channels > 16)
      hipLaunchKernelGGL((wgrad_patch_kernel<2>), pgrid, dim3(256), 0, st, d);
    else
      hipLaunchKernelGGL((wgrad_patch_kernel<1>), pgrid, dim3(256), 0, st, d);
    return check_launch("wgrad_patch_kernel");
  }
  if (a->dtype == RGBAC_BF16 && !a->square_input && ring_env) {
    // (128 x 128 tiles, wgrad_ring_kernel<4, 4, 3>: one workgroup per CU -- measured no faster
    // on the slice-stack shapes and -4 % on the training step, so not dispatched)
    if (big) {
      hipLaunchKernelGGL((wgrad_ring_kernel<4, 4, 3, 2, 4>), grid, dim3(512), 0, st, d);
    } else if (wide) {
      hipLaunchKernelGGL((wgrad_ring_kernel<2, 4, 3>), grid, dim3(256), 0, st, d);
    } else {
      hipLaunchKernelGGL((wgrad_ring_kernel<2, 2, 4>), grid, dim3(256), 0, st, d);
    }
    return check_launch("wgrad_ring_kernel");
  }
  if (a->dtype == RGBAC_F32)
    hipLaunchKernelGGL((wgrad_kernel<float, 2>), grid, dim3(256), 0, st, d);
  else if (wide)
    hipLaunchKernelGGL((wgrad_kernel<bf16_t, 4>), grid, dim3(256), 0, st, d);
  else
    hipLaunchKernelGGL((wgrad_kernel<bf16_t, 2>), grid, dim3(256), 0, st, d);
  return check_launch("wgrad_kernel");
}

extern "C" int rgbac_wgrad_reduce(int64_t nslot, const int32_t* fmap, const float* partial,
                                  int nsplit, int64_t slab, float* dw, int nbias,
                                  const float* bias_partial, int n_pad, float* db, int accumulate,
                                  void* stream) {
  RGBAC_REQUIRE(nslot >= 0 && nsplit >= 1 && slab > 0 && nslot <= slab, "shape");
  RGBAC_REQUIRE((nslot == 0 || (fmap && partial && dw)) && (nbias == 0 || (bias_partial && db)),
                "null pointer");
  RGBAC_REQUIRE(nbias <= n_pad, "nbias > n_pad");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (nsplit >= 16) {
    const long long nblk = (nslot + nbias + 31) / 32;
    if (nblk == 0) return RGBAC_OK;
    hipLaunchKernelGGL(wgrad_reduce_wide_kernel, dim3((unsigned)nblk), dim3(256), 0, st, nslot,
                       fmap, partial, nsplit, slab, dw, nbias, bias_partial, n_pad, db, accumulate);
    return check_launch("wgrad_reduce_wide_kernel");
  }
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(grid_for(nslot + nbias)), dim3(256), 0, st, nslot,
                     fmap, partial, nsplit, slab, dw, nbias, bias_partial, n_pad, db, accumulate);
  return check_launch("wgrad_reduce_kernel");
}

extern "C" int rgbac_wgrad_reduce_multi(int ntasks, const int64_t* tasks, void* stream) {
  RGBAC_REQUIRE(ntasks >= 1 && ntasks <= 8 && tasks, "1..8 tasks");
  ReduceTasks tk{};
  tk.ntask = ntasks;
  tk.blk0[0] = 0;
  for (int i = 0; i < ntasks; ++i) {
    const int64_t* d = tasks + 11 * i;
    ReduceTask& k = tk.t[i];
    k.nslot = d[0];
    k.fmap = reinterpret_cast<const int*>(d[1]);
    k.part = reinterpret_cast<const float*>(d[2]);
    k.nsplit = (int)d[3];
    k.slab = d[4];
    k.dw = reinterpret_cast<float*>(d[5]);
    k.nbias = (int)d[6];
    k.bpart = reinterpret_cast<const float*>(d[7]);
    k.n_pad = (int)d[8];
    k.db = reinterpret_cast<float*>(d[9]);
    k.acc = (int)d[10];
    RGBAC_REQUIRE(k.nslot >= 0 && k.nsplit >= 1 && k.slab > 0 && k.nslot <= k.slab, "shape");
    RGBAC_REQUIRE((k.nslot == 0 || (k.fmap && k.part && k.dw)) &&
                      (k.nbias == 0 || (k.bpart && k.db)), "null pointer");
    RGBAC_REQUIRE(k.nbias <= k.n_pad, "nbias > n_pad");
    const long long nb = (k.nslot + k.nbias + 31) / 32;
    RGBAC_REQUIRE(tk.blk0[i] + nb < (1ll << 31), "too many blocks");
    tk.blk0[i + 1] = tk.blk0[i] + (int)nb;
  }
  if (tk.blk0[ntasks] == 0) return RGBAC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(wgrad_reduce_multi_kernel, dim3((unsigned)tk.blk0[ntasks]), dim3(256), 0, st, tk);
  return check_launch("wgrad_reduce_multi_kernel");
}

template <typename T, int WS, int DH>
static void launch_attn_bwd_mfma(dim3 grid, hipStream_t st, int batch, int h, int w, int channels,
                                 int heads, int shift, int masked, float scale, const void* qkv,
                                 int64_t ldq, const float* alpha, const float* bias,
                                 const void* dout, int64_t ldo, void* dqkv, int64_t lddq,
                                 float* bias_partial, const float* amask, int amask_nw) {
  constexpr int bytes = wbwd::Lay<T, DH>::BYTES;
  static unsigned long long attr = 0;             // > 64 KiB of dynamic LDS for f32; per device
  lds_optin(reinterpret_cast<const void*>(winattn_bwd_mfma_kernel<T, WS, DH>), bytes, &attr);
  hipLaunchKernelGGL((winattn_bwd_mfma_kernel<T, WS, DH>), grid, dim3(256), bytes, st, batch, h, w,
                     channels, heads, shift, masked, scale, (const T*)qkv, ldq, alpha, bias,
                     (const T*)dout, ldo, (T*)dqkv, lddq, bias_partial, amask, amask_nw);
}

extern "C" int rgbac_winattn_core_bwd_ex(int dtype, int batch, int h, int w, int channels,
                                         int heads, int ws, int shift, int masked, float scale,
                                         const void* qkv, int64_t ldq, const float* alpha,
                                         const float* bias, const void* dout, int64_t ldo,
                                         void* dqkv, int64_t lddq, int nblk, float* bias_partial,
                                         const float* amask, int amask_nw, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(ws == 4 || ws == 8, "window size must be 4 or 8");
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && h % ws == 0 && w % ws == 0, "shape");
  RGBAC_REQUIRE(heads > 0 && channels % heads == 0 && channels / heads <= 24, "head dim");
  RGBAC_REQUIRE(shift >= 0 && shift < ws, "shift");
  RGBAC_REQUIRE(qkv && dout && dqkv && bias && bias_partial, "null pointer");
  RGBAC_REQUIRE(!masked || alpha, "masked attention needs alpha");
  RGBAC_REQUIRE(nblk >= 1 && nblk <= 65535, "nblk");
  RGBAC_REQUIRE(!amask || amask_nw > 0, "an explicit mask needs nW > 0");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(nblk, heads);
  // MFMA path for the model's two shapes (as the forward's winattn_mfma_kernel);
  // RGBAC_ATTN_BWD_VALU=1 keeps the VALU kernel (A/B)
  static const bool force_valu = [] {
    const char* e = getenv("RGBAC_ATTN_BWD_VALU");
    return e && e[0] == '1';
  }();
  const int dh = channels / heads;
  // the MFMA kernel moves q/k/v, dO and dQKV rows in vectors of up to 16 bytes: it needs
  // 16-byte aligned bases and row strides; any other layout takes the VALU kernel (scalar
  // accesses, any stride)
  const int64_t esz = dtype == RGBAC_F32 ? 4 : 2;
  const bool vec_ok =
      ((reinterpret_cast<uintptr_t>(qkv) | reinterpret_cast<uintptr_t>(dout) |
        reinterpret_cast<uintptr_t>(dqkv)) & 15) == 0 &&
      (ldq * esz) % 16 == 0 && (ldo * esz) % 16 == 0 && (lddq * esz) % 16 == 0;
  if (!force_valu && vec_ok && ((ws == 8 && dh == 24) || (ws == 4 && dh == 10))) {
    if (dtype == RGBAC_F32) {
      if (ws == 8) launch_attn_bwd_mfma<float, 8, 24>(grid, st, batch, h, w, channels, heads, shift, masked, scale, qkv, ldq, alpha, bias, dout, ldo, dqkv, lddq, bias_partial, amask, amask_nw);
      else launch_attn_bwd_mfma<float, 4, 10>(grid, st, batch, h, w, channels, heads, shift, masked, scale, qkv, ldq, alpha, bias, dout, ldo, dqkv, lddq, bias_partial, amask, amask_nw);
    } else {
      if (ws == 8) launch_attn_bwd_mfma<bf16_t, 8, 24>(grid, st, batch, h, w, channels, heads, shift, masked, scale, qkv, ldq, alpha, bias, dout, ldo, dqkv, lddq, bias_partial, amask, amask_nw);
      else launch_attn_bwd_mfma<bf16_t, 4, 10>(grid, st, batch, h, w, channels, heads, shift, masked, scale, qkv, ldq, alpha, bias, dout, ldo, dqkv, lddq, bias_partial, amask, amask_nw);
    }
    return check_launch("winattn_bwd_mfma_kernel");
  }
#define K_(T, WS_)                                                                              \
  hipLaunchKernelGGL((winattn_bwd_kernel<T, WS_>), grid, dim3(256), 0, st, batch, h, w, channels, \
                     heads, shift, masked, scale, (const T*)qkv, ldq, alpha, bias,                \
                     (const T*)dout, ldo, (T*)dqkv, lddq, bias_partial, amask, amask_nw)
  if (ws == 8) { RGBAC_DT_DISPATCH(dtype, K_, 8); }
  else { RGBAC_DT_DISPATCH(dtype, K_, 4); }
#undef K_
  return check_launch("winattn_bwd_kernel");
}

extern "C" int rgbac_winattn_core_bwd(int dtype, int batch, int h, int w, int channels, int heads,
                                      int ws, int shift, int masked, float scale, const void* qkv,
                                      int64_t ldq, const float* alpha, const float* bias,
                                      const void* dout, int64_t ldo, void* dqkv, int64_t lddq,
                                      int nblk, float* bias_partial, void* stream) {
  return rgbac_winattn_core_bwd_ex(dtype, batch, h, w, channels, heads, ws, shift, masked, scale,
                                   qkv, ldq, alpha, bias, dout, ldo, dqkv, lddq, nblk, bias_partial,
                                   nullptr, 0, stream);
}

extern "C" int rgbac_relpos_bwd(int nblk, int heads, int ws, const float* bias_partial,
                                const int32_t* csr_off, const int32_t* csr_ij, float* dense,
                                float* dtable, void* stream) {
  RGBAC_REQUIRE(ws == 4 || ws == 8, "window size");
  RGBAC_REQUIRE(nblk >= 1 && heads > 0 && bias_partial && csr_off && csr_ij && dense && dtable,
                "args");
  const int N = ws * ws;
  const int ntab = (2 * ws - 1) * (2 * ws - 1);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(relpos_reduce_kernel, dim3(grid_for((long long)heads * N * N)), dim3(256), 0,
                     st, nblk, heads, N, bias_partial, dense);
  int rc = check_launch("relpos_reduce_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(relpos_scatter_kernel, dim3(grid_for((long long)ntab * heads)), dim3(256), 0,
                     st, ntab, heads, N, csr_off, csr_ij, dense, dtable);
  return check_launch("relpos_scatter_kernel");
}

extern "C" int rgbac_gaussian_bwd(int dtype, int64_t npix, int nch, const void* y, int64_t ldy,
                                  const void* mu, int64_t ldmu, const void* scale, int64_t lds,
                                  const float* noise, const float* gbits, const void* dhat,
                                  int64_t lddh, void* dy, int64_t lddy, void* dmu, int64_t lddmu,
                                  void* dscale, int64_t lddsc, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(npix > 0 && nch > 0, "empty slice");
  RGBAC_REQUIRE(y && mu && scale && gbits && dy && dmu && dscale, "null pointer");
  const long long n = npix * (long long)nch;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define K_(T, ...)                                                                              \
  hipLaunchKernelGGL(gaussian_bwd_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, n, nch,      \
                     (const T*)y, ldy, (const T*)mu, ldmu, (const T*)scale, lds, noise, gbits,  \
                     (const T*)dhat, lddh, (T*)dy, lddy, (T*)dmu, lddmu, (T*)dscale, lddsc)
  RGBAC_DT_DISPATCH(dtype, K_, 0);
#undef K_
  return check_launch("gaussian_bwd_kernel");
}

extern "C" int rgbac_eb_bwd(int dtype, int64_t npix, int channels, const void* z, int64_t ldz,
                            const float* params, const float* noise, const float* gbits,
                            const void* dzhat, int64_t lddh, void* dz, int64_t lddz,
                            float* dparams, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(npix > 0 && channels > 0, "empty tensor");
  RGBAC_REQUIRE(z && params && gbits && dz && dparams, "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define K_(T, ...)                                                                              \
  hipLaunchKernelGGL(eb_bwd_kernel<T>, dim3(channels), dim3(256), 0, st, npix, channels,        \
                     (const T*)z, ldz, params, noise, gbits, (const T*)dzhat, lddh, (T*)dz, lddz, \
                     dparams)
  RGBAC_DT_DISPATCH(dtype, K_, 0);
#undef K_
  return check_launch("eb_bwd_kernel");
}

extern "C" int rgbac_mse_bwd(int dtype, int mode, int batch, int cx, int h, int w, const float* x,
                             const void* x_hat, int64_t ldh, const float* mask,
                             const double* scratch, const float* gmse, void* dx_hat, int64_t lddx,
                             void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(mode == 0 || mode == 1, "mode");
  RGBAC_REQUIRE(batch > 0 && cx > 0 && h > 0 && w > 0 && lddx >= cx, "shape");
  RGBAC_REQUIRE(x && x_hat && gmse && dx_hat && (mode == 1 || (mask && scratch)), "null pointer");
  const int nblk = rgbac_finalize_blocks(h, w);   // the forward's scratch layout
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  dim3 grid(64, batch);
#define K_(T, ...)                                                                              \
  hipLaunchKernelGGL(mse_bwd_kernel<T>, grid, dim3(256), 0, st, mode, batch, cx, h * w, nblk, x,   \
                     (const T*)x_hat, ldh, mask, scratch, gmse, (T*)dx_hat, lddx)
  RGBAC_DT_DISPATCH(dtype, K_, 0);
#undef K_
  return check_launch("mse_bwd_kernel");
}

extern "C" int rgbac_adam_clamp(int64_t n, float* param, float* grad, float* exp_avg,
                                float* exp_avg_sq, double lr, double beta1, double beta2,
                                double eps, int64_t step, float clip, float grad_scale,
                                void* stream) {
  RGBAC_REQUIRE(n >= 0 && step >= 1, "shape/step");
  RGBAC_REQUIRE(n == 0 || (param && grad && exp_avg && exp_avg_sq), "null pointer");
  if (n == 0) return RGBAC_OK;
  // scalars exactly as torch.optim.Adam forms them (python doubles, applied in fp32)
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(adam_clamp_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, param, grad,
                     exp_avg, exp_avg_sq, (float)(1.0 - beta1), (float)beta2,
                     (float)(1.0 - beta2), (float)std::sqrt(bc2), (float)eps,
                     (float)(lr / bc1), clip, grad_scale);
  return check_launch("adam_clamp_kernel");
}

extern "C" int rgbac_adam_clamp_dstep(int64_t n, float* param, float* grad, float* exp_avg,
                                      float* exp_avg_sq, double lr, double beta1, double beta2,
                                      double eps, int64_t* step_dev, float clip, float grad_scale,
                                      void* stream) {
  RGBAC_REQUIRE(n >= 0 && step_dev, "shape/step");
  RGBAC_REQUIRE(n == 0 || (param && grad && exp_avg && exp_avg_sq), "null pointer");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (n > 0) {
    hipLaunchKernelGGL(adam_clamp_dstep_kernel, dim3(grid_for(n)), dim3(256), 0, st, n, param,
                       grad, exp_avg, exp_avg_sq, reinterpret_cast<const long long*>(step_dev),
                       lr, beta1, beta2, eps, clip, grad_scale);
    int rc = check_launch("adam_clamp_dstep_kernel");
    if (rc) return rc;
  }
  hipLaunchKernelGGL(step_advance_kernel, dim3(1), dim3(64), 0, st,
                     reinterpret_cast<long long*>(step_dev));
  return check_launch("step_advance_kernel");
}

extern "C" int rgbac_pixel_shuffle(int dtype, int dir, int batch, int h, int w, int c,
                                   const void* in, int64_t ldi, void* out, int64_t ldo,
                                   void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(dir == 0 || dir == 1, "dir");
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && c > 0 && in && out, "shape");
  RGBAC_REQUIRE(dir == 0 ? (ldi >= 4 * c && ldo >= c) : (ldi >= c && ldo >= 4 * c), "strides");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long long n = (long long)batch * h * w * 4 * c;
#define K_(T, ...)                                                                              \
  hipLaunchKernelGGL(pixel_shuffle_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, dir, batch, h, \
                     w, c, (const T*)in, ldi, (T*)out, ldo)
  RGBAC_DT_DISPATCH(dtype, K_, 0);
#undef K_
  return check_launch("pixel_shuffle_kernel");
}

extern "C" int rgbac_channel_copy(int dtype, int64_t npix, int channels, const void* src,
                                  int64_t lds, int scoff, void* dst, int64_t ldd, int dcoff,
                                  void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(npix >= 0 && channels > 0 && src && dst, "shape");
  RGBAC_REQUIRE(scoff + channels <= lds && dcoff + channels <= ldd, "channel range");
  if (npix == 0) return RGBAC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const long long n = npix * channels;
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(channel_copy_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, npix,
                       channels, (const float*)src, lds, scoff, (float*)dst, ldd, dcoff);
  else
    hipLaunchKernelGGL(channel_copy_kernel<uint16_t>, dim3(grid_for(n)), dim3(256), 0, st, npix,
                       channels, (const uint16_t*)src, lds, scoff, (uint16_t*)dst, ldd, dcoff);
  return check_launch("channel_copy_kernel");
}

static int copy_multi(int dtype, int64_t npix, int ntasks, const int64_t* desc, int nfield,
                      void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(npix >= 0 && ntasks >= 1 && ntasks <= 16 && desc, "shape");
  if (npix == 0) return RGBAC_OK;
  const int es = dtype == RGBAC_F32 ? 4 : 2, epv = 16 / es;
  CopyTasks tk;
  long long maxc = 0;
  for (int i = 0; i < ntasks; ++i) {
    const int64_t* d = desc + nfield * i;     // src, lds, scoff, channels, dst, ldd, dcoff[, acc]
    CopyTask& k = tk.t[i];
    k.acc = nfield > 7 ? (int)d[7] : 0;
    k.src = reinterpret_cast<const void*>(d[0]);
    k.lds = d[1];
    k.scoff = (int)d[2];
    k.C = (int)d[3];
    k.dst = reinterpret_cast<void*>(d[4]);
    k.ldd = d[5];
    k.dcoff = (int)d[6];
    RGBAC_REQUIRE(k.src && k.dst && k.C > 0, "null pointer / empty copy");
    RGBAC_REQUIRE(k.scoff >= 0 && k.dcoff >= 0 && k.scoff + k.C <= k.lds && k.dcoff + k.C <= k.ldd,
                  "channel range");
    k.vec = (k.C % epv == 0 && k.scoff % epv == 0 && k.dcoff % epv == 0 && k.lds % epv == 0 &&
             k.ldd % epv == 0 && d[0] % 16 == 0 && d[4] % 16 == 0);
    maxc = std::max<long long>(maxc, k.vec ? k.C / epv : k.C);
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid(grid_for(npix * maxc), ntasks);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(channel_copy_multi_kernel<float>, grid, dim3(256), 0, st, npix, tk);
  else
    hipLaunchKernelGGL(channel_copy_multi_kernel<uint16_t>, grid, dim3(256), 0, st, npix, tk);
  return check_launch("channel_copy_multi_kernel");
}

extern "C" int rgbac_channel_copy_multi(int dtype, int64_t npix, int ntasks, const int64_t* desc,
                                        void* stream) {
  return copy_multi(dtype, npix, ntasks, desc, 7, stream);
}

extern "C" int rgbac_channel_copy_multi_ex(int dtype, int64_t npix, int ntasks,
                                           const int64_t* desc, void* stream) {
  return copy_multi(dtype, npix, ntasks, desc, 8, stream);
}

extern "C" int rgbac_weight_gather(int dtype, int64_t n, const float* src, const int32_t* idx,
                                   void* dst, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(n >= 0 && (n == 0 || (src && idx && dst)), "args");
  if (n == 0) return RGBAC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(gather_kernel<float>, dim3(grid_for(n)), dim3(256), 0, st, n, src, idx,
                       (float*)dst);
  else
    hipLaunchKernelGGL(gather_kernel<bf16_t>, dim3(grid_for(n)), dim3(256), 0, st, n, src, idx,
                       (bf16_t*)dst);
  return check_launch("gather_kernel");
}

extern "C" int rgbac_weight_gather_multi(int ntask, const int64_t* tasks, const int64_t* blk0,
                                         int64_t nblk, void* stream) {
  RGBAC_REQUIRE(ntask >= 0 && nblk >= 0 && (ntask == 0 || (tasks && blk0)), "args");
  RGBAC_REQUIRE(nblk < (1ll << 31), "too many blocks");
  if (ntask == 0 || nblk == 0) return RGBAC_OK;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(gather_multi_kernel, dim3((unsigned)nblk), dim3(256), 0, st, ntask,
                     reinterpret_cast<const long long*>(tasks),
                     reinterpret_cast<const long long*>(blk0));
  return check_launch("gather_multi_kernel");
}

extern "C" int rgbac_weight_repack_multi(int ntask, const int64_t* tasks, const int64_t* blk0,
                                         int64_t nblk, void* stream) {
  RGBAC_REQUIRE(ntask >= 1 && tasks && blk0, "tasks");
  RGBAC_REQUIRE(nblk >= 1 && nblk < (1ll << 31), "block count");
  hipLaunchKernelGGL(repack_multi_kernel, dim3((unsigned)nblk), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), ntask,
                     reinterpret_cast<const long long*>(tasks), reinterpret_cast<const long long*>(blk0));
  return check_launch("repack_multi_kernel");
}

extern "C" int rgbac_colsum(int dtype, int64_t npix, int channels, const void* x, int64_t ldx,
                            int nsplit, float* partial, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(npix > 0 && channels > 0 && ldx >= channels && x && partial, "args");
  RGBAC_REQUIRE(nsplit >= 1 && nsplit <= 65535, "nsplit");
  const long long chunk = (npix + nsplit - 1) / nsplit;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (dtype == RGBAC_F32)
    hipLaunchKernelGGL(colsum_kernel<float>, dim3(nsplit), dim3(256), 0, st, npix, channels,
                       (const float*)x, ldx, chunk, partial);
  else
    hipLaunchKernelGGL(colsum_kernel<bf16_t>, dim3(nsplit), dim3(256), 0, st, npix, channels,
                       (const bf16_t*)x, ldx, chunk, partial);
  return check_launch("colsum_kernel");
}

extern "C" int rgbac_sum_partials(int rows, int n, const double* partial, float* out,
                                  void* stream) {
  RGBAC_REQUIRE(rows >= 1 && n >= 1 && partial && out, "args");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sum_rows_kernel, dim3(1), dim3(256), 0, st, rows, n, partial, out);
  return check_launch("sum_rows_kernel");
}
