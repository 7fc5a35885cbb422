// Fused analysis stem: conv5x5/s2 (Cin <= 8 -> 192) + GDN, bf16
// (reference: layers/TransformRGB.py:55-56,66 -- self.x1 then self.gdn1; layers/GDN.py:64-94).
//
//   y   = bf16( W1 (*) x + b1 )                              (the stem conv, 3 -> 192)
//   out = y / sqrt( beta' + gamma' . bf16(y^2) )             (GDN; IGDN: * sqrt)
//
// i.e. exactly the unfused bf16 path (conv -> bf16 store -> GDN norm pool on bf16(y^2) with
// the y/sqrt epilogue), without writing y to HBM and reading it back twice.  The stem's
// output at 128x128 is the largest activation of the encoder (50 MB per 8 images), so the
// two unfused kernels are HBM-bound; the fused one reads the 3-channel image and writes
// the GDN output once.
//
// One persistent workgroup per CU holds both weight panels in LDS (W1: 192 x 208 bf16,
// W2 = gamma': 192 x 192 bf16, 150 KB); each WAVE streams 32-pixel tiles on its own:
//   stem : 13 k-steps of v_mfma_f32_32x32x16_bf16, B = im2col fragment (pixel lane&31,
//          tap 2*ks + (lane>>5), its 8 channels = one 16-byte load straight to VGPRs),
//          A = W1 fragments from LDS; acc1 = 6 x (32 ch x 32 px).
//   gdn  : the accumulator holds, per lane, pixel lane&31 and channel quads
//          32t + 8g + 4h (h = lane>>5); the GDN GEMM's B fragment for k-step ks needs
//          channels 16ks + 8h .. +7 of the same pixel: one quad is the lane's own, the
//          other is the partner lane's (lane ^ 32) -- one v_permlane32_swap per k-step.
//   out  : y / sqrt(norm + beta') in the accumulator layout, 8-byte stores.
#include "common.h"

namespace rgbac {

constexpr int kStemC = 192;          // output channels (N of the reference)
constexpr int kStemNT = kStemC / 32; // 32-channel MFMA tiles
constexpr int kStemKS1 = 13;         // stem k-steps of 16: 25 taps x 8 channels = 200 -> 208
constexpr int kStemKS2 = kStemC / 16;
constexpr int kW1Chunks = 2 * kStemKS1 + 1;   // 16-byte chunks per W1 row (26 + 1 pad:
                                               // 16 consecutive rows hit distinct banks)
constexpr int kW2Chunks = kStemC / 8;     // 24

typedef __attribute__((ext_vector_type(16))) float f32x16_s;
// waves per workgroup: two per SIMD, so one wave's VALU epilogues (bias / GDN B fragments /
// rsqrt) issue beside the other wave's MFMAs (at one wave per SIMD they serialised)
#ifndef RGBAC_STEM_NW
#define RGBAC_STEM_NW 8
#endif
constexpr int kStemNW = RGBAC_STEM_NW;

__device__ uint4 g_stem_zero[64];           // source of the W1 rows' padding chunk

__device__ __forceinline__ void stem_dma16(const void* src, uint32_t lds) {
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

__device__ __forceinline__ int w1_slot(int row, int chunk) { return row * kW1Chunks + chunk; }
__device__ __forceinline__ int w2_slot(int row, int chunk) {
  return row * kW2Chunks + (chunk ^ (row & 7));
}


__global__ void __launch_bounds__(kStemNW * 64, 1)
stem_gdn_kernel(int batch, int in_h, int in_w, const bf16_t* __restrict__ x, int x_ldc,
                const bf16_t* __restrict__ w1, int w1_kpad, const float* __restrict__ b1,
                const bf16_t* __restrict__ w2, int w2_kpad, const float* __restrict__ beta,
                int inverse, bf16_t* __restrict__ out, long long out_ldc) {
  __shared__ __attribute__((aligned(16))) uint4 W1s[kStemC * kW1Chunks];
  __shared__ __attribute__((aligned(16))) uint4 W2s[kStemC * kW2Chunks];
  __shared__ float B1s[kStemC], BEs[kStemC];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // panel staging by LDS-DMA: 1-KiB pieces (64 16-byte slots) straight into the (padded /
  // swizzled) panel images, every piece in flight at once and one wait for all -- the
  // register round trip (load 4 chunks, wait, store) paid ~10 memory latencies per CU
  {
    const uint32_t l1 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(size_t)(__attribute__((address_space(3))) void*)W1s);
    const uint32_t l2 = __builtin_amdgcn_readfirstlane(
        (uint32_t)(size_t)(__attribute__((address_space(3))) void*)W2s);
    constexpr int P1 = kStemC * kW1Chunks / 64, P2 = kStemC * kW2Chunks / 64;
    static_assert(P1 * 64 == kStemC * kW1Chunks && P2 * 64 == kStemC * kW2Chunks, "whole pieces");
    for (int p = wave; p < P1 + P2; p += kStemNW) {
      if (p < P1) {
        const int e = p * 64 + lane, r = e / kW1Chunks, ch = e - r * kW1Chunks;
        stem_dma16(ch < kW1Chunks - 1 ? (const void*)(w1 + (size_t)r * w1_kpad + ch * 8)
                                      : (const void*)g_stem_zero,
                   l1 + p * 1024);
      } else {
        const int e = (p - P1) * 64 + lane, r = e / kW2Chunks, sl = e - r * kW2Chunks;
        stem_dma16(w2 + (size_t)r * w2_kpad + (sl ^ (r & 7)) * 8, l2 + (p - P1) * 1024);
      }
    }
  }
  if (tid < kStemC) {
    B1s[tid] = b1 ? b1[tid] : 0.0f;
    BEs[tid] = beta[tid];
  }

  const int r32 = lane & 31, h = lane >> 5;
  const int Ho = (in_h + 1) / 2, Wo = (in_w + 1) / 2;
  const int M = batch * Ho * Wo;
  const int ntile = (M + 31) / 32;
  const int tstride = gridDim.x * kStemNW;
  // XCD-contiguous tile runs: the hardware deals block b to XCD b mod 8, so with the plain
  // order the 4 x 32-pixel tiles of one output row and its neighbour rows -- whose 5x5/s2
  // windows share input rows -- land on 8 different L2s and every L2 fetches the shared rows
  // from HBM (PMC: 23.2 MB fetched for an 8.4 MB input).  Remapped, the blocks of one XCD run
  // consecutive tiles (32 output rows at 128^2 per round), and the row overlap stays in its L2.
  int vb = blockIdx.x;
  {
    const int nwg = gridDim.x, xcd = vb & 7, q = nwg >> 3, rr = nwg & 7;
    vb = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (vb >> 3);
  }
  // im2col fragment of stem k-step ks for the pixel decoded as (pb, oy, ox) / valid:
  // tap = 2*ks + h (taps >= 25 are the zero padding of K)
  auto load_b = [&](int ks, int pb, int oy, int ox, bool valid) -> uint4 {
    const int tap = 2 * ks + h;
    const int ty = tap / 5, tx = tap - ty * 5;
    const int iy = 2 * oy + ty - 2, ix = 2 * ox + tx - 2;
    const bool ok = valid & (tap < 25) & ((unsigned)iy < (unsigned)in_h) &
                    ((unsigned)ix < (unsigned)in_w);
    const uint4* p = ok ? reinterpret_cast<const uint4*>(
                              x + ((size_t)(pb * in_h + iy) * in_w + ix) * x_ldc)
                        : reinterpret_cast<const uint4*>(x);
    const uint4 v = *p;
    return ok ? v : make_uint4(0, 0, 0, 0);
  };

  auto decode = [&](int tl, int& pb, int& oy, int& ox) -> bool {
    const int m = tl * 32 + r32;
    const bool valid = (tl < ntile) & (m < M);
    const int mm = valid ? m : 0;
    ox = mm % Wo;
    const int t2 = mm / Wo;
    oy = t2 % Ho;
    pb = t2 / Ho;
    return valid;
  };
  // the panels, one wait
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int tile = vb * kStemNW + wave; tile < ntile; tile += tstride) {
    const int m = tile * 32 + r32;
    const bool valid = m < M;
    // this tile's im2col fragments (register budget at two waves per SIMD: no cross-tile
    // prefetch; the SIMD's other wave computes while these are in flight)
    uint4 bv[kStemKS1];
    {
      int pb, oy, ox;
      const bool v = decode(tile, pb, oy, ox);
#pragma unroll
      for (int ks = 0; ks < kStemKS1; ++ks) bv[ks] = load_b(ks, pb, oy, ox, v);
    }

    // ---- stem conv
    f32x16_s acc[kStemNT];
    const f32x16_s zero16 = {};
    // A fragments one k-step ahead: k-step ks + 1's LDS reads are in flight under k-step ks's
    // six MFMAs (the scheduling barrier keeps the compiler from hoisting all 78 and spilling)
    uint4 an[kStemNT];
#pragma unroll
    for (int t = 0; t < kStemNT; ++t) an[t] = W1s[w1_slot(32 * t + r32, h)];
#pragma unroll
    for (int ks = 0; ks < kStemKS1; ++ks) {
      const bf16x8 bb = __builtin_bit_cast(bf16x8, bv[ks]);
      uint4 a[kStemNT];
#pragma unroll
      for (int t = 0; t < kStemNT; ++t) a[t] = an[t];
      if (ks + 1 < kStemKS1) {
#pragma unroll
        for (int t = 0; t < kStemNT; ++t) an[t] = W1s[w1_slot(32 * t + r32, 2 * (ks + 1) + h)];
      }
#pragma unroll
      for (int t = 0; t < kStemNT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[t]), bb,
                                                         ks ? acc[t] : zero16, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }


    // ---- y = bf16(acc + b1), kept packed per channel quad (channels 32t + 8g + 4h + r)
    uint32_t ypk[kStemNT][4][2];
#pragma unroll
    for (int t = 0; t < kStemNT; ++t)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int c = 32 * t + 8 * g + 4 * h;
        ypk[t][g][0] = pack_bf16x2(acc[t][4 * g] + B1s[c], acc[t][4 * g + 1] + B1s[c + 1]);
        ypk[t][g][1] = pack_bf16x2(acc[t][4 * g + 2] + B1s[c + 2], acc[t][4 * g + 3] + B1s[c + 3]);
      }
    // bf16(y^2) of a packed pair, as the unfused GDN's square_chunk forms it
    auto sq2 = [](uint32_t w) -> uint32_t {
      const float lo = bf2f((uint16_t)(w & 0xFFFF)), hi = bf2f((uint16_t)(w >> 16));
      return pack_bf16x2(lo * lo, hi * hi);
    };

    // ---- GDN norm pool: norm[n][px] = sum_j gamma'[n][j] * y[j][px]^2 on MFMA
    uint4 wn[kStemNT];
#pragma unroll
    for (int t = 0; t < kStemNT; ++t) wn[t] = W2s[w2_slot(32 * t + r32, h)];
#pragma unroll
    for (int ks = 0; ks < kStemKS2; ++ks) {
      // B fragment: channels 16ks + 8h .. +7 = quad g_need = 2(ks&1) + h of tile ks/2, both
      // halves; the lane's own half (4h) is local, the other comes from lane ^ 32, which in
      // turn needs this lane's quad 2(ks&1) + (1-h).
      const int tt = ks >> 1;
      const int g_need = 2 * (ks & 1) + h, g_send = 2 * (ks & 1) + (1 - h);
      const int ga = 2 * (ks & 1), gb = ga + 1;
      const uint32_t s0 = sq2(h ? ypk[tt][ga][0] : ypk[tt][gb][0]);
      const uint32_t s1 = sq2(h ? ypk[tt][ga][1] : ypk[tt][gb][1]);
      (void)g_send;
      // the partner half's quad: v_permlane32_swap (a VALU lane exchange, no LDS round trip)
      const uint32_t r0 = xor32_u(s0);
      const uint32_t r1 = xor32_u(s1);
      const uint32_t o0 = sq2(h ? ypk[tt][gb][0] : ypk[tt][ga][0]);
      const uint32_t o1 = sq2(h ? ypk[tt][gb][1] : ypk[tt][ga][1]);
      (void)g_need;
      // channels 0..3 of the chunk come from half 0, 4..7 from half 1
      uint4 b;
      if (h == 0) b = make_uint4(o0, o1, r0, r1);
      else b = make_uint4(r0, r1, o0, o1);
      const bf16x8 bb = __builtin_bit_cast(bf16x8, b);
      uint4 a[kStemNT];
#pragma unroll
      for (int t = 0; t < kStemNT; ++t) a[t] = wn[t];
      if (ks + 1 < kStemKS2) {
#pragma unroll
        for (int t = 0; t < kStemNT; ++t) wn[t] = W2s[w2_slot(32 * t + r32, 2 * (ks + 1) + h)];
      }
#pragma unroll
      for (int t = 0; t < kStemNT; ++t)
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a[t]), bb,
                                                         ks ? acc[t] : zero16, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- out = y / sqrt(norm + beta')  (IGDN: * sqrt)
    if (valid) {
      bf16_t* op = out + (size_t)m * out_ldc;
#pragma unroll
      for (int t = 0; t < kStemNT; ++t)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          float o[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const uint32_t w = ypk[t][g][r >> 1];
            const float y = bf2f((r & 1) ? (uint16_t)(w >> 16) : (uint16_t)(w & 0xFFFF));
            const float v = acc[t][4 * g + r] + BEs[32 * t + 8 * g + 4 * h + r];
            // bf16 output: hardware rsq / sqrt (~1 ulp fp32) instead of IEEE sqrt + divide
            o[r] = inverse ? y * __builtin_amdgcn_sqrtf(v) : y * __builtin_amdgcn_rsqf(v);
          }
          uint2 st;
          st.x = pack_bf16x2(o[0], o[1]);
          st.y = pack_bf16x2(o[2], o[3]);
          *reinterpret_cast<uint2*>(op + 32 * t + 8 * g + 4 * h) = st;
        }
    }
  }
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_stem_gdn(int batch, int in_h, int in_w, const void* x, int64_t x_ldc,
                              const void* w1, int w1_kpad, const float* b1, const void* w2,
                              int w2_kpad, const float* beta, int inverse, void* out,
                              int64_t out_ldc, void* stream) {
  RGBAC_REQUIRE(batch > 0 && in_h > 0 && in_w > 0, "bad input shape");
  RGBAC_REQUIRE(x && w1 && w2 && beta && out, "null pointer");
  RGBAC_REQUIRE(x_ldc == 8, "the stem input must be NHWC with 8 (padded) channels");
  RGBAC_REQUIRE(w1_kpad >= 8 * 26 && w1_kpad % 8 == 0, "w1 k_pad must cover 26 x 8 (zero-padded)");
  RGBAC_REQUIRE(w2_kpad >= kStemC && w2_kpad % 8 == 0, "w2 k_pad must be >= 192");
  RGBAC_REQUIRE(out_ldc >= kStemC && out_ldc % 4 == 0, "out_ldc");
  RGBAC_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)w1 % 16) == 0 && ((uintptr_t)w2 % 16) == 0,
                "16-byte alignment");
  const long long M = (long long)batch * ((in_h + 1) / 2) * ((in_w + 1) / 2);
  RGBAC_REQUIRE(M < (1ll << 31), "too many output pixels");
  const int ncu = device_cus();
  const long long ntile = (M + 31) / 32;
  long long g = (ntile + kStemNW - 1) / kStemNW;
  if (g > ncu) g = ncu;
  hipLaunchKernelGGL(stem_gdn_kernel, dim3((unsigned)g), dim3(kStemNW * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), batch, in_h, in_w,
                     reinterpret_cast<const bf16_t*>(x), (int)x_ldc,
                     reinterpret_cast<const bf16_t*>(w1), w1_kpad, b1,
                     reinterpret_cast<const bf16_t*>(w2), w2_kpad, beta, inverse,
                     reinterpret_cast<bf16_t*>(out), (long long)out_ldc);
  return check_launch("stem_gdn_kernel");
}
