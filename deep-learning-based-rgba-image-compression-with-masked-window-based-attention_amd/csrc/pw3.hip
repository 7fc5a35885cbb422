// Pointwise GDN / IGDN / gate forward with a two-deep input pipeline (conv_pw3_kernel).
// Reference: layers/GDN.py:64-94 -- out = x / sqrt(beta' + gamma' . x^2) (IGDN: * sqrt), the
// norm pool a 1x1 conv over bf16(x^2).
//
// conv_pw2_kernel (conv.hip) keeps ONE 16-pixel input tile per wave in LDS: the next tile's
// LDS-DMA goes out after this tile's MFMAs and has to land before the next MFMAs start, so a
// wave has at most one tile in flight and waits one memory latency per tile.  On the
// multi-round launches (the 256^2 and 512^2 GDN / IGDN of config 4: 16-64 tiles per wave) that
// latency, not HBM or the MFMAs, set the time (2.66 TB/s on the 512^2 IGDN).  Here each wave
// owns TWO tile slots: tile k+2's DMA is issued while tile k computes, and the wait before
// tile k+1 retires only the DMA issued one iteration earlier (counted vmcnt: the epilogue's
// stores and the newest DMA stay in flight).  The residual-register sets of conv_pw2_kernel
// (res0 / res1 / res2 quads, double-buffered) are gone: the only epilogue operand, x, comes
// from the LDS tile the MFMAs consumed.  The attention gate (a * sigmoid(W b + bias) + x,
// layers/Masked_Attention.py:182-189) loads its a / x quads into registers one tile ahead,
// issued behind each tile DMA.  Seven waves (two slots of 6 KiB each + the 72 KiB weight
// panel = 156 KiB of LDS).
//
// Same MFMA order, the same bf16(x^2) B fragments and the same epilogue arithmetic as
// conv_pw2_kernel's GDN / IGDN instance, so the two are bit-identical.
#include <cstdlib>

#include "common.h"
#include "conv_common.h"

namespace rgbac {

#ifndef RGBAC_PW3_WAVES
#define RGBAC_PW3_WAVES 7
#endif
// waves per workgroup: 7 x two 6 KiB slots + the 72 KiB panel = 156 KiB of LDS
constexpr int kPw3Waves = RGBAC_PW3_WAVES;

template <int NKS, int ACT>
__global__ void __launch_bounds__(64 * kPw3Waves, 1) conv_pw3_kernel(const ConvArgsDev args) {
  constexpr int NT = 12, BN = 192, NCH = 4 * NKS, NW = kPw3Waves, TS = 24;
  static_assert(NCH % 8 == 0 && NCH <= TS, "swizzle groups of 8 chunks");
  constexpr int NPIECE = BN * NCH / 64;            // 1-KiB LDS-DMA pieces of the panel
  constexpr int XP = 16 * TS / 64;                 // pieces of one 16-pixel tile (6)
  constexpr int XS = 16 * TS;                      // uint4 slots of one tile
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  __shared__ float bl[BN];
  const ConvShared& s = args.s;
  const ConvGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int nchunk = g.cin_pad >> 3;
  const int Mtot = s.M;
  const int ld = (int)g.sld0;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)lds);
  const uint32_t xbase = lbase + (uint32_t)(BN * NCH + wave * 2 * XS) * 16u;
  const uint4* const X0 = lds + BN * NCH + wave * 2 * XS;
  {
    const bf16_t* wbase = reinterpret_cast<const bf16_t*>(g.w);
    for (int p = wave; p < NPIECE; p += NW) {
      const int d = p * 64 + lane;
      const int row = d / NCH, slot = d - (d / NCH) * NCH;
      const int ch = slot ^ (row & 7);
      const bool ok = row < g.rows && ch < nchunk;
      dma16_l(ok ? (const void*)(wbase + (size_t)row * g.k_pad + ch * 8) : (const void*)g_zero_page,
              lbase + p * 1024);
    }
  }
  for (int e = tid; e < BN; e += 64 * NW) bl[e] = g.bias ? g.bias[e] : 0.0f;

  const char* const src = reinterpret_cast<const char*>(g.sp0);
  constexpr bool GATE = ACT == RGBAC_ACT_GATE;
  const bf16_t* const R1 = reinterpret_cast<const bf16_t*>(g.res1);
  const bf16_t* const R2 = reinterpret_cast<const bf16_t*>(g.res2);
  const int ntile = (Mtot + 15) / 16;
  const int tstride = gridDim.x * NW;
  int tile = blockIdx.x * NW + wave;

  // tile t_ -> slot sl_ of this wave (rows past M and padding chunks read the zero page);
  // always XP pieces, so the counted waits below are exact
  auto dma_tile = [&](int t_, int sl_) {
#pragma unroll
    for (int p = 0; p < XP; ++p) {
      const int d = p * 64 + lane;
      const int row = d / TS, slot = d - (d / TS) * TS;
      const int ch = slot ^ (row & 7);
      const int m = t_ * 16 + row;
      const bool ok = m < Mtot && ch < nchunk;
      dma16_l(ok ? (const void*)(src + ((size_t)m * ld + ch * 8) * 2) : (const void*)g_zero_page,
              xbase + (uint32_t)(sl_ * XS * 16) + p * 1024);
    }
  };
  // GATE: the epilogue's a / x quads of tile t_ (rows past M read row 0: always 2 NT loads)
  auto load_res = [&](int t_, uint2 (&ea)[NT], uint2 (&er)[NT]) {
    const int m_ = t_ * 16 + fr;
    const long long mm = m_ < Mtot ? m_ : 0;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = 16 * j + 4 * fq;
      ea[j] = *reinterpret_cast<const uint2*>(R1 + mm * g.ld1 + n);
      er[j] = *reinterpret_cast<const uint2*>(R2 + mm * g.ld2 + n);
    }
  };
  uint2 ca[NT], cr[NT], na[NT], nr[NT];
  dma_tile(tile, 0);
  dma_tile(tile + tstride, 1);
  if constexpr (GATE) load_res(tile, ca, cr);
  if constexpr (GATE) wait_vm<2 * NT + XP>();      // the panel and slot 0
  else wait_vm<XP>();                              // (slot 1, and the quads, in flight)
  __syncthreads();
  bf16_t* const out = reinterpret_cast<bf16_t*>(g.out);
  // one tile; ua / ur hold its gate quads, va / vr receive the next tile's (the loop below
  // alternates the two sets: a loop-carried copy would make the compiler wait for every
  // outstanding load, DMAs included, at the top of each iteration)
  auto step = [&](int k, const uint2 (&ua)[NT], const uint2 (&ur)[NT], uint2 (&va)[NT],
                  uint2 (&vr)[NT]) {
    // slot k & 1 holds tile k: its DMA was issued two iterations back (or in the prologue);
    // younger than it are that iteration's stores (NT), the next DMA (XP) and the last
    // iteration's stores (NT).  The counts are lower bounds that hold for any codegen: the DMA
    // is always XP pieces (asm), and the NT quad stores of a lane are 8-byte stores 32 bytes
    // apart (nothing to merge; a split store only adds younger operations, i.e. waits more);
    // every iteration has a valid lane (fr = 0), so no store block is skipped
    // (GATE: plus the 2 NT quad loads of the next tile issued behind each tile DMA; past
    // vmcnt's 63 the wait also retires some older quad loads, which the epilogue before
    // already needed)
    if constexpr (GATE) {
      if (k > 0) wait_vm<63>();                    // (66 / 78 younger: k == 1 / k > 1)
    } else {
      if (k == 1) wait_vm<XP + NT>();
      else if (k > 1) wait_vm<2 * NT + XP>();
    }
    const uint4* const Xl = X0 + (k & 1) * XS;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      const int slot = (4 * st + fq) ^ (fr & 7);
      uint4 b = Xl[fr * TS + slot];
      if constexpr (!GATE) b = square_chunk<bf16_t>(b);
#pragma unroll
      for (int j = 0; j < NT; ++j) mma_step<bf16_t>(acc[j], lds[(16 * j + fr) * NCH + slot], b);
    }
    uint2 xq[NT];                                  // the epilogue's x quads, from the same tile
    if constexpr (!GATE) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int c = 2 * j + (fq >> 1);
        xq[j] = *reinterpret_cast<const uint2*>(
            reinterpret_cast<const char*>(Xl + fr * TS + (c ^ (fr & 7))) + 8 * (fq & 1));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // slot reads done before its refill
    dma_tile(tile + 2 * tstride, k & 1);
    if constexpr (GATE) load_res(tile + tstride, va, vr);
    const int m = tile * 16 + fr;
    if (m < Mtot) {
      bf16_t* const orow = out + (long long)m * g.out_ldc + g.out_coff;
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = 16 * j + 4 * fq;
        float v[4];
        if constexpr (GATE) {                      // a * sigmoid(conv + b) + x
          const float a4[4] = {bf2f(ua[j].x & 0xFFFF), bf2f(ua[j].x >> 16),
                               bf2f(ua[j].y & 0xFFFF), bf2f(ua[j].y >> 16)};
          const float r4[4] = {bf2f(ur[j].x & 0xFFFF), bf2f(ur[j].x >> 16),
                               bf2f(ur[j].y & 0xFFFF), bf2f(ur[j].y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = a4[r] * sigmoid_f(acc[j][r] + bl[n + r]) + r4[r];
        } else {
          const float x4[4] = {bf2f(xq[j].x & 0xFFFF), bf2f(xq[j].x >> 16),
                               bf2f(xq[j].y & 0xFFFF), bf2f(xq[j].y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float nrm = acc[j][r] + bl[n + r];
            v[r] = ACT == RGBAC_ACT_GDN ? gdn_t<bf16_t>(x4[r], nrm) : igdn_t<bf16_t>(x4[r], nrm);
          }
        }
        Elem<bf16_t>::st4(orow + n, v);
      }
    }
  };
  for (int k = 0;; k += 2) {
    if (tile >= ntile) break;
    step(k, ca, cr, na, nr);
    tile += tstride;
    if (tile >= ntile) break;
    step(k + 1, na, nr, ca, cr);
    tile += tstride;
  }
  wait_vm<0>();                                    // no DMA may land after the workgroup ends
}

// conv_pw3_kernel's shapes: the bf16 GDN / IGDN norm pool -- one source whose x is also the
// epilogue's (square input, res1 == the input), 192 outputs, no other residual, no
// pre-activation store.  RGBAC_PW3=0 keeps conv_pw2_kernel (A/B switch).
bool pw3_ok(const ConvArgsDev& d, int cin_max) {
  const char* e = getenv("RGBAC_PW3");              // read per launch (tests switch it)
  const bool on = !(e && e[0] == '0');
  // the gate only on multi-round launches (>= 8192 tiles: config 4's 256^2 gates, 216 vs
  // 240 us); at config 2's 2048 tiles its register-prefetched quads lose (50 vs 45 us)
  const bool gate = d.s.act == RGBAC_ACT_GATE && d.s.M >= 8192 * 16;
  if (!on || (d.s.act != RGBAC_ACT_GDN && d.s.act != RGBAC_ACT_IGDN && !gate) ||
      (d.s.square != 0) == gate || d.s.mode != RGBAC_CONV || cin_max <= 128 || cin_max > 192)
    return false;
  for (int i = 0; i < d.s.ngroups; ++i) {
    const ConvGroup& g = d.g[i];
    if (g.res0 || g.zout || g.cout != 192 || g.rows < 192 || g.out_coff % 8 || g.out_ldc % 8 ||
        g.sld0 % 8 || g.k_pad < g.cin_pad)
      return false;
    if (gate ? (!g.res1 || !g.res2 || g.ld1 % 4 || g.ld2 % 4)
             : (g.res1 != g.sp0 || g.ld1 != g.sld0 || g.res2))
      return false;
  }
  return true;
}

template <int ACT>
static void launch_pw3_k(const ConvArgsDev& d, hipStream_t st) {
  auto kern = conv_pw3_kernel<6, ACT>;
  constexpr size_t lds = ((size_t)192 * 24 + (size_t)kPw3Waves * 2 * 16 * 24) * 16;
  static unsigned long long attr = 0;                 // per device (lds_optin, common.h)
  lds_optin((const void*)kern, (int)lds, &attr);
  const int ncu = device_cus();
  const int nz = d.s.ngroups;
  const int ntile = (d.s.M + 15) / 16;
  int gx = (ncu + nz - 1) / nz;
  const int need = (ntile + kPw3Waves - 1) / kPw3Waves;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(kern, dim3(gx, 1, nz), dim3(64 * kPw3Waves), lds, st, d);
}

void launch_pw3(const ConvArgsDev& d, hipStream_t st) {
  if (d.s.act == RGBAC_ACT_GDN) launch_pw3_k<RGBAC_ACT_GDN>(d, st);
  else if (d.s.act == RGBAC_ACT_IGDN) launch_pw3_k<RGBAC_ACT_IGDN>(d, st);
  else launch_pw3_k<RGBAC_ACT_GATE>(d, st);
}

}  // namespace rgbac
