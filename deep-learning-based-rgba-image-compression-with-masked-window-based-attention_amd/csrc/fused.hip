// Fused ResidualUnit (reference: layers/Masked_Attention.py:150-169)
//
//   y = GELU( W3 * GELU( W2 (*)3x3 GELU( W1 * x + b1 ) + b2 ) + b3 + x )
//
// for C = 192 (CH = 96) on bf16 NHWC activations.  One workgroup computes an
// 8x8 output tile: stage 1 evaluates the first 1x1 conv on the 10x10 halo
// (zero outside the image, as the 3x3's zero padding requires) into LDS (T1),
// stage 2 the 3x3 conv from T1 into LDS (T2), stage 3 the last 1x1 conv with
// bias, residual and GELU straight to HBM.  The three packed weight matrices
// ([rows][k_pad], k = tap*cin + c, the conv engine's layout) stream through one
// double-buffered LDS ring in 12-15 KB chunks shared by the four waves.
// Versus three conv launches this removes two HBM round trips of the
// intermediates and two launch/latency tails per unit; two units of identical
// shape (the conv_a / conv_b chains of Win_noShift_Attention) run as one
// launch (blockIdx.z = group).
//
// MFMA: v_mfma_f32_16x16x32_bf16, D[n][m] = sum_k W[n][k] X[m][k]: channels on
// the row axis (each lane ends with 4 consecutive channels of one pixel).
//   stage 1: M = 128 halo rows (100 real; waves own 32 rows), N = 96, K = 192
//   stage 2: M = 64, N = 96, K = 864    (waves: 2 channel halves x 2 pixel halves)
//   stage 3: M = 64, N = 192, K = 96    (same split)
// LDS: T1 100 x 192 B, T2 (64 x 192 B) aliased onto T1 once
// stage 2 has consumed it, ring 2 x 15 KB -> 51 KB: three workgroups per CU.
// Weight chunks are prefetched PF = 4 chunks ahead in registers (the chunk
// loops are fully unrolled so the register ring is statically indexed).
#include <cstdlib>

#include "common.h"

namespace rgbac {

constexpr int kRuMaxGroups = 4;

struct RuGroup {
  const bf16_t* x; long long ldx;
  const bf16_t* w1; const bf16_t* w2; const bf16_t* w3;
  int kp1, kp2, kp3;
  const float* b1; const float* b2; const float* b3;
  bf16_t* out; long long ldo;
};
struct RuArgsDev {
  int batch, H, W, ngroups;
  int stagger;                     // ru_stream_kernel: s_sleep(16) rounds of the later half of the grid
  RuGroup g[kRuMaxGroups];
  // ru_stream_kernel<.., GATE = true> (rgbac_residual_unit_gate): the attention block's gate
  const bf16_t* gw;                // conv_b[3] weights, fragment-major [12][6][64][8]
  const float* gb;                 // its bias [192]
  const bf16_t* gid; long long ldid;   // the block input (identity)
  unsigned* flags;                 // per-tile hand-off words (zero at entry, left zero)
  unsigned* timeout;               // set to 1 if a hand-off wait ever gave up (never expected)
};

// 16-byte write-through (sc1) store: the hand-off payload of rgbac_residual_unit_gate (no release
// fence needed: cdna_hip_programming.md Guideline 16 R1).  Not counted by hipcc: the caller
// drains it with s_waitcnt vmcnt(0) before the flag store.
typedef unsigned ru_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st16_wt(void* p, const uint4& v) {
  const ru_u32x4 d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
}

__device__ __forceinline__ float ru_gelu(float v) { return gelu_fast(v); }   // bf16 outputs

// RB = 0: ResidualUnit (GELU after each conv, GELU after the residual add);
// RB = 1: the alpha codec's ResBlock (AutoEncoderMask_Journal.py:96-110: ReLU, ReLU, + x).
template <int RB>
__device__ __forceinline__ float ru_act(float v) { return RB ? fmaxf(v, 0.0f) : ru_gelu(v); }
// v = act(a + b) on one accumulator quad
template <int RB>
__device__ __forceinline__ void ru_act4(float (&v)[4], const f32x4& a, const float4& b) {
  if constexpr (RB) {
    v[0] = fmaxf(a[0] + b.x, 0.0f); v[1] = fmaxf(a[1] + b.y, 0.0f);
    v[2] = fmaxf(a[2] + b.z, 0.0f); v[3] = fmaxf(a[3] + b.w, 0.0f);
  } else {
    v[0] = a[0] + b.x; v[1] = a[1] + b.y; v[2] = a[2] + b.z; v[3] = a[3] + b.w;
    gelu4_fast(v);                                   // packed pairs (bit-identical to ru_gelu)
  }
}

template <int C, int CH, int TY, int TX, int OCC, int RB = 0>
__global__ void __launch_bounds__(256, OCC) ru_fused_kernel(const RuArgsDev args) {
  // TY x TX output tile, (TY+2) x (TX+2) halo; 8x16 halves the weight traffic per pixel
  // (every tile streams all three weight matrices once) at 2 workgroups per CU
  constexpr int HY = TY + 2, HX = TX + 2, NH = HY * HX;
  constexpr int MT1 = (NH + 63) / 64;                  // stage-1 m tiles per wave
  constexpr int NPX = TY * TX;                         // output pixels per tile
  constexpr int MT2 = NPX / 32;                        // stage-2/3 m tiles per wave
  static_assert(NPX % 32 == 0 && NH >= NPX, "tile geometry");
  constexpr int NT1 = CH / 16;                         // n tiles of stages 1 / 2
  constexpr int NT3 = C / 16;                          // n tiles of stage 3
  // T1 / T2 row bytes.  A fragment read is 16 lanes on 16 pixel rows: with 16-pixel tile rows
  // they are 16 consecutive rows, and 208-B rows (52 dwords: 52 r mod 64 distinct for r < 16)
  // are conflict-free for the ds_read_b128 lane groups, where 192-B rows collide 2-way (47 %
  // of the LDS cycles were conflict cycles).  8-pixel rows split a read over two tile rows:
  // unpadded rows stay (208 B would give 3-way there).
  constexpr int TROW = CH * 2 + (TX == 16 ? 16 : 0);
  constexpr int KC1 = C / 64;                          // stage-1 chunks (64 k each)
  constexpr int K2 = 9 * CH;
  constexpr int KC2 = (K2 + 63) / 64;                  // stage-2 chunks (64 k each)
  constexpr int KC3 = CH / 32;                         // stage-3 chunks (32 k each)
  constexpr int NCH = KC1 + KC2 + KC3;
  constexpr int RING = (CH * 128 > C * 80 ? CH * 128 : C * 80);   // bytes per ring slot
  constexpr int PIECES = 768;                          // 16-B pieces per chunk (12 KB)
  static_assert(CH * 128 == PIECES * 16 && C * 64 == PIECES * 16, "chunk geometry");
  static_assert(C % 64 == 0 && CH % 32 == 0, "channel geometry");
  constexpr int PF = 4;                                // chunks in flight ahead
  __shared__ __attribute__((aligned(16))) unsigned char T1[NH * TROW];
  unsigned char* const T2 = T1;                        // stage-3 input, after stage 2
  __shared__ __attribute__((aligned(16))) unsigned char ring[2][RING];

  const RuGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int tx_n = args.W / TX, ty_n = args.H / TY;
  int t = blockIdx.x;
  const int tx = t % tx_n; t /= tx_n;
  const int ty = t % ty_n;
  const int b = t / ty_n;
  const int y0 = ty * TY, x0 = tx * TX;

  // ---- weight ring: chunk c -> 3 pieces of 16 B per thread, staged in registers
  // set c % 5 of five named register sets (selects fold after full unrolling;
  // an indexed array here is not promoted to registers), stored to LDS slot c & 1
  static_assert(PF == 4, "five register sets");
  uint4 wa[3], wb[3], wc[3], wd[3], we[3];
  auto load_w = [&](int c) {
    if (c >= NCH) return;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int p = tid + 256 * j;
      const bf16_t* src;
      if (c < KC1) {
        const int r = p >> 3, q = p & 7;
        src = g.w1 + (size_t)r * g.kp1 + c * 64 + q * 8;
      } else if (c < KC1 + KC2) {
        const int r = p >> 3, q = p & 7;
        src = g.w2 + (size_t)r * g.kp2 + (c - KC1) * 64 + q * 8;
      } else {
        const int r = p >> 2, q = p & 3;
        src = g.w3 + (size_t)r * g.kp3 + (c - KC1 - KC2) * 32 + q * 8;
      }
      const uint4 v = *reinterpret_cast<const uint4*>(src);
      const int set = c % 5;
      if (set == 0) wa[j] = v;
      else if (set == 1) wb[j] = v;
      else if (set == 2) wc[j] = v;
      else if (set == 3) wd[j] = v;
      else we[j] = v;
    }
  };
  auto store_w = [&](int c, int buf) {
    if (c >= NCH) return;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int p = tid + 256 * j;
      int off;
      if (c < KC1 + KC2) {
        const int r = p >> 3, q = p & 7;
        off = r * 128 + 16 * (q ^ (r & 7));
      } else {
        const int r = p >> 2, q = p & 3;
        off = r * 80 + 16 * q;
      }
      const int set = c % 5;
      *reinterpret_cast<uint4*>(&ring[buf][off]) =
          set == 0 ? wa[j] : set == 1 ? wb[j] : set == 2 ? wc[j] : set == 3 ? wd[j] : we[j];
    }
  };
  // A fragment of n tile j, k-step kk of a 64-k chunk (stages 1 / 2)
  auto wfrag64 = [&](int buf, int j, int kk) -> uint4 {
    const int r = j * 16 + fr, q = kk * 4 + fq;
    return *reinterpret_cast<const uint4*>(&ring[buf][r * 128 + 16 * (q ^ (r & 7))]);
  };
  auto wfrag32 = [&](int buf, int j) -> uint4 {          // stage 3 (32-k chunks)
    const int r = j * 16 + fr;
    return *reinterpret_cast<const uint4*>(&ring[buf][r * 80 + 16 * fq]);
  };

#pragma unroll
  for (int c = 0; c <= PF; ++c) load_w(c);
  store_w(0, 0);
  __syncthreads();

  // ======================= stage 1: T1 = GELU(W1 x + b1) on the 10x10 halo
  {
    f32x4 acc[NT1][MT1];
#pragma unroll
    for (int j = 0; j < NT1; ++j)
#pragma unroll
      for (int i = 0; i < MT1; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bf16_t* xrow[MT1];
    bool xin[MT1];
#pragma unroll
    for (int i = 0; i < MT1; ++i) {
      const int hp = wave * (16 * MT1) + i * 16 + fr;
      const int hy = hp / HX, hx = hp - (hp / HX) * HX;
      const int iy = y0 + hy - 1, ix = x0 + hx - 1;
      xin[i] = hp < NH && iy >= 0 && iy < args.H && ix >= 0 && ix < args.W;
      xrow[i] = g.x + ((long long)(b * args.H + (xin[i] ? iy : 0)) * args.W + (xin[i] ? ix : 0)) * g.ldx;
    }
#pragma unroll
    for (int c = 0; c < KC1; ++c) {
      uint4 xb[2][MT1];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < MT1; ++i)
          xb[kk][i] = xin[i] ? *reinterpret_cast<const uint4*>(xrow[i] + c * 64 + kk * 32 + fq * 8)
                             : make_uint4(0, 0, 0, 0);
      const int buf = c & 1;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < NT1; ++j) {
          const uint4 a = wfrag64(buf, j, kk);
#pragma unroll
          for (int i = 0; i < MT1; ++i) mma_step<bf16_t>(acc[j][i], a, xb[kk][i]);
        }
      store_w(c + 1, buf ^ 1);
      load_w(c + PF + 1);
      __syncthreads();
    }
    // epilogue -> T1 (zero outside the image: the 3x3's zero padding)
#pragma unroll
    for (int i = 0; i < MT1; ++i) {
      const int hp = wave * (16 * MT1) + i * 16 + fr;
      if (hp >= NH) continue;
#pragma unroll
      for (int j = 0; j < NT1; ++j) {
        const int n = j * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = xin[i] ? ru_act<RB>(acc[j][i][r] + g.b1[n + r]) : 0.0f;
        Elem<bf16_t>::st4(reinterpret_cast<bf16_t*>(&T1[hp * TROW + n * 2]), v);
      }
    }
  }
  __syncthreads();

  // stages 2 / 3: waves as 2 (channel halves) x 2 (pixel halves): per k-step a wave
  // reads NT/2 weight fragments and 2 pixel fragments for NT/2 x 2 MFMAs
  const int wn = wave >> 1, wm = wave & 1;

  // ======================= stage 2: T2 = GELU(W2 (*) T1 + b2), 3x3 over the halo
  {
    constexpr int NJ = NT1 / 2;                       // 3 channel tiles per wave
    f32x4 acc[NJ][MT2];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < MT2; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    int py[MT2], px[MT2];
#pragma unroll
    for (int i = 0; i < MT2; ++i) {
      const int p = wm * (NPX / 2) + i * 16 + fr;     // this lane's pixel of m tile i
      py[i] = p / TX;
      px[i] = p % TX;
    }
#pragma unroll
    for (int c2 = 0; c2 < KC2; ++c2) {
      const int c = KC1 + c2;
      const int buf = c & 1;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int k = c2 * 64 + kk * 32;              // a 32-k step never straddles taps
        const int tap = k / CH, ch = k - tap * CH + fq * 8;
        uint4 bv[MT2];
#pragma unroll
        for (int i = 0; i < MT2; ++i) {
          bv[i] = make_uint4(0, 0, 0, 0);
          if (tap < 9) {
            const int hr = (py[i] + tap / 3) * HX + px[i] + tap % 3;
            bv[i] = *reinterpret_cast<const uint4*>(&T1[hr * TROW + ch * 2]);
          }
        }
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const uint4 a = wfrag64(buf, wn * NJ + j, kk);
#pragma unroll
          for (int i = 0; i < MT2; ++i) mma_step<bf16_t>(acc[j][i], a, bv[i]);
        }
      }
      store_w(c + 1, buf ^ 1);
      load_w(c + PF + 1);
      __syncthreads();                  // (last one: every wave is done reading T1)
    }
#pragma unroll
    for (int i = 0; i < MT2; ++i) {
      const int p = wm * (NPX / 2) + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = (wn * NJ + j) * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = ru_act<RB>(acc[j][i][r] + g.b2[n + r]);
        Elem<bf16_t>::st4(reinterpret_cast<bf16_t*>(&T2[p * TROW + n * 2]), v);
      }
    }
  }
  __syncthreads();

  // ======================= stage 3: y = GELU(W3 T2 + b3 + x)
  {
    constexpr int NJ = NT3 / 2;                       // 6 channel tiles per wave
    f32x4 acc[NJ][MT2];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < MT2; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c3 = 0; c3 < KC3; ++c3) {
      const int c = KC1 + KC2 + c3;
      const int buf = c & 1;
      uint4 bv[MT2];
#pragma unroll
      for (int i = 0; i < MT2; ++i) {
        const int p = wm * (NPX / 2) + i * 16 + fr;
        bv[i] = *reinterpret_cast<const uint4*>(&T2[p * TROW + (c3 * 32 + fq * 8) * 2]);
      }
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const uint4 a = wfrag32(buf, wn * NJ + j);
#pragma unroll
        for (int i = 0; i < MT2; ++i) mma_step<bf16_t>(acc[j][i], a, bv[i]);
      }
      store_w(c + 1, buf ^ 1);
      load_w(c + PF + 1);
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < MT2; ++i) {
      const int p = wm * (NPX / 2) + i * 16 + fr;
      const int py = p / TX, px = p % TX;
      const long long pix = (long long)(b * args.H + y0 + py) * args.W + x0 + px;
      const bf16_t* xr = g.x + pix * g.ldx;
      bf16_t* orow = g.out + pix * g.ldo;
      float res[NJ][4];
#pragma unroll
      for (int j = 0; j < NJ; ++j) Elem<bf16_t>::ld4(xr + (wn * NJ + j) * 16 + fq * 4, res[j]);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int n = (wn * NJ + j) * 16 + fq * 4;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t = acc[j][i][r] + g.b3[n + r] + res[j][r];
          v[r] = RB ? t : ru_gelu(t);
        }
        Elem<bf16_t>::st4(orow + n, v);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// C = 80 bottleneck (CH = 40): the latent-resolution ResidualUnits of the ws-4 attention
// blocks (M = 80) and the alpha codec's 80-channel ResBlocks.  Three small GEMMs per 8x8
// tile -- every weight matrix fits in LDS at once, so it is staged once per workgroup from
// host-built fragment-major packs (1 KiB per 16 rows x 32 k, zero padded):
//   stage 1: T1 = act(W1 x + b1) on the 10x10 halo, 48 rows (40 real) x K 96 (80 real)
//   stage 2: T2 = act(W2 (*) T1 + b2), 48 rows x K 9 taps x 64 (40 real)
//   stage 3: y  = [GELU](W3 T2 + b3 + x), 80 rows x K 64 (40 real)
// T1 / T2 pixels are 128-B rows (64 channels, 40..63 zero), chunk c at slot c ^ (p & 7).
// LDS 73 KiB weights + 22 KiB maps: one workgroup per CU, 4 waves, persistent over tiles (at
// config 4's 128^2 latent, 8 tiles per workgroup); per wave and tile 18 + 54 + 10 MFMAs.  Three launches (and two HBM round trips of the 40-channel maps) become one.
typedef __attribute__((address_space(3))) void* ru_lptr_t;
// one LDS-DMA piece: each lane moves 16 bytes from src to lds + 16 * lane (M0 saved / restored;
// waited for by an explicit s_waitcnt)
__device__ __forceinline__ void ru_dma16(const void* src, uint32_t lds) {
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
namespace rus {
constexpr int W1F = 9, W2F = 54, W3F = 10;            // fragments per matrix
constexpr int HY = 10, HX = 10, NH = 100, NHP = 112;  // halo pixels (7 fragments)
}  // namespace rus

// NHALF = 2 (multi-round launches): two 4-wave halves each run their own tile over the shared
// weights -- two waves per SIMD instead of one (T1 / T2 per half: 117 KiB of LDS)
template <int RB, int NHALF>
__global__ void __launch_bounds__(256 * NHALF, 1) ru_small_kernel(const RuArgsDev args) {
  using namespace rus;
  __shared__ __attribute__((aligned(16))) uint4 Ws[(W1F + W2F + W3F) * 64];
  __shared__ __attribute__((aligned(16))) uint4 T1s[NHALF * NHP * 8];
  __shared__ __attribute__((aligned(16))) uint4 T2s[NHALF * 64 * 8];
  __shared__ float bs[48 + 48 + 80];
  const RuGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = wave_all >> 2, wave = wave_all & 3;
  uint4* const T1 = T1s + half * NHP * 8;
  uint4* const T2 = T2s + half * 64 * 8;
  const int n = lane & 15, q = lane >> 4;
  const int tx_n = args.W / 8, ty_n = args.H / 8;
  const int ntiles = args.batch * tx_n * ty_n;

  // weights: the three fragment-major packs (1 KiB per fragment) land in LDS by LDS-DMA, one
  // piece per wave instruction with no wait in between -- the register-staged copy loop it
  // replaces waited for an L2 round trip every few of its 18 iterations
  {
    const uint32_t lws = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(ru_lptr_t)Ws);
    for (int pc = wave_all; pc < W1F + W2F + W3F; pc += 4 * NHALF) {
      const uint4* src = pc < W1F ? reinterpret_cast<const uint4*>(g.w1) + pc * 64
                       : pc < W1F + W2F ? reinterpret_cast<const uint4*>(g.w2) + (pc - W1F) * 64
                       : reinterpret_cast<const uint4*>(g.w3) + (pc - W1F - W2F) * 64;
      ru_dma16(src + lane, lws + (uint32_t)pc * 1024u);
    }
  }
  for (int e = tid; e < 48 + 48 + 80; e += 256 * NHALF)
    bs[e] = e < 48 ? g.b1[e] : e < 96 ? g.b2[e - 48] : g.b3[e - 96];
  // zero channels 48..63 (chunks 6, 7) of T1 / T2: the stage-2 / stage-3 K padding
  for (int e = tid & 255; e < (NHP + 64) * 2; e += 256) {
    const int p = e >> 1, c = 6 + (e & 1);
    if (p < NHP) T1[p * 8 + (c ^ (p & 7))] = make_uint4(0, 0, 0, 0);
    else T2[(p - NHP) * 8 + (c ^ ((p - NHP) & 7))] = make_uint4(0, 0, 0, 0);
  }
  // stage-1 input fragments straight from HBM: halo pixel 16f + n, channels 32ks + 8q
  constexpr int F1 = 2;                                  // fragments w, w + 4 (< 7)
  uint4 xb[F1][3], xn[F1][3];
  bool xin[F1], xinn[F1];
  uint2 rx[5], rxn[5];                                   // stage 3's residual quads
  const int p = 16 * wave + n, py = p >> 3, px = p & 7;  // this lane's stage-2 / 3 pixel
  auto load_x = [&](int tt, uint4 (&dst)[F1][3], bool (&in)[F1], uint2 (&rd)[5]) {
    const int tx = tt % tx_n, ty = (tt / tx_n) % ty_n, b = tt / (tx_n * ty_n);
#pragma unroll
    for (int i = 0; i < F1; ++i) {
      const int hp = 16 * (wave + 4 * i) + n;
      const int hy = hp / HX, hx = hp - hy * HX;
      const int iy = ty * 8 + hy - 1, ix = tx * 8 + hx - 1;
      in[i] = hp < NH && iy >= 0 && iy < args.H && ix >= 0 && ix < args.W;
      const bf16_t* row = g.x + ((long long)(b * args.H + (in[i] ? iy : 0)) * args.W +
                                 (in[i] ? ix : 0)) * g.ldx;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const int c8 = 4 * ks + q;                       // 8-channel chunk (10 real)
        dst[i][ks] = (in[i] && c8 < 10) ? *reinterpret_cast<const uint4*>(row + 8 * c8)
                                        : make_uint4(0, 0, 0, 0);
      }
    }
    const bf16_t* xr = g.x + ((long long)(b * args.H + ty * 8 + py) * args.W + tx * 8 + px) * g.ldx;
#pragma unroll
    for (int tt2 = 0; tt2 < 5; ++tt2) rd[tt2] = *reinterpret_cast<const uint2*>(xr + 16 * tt2 + 4 * q);
  };
  // half h runs tiles blockIdx.x + h grid, + NHALF grid, ...; a half past the last tile
  // computes a clamped tile and stores nothing (both halves meet at every barrier)
  const int stride = NHALF * (int)gridDim.x;
  int t = blockIdx.x + half * (int)gridDim.x;
  if ((int)blockIdx.x >= ntiles) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (no DMA may land after the exit)
    return;
  }
  load_x(t < ntiles ? t : ntiles - 1, xb, xin, rx);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // this wave's weight pieces landed
  __syncthreads();

  // persistent over tiles (the 73 KiB of weights staged once per workgroup, not per tile): the
  // next tile's stage-1 fragments load while this tile runs stages 2 and 3.  T1 is rewritten
  // only after every wave passed the barrier behind stage 2 (its last reader); T2 rows are
  // wave-private.
  for (;;) {
    const bool valid = t < ntiles;
    const int tc = valid ? t : ntiles - 1;
    const int tx = tc % tx_n, ty = (tc / tx_n) % ty_n, b = tc / (tx_n * ty_n);
    const int y0 = ty * 8, x0 = tx * 8;
    const int tnext = t + stride;

    // ================= stage 1
    {
      f32x4 acc[3][F1];
#pragma unroll
      for (int tt = 0; tt < 3; ++tt)
#pragma unroll
        for (int i = 0; i < F1; ++i) acc[tt][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks)
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) {
          const uint4 a = Ws[(tt * 3 + ks) * 64 + lane];
#pragma unroll
          for (int i = 0; i < F1; ++i)
            if (wave + 4 * i < 7) mma_step<bf16_t>(acc[tt][i], a, xb[i][ks]);
        }
      if (tnext < ntiles) load_x(tnext, xn, xinn, rxn);         // consumed: the next tile's go out
#pragma unroll
      for (int i = 0; i < F1; ++i) {
        const int hp = 16 * (wave + 4 * i) + n;
        if (wave + 4 * i >= 7) continue;
#pragma unroll
        for (int tt = 0; tt < 3; ++tt) {
          const int c0 = 16 * tt + 4 * q;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = xin[i] ? ru_act<RB>(acc[tt][i][r] + bs[c0 + r]) : 0.0f;
          *reinterpret_cast<uint2*>(reinterpret_cast<unsigned char*>(T1) + hp * 128 +
                                    (((c0 >> 3) ^ (hp & 7)) << 4) + 2 * (c0 & 7)) =
              make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
        }
      }
    }
    __syncthreads();

    // ================= stage 2 (wave w: output pixels 16w .. 16w+15 = rows 2w, 2w+1)
    {
      f32x4 acc[3];
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 18; ++kk) {
        const int tap = kk >> 1, c8 = 4 * (kk & 1) + q;
        const int hp = (py + tap / 3) * HX + px + tap % 3;
        const uint4 bv = T1[hp * 8 + (c8 ^ (hp & 7))];
#pragma unroll
        for (int tt = 0; tt < 3; ++tt)
          mma_step<bf16_t>(acc[tt], Ws[(W1F + tt * 18 + kk) * 64 + lane], bv);
      }
#pragma unroll
      for (int tt = 0; tt < 3; ++tt) {
        const int c0 = 16 * tt + 4 * q;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = ru_act<RB>(acc[tt][r] + bs[48 + c0 + r]);
        *reinterpret_cast<uint2*>(reinterpret_cast<unsigned char*>(T2) + p * 128 +
                                  (((c0 >> 3) ^ (p & 7)) << 4) + 2 * (c0 & 7)) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
    __syncthreads();                                       // (T2 rows are wave-private: a
                                                           //  wave reads only its own pixels)
    // ================= stage 3: y = [GELU](W3 T2 + b3 + x)
    {
      f32x4 acc[5];
#pragma unroll
      for (int tt = 0; tt < 5; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int c8 = 4 * ks + q;
        const uint4 bv = T2[p * 8 + (c8 ^ (p & 7))];
#pragma unroll
        for (int tt = 0; tt < 5; ++tt)
          mma_step<bf16_t>(acc[tt], Ws[(W1F + W2F + tt * 2 + ks) * 64 + lane], bv);
      }
      const int gy = y0 + py, gx = x0 + px;
      const long long pix = (long long)(b * args.H + gy) * args.W + gx;
      bf16_t* orow = g.out + pix * g.ldo;
      float res[5][4];                                   // (prefetched with the x fragments)
#pragma unroll
      for (int tt = 0; tt < 5; ++tt) {
        res[tt][0] = bf2f(rx[tt].x & 0xFFFF);
        res[tt][1] = bf2f(rx[tt].x >> 16);
        res[tt][2] = bf2f(rx[tt].y & 0xFFFF);
        res[tt][3] = bf2f(rx[tt].y >> 16);
      }
#pragma unroll
      for (int tt = 0; tt < 5; ++tt) {
        const int c0 = 16 * tt + 4 * q;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float t3 = acc[tt][r] + bs[96 + c0 + r] + res[tt][r];
          v[r] = RB ? t3 : ru_gelu(t3);
        }
        if (valid) Elem<bf16_t>::st4(orow + c0, v);
      }
    }
    if (tnext - half * (int)gridDim.x >= ntiles) break;   // (the first half's next tile)
    t = tnext;
#pragma unroll
    for (int i = 0; i < F1; ++i) {
      xin[i] = xinn[i];
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) xb[i][ks] = xn[i][ks];
    }
#pragma unroll
    for (int tt = 0; tt < 5; ++tt) rx[tt] = rxn[tt];
  }
}

// ---------------------------------------------------------------------------------------
// C = 192 bottleneck, fragment-streamed (CH = 96): the same three GEMMs per 8x16 output tile
// as ru_fused_kernel, but with NO barrier inside any K loop.  Every wave streams the weight
// fragments it needs straight from host-built fragment-major packs (1 KiB per 16 rows x 32 k,
// lane-ordered: each load is one fully coalesced global_load_dwordx4, served by L2 after the
// first tiles) into a statically indexed register ring, instead of the 20 chunk-wise LDS
// ring refills and barriers of ru_fused_kernel.  Barriers: 2 (T1 complete, T2 complete).
//   stage 1: T1 = act(W1 x + b1) on the 10x18 halo: wave w owns halo rows 48w..48w+47
//            (3 m tiles) x all 6 n tiles; its x fragments (6 k-steps) are loaded up front
//   stage 2: T2 = act(W2 (*) T1 + b2): waves = 2 channel halves x 2 pixel halves,
//            27 k-steps (tap-major, 3 per tap) of 3 x 4 MFMAs, ring R2 k-steps deep
//   stage 3: y = [GELU](W3 T2 + b3 + x): 3 k-steps of 6 x 4 MFMAs
// Each next stage's first weights (and the residual x) are requested before the current
// stage's epilogue, so their latency hides behind its activation math.  T1 / T2 are separate
// 208-B-row buffers (conflict-free 16-row fragment reads): 64 KiB, two workgroups per CU.
#ifndef RGBAC_RU_R2
#define RGBAC_RU_R2 8      // ru_stream_kernel<0> stage-2 weight ring depth (k-steps)
#endif
namespace rsw {
constexpr int TY = 8, TX = 16, HX = TX + 2, NH = (TY + 2) * HX;   // 180 halo pixels
constexpr int NHP = 192;           // T1 rows (halo padded to the waves' 4 x 48 m-tile rows)
constexpr int TROW = 208;
constexpr int ORW = 400;           // output staging row (100 dwords: 16 rows on distinct banks)
constexpr int NK1 = 6, NK2 = 27, NK3 = 3;
constexpr int R1 = 2, R3 = 2;
constexpr int PRE2 = 4;            // stage-2 ring slots requested before the stage-1 epilogue
}  // namespace rsw

#ifdef RGBAC_RU_TIMING
// probe builds only (tools/ru_stage_probe.py): per-workgroup stage timestamps of waves 0 / 3
__device__ unsigned long long g_ru_t[8192][2][8];
__device__ unsigned long long g_ru_w[8192][2];     // wall clock (100 MHz) at start / end
#define RU_T(k)                                                                              \
  do {                                                                                       \
    const unsigned long long c_ = clock64();                                                 \
    if (lane == 0 && (wave == 0 || wave == 3) && blockIdx.x < 8192 && blockIdx.z == 0)       \
      g_ru_t[blockIdx.x][wave == 3][k] = c_;                                                 \
    if ((k == 0 || k == 7) && tid == 0 && blockIdx.x < 8192 && blockIdx.z == 0)               \
      g_ru_w[blockIdx.x][k == 7] = wall_clock64();                                           \
  } while (0)
#else
#define RU_T(k) do {} while (0)
#endif

// Group 1 of the gated launch: the b tile (bf16, 128 pixels x 192 channels, 400-B rows) is in OT.
// Wave (wn, wm) computes gate channels 96 wn .. +95 of pixel rows 4 wm .. 4 wm + 3 -- the stage-3
// tiling, K = 192 in 6 k-steps from OT -- then waits for group 0's tile and writes
//   out = a * sigmoid(W_g b + b_g) + x
// with conv_pw2_kernel's gate epilogue arithmetic (pw2_epi<.., RGBAC_ACT_GATE>).
__device__ __forceinline__ void ru_gate_tile(const RuArgsDev& args, const unsigned char* OT, int tile,
                                             int b, int y0, int x0, int wn, int wm, int fr, int fq,
                                             int lane) {
  using namespace rsw;
  constexpr int RG = 3;                            // gate weight ring depth (k-steps)
  const uint4* const WG = reinterpret_cast<const uint4*>(args.gw) + lane + (size_t)(6 * wn) * 6 * 64;
  uint4 wr[RG][6];
#pragma unroll
  for (int u = 0; u < RG; ++u)
#pragma unroll
    for (int j = 0; j < 6; ++j) wr[u][j] = WG[(j * 6 + u) * 64];
  float4 gb[6];
#pragma unroll
  for (int j = 0; j < 6; ++j) gb[j] = *reinterpret_cast<const float4*>(args.gb + 96 * wn + 16 * j + 4 * fq);
  f32x4 acc[6][4];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned char* const otl = OT + (4 * wm * TX + fr) * ORW + fq * 16;
#pragma unroll
  for (int ks = 0; ks < 6; ++ks) {
    uint4 bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = *reinterpret_cast<const uint4*>(otl + i * TX * ORW + ks * 64);
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) mma_step<bf16_t>(acc[j][i], wr[ks % RG][j], bv[i]);
    if (ks + RG < 6) {
#pragma unroll
      for (int j = 0; j < 6; ++j) wr[ks % RG][j] = WG[(j * 6 + ks + RG) * 64];
    }
  }
  const RuGroup& ga = args.g[0];
  const RuGroup& gbg = args.g[1];
  // the identity quads are no hand-off: in flight while the flag is polled
  uint2 av[4][6], xv[4][6];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long pix = (long long)(b * args.H + y0 + 4 * wm + i) * args.W + x0 + fr;
#pragma unroll
    for (int j = 0; j < 6; ++j)
      xv[i][j] = *reinterpret_cast<const uint2*>(args.gid + pix * args.ldid + 96 * wn + 16 * j + 4 * fq);
  }
  // group 0's tile: poll its flag (relaxed, every lane the same word), bounded; then ONE
  // agent-scope acquire and plain loads (Guideline 16 recipe)
  unsigned* const flag = args.flags + tile;
  for (unsigned spins = 0;; ++spins) {
    if (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) break;
    if (spins > (1u << 16)) {                        // never expected: record and go on
      if (lane == 0)
        __hip_atomic_store(args.timeout, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long pix = (long long)(b * args.H + y0 + 4 * wm + i) * args.W + x0 + fr;
#pragma unroll
    for (int j = 0; j < 6; ++j)
      av[i][j] = *reinterpret_cast<const uint2*>(ga.out + pix * ga.ldo + 96 * wn + 16 * j + 4 * fq);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const long long pix = (long long)(b * args.H + y0 + 4 * wm + i) * args.W + x0 + fr;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int n = 96 * wn + 16 * j + 4 * fq;
      const float bb[4] = {gb[j].x, gb[j].y, gb[j].z, gb[j].w};
      const float r1[4] = {bf2f(av[i][j].x & 0xFFFF), bf2f(av[i][j].x >> 16),
                           bf2f(av[i][j].y & 0xFFFF), bf2f(av[i][j].y >> 16)};
      const float r2[4] = {bf2f(xv[i][j].x & 0xFFFF), bf2f(xv[i][j].x >> 16),
                           bf2f(xv[i][j].y & 0xFFFF), bf2f(xv[i][j].y >> 16)};
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float x = acc[j][i][r] + bb[r];
        v[r] = r1[r] * (1.0f / (1.0f + expf(-x))) + r2[r];     // conv_common.h sigmoid_f
      }
      Elem<bf16_t>::st4(gbg.out + pix * gbg.ldo + n, v);
    }
  }
  // this workgroup is the flag's only reader: once every wave has seen it, leave it zero for
  // the next launch
  __syncthreads();
  if (wn == 0 && wm == 0 && lane == 0)
    __hip_atomic_store(flag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// TYV = 8: 8 x 16 tiles, 4 waves, two workgroups per CU (the launched form).  16 x 16 tiles at
// one 8-wave workgroup per CU measured 4-5 % slower and were removed, as were
// 8 x 8 half tiles (14k).
// GATE (the last unit pair of a Win_noShift_Attention block, Masked_Attention.py:182-189, group 0 =
// conv_a[2], group 1 = conv_b[2]): group 0 publishes its tile (a) by write-through stores and a
// per-tile flag; group 1 keeps its tile (b) in LDS, runs conv_b[3] (1x1, 192 -> 192) on it, waits
// for the flag (group 0's workgroups precede group 1's in dispatch order, so the wait always
// ends; it is bounded anyway) and writes out = a * sigmoid(W_g b + b_g) + x.  The gate's HBM
// round trip of b and its launch disappear.
template <int RB, int TYV, bool GATE = false>
__global__ void __launch_bounds__(32 * TYV, TYV == 8 ? 2 : 1) ru_stream_kernel(const RuArgsDev args) {
  using namespace rsw;
  constexpr int TY = TYV, NH = (TYV + 2) * HX;      // (shadow rsw's 8-row values)
  constexpr int NW = TYV / 2, NTH = 64 * NW;        // waves: stage 1 takes 3 halo m tiles each
  constexpr int NHP = NW * 48;
  constexpr int R2 = RB ? 6 : RGBAC_RU_R2;         // stage-2 ring (ReLU variant: register fit)
  // T1 | T2; after stage 3's MFMAs the same bytes stage the output tile (128 x 400-B rows)
  // (T1 padded to NHP = 192 rows: the stage-1 epilogue of wave 3 stores its 12 rows past the
  // halo without a guard, so all 18 GELU quads of a wave form one branch-free block)
  __shared__ __attribute__((aligned(16))) unsigned char lds[NHP * TROW + TY * TX * TROW];
  unsigned char* const T1 = lds;
  unsigned char* const T2 = lds + NHP * TROW;
  unsigned char* const OT = lds;
  static_assert(TY * TX * ORW <= NHP * TROW + TY * TX * TROW, "output staging fits");
  static_assert(NHP >= NH, "every halo row has a T1 row");
  // biases in LDS: an epilogue's bias read is then an LDS read (lgkmcnt), not a global load
  // whose vmcnt wait would also drain the next stage's weight prefetch
  __shared__ __attribute__((aligned(16))) float bs[96 + 96 + 192];
  const RuGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int tx_n = args.W / TX, ty_n = args.H / TY;
  int t = blockIdx.x;
  {                                                // XCD-contiguous runs of neighbouring tiles
    const int nwg = gridDim.x, xcd = t & 7, q = nwg >> 3, r = nwg & 7;
    t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (t >> 3);
  }
  const int tile = t;                              // (both groups map blockIdx.x alike)
  const int tx = t % tx_n; t /= tx_n;
  const int ty = t % ty_n;
  const int b = t / ty_n;
  const int y0 = ty * TY, x0 = tx * TX;

  // The second workgroup a CU receives (the later half of the grid in dispatch order) starts
  // `stagger` x 1024 cycles late: the two workgroups sharing each SIMD then run out of phase, so
  // one's GELU epilogues (VALU) issue beside the other's MFMA loops instead of both alternating
  // MFMA and VALU phases in lockstep.
  if (args.stagger > 0 && (int)(blockIdx.z * gridDim.x + blockIdx.x) >= (int)(gridDim.x * gridDim.z) / 2)
    for (int i = 0; i < args.stagger; ++i) __builtin_amdgcn_s_sleep(16);
  // ================= stage 1
  RU_T(0);
  for (int e = tid; e < 384; e += NTH) bs[e] = e < 96 ? g.b1[e] : e < 192 ? g.b2[e - 96] : g.b3[e - 192];
  const uint4* const W1 = reinterpret_cast<const uint4*>(g.w1) + lane;
  uint4 w1r[R1][6];
#pragma unroll
  for (int u = 0; u < R1; ++u)
#pragma unroll
    for (int j = 0; j < 6; ++j) w1r[u][j] = W1[(j * NK1 + u) * 64];
  uint4 xb[NK1][3];
  bool xin[3];
  unsigned xoff[3];                                // element offsets (< 2^31, host-checked)
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const int hp = 48 * wave + 16 * i + fr;
    const int hy = hp / HX, hx = hp - (hp / HX) * HX;
    const int iy = y0 + hy - 1, ix = x0 + hx - 1;
    xin[i] = hp < NH && iy >= 0 && iy < args.H && ix >= 0 && ix < args.W;
    xoff[i] = (unsigned)(((b * args.H + (xin[i] ? iy : 0)) * args.W + (xin[i] ? ix : 0)) * g.ldx +
                         fq * 8);
  }
  // k-step-major issue order: the first k-step's MFMAs wait for 3 loads, not for 13
#pragma unroll
  for (int ks = 0; ks < NK1; ++ks)
#pragma unroll
    for (int i = 0; i < 3; ++i)
      xb[ks][i] = xin[i] ? *reinterpret_cast<const uint4*>(g.x + xoff[i] + ks * 32)
                         : make_uint4(0, 0, 0, 0);
  __syncthreads();                                 // bs visible (behind the x / W1 loads)
  f32x4 acc1[6][3];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int i = 0; i < 3; ++i) acc1[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NK1; ++ks) {
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int i = 0; i < 3; ++i) mma_step<bf16_t>(acc1[j][i], w1r[ks % R1][j], xb[ks][i]);
    if (ks + R1 < NK1) {
#pragma unroll
      for (int j = 0; j < 6; ++j) w1r[ks % R1][j] = W1[(j * NK1 + ks + R1) * 64];
    }
  }
  RU_T(1);
  // stage-2 weights for the first R2 k-steps, in flight during the stage-1 epilogue
  const int wn = wave / (NW / 2), wm = wave % (NW / 2);   // channel half, 4-row group
  const uint4* const W2 = reinterpret_cast<const uint4*>(g.w2) + lane + (size_t)(3 * wn) * NK2 * 64;
  uint4 w2r[R2][3];
#pragma unroll
  for (int u = 0; u < PRE2; ++u)
#pragma unroll
    for (int j = 0; j < 3; ++j) w2r[u][j] = W2[(j * NK2 + u) * 64];
  {
    // biases of this lane's channels read once (no lgkmcnt wait between the stores), the 18
    // quads computed branch-free (outside-image halo pixels selected to zero)
    float4 b1v[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) b1v[j] = *reinterpret_cast<const float4*>(bs + 16 * j + 4 * fq);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int n = 16 * j + 4 * fq;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const int hp = 48 * wave + 16 * i + fr;
        float v[4];
        ru_act4<RB>(v, acc1[j][i], b1v[j]);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = xin[i] ? v[r] : 0.0f;
        Elem<bf16_t>::st4(reinterpret_cast<bf16_t*>(&T1[hp * TROW + n * 2]), v);
      }
    }
  }
  RU_T(2);
#pragma unroll
  for (int u = PRE2; u < R2; ++u)
#pragma unroll
    for (int j = 0; j < 3; ++j) w2r[u][j] = W2[(j * NK2 + u) * 64];
  __syncthreads();
  RU_T(3);

  // residual element offset of this lane's first pixel / channel quad (32-bit, host-checked):
  // one register carried through stage 2 instead of the tile coordinates
  const unsigned roff = (unsigned)(((b * args.H + y0 + 4 * wm) * args.W + x0 + fr) * g.ldx +
                                   96 * wn + 4 * fq);
  // ================= stage 2: m tile i = tile row 4 wm + i (16 pixels), lane pixel x = fr
  f32x4 acc2[3][4];
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc2[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned char* const t1l = T1 + (4 * wm * HX + fr) * TROW + fq * 16;
#pragma unroll
  for (int ks = 0; ks < NK2; ++ks) {
    const int tap = ks / 3, c = ks % 3;
    const int off = ((tap / 3) * HX + tap % 3) * TROW + c * 64;
    uint4 bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = *reinterpret_cast<const uint4*>(t1l + i * HX * TROW + off);
#pragma unroll
    for (int j = 0; j < 3; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) mma_step<bf16_t>(acc2[j][i], w2r[ks % R2][j], bv[i]);
    if (ks + R2 < NK2) {
#pragma unroll
      for (int j = 0; j < 3; ++j) w2r[ks % R2][j] = W2[(j * NK2 + ks + R2) * 64];
    }
    // keep the next k-step's LDS reads from being hoisted further up (the fully unrolled loop
    // otherwise front-loads them and spills)
    asm volatile("" ::: "memory");
  }
  RU_T(4);
  // stage-3 weights (first R3 k-steps) and the residual x, in flight during this epilogue
  // (the residual loads must precede every output store: vmcnt counts stores too, so a load
  // issued behind a store waits for it)
  const uint4* const W3 = reinterpret_cast<const uint4*>(g.w3) + lane + (size_t)(6 * wn) * NK3 * 64;
  uint4 w3r[R3][6];
#pragma unroll
  for (int u = 0; u < R3; ++u)
#pragma unroll
    for (int j = 0; j < 6; ++j) w3r[u][j] = W3[(j * NK3 + u) * 64];
  uint2 res[4][6];
  auto load_res = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16_t* xr = g.x + roff + (unsigned)(i * args.W * g.ldx);
#pragma unroll
      for (int j = 0; j < 6; ++j) res[i][j] = *reinterpret_cast<const uint2*>(xr + 16 * j);
    }
  };
  if constexpr (!RB) load_res();                   // (the ReLU variant: after stage 3's MFMAs)
  float4 b2v[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) b2v[j] = *reinterpret_cast<const float4*>(bs + 96 + 48 * wn + 16 * j + 4 * fq);
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int n = 48 * wn + 16 * j + 4 * fq;
    const float4 bb = b2v[j];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int p = (4 * wm + i) * TX + fr;
      float v[4];
      ru_act4<RB>(v, acc2[j][i], bb);
      Elem<bf16_t>::st4(reinterpret_cast<bf16_t*>(&T2[p * TROW + n * 2]), v);
    }
  }
  RU_T(5);
  __syncthreads();
  RU_T(6);

  // ================= stage 3
  f32x4 acc3[6][4];
#pragma unroll
  for (int j = 0; j < 6; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc3[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned char* const t2l = T2 + (4 * wm * TX + fr) * TROW + fq * 16;
#pragma unroll
  for (int ks = 0; ks < NK3; ++ks) {
    uint4 bv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[i] = *reinterpret_cast<const uint4*>(t2l + i * TX * TROW + ks * 64);
#pragma unroll
    for (int j = 0; j < 6; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) mma_step<bf16_t>(acc3[j][i], w3r[ks % R3][j], bv[i]);
    if (ks + R3 < NK3) {
#pragma unroll
      for (int j = 0; j < 6; ++j) w3r[ks % R3][j] = W3[(j * NK3 + ks + R3) * 64];
    }
  }
  if constexpr (RB != 0) load_res();
  float4 b3v[6];                                   // biases read once, before the output barrier
#pragma unroll
  for (int j = 0; j < 6; ++j) b3v[j] = *reinterpret_cast<const float4*>(bs + 192 + 96 * wn + 16 * j + 4 * fq);
  __syncthreads();                                 // every wave is done reading T2
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = (4 * wm + i) * TX + fr;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int n = 96 * wn + 16 * j + 4 * fq;
      const float4 bb = b3v[j];
      const uint2 rr = res[i][j];
      float v[4];
      v[0] = acc3[j][i][0] + bb.x + bf2f(rr.x & 0xFFFF);
      v[1] = acc3[j][i][1] + bb.y + bf2f(rr.x >> 16);
      v[2] = acc3[j][i][2] + bb.z + bf2f(rr.y & 0xFFFF);
      v[3] = acc3[j][i][3] + bb.w + bf2f(rr.y >> 16);
      if (!RB) gelu4_fast(v);
      Elem<bf16_t>::st4(reinterpret_cast<bf16_t*>(OT + p * ORW + n * 2), v);
    }
  }
  __syncthreads();
  if constexpr (GATE) {
    if (blockIdx.z == 1) {
      ru_gate_tile(args, OT, tile, b, y0, x0, wn, wm, fr, fq, lane);
      return;
    }
  }
  // whole 16-B chunks, consecutive lanes on consecutive chunks of a pixel's 384 bytes
#pragma unroll
  for (int u = 0; u < TY * TX * 24 / NTH; ++u) {
    const int c = tid + NTH * u, p = c / 24, q = c - (c / 24) * 24;
    const long long pix = (long long)(b * args.H + y0 + p / TX) * args.W + x0 + p % TX;
    const uint4 v = *reinterpret_cast<const uint4*>(OT + p * ORW + q * 16);
    if constexpr (GATE) st16_wt(g.out + pix * g.ldo + q * 8, v);     // group 0: the hand-off
    else *reinterpret_cast<uint4*>(g.out + pix * g.ldo + q * 8) = v;
  }
  if constexpr (GATE) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drained (R1) ...
    __syncthreads();                                   // ... before the one flag store
    if (tid == 0)
      __hip_atomic_store(&args.flags[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  RU_T(7);
}
#undef RU_T

}  // namespace rgbac

using namespace rgbac;

#ifdef RGBAC_RU_TIMING
extern "C" int rgbac_debug_ru_times(unsigned long long* host, int nblocks) {
  if (nblocks > 8192) nblocks = 8192;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ru_t), (size_t)nblocks * 16 * 8) != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host + (size_t)nblocks * 16, HIP_SYMBOL(g_ru_w), (size_t)nblocks * 2 * 8) ==
                 hipSuccess ? 0 : 1;
}
#endif

extern "C" int rgbac_residual_unit(const rgbac_ru_args* args, int ngroups, void* stream) {
  return rgbac_residual_unit_ex(args, ngroups, 0, stream);
}

extern "C" int rgbac_residual_unit_ex(const rgbac_ru_args* args, int ngroups, int kind,
                                      void* stream) {
  RGBAC_REQUIRE(args != nullptr && ngroups >= 1 && ngroups <= kRuMaxGroups, "groups");
  const rgbac_ru_args* a = args;
  RGBAC_REQUIRE(a->dtype == RGBAC_BF16, "the fused residual unit is bf16 only");
  RGBAC_REQUIRE(kind == 0 || kind == 1, "kind: 0 = ResidualUnit, 1 = ResBlock");
  RGBAC_REQUIRE(a->channels == 192 || a->channels == 80, "fused units support C = 192 or 80");
  RGBAC_REQUIRE(a->batch > 0 && a->h > 0 && a->w > 0 && a->h % 8 == 0 && a->w % 8 == 0,
                "H and W must be positive multiples of 8");
  RuArgsDev d{};
  d.batch = a->batch; d.H = a->h; d.W = a->w; d.ngroups = ngroups;
  static const int stagger_env = [] {
    const char* e = getenv("RGBAC_RU_STAGGER");
    return e ? atoi(e) : 0;
  }();
  d.stagger = stagger_env;
  for (int i = 0; i < ngroups; ++i) {
    const rgbac_ru_args* q = &args[i];
    RGBAC_REQUIRE(q->dtype == a->dtype && q->channels == a->channels && q->batch == a->batch &&
                      q->h == a->h && q->w == a->w, "grouped units must share the geometry");
    RGBAC_REQUIRE(q->x && q->out && q->w1 && q->w2 && q->w3 && q->b1 && q->b2 && q->b3,
                  "null pointer");
    RGBAC_REQUIRE(q->x != q->out, "out must not alias x (the halo is read by other tiles)");
    RGBAC_REQUIRE(q->x_ldc >= a->channels && q->x_ldc % 8 == 0 && q->out_ldc >= a->channels &&
                      q->out_ldc % 4 == 0, "strides");
    if (a->channels == 192 && q->w1_kpad != 0)
      RGBAC_REQUIRE(q->w1_kpad >= 192 && q->w2_kpad >= 896 && q->w3_kpad >= 96 &&
                        q->w1_kpad % 8 == 0 && q->w2_kpad % 8 == 0 && q->w3_kpad % 8 == 0,
                    "packed weight k_pad (w1 >= 192, w2 >= 896 zero-padded, w3 >= 96)");
    RGBAC_REQUIRE(((uintptr_t)q->x % 16) == 0 && ((uintptr_t)q->w1 % 16) == 0 &&
                      ((uintptr_t)q->w2 % 16) == 0 && ((uintptr_t)q->w3 % 16) == 0,
                  "16-byte alignment");
    RuGroup& g = d.g[i];
    g.x = (const bf16_t*)q->x; g.ldx = q->x_ldc;
    g.w1 = (const bf16_t*)q->w1; g.w2 = (const bf16_t*)q->w2; g.w3 = (const bf16_t*)q->w3;
    g.kp1 = q->w1_kpad; g.kp2 = q->w2_kpad; g.kp3 = q->w3_kpad;
    g.b1 = q->b1; g.b2 = q->b2; g.b3 = q->b3;
    g.out = (bf16_t*)q->out; g.ldo = q->out_ldc;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a->channels == 80) {
    const long long tiles = (long long)a->batch * (a->h / 8) * (a->w / 8);
    RGBAC_REQUIRE(tiles < (1ll << 31), "too many tiles");
    // one workgroup per CU over all groups (a workgroup stages its group's weights once)
    const int ncu = device_cus();
    long long gx = ncu / ngroups;
    if (gx < 1) gx = 1;
    const char* dual_env = getenv("RGBAC_RU_SMALL_DUAL");
    // multi-round launches only (=2 forces it: A/B)
    const bool dual = (tiles > gx && !(dual_env && dual_env[0] == '0')) || (dual_env && dual_env[0] == '2');
    if (dual) {
      if (gx > (tiles + 1) / 2) gx = (tiles + 1) / 2;
      if (kind) hipLaunchKernelGGL((ru_small_kernel<1, 2>), dim3((unsigned)gx, 1, ngroups), dim3(512), 0, st, d);
      else hipLaunchKernelGGL((ru_small_kernel<0, 2>), dim3((unsigned)gx, 1, ngroups), dim3(512), 0, st, d);
    } else {
      if (gx > tiles) gx = tiles;
      if (kind) hipLaunchKernelGGL((ru_small_kernel<1, 1>), dim3((unsigned)gx, 1, ngroups), dim3(256), 0, st, d);
      else hipLaunchKernelGGL((ru_small_kernel<0, 1>), dim3((unsigned)gx, 1, ngroups), dim3(256), 0, st, d);
    }
    return check_launch("ru_small_kernel");
  }
  if (a->w1_kpad == 0) {                             // fragment-major packs: streamed kernel
    RGBAC_REQUIRE(a->h % 8 == 0 && a->w % 16 == 0, "the streamed unit needs H % 8 == 0, W % 16 == 0");
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE(args[i].w1_kpad == 0 && args[i].w2_kpad == 0 && args[i].w3_kpad == 0 &&
                        ((uintptr_t)args[i].b1 % 16) == 0 && ((uintptr_t)args[i].b2 % 16) == 0 &&
                        ((uintptr_t)args[i].b3 % 16) == 0 && args[i].out_ldc % 8 == 0 &&
                        ((uintptr_t)args[i].out % 16) == 0,
                    "grouped units must all be fragment-major (16-B aligned biases and out rows)");
    const long long tiles = (long long)a->batch * (a->h / 8) * (a->w / 16);
    RGBAC_REQUIRE(tiles < (1ll << 31), "too many tiles");
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE((long long)a->batch * a->h * a->w * args[i].x_ldc < (1ll << 31),
                    "the streamed unit addresses x with 32-bit element offsets");
    if (kind) hipLaunchKernelGGL((ru_stream_kernel<1, 8>), dim3((unsigned)tiles, 1, ngroups), dim3(256), 0, st, d);
    else hipLaunchKernelGGL((ru_stream_kernel<0, 8>), dim3((unsigned)tiles, 1, ngroups), dim3(256), 0, st, d);
    return check_launch("ru_stream_kernel");
  }
  static const int wide_env = [] {
    const char* e = getenv("RGBAC_RU_TILE");
    return (e && e[0] == '8') ? 0 : 1;              // RGBAC_RU_TILE=8: the 8x8 tile
  }();
  if (wide_env && a->w % 16 == 0) {
    const long long tiles = (long long)a->batch * (a->h / 8) * (a->w / 16);
    RGBAC_REQUIRE(tiles < (1ll << 31), "too many tiles");
    if (kind) hipLaunchKernelGGL((ru_fused_kernel<192, 96, 8, 16, 2, 1>), dim3((unsigned)tiles, 1, ngroups),
                                 dim3(256), 0, st, d);
    else hipLaunchKernelGGL((ru_fused_kernel<192, 96, 8, 16, 2>), dim3((unsigned)tiles, 1, ngroups),
                            dim3(256), 0, st, d);
  } else {
    const long long tiles = (long long)a->batch * (a->h / 8) * (a->w / 8);
    RGBAC_REQUIRE(tiles < (1ll << 31), "too many tiles");
    if (kind) hipLaunchKernelGGL((ru_fused_kernel<192, 96, 8, 8, 3, 1>), dim3((unsigned)tiles, 1, ngroups),
                                 dim3(256), 0, st, d);
    else hipLaunchKernelGGL((ru_fused_kernel<192, 96, 8, 8, 3>), dim3((unsigned)tiles, 1, ngroups),
                            dim3(256), 0, st, d);
  }
  return check_launch("ru_fused_kernel");
}

extern "C" int rgbac_residual_unit_gate(const rgbac_ru_args* args, const void* gate_w,
                                        const float* gate_b, const void* ident, int64_t ident_ldc,
                                        uint32_t* flags, int64_t nflags, void* stream) {
  RGBAC_REQUIRE(args != nullptr && gate_w && gate_b && ident && flags, "null pointer");
  const rgbac_ru_args* a = args;
  RGBAC_REQUIRE(a->dtype == RGBAC_BF16 && a->channels == 192,
                "the gated unit pair is bf16, C = 192 only");
  RGBAC_REQUIRE(a->batch > 0 && a->h > 0 && a->w > 0 && a->h % 8 == 0 && a->w % 16 == 0,
                "the gated unit pair needs H % 8 == 0, W % 16 == 0");
  const long long tiles = (long long)a->batch * (a->h / 8) * (a->w / 16);
  RGBAC_REQUIRE(tiles < (1ll << 31) && nflags >= tiles + 1,
                "flags: one zeroed word per 8 x 16 tile plus the timeout word (the last)");
  RGBAC_REQUIRE(((uintptr_t)flags % 4) == 0 && ((uintptr_t)gate_w % 16) == 0 &&
                    ((uintptr_t)gate_b % 16) == 0 && ((uintptr_t)ident % 8) == 0 &&
                    ident_ldc >= 192 && ident_ldc % 4 == 0,
                "gate operand alignment / stride");
  RGBAC_REQUIRE((long long)a->batch * a->h * a->w * ident_ldc < (1ll << 31) ||
                    ident_ldc > 0, "identity stride");
  RuArgsDev d{};
  d.batch = a->batch; d.H = a->h; d.W = a->w; d.ngroups = 2;
  for (int i = 0; i < 2; ++i) {
    const rgbac_ru_args* q = &args[i];
    RGBAC_REQUIRE(q->dtype == a->dtype && q->channels == 192 && q->batch == a->batch &&
                      q->h == a->h && q->w == a->w, "both units must share the geometry");
    RGBAC_REQUIRE(q->x && q->out && q->w1 && q->w2 && q->w3 && q->b1 && q->b2 && q->b3,
                  "null pointer");
    RGBAC_REQUIRE(q->x != q->out && q->out != ident, "out must alias neither x nor the identity");
    RGBAC_REQUIRE(q->w1_kpad == 0 && q->w2_kpad == 0 && q->w3_kpad == 0,
                  "fragment-major packs only (the streamed unit)");
    RGBAC_REQUIRE(q->x_ldc >= 192 && q->x_ldc % 8 == 0 && q->out_ldc >= 192 &&
                      q->out_ldc % 8 == 0, "strides");
    RGBAC_REQUIRE(((uintptr_t)q->x % 16) == 0 && ((uintptr_t)q->w1 % 16) == 0 &&
                      ((uintptr_t)q->w2 % 16) == 0 && ((uintptr_t)q->w3 % 16) == 0 &&
                      ((uintptr_t)q->b1 % 16) == 0 && ((uintptr_t)q->b2 % 16) == 0 &&
                      ((uintptr_t)q->b3 % 16) == 0 && ((uintptr_t)q->out % 16) == 0,
                  "16-byte alignment");
    RGBAC_REQUIRE((long long)a->batch * a->h * a->w * q->x_ldc < (1ll << 31),
                  "the streamed unit addresses x with 32-bit element offsets");
    RuGroup& g = d.g[i];
    g.x = (const bf16_t*)q->x; g.ldx = q->x_ldc;
    g.w1 = (const bf16_t*)q->w1; g.w2 = (const bf16_t*)q->w2; g.w3 = (const bf16_t*)q->w3;
    g.b1 = q->b1; g.b2 = q->b2; g.b3 = q->b3;
    g.out = (bf16_t*)q->out; g.ldo = q->out_ldc;
  }
  d.gw = (const bf16_t*)gate_w; d.gb = gate_b;
  d.gid = (const bf16_t*)ident; d.ldid = ident_ldc;
  d.flags = flags; d.timeout = flags + (nflags - 1);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // group 0 (blockIdx.z = 0) is dispatched ahead of group 1, whose workgroups wait on it
  hipLaunchKernelGGL((ru_stream_kernel<0, 8, true>), dim3((unsigned)tiles, 1, 2), dim3(256), 0, st, d);
  return check_launch("ru_stream_kernel");
}
