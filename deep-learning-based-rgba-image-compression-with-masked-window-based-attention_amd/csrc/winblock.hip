// Fused masked shifted-window attention block, bf16, ws 8, C 192, 8 heads of 24
// (reference: layers/masked_win_attention.py:96-131 WindowAttention.forward and :169-251
// WinBasedAttention.forward; the block of Win_noShift_Attention, layers/Masked_Attention.py).
//
//   out = x + proj( softmax(q k^T * scale + B_rel + M_shift) v )   on windows with any alpha,
//   out = x                                                         on all-transparent windows
//
// One launch replaces three (qkv 1x1 GEMM -> HBM, attention core, proj GEMM + MASKSEL):
// the 576-channel qkv tensor (37.7 MB at 64x64 B8) never leaves the chip.
//
// One workgroup = 2 windows = 128 tokens, 8 waves; wave w owns the 16 tokens 16w..16w+15
// (token tile w & 3 of window w >> 2).  The attention chain runs in REGISTERS: every product
// after the qkv GEMM takes its operand straight from the accumulator of the one before
// (v_mfma_f32_16x16x32_bf16: an accumulator tile holds column lane&15, rows 4(lane>>4)+r, so
// two 16-row tiles side by side are one 32-deep k-step whose k order is permuted the same way
// in both operands of the next product):
//   q^T, k^T = Wq|Wk X^T  (channels x tokens)        v = X Wv^T  (tokens x channels)
//   S^T = K Q^T    per head: ONE k-step (channel tiles (0, 1) or (1, 2) of the pair, the other
//                  head's 8 channels of tile 1 zeroed in q)
//   P^T = softmax over keys (rows: 4 lanes apart, reduced by two permlane swaps; exp2 with
//                  log2 e folded into the q scale and the bias tables)
//   O^T = V^T P^T  (key-tile pairs as k-steps; tile 1's rows masked per head)
//   out^T += Wp O^T every two head pairs (3 k-steps of O^T tile pairs; the proj weights are
//                  packed in that permuted k order on the host)
// Only k^T and v cross waves (the four token tiles of a window share the keys): each wave
// stores its k^T / v fragments to LDS once per head pair (14 KiB per window) and reads the
// window's.  Weights are pre-packed fragment-major (1 KiB per 16 rows x 32 k) and streamed
// into LDS by LDS-DMA one pair ahead, waited on at the pair's barrier (counted vmcnt where a
// younger stream may stay in flight).  Two barriers per head pair (exchange visible /
// exchange free), nine in all.
//
// MFMAs per 16 tokens: 54 x 4 (qkv) + 8 x (4 + 4) (scores, PV) + 36 x 2 (proj) = 352.
//
// LDS (bytes): WQ 54 KiB | WP 36 KiB | K^T [2 win][2 heads][4 key tiles] 16 KiB |
// V^T [2 win][3 channel tiles][2 key pairs] 12 KiB | relative-position bias [table,
// table - 100 (the shift mask folded in)][8 heads][225] fp32 | proj bias -> 136,000 B.
// All fragment images are lane-major (16 B per lane): conflict-free ds_read/write_b128.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace rgbac {

namespace wb {
constexpr int WS = 8, C = 192, HEADS = 8, TOK = 128;
constexpr int WQF = 54;                                // qkv fragments per head pair
constexpr int WPF = 36;                                // proj fragments per two head pairs
constexpr int L_WQ = 0;
constexpr int L_WP = L_WQ + WQF * 1024;                // 55296
constexpr int L_XK = L_WP + WPF * 1024;                // 92160
constexpr int L_XV = L_XK + 2 * 2 * 4 * 1024;          // 108544
constexpr int L_TB = L_XV + 2 * 3 * 2 * 1024;          // 120832: bias [2][8 heads][225]
constexpr int L_BQ = L_TB + 2 * 8 * 225 * 4;           // 135232: bproj[192]
constexpr int LDS = L_BQ + 192 * 4;                    // 136000
constexpr int WQ_W = (WQF + 7) / 8;                    // DMA pieces per wave (7)
constexpr int WP_W = (WPF + 7) / 8;                    // (5)
}  // namespace wb

struct WinBlockArgs {
  int batch, H, W, shift, masked;
  float scale;
  const bf16_t* x; long long ldx;
  const float* alpha;                    // (B, H, W) fp32 when masked
  const bf16_t* wq;                      // [4 pairs][54][64 lanes][8]
  const float* bqkv;                     // [576] (ws 4) | the ws-8 bias pack [5][256]
  const bf16_t* wp;                      // [2 pair pairs][12 m][3 k-steps][64][8] (permuted k)
  const float* bproj;                    // [80] (ws 4) | the ws-8 bias pack (row 0 = bproj)
  const float* table;                    // [49][8] (ws 4) | the ws-8 per-pair pack [4][1024]
  bf16_t* out; long long ldo;
};

__device__ __forceinline__ void wb_dma16(const void* src, uint32_t lds) {
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
__device__ __forceinline__ void wb_wait_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wb_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Reductions over the lane pairs l ^ 16 and l ^ 32 without an LDS round trip
// (v_permlane16_swap / v_permlane32_swap, gfx950): with the same value in both operands, the
// two results hold the pair's two values in the same order on both lanes, so op(r0, r1) is the
// pair's reduction, bit-identical on both lanes.
__device__ __forceinline__ float pair16_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float pair16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float pair32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ uint2 pk4(const f32x4& v) {
  return make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
}
__device__ __forceinline__ uint4 cat2(uint2 lo, uint2 hi) { return make_uint4(lo.x, lo.y, hi.x, hi.y); }

#ifdef RGBAC_WB_TIMING
// probe builds only (tools/winblock_stage_probe.py): per-workgroup phase stamps of wave 0
__device__ unsigned long long g_wb_t[8192][18];
__device__ unsigned long long g_wb_w[8192][2];     // wall clock (100 MHz) at start / end
#define WB_T(k)                                                                              \
  do {                                                                                       \
    const unsigned long long c_ = clock64();                                                 \
    if (tid == 0 && blockIdx.x < 8192) g_wb_t[blockIdx.x][k] = c_;                           \
    if (((k) == 0 || (k) == 17) && tid == 0 && blockIdx.x < 8192)                            \
      g_wb_w[blockIdx.x][(k) == 17] = wall_clock64();                                        \
  } while (0)
#else
#define WB_T(k) do {} while (0)
#endif

__global__ void __launch_bounds__(512, 1) winblock_v2_kernel(const WinBlockArgs a) {
  using namespace wb;
  constexpr float LOG2E = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  __shared__ int pix_s[TOK];
  __shared__ int rid_s[TOK];
  __shared__ int act_s[2];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, qq = lane >> 4;
  const int H = a.H, W = a.W, shift = a.shift;
  const int nwx = W / WS, nwy = H / WS;
  const int total = a.batch * nwx * nwy;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) void*)sm;
  const int tok0 = 16 * w;                             // this wave's first token (of 128)
  const int win = w >> 2, tt = w & 3;                  // its window and token tile in it
  WB_T(0);

  // ---- weight streams (pieces past the end repeat the last one: same bytes to the same
  // place, so every wave issues as many)
  auto dma_wq = [&](int p) {
#pragma unroll
    for (int i = 0; i < WQ_W; ++i) {
      int f = w + 8 * i;
      if (f >= WQF) f = WQF - 1;
      wb_dma16(a.wq + ((size_t)(p * WQF + f) * 64 + lane) * 8, lds0 + L_WQ + f * 1024);
    }
  };
  auto dma_wp = [&](int u) {
#pragma unroll
    for (int i = 0; i < WP_W; ++i) {
      int f = w + 8 * i;
      if (f >= WPF) f = WPF - 1;
      wb_dma16(a.wp + ((size_t)(u * WPF + f) * 64 + lane) * 8, lds0 + L_WP + f * 1024);
    }
  };
  // pair 0's qkv weights are requested first thing: they depend on nothing, and the first
  // pair's MFMAs wait for them (the proj weights of pairs 0-1 stream behind pair 0; a
  // workgroup's weight stream, 288 KiB, is what bounds it: every CU pulls its own copy at
  // ~12 B/cycle, MI355X_MICROARCH.md prologue-burst row)
  dma_wq(0);

  // ---- this wave's x tile as MFMA fragments: X[ks] = tokens tok0+n, k-chunk 4ks+qq; the
  // lane's pixel is derived here (the same map as the gather below), so the loads go out
  // before the first barrier instead of behind the alpha gather's round trip
  uint4 X[6];
  {
    const int gw = blockIdx.x * 2 + win;
    int pix = -1;
    if (gw < total) {
      const int b = gw / (nwx * nwy);
      const int rem = gw - b * nwx * nwy;
      const int wy = rem / nwx, wx = rem - wy * nwx;
      const int lt = 16 * tt + n;
      int oy = wy * WS + (lt >> 3) + shift; if (oy >= H) oy -= H;
      int ox = wx * WS + (lt & 7) + shift; if (ox >= W) ox -= W;
      pix = (b * H + oy) * W + ox;
    }
    const bf16_t* row = a.x + (long long)(pix < 0 ? 0 : pix) * a.ldx;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks)
      X[ks] = pix < 0 ? make_uint4(0, 0, 0, 0) : *reinterpret_cast<const uint4*>(row + 32 * ks + 8 * qq);
  }

  // ---- tables (in log2 units: softmax runs on exp2; the host's per-pair pack [var][head][225],
  // the shift mask's -100 folded into var 1) -> [var][8 heads][225]: global reads issued before
  // the gather
  float* tb = reinterpret_cast<float*>(sm + L_TB);
  for (int e = tid; e < 2 * 8 * 225; e += 512) {
    const int var = e >= 8 * 225 ? 1 : 0, rem = e - 8 * 225 * var;
    const int hd = rem / 225, idx = rem - 225 * hd;
    tb[e] = a.table[(hd >> 1) * 1024 + var * 450 + (hd & 1) * 225 + idx];
  }
  float* bq = reinterpret_cast<float*>(sm + L_BQ);
  for (int e = tid; e < 192; e += 512) bq[e] = a.bproj[e];   // the bias pack's row 0

  // ---- window gather: token -> pixel (cyclic shift folded in), shifted-frame region id
  if (tid < 2) act_s[tid] = a.masked ? 0 : 1;
  __syncthreads();
  if (tid < TOK) {
    const int wi = tid >> 6, lt = tid & 63;
    const int gw = blockIdx.x * 2 + wi;
    int pix = -1, rid = 0;
    if (gw < total) {
      const int b = gw / (nwx * nwy);
      const int rem = gw - b * nwx * nwy;
      const int wy = rem / nwx, wx = rem - wy * nwx;
      const int r = wy * WS + (lt >> 3), c = wx * WS + (lt & 7);
      int oy = r + shift; if (oy >= H) oy -= H;
      int ox = c + shift; if (ox >= W) ox -= W;
      pix = (b * H + oy) * W + ox;
      if (a.masked && a.alpha[pix] != 0.0f) act_s[wi] = 1;     // remove_zero_windows (:38-47)
      rid = 3 * (r < H - WS ? 0 : (r < H - shift ? 1 : 2)) + (c < W - WS ? 0 : (c < W - shift ? 1 : 2));
    }
    pix_s[tid] = pix;
    rid_s[tid] = rid;
  }
  __syncthreads();
  const bool act = act_s[win] != 0 && pix_s[tok0] >= 0;         // wave-uniform
  if (act_s[0] == 0 && act_s[1] == 0) {
    // both windows transparent: out = x on their tokens.  The weight DMA issued above lands
    // in this workgroup's LDS: it must complete before the workgroup exits.
    wb_wait_all();
    for (int e = tid; e < TOK * (C / 8); e += 512) {
      const int t = e / (C / 8), c8 = e - t * (C / 8);
      const int pix = pix_s[t];
      if (pix >= 0)
        *reinterpret_cast<uint4*>(a.out + (long long)pix * a.ldo + 8 * c8) =
            *reinterpret_cast<const uint4*>(a.x + (long long)pix * a.ldx + 8 * c8);
    }
    return;
  }

  // ---- per-lane relative-position-bias offsets (head-invariant; +900 h per head), into the
  // "- 100" copy where the shift mask separates query and key:
  // S^T element (kt, r) = (key 16kt+4qq+r, query 16tt+n) of the window
  int toff[4][4];
  {
    const int iq = 16 * tt + n;
    const int qrid = rid_s[64 * win + iq];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int jk = 16 * kt + 4 * qq + r;
        const int idx = ((iq >> 3) - (jk >> 3) + 7) * 15 + ((iq & 7) - (jk & 7) + 7);
        const bool cut = shift > 0 && rid_s[64 * win + jk] != qrid;
        toff[kt][r] = L_TB + (cut ? 8 * 225 * 4 : 0) + idx * 4;
      }
  }

  f32x4 acc[12];                                       // proj output^T: 16-channel tiles
#pragma unroll
  for (int m = 0; m < 12; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  uint2 prevO[3];                                      // O^T of the even pair (packed bf16)
#pragma unroll
  for (int c = 0; c < 3; ++c) prevO[c] = make_uint2(0, 0);

  const float qscale = a.scale * LOG2E;                // q * scale, in log2 units
  const uint32_t lo8 = n < 8 ? 0xFFFFFFFFu : 0u;       // lane holds channel row < 8 of a tile
  const uint32_t qlo = qq < 2 ? 0xFFFFFFFFu : 0u;      // lane's accumulator rows are < 8
  unsigned char* const xk = sm + L_XK + win * 8192;
  unsigned char* const xv = sm + L_XV + win * 6144;
  wb_wait_all();
  __syncthreads();

  for (int p = 0; p < 4; ++p) {
    if (p > 0) {
      if (p == 1) wb_wait_vm<WP_W>();                  // WQ(1) landed (WP(0), issued after it,
      else wb_wait_all();                              //  may be in flight); WQ(p) (+ WP(1))
      __syncthreads();                                 // ... everywhere; exchange free
      if (p == 2) dma_wp(1);                           // proj(0) done in every wave
    }
    WB_T(1 + 4 * p);
    // ================= q^T, k^T, v of heads 2p, 2p+1 for this wave's 16 tokens
    uint4 qf[2];
    if (act) {
      f32x4 aq[3], ak[3], av[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) aq[t] = ak[t] = av[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      float4 bq4[3], bk4[3];
      float bv[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        bq4[t] = *reinterpret_cast<const float4*>(a.bqkv + 256 * (1 + p) + 16 * t + 4 * qq);
        bk4[t] = *reinterpret_cast<const float4*>(a.bqkv + 256 * (1 + p) + 48 + 16 * t + 4 * qq);
        bv[t] = a.bqkv[256 * (1 + p) + 96 + 16 * t + n];
      }
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        uint4 fq[3], fk[3], fv[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          fq[t] = *reinterpret_cast<const uint4*>(sm + L_WQ + (t * 6 + ks) * 1024 + lane * 16);
          fk[t] = *reinterpret_cast<const uint4*>(sm + L_WQ + (18 + t * 6 + ks) * 1024 + lane * 16);
          fv[t] = *reinterpret_cast<const uint4*>(sm + L_WQ + (36 + t * 6 + ks) * 1024 + lane * 16);
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          mma_step<bf16_t>(aq[t], fq[t], X[ks]);
          mma_step<bf16_t>(ak[t], fk[t], X[ks]);
          mma_step<bf16_t>(av[t], X[ks], fv[t]);
        }
      }
      // q^T (x scale), k^T: rows = pair channels 16t + 4qq + r, column = token n
      uint2 q2[3], k2[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        q2[t] = make_uint2(pack_bf16x2((aq[t][0] + bq4[t].x) * qscale, (aq[t][1] + bq4[t].y) * qscale),
                           pack_bf16x2((aq[t][2] + bq4[t].z) * qscale, (aq[t][3] + bq4[t].w) * qscale));
        k2[t] = make_uint2(pack_bf16x2(ak[t][0] + bk4[t].x, ak[t][1] + bk4[t].y),
                           pack_bf16x2(ak[t][2] + bk4[t].z, ak[t][3] + bk4[t].w));
      }
      // head 2p: channels 0..23 = tile 0 + rows 0..7 of tile 1; head 2p+1: rows 8..15 of
      // tile 1 + tile 2.  Zeroing the other head's rows in q alone cuts them from q . k.
      qf[0] = make_uint4(q2[0].x, q2[0].y, q2[1].x & qlo, q2[1].y & qlo);
      qf[1] = make_uint4(q2[1].x & ~qlo, q2[1].y & ~qlo, q2[2].x, q2[2].y);
      // K (keys x channels) fragments of this token tile for both heads
      *reinterpret_cast<uint4*>(xk + (0 * 4 + tt) * 1024 + lane * 16) = cat2(k2[0], k2[1]);
      *reinterpret_cast<uint4*>(xk + (1 * 4 + tt) * 1024 + lane * 16) = cat2(k2[1], k2[2]);
      // V^T (channels x keys): this token tile is one half of key pair tt >> 1
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const float4 vv = make_float4(av[t][0] + bv[t], av[t][1] + bv[t], av[t][2] + bv[t], av[t][3] + bv[t]);
        *reinterpret_cast<uint2*>(xv + (t * 2 + (tt >> 1)) * 1024 + lane * 16 + 8 * (tt & 1)) =
            make_uint2(pack_bf16x2(vv.x, vv.y), pack_bf16x2(vv.z, vv.w));
      }
    }
    WB_T(2 + 4 * p);
    if (p == 1) wb_wait_all();                         // WP(0) landed (proj(0) ends this pair)
    __syncthreads();                                   // K / V^T of the window visible; WQ free
    WB_T(3 + 4 * p);
    if (p < 3) dma_wq(p + 1);
    if (p == 0) dma_wp(0);

    if (act) {
      f32x4 o[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) o[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int h = 2 * p + hh;
        // ---- S^T = K Q^T: rows = keys 16kt + 4qq + r, column = query n
        f32x4 s[4];
#pragma unroll
        for (int kt = 0; kt < 4; ++kt) {
          const uint4 kf = *reinterpret_cast<const uint4*>(xk + (hh * 4 + kt) * 1024 + lane * 16);
          s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
          mma_step<bf16_t>(s[kt], kf, qf[hh]);
        }
        // ---- + B_rel + shift mask, softmax over the 64 keys (lane + lanes ^16, ^32, ^48)
        float mx = -INFINITY;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float v = s[kt][r] + *reinterpret_cast<const float*>(sm + toff[kt][r] + 900 * h);
            s[kt][r] = v;
            mx = fmaxf(mx, v);
          }
        mx = pair16_max(mx);
        mx = pair32_max(mx);
        float sum = 0.f;
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float ex = __builtin_amdgcn_exp2f(s[kt][r] - mx);
            s[kt][r] = ex;
            sum += ex;
          }
        sum = pair16_sum(sum);
        sum = pair32_sum(sum);
        const float inv = __builtin_amdgcn_rcpf(sum);
        uint4 pf[2];                                   // P^T key pairs (0,1), (2,3)
#pragma unroll
        for (int kp = 0; kp < 2; ++kp) {
          f32x4 a0 = s[2 * kp], a1 = s[2 * kp + 1];
#pragma unroll
          for (int r = 0; r < 4; ++r) { a0[r] *= inv; a1[r] *= inv; }
          pf[kp] = cat2(pk4(a0), pk4(a1));
        }
        // ---- O^T = V^T P^T over this head's channel tiles (tile 1: its 8 rows only)
#pragma unroll
        for (int ci = 0; ci < 2; ++ci) {
          const int c = hh + ci;
#pragma unroll
          for (int kp = 0; kp < 2; ++kp) {
            uint4 vf = *reinterpret_cast<const uint4*>(xv + (c * 2 + kp) * 1024 + lane * 16);
            if (c == 1) {
              const uint32_t keep = hh == 0 ? lo8 : ~lo8;
              vf.x &= keep; vf.y &= keep; vf.z &= keep; vf.w &= keep;
            }
            mma_step<bf16_t>(o[c], vf, pf[kp]);
          }
        }
      }
      if ((p & 1) == 0) {
#pragma unroll
        for (int c = 0; c < 3; ++c) prevO[c] = pk4(o[c]);
      } else {
        // ---- out^T += Wp[:, 96u .. 96u + 95] O^T (pairs 2u, 2u+1: six channel tiles as
        // three k-steps of tile pairs)
        uint4 ob[3];
        ob[0] = cat2(prevO[0], prevO[1]);
        ob[1] = cat2(prevO[2], pk4(o[0]));
        ob[2] = cat2(pk4(o[1]), pk4(o[2]));
#pragma unroll
        for (int m = 0; m < 12; ++m)
#pragma unroll
          for (int s = 0; s < 3; ++s) {
            const uint4 wf = *reinterpret_cast<const uint4*>(sm + L_WP + (m * 3 + s) * 1024 + lane * 16);
            mma_step<bf16_t>(acc[m], wf, ob[s]);
          }
      }
    }
    WB_T(4 + 4 * p);
  }

  // ---- epilogue: out = x + proj + b (active window) or x (MASKSEL, :236-240)
  const float* bp = reinterpret_cast<const float*>(sm + L_BQ);
  const int pix = pix_s[tok0 + n];
  WB_T(17);
  if (pix < 0) return;
  const bf16_t* xr = a.x + (long long)pix * a.ldx;
  bf16_t* orow = a.out + (long long)pix * a.ldo;
  uint2 xv4[12];
#pragma unroll
  for (int m = 0; m < 12; ++m) xv4[m] = *reinterpret_cast<const uint2*>(xr + 16 * m + 4 * qq);
#pragma unroll
  for (int m = 0; m < 12; ++m) {
    const int c0 = 16 * m + 4 * qq;
    const uint2 xv = xv4[m];
    float v[4] = {bf2f(xv.x & 0xFFFF), bf2f(xv.x >> 16), bf2f(xv.y & 0xFFFF), bf2f(xv.y >> 16)};
    if (act) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += acc[m][r] + bp[c0 + r];
    }
    *reinterpret_cast<uint2*>(orow + c0) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
  }
}


// ---------------------------------------------------------------------------------------
// Round 6: the ws-8 block as persistent kernels over the ACTIVE windows.
//
// winblock_v2_kernel (round 3, kept for the A/B until it is removed) runs one 8-wave workgroup
// per window PAIR and streams all four head pairs' weights (288 KiB) through its LDS for those
// 128 tokens: a 42k-cycle chain per workgroup, one round of workgroups at config 2 (DESIGN
// 12c).  Here:
//   winflag_kernel   one wave per window: flag = alpha non-zero anywhere in the (shifted)
//                    window (remove_zero_windows, :38-47), no host sync;
//   winblock_kernel  one workgroup per (head pair, slot), persistent: the pair's 54 KiB qkv
//                    panel stays in LDS; a block scan of the flags deals active window r to
//                    slot r % slots (device-side compaction), and the workgroup walks its
//                    windows two at a time -- 8 waves, token tile w & 3, role w >> 2 (0: q^T
//                    tiles 0-2 + k^T tiles 0-1, 1: k^T tile 2 + v tiles 0-2), so every qkv
//                    weight fragment read from LDS feeds two MFMAs and each SIMD (waves w,
//                    w + 4) issues 108 of the pair's 432 qkv MFMAs; x fragments arrive by
//                    LDS-DMA (the next pair's during this pair's attention); K, V^T and the
//                    head-1 q^T fragments cross waves through LDS; wave (head w >> 2, query
//                    tile w & 3) runs S^T = K Q^T, the softmax and O^T = V^T P^T in registers
//                    and stores O^T (bf16) to the window's slot of the workspace.  Inactive
//                    windows are copied out = x (MASKSEL, :236-240) by the workgroups in
//                    inactive-rank order; pair 0's workgroups publish the compacted list;
//   winproj_kernel   persistent over that list: out = x + Wp O^T + b for every token of an
//                    active window, the 72 KiB proj panel resident, each window's O^T
//                    fragments LDS-DMA'd one window ahead.
// The four workgroups of a slot have the same blockIdx & 7, so they sit on one XCD and share
// the windows' x in L2.  Every product, rounding point and accumulation order is
// winblock_v2_kernel's (O^T is rounded to bf16 exactly where that kernel rounds it before the
// proj), so the two paths are bit-identical.
namespace wb3 {
constexpr int WQF = 54, WPF = 72;
// winblock_kernel
constexpr int L_WQ = 0;                                // the pair's qkv fragments
constexpr int L_X = L_WQ + WQF * 1024;                 // 55296: x [win 2][token tile 4][k-step 6]
constexpr int L_K = L_X + 48 * 1024;                   // 104448: K [win 2][head 2][key tile 4]
constexpr int L_V = L_K + 16 * 1024;                   // 120832: V^T [win 2][channel tile 3][key pair 2]
constexpr int L_Q = L_V + 12 * 1024;                   // 133120: q^T [win 2][head 2][token tile 4]
constexpr int L_TB = L_Q + 16 * 1024;                  // 149504: bias [var 2][head 2][225] fp32 (4 KiB)
constexpr int L_BQ = L_TB + 4 * 1024;                  // 153600: [bq 48 | bk 48 | bv 48] (1 KiB piece)
constexpr int L_LA = L_BQ + 1024;                      // 154624: this workgroup's active windows
constexpr int MAXA = 256;
constexpr int L_LC = L_LA + MAXA * 2;                  // 155136: its inactive windows
constexpr int MAXC = 64;
constexpr int L_MS = L_LC + MAXC * 2;                  // 155264: scan partials [8]
constexpr int LDS_A = L_MS + 64;                       // 155328
static_assert(LDS_A <= 160 * 1024, "LDS");
// prologue staging, free until the first x DMA: the launch's flags at L_X (<= 8 KiB)
// winproj_kernel
constexpr int P_WP = 0;                                // all proj fragments [u][m][s]
constexpr int P_O = P_WP + WPF * 1024;                 // 73728: O^T [buf 2][token tile 4][k-step 6]
constexpr int P_BP = P_O + 48 * 1024;                  // 122880: bproj (1 KiB piece)
constexpr int LDS_B = P_BP + 1024;                     // 123904
constexpr int CHUNK = 8192;                            // windows per launch: 16 flags per thread
constexpr int OSLOT = 4 * 6 * 64 * 2;                  // 8-byte words of one window's O^T (24 KiB)
}  // namespace wb3

struct WinBlock3Args {
  int batch, H, W, shift, masked;
  int w0, nwc, slots, chunk;             // window range of this launch; workgroups per pair
  float scale;
  const bf16_t* x; long long ldx;
  const float* alpha;                    // (B, H, W) fp32 (masked; winflag_kernel only)
  uint8_t* flags;                        // [windows]: alpha non-zero somewhere in the window
  const bf16_t* wq;                      // [4 pairs][54][64 lanes][8]
  const float* bias;                     // [5][256]: bproj | pair p: bq, bk, bv (48 each)
  const bf16_t* wp;                      // [2][12][3][64][8] (permuted k)
  const float* table;                    // [4 pairs][1024]: [var 2][head 2][225] in log2 units
  bf16_t* out; long long ldo;
  unsigned long long* oscr;              // [windows][4 token tiles][6 k-steps][64 lanes][2]
  int* alist;                            // [windows]: active rank -> window (per launch at w0)
  int* acount;                           // [launches]: active windows of the launch
};

// per-window alpha flags: one wave per window, the 64 alpha values of its (shifted) pixels
__global__ void __launch_bounds__(256) winflag_kernel(const WinBlock3Args a) {
  const int lane = threadIdx.x & 63;
  const int win = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwx = a.W >> 3, nwimg = nwx * (a.H >> 3);
  if (win >= a.batch * nwimg) return;
  const int b = win / nwimg, rem = win - b * nwimg;
  const int wy = rem / nwx, wx = rem - wy * nwx;
  int oy = wy * 8 + (lane >> 3) + a.shift; if (oy >= a.H) oy -= a.H;
  int ox = wx * 8 + (lane & 7) + a.shift; if (ox >= a.W) ox -= a.W;
  const bool act = __any(a.alpha[((long long)b * a.H + oy) * a.W + ox] != 0.0f);
  if (lane == 0) a.flags[win] = act ? 1 : 0;
}

__device__ __forceinline__ int wb_win_pix(int wg, int lt, int H, int W, int nwx, int nwimg,
                                          int shift) {               // token lt of window wg
  const int b = wg / nwimg, rem = wg - b * nwimg;
  const int wy = rem / nwx, wx = rem - wy * nwx;
  int oy = wy * 8 + (lt >> 3) + shift; if (oy >= H) oy -= H;
  int ox = wx * 8 + (lt & 7) + shift; if (ox >= W) ox -= W;
  return (b * H + oy) * W + ox;
}

__global__ void __launch_bounds__(512, 1) winblock_kernel(const WinBlock3Args a) {
  using namespace wb3;
  constexpr float LOG2E = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, qq = lane >> 4;
  const int g = blockIdx.x, slots = a.slots, G = 4 * slots;
  const int p = (g >> 3) & 3;                          // head pair
  const int slot = ((g >> 5) << 3) | (g & 7);          // a slot's four pair workgroups: one XCD
  const int H = a.H, W = a.W, shift = a.shift;
  const int nwx = W >> 3, nwimg = nwx * (H >> 3);
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) void*)sm;
  const int tt = w & 3, hr = w >> 2;                   // token tile; role and attention head
  WB_T(0);

  // ---- prologue DMA, two staging pieces per wave (the launch's flags, the pair's bias table
  // and biases), then the pair's qkv panel.  Pieces past the end repeat the last one (same
  // bytes, same place).  The panel pieces start at a per-slot rotation: the 32 workgroups of
  // an XCD would otherwise request the same lines in the same order (one L2 channel at a time).
  const int nflag = (a.nwc + 1023) >> 10;              // 1 KiB flag pieces of this launch
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int k = w + 8 * i;
    if (k > nflag + 4) k = nflag + 4;
    const void* src;
    int dst;
    if (k < nflag) { src = a.flags + a.w0 + k * 1024 + lane * 16; dst = L_X + k * 1024; }
    else if (k < nflag + 4) { src = a.table + 1024 * p + (k - nflag) * 256 + lane * 4; dst = L_TB + (k - nflag) * 1024; }
    else { src = a.bias + 256 * (1 + p) + lane * 4; dst = L_BQ; }
    wb_dma16(src, lds0 + dst);
  }
  const bf16_t* wqp = a.wq + (size_t)p * WQF * 512;
  const int rot = ((g >> 5) * 7) % WQF;
#pragma unroll
  for (int i = 0; i < 7; ++i) {
    int f = w + 8 * i;
    if (f >= WQF) f = WQF - 1;
    f += rot;
    if (f >= WQF) f -= WQF;
    wb_dma16(wqp + ((size_t)f * 64 + lane) * 8, lds0 + L_WQ + f * 1024);
  }
  wb_wait_vm<7>();                                     // the staging pieces landed
  __syncthreads();

  // ---- this workgroup's windows: block scan of the active flags (16 windows per thread)
  short* const la = reinterpret_cast<short*>(sm + L_LA);
  short* const lc = reinterpret_cast<short*>(sm + L_LC);
  int* const ms = reinterpret_cast<int*>(sm + L_MS);
  const int nwc = a.nwc;
  unsigned bits = 0;
  {
    const uint4 fv = *reinterpret_cast<const uint4*>(sm + L_X + 16 * tid);
    const uint32_t fw[4] = {fv.x, fv.y, fv.z, fv.w};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const bool on = 16 * tid + e < nwc && (!a.masked || ((fw[e >> 2] >> (8 * (e & 3))) & 0xFFu) != 0);
      bits |= (on ? 1u : 0u) << e;
    }
  }
  const int cntv = __popc(bits);
  int inc = cntv;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(inc, d);
    if (lane >= d) inc += y;
  }
  if (lane == 63) ms[w] = inc;
  __syncthreads();
  int nact = 0, before = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int v = ms[i];
    nact += v;
    before += i < w ? v : 0;
  }
  {
    const int r = before + inc - cntv;                 // active windows before 16 tid
    int rq = r / slots, rm = r - rq * slots;
    const int q0 = min(16 * tid, nwc) - r;             // inactive windows before 16 tid
    int iq = q0 / G, im = q0 - iq * G;
    for (int e = 0; e < 16; ++e) {
      const int idx = 16 * tid + e;
      if (idx >= nwc) break;
      if ((bits >> e) & 1u) {
        if (rm == slot) la[rq] = (short)idx;
        if (g == 0) a.alist[a.w0 + rq * slots + rm] = a.w0 + idx;   // the compacted list
        if (++rm == slots) { rm = 0; ++rq; }
      } else {
        if (im == g) lc[iq] = (short)idx;
        if (++im == G) { im = 0; ++iq; }
      }
    }
  }
  if (g == 0 && tid == 0) a.acount[a.chunk] = nact;
  const int nmine = nact > slot ? (nact - 1 - slot) / slots + 1 : 0;
  const int ninact = nwc - nact;
  const int ncopy = ninact > g ? (ninact - 1 - g) / G + 1 : 0;
  const int npair = (nmine + 1) >> 1;
  __syncthreads();                                     // lists visible; the staging area free
  WB_T(1);

  // x of windows (wa, wb) as fragment images [win][tt][ks] by LDS-DMA: 48 pieces, 6 per wave
  // (piece k: window k / 24, token tile (k / 6) & 3, k-step k % 6; lane (n, qq) fetches token
  // 16 tt + n, channels 32 ks + 8 qq ..)
  auto dma_x = [&](int wa, int wb) {
#pragma unroll
    for (int i = 0; i < 6; ++i) {
      const int k = w + 8 * i;
      const int wi = k / 24, t4 = (k / 6) & 3, ks = k % 6;
      const int pix = wb_win_pix(wi ? wb : wa, 16 * t4 + n, H, W, nwx, nwimg, shift);
      wb_dma16(a.x + (long long)pix * a.ldx + 32 * ks + 8 * qq, lds0 + L_X + k * 1024);
    }
  };
  if (npair > 0) dma_x(a.w0 + la[0], a.w0 + la[nmine > 1 ? 1 : 0]);
  wb_wait_all();                                       // qkv panel and the first windows' x
  __syncthreads();

  // relative-position bias of this lane's S^T elements (key 16 kt + 4 qq + r, query 16 tt + n)
  // for this wave's head, held in registers for the launch: idx(kt, r) = idx(3, 3) +
  // 30 (3 - kt) + 3 - r; the "- 100" copy (bcut) where the shift mask separates query and key
  const int iq = 16 * tt + n;
  const int tbase = L_TB + hr * 900 +
                    4 * (((iq >> 3) - 6 - (qq >> 1) + 7) * 15 + ((iq & 7) - 4 * (qq & 1) - 3 + 7));
  float breg[16], bcut[16];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int off = tbase + 4 * (30 * (3 - (e >> 2)) + 3 - (e & 3));
    breg[e] = *reinterpret_cast<const float*>(sm + off);
    bcut[e] = shift > 0 ? *reinterpret_cast<const float*>(sm + off + 1800) : 0.0f;
  }
  auto make_cut = [&](int wg) -> unsigned {
    if (shift == 0) return 0u;
    const int rem = wg % nwimg;
    const int wy = rem / nwx, wx = rem - wy * nwx;
    auto rid = [&](int t) {
      const int r = wy * 8 + (t >> 3), c = wx * 8 + (t & 7);
      return 3 * (r < H - 8 ? 0 : (r < H - shift ? 1 : 2)) + (c < W - 8 ? 0 : (c < W - shift ? 1 : 2));
    };
    const int qrid = rid(iq);
    unsigned m = 0;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) m |= (rid(16 * kt + 4 * qq + r) != qrid ? 1u : 0u) << (4 * kt + r);
    return m;
  };
  WB_T(2);

  const float qscale = a.scale * LOG2E;                // q * scale, in log2 units
  const uint32_t lo8 = n < 8 ? 0xFFFFFFFFu : 0u;       // lane holds channel row < 8 of a tile
  const uint32_t qlo = qq < 2 ? 0xFFFFFFFFu : 0u;      // lane's accumulator rows are < 8
  const float* bqs = reinterpret_cast<const float*>(sm + L_BQ);

  // q^T, k^T, v of the pair's heads for this wave's 16 tokens of NWIN windows: every weight
  // fragment read once, used for each window
  auto gemm = [&](auto nw_c) {
    constexpr int NWIN = decltype(nw_c)::value;
    if (hr == 0) {
      f32x4 aq[NWIN][3], ak[NWIN][2];
#pragma unroll
      for (int v = 0; v < NWIN; ++v) {
#pragma unroll
        for (int t = 0; t < 3; ++t) aq[v][t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 2; ++t) ak[v][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        uint4 X[NWIN];
#pragma unroll
        for (int v = 0; v < NWIN; ++v)
          X[v] = *reinterpret_cast<const uint4*>(sm + L_X + ((v * 4 + tt) * 6 + ks) * 1024 + lane * 16);
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const uint4 f = *reinterpret_cast<const uint4*>(sm + L_WQ + (t * 6 + ks) * 1024 + lane * 16);
#pragma unroll
          for (int v = 0; v < NWIN; ++v) mma_step<bf16_t>(aq[v][t], f, X[v]);
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const uint4 f = *reinterpret_cast<const uint4*>(sm + L_WQ + (18 + t * 6 + ks) * 1024 + lane * 16);
#pragma unroll
          for (int v = 0; v < NWIN; ++v) mma_step<bf16_t>(ak[v][t], f, X[v]);
        }
      }
      float4 bq4[3], bk4[2];
#pragma unroll
      for (int t = 0; t < 3; ++t) bq4[t] = *reinterpret_cast<const float4*>(bqs + 16 * t + 4 * qq);
#pragma unroll
      for (int t = 0; t < 2; ++t) bk4[t] = *reinterpret_cast<const float4*>(bqs + 48 + 16 * t + 4 * qq);
#pragma unroll
      for (int v = 0; v < NWIN; ++v) {
        uint2 q2[3], k2[2];
#pragma unroll
        for (int t = 0; t < 3; ++t)
          q2[t] = make_uint2(pack_bf16x2((aq[v][t][0] + bq4[t].x) * qscale, (aq[v][t][1] + bq4[t].y) * qscale),
                             pack_bf16x2((aq[v][t][2] + bq4[t].z) * qscale, (aq[v][t][3] + bq4[t].w) * qscale));
#pragma unroll
        for (int t = 0; t < 2; ++t)
          k2[t] = make_uint2(pack_bf16x2(ak[v][t][0] + bk4[t].x, ak[v][t][1] + bk4[t].y),
                             pack_bf16x2(ak[v][t][2] + bk4[t].z, ak[v][t][3] + bk4[t].w));
        // head 2p: channels 0..23 = tile 0 + rows 0..7 of tile 1; head 2p+1: rows 8..15 of
        // tile 1 + tile 2.  Zeroing the other head's rows in q alone cuts them from q . k.
        *reinterpret_cast<uint4*>(sm + L_Q + (v * 8 + tt) * 1024 + lane * 16) =
            make_uint4(q2[0].x, q2[0].y, q2[1].x & qlo, q2[1].y & qlo);
        *reinterpret_cast<uint4*>(sm + L_Q + (v * 8 + 4 + tt) * 1024 + lane * 16) =
            make_uint4(q2[1].x & ~qlo, q2[1].y & ~qlo, q2[2].x, q2[2].y);
        *reinterpret_cast<uint4*>(sm + L_K + ((v * 2 + 0) * 4 + tt) * 1024 + lane * 16) = cat2(k2[0], k2[1]);
        *reinterpret_cast<uint2*>(sm + L_K + ((v * 2 + 1) * 4 + tt) * 1024 + lane * 16) = k2[1];
      }
    } else {
      f32x4 ak2[NWIN], av[NWIN][3];
#pragma unroll
      for (int v = 0; v < NWIN; ++v) {
        ak2[v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int t = 0; t < 3; ++t) av[v][t] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int ks = 0; ks < 6; ++ks) {
        uint4 X[NWIN];
#pragma unroll
        for (int v = 0; v < NWIN; ++v)
          X[v] = *reinterpret_cast<const uint4*>(sm + L_X + ((v * 4 + tt) * 6 + ks) * 1024 + lane * 16);
        {
          const uint4 f = *reinterpret_cast<const uint4*>(sm + L_WQ + (30 + ks) * 1024 + lane * 16);
#pragma unroll
          for (int v = 0; v < NWIN; ++v) mma_step<bf16_t>(ak2[v], f, X[v]);
        }
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const uint4 f = *reinterpret_cast<const uint4*>(sm + L_WQ + (36 + t * 6 + ks) * 1024 + lane * 16);
#pragma unroll
          for (int v = 0; v < NWIN; ++v) mma_step<bf16_t>(av[v][t], X[v], f);
        }
      }
      const float4 bk4 = *reinterpret_cast<const float4*>(bqs + 48 + 32 + 4 * qq);
      float bv[3];
#pragma unroll
      for (int t = 0; t < 3; ++t) bv[t] = bqs[96 + 16 * t + n];
#pragma unroll
      for (int v = 0; v < NWIN; ++v) {
        *reinterpret_cast<uint2*>(sm + L_K + ((v * 2 + 1) * 4 + tt) * 1024 + lane * 16 + 8) =
            make_uint2(pack_bf16x2(ak2[v][0] + bk4.x, ak2[v][1] + bk4.y),
                       pack_bf16x2(ak2[v][2] + bk4.z, ak2[v][3] + bk4.w));
        // V^T (channels x keys): this token tile is one half of key pair tt >> 1
#pragma unroll
        for (int t = 0; t < 3; ++t)
          *reinterpret_cast<uint2*>(sm + L_V + ((v * 3 + t) * 2 + (tt >> 1)) * 1024 + lane * 16 + 8 * (tt & 1)) =
              make_uint2(pack_bf16x2(av[v][t][0] + bv[t], av[v][t][1] + bv[t]),
                         pack_bf16x2(av[v][t][2] + bv[t], av[v][t][3] + bv[t]));
      }
    }
  };

  // attention of head 2p + hr, query tile tt, for NWIN windows (global windows wg[v]) phase by
  // phase, so the windows' independent chains interleave: O^T to each window's slot of the
  // workspace (channel tile 3p + c is half (3p + c) & 1 of the proj's k-step (3p + c) >> 1);
  // two store instructions per window
  auto attend = [&](auto nw_c, int wg0, int wg1) {
    constexpr int NWIN = decltype(nw_c)::value;
    const int wgv[2] = {wg0, wg1};
    f32x4 s[NWIN][4];
#pragma unroll
    for (int v = 0; v < NWIN; ++v) {
      const uint4 qf = *reinterpret_cast<const uint4*>(sm + L_Q + (v * 8 + hr * 4 + tt) * 1024 + lane * 16);
#pragma unroll
      for (int kt = 0; kt < 4; ++kt) {
        const uint4 kf = *reinterpret_cast<const uint4*>(sm + L_K + ((v * 2 + hr) * 4 + kt) * 1024 + lane * 16);
        s[v][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
        mma_step<bf16_t>(s[v][kt], kf, qf);
      }
    }
    unsigned cutm[NWIN];
#pragma unroll
    for (int v = 0; v < NWIN; ++v) cutm[v] = make_cut(wgv[v]);
    // + B_rel + shift mask, softmax over the 64 keys (lane + lanes ^16, ^32, ^48)
    float mx[NWIN], sum[NWIN];
#pragma unroll
    for (int v = 0; v < NWIN; ++v) {
      mx[v] = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float val = s[v][kt][r] + (((cutm[v] >> (4 * kt + r)) & 1u) ? bcut[4 * kt + r] : breg[4 * kt + r]);
          s[v][kt][r] = val;
          mx[v] = fmaxf(mx[v], val);
        }
    }
#pragma unroll
    for (int v = 0; v < NWIN; ++v) mx[v] = pair16_max(mx[v]);
#pragma unroll
    for (int v = 0; v < NWIN; ++v) mx[v] = pair32_max(mx[v]);
#pragma unroll
    for (int v = 0; v < NWIN; ++v) {
      sum[v] = 0.f;
#pragma unroll
      for (int kt = 0; kt < 4; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float ex = __builtin_amdgcn_exp2f(s[v][kt][r] - mx[v]);
          s[v][kt][r] = ex;
          sum[v] += ex;
        }
    }
#pragma unroll
    for (int v = 0; v < NWIN; ++v) sum[v] = pair16_sum(sum[v]);
#pragma unroll
    for (int v = 0; v < NWIN; ++v) sum[v] = pair32_sum(sum[v]);
#pragma unroll
    for (int v = 0; v < NWIN; ++v) {
      const float inv = __builtin_amdgcn_rcpf(sum[v]);
      uint4 pf[2];                                     // P^T key pairs (0,1), (2,3)
#pragma unroll
      for (int kp = 0; kp < 2; ++kp) {
        f32x4 a0 = s[v][2 * kp], a1 = s[v][2 * kp + 1];
#pragma unroll
        for (int r = 0; r < 4; ++r) { a0[r] *= inv; a1[r] *= inv; }
        pf[kp] = cat2(pk4(a0), pk4(a1));
      }
      uint2* dst = reinterpret_cast<uint2*>(a.oscr + (size_t)wgv[v] * OSLOT);
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) {
        const int c = hr + ci;
        f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kp = 0; kp < 2; ++kp) {
          uint4 vf = *reinterpret_cast<const uint4*>(sm + L_V + ((v * 3 + c) * 2 + kp) * 1024 + lane * 16);
          if (c == 1) {
            const uint32_t keep = hr == 0 ? lo8 : ~lo8;
            vf.x &= keep; vf.y &= keep; vf.z &= keep; vf.w &= keep;
          }
          mma_step<bf16_t>(o, vf, pf[kp]);
        }
        const int ct = 3 * p + c;
        if (c != 1 || (hr == 0 ? qq < 2 : qq >= 2))
          dst[((tt * 6 + (ct >> 1)) * 64 + lane) * 2 + (ct & 1)] = pk4(o);
      }
    }
  };

  // inactive windows: out = x (MASKSEL, :236-240), 64 tokens x 24 chunks of 16 bytes, 3 per
  // thread; one window per pair iteration rides under the attention (loads after the exchange
  // barrier, stores after the attention), the rest follow the loop
  uint4 cv0, cv1, cv2;
  long long cp0 = 0, cp1 = 0, cp2 = 0;
  const int ce0 = tid, ce1 = tid + 512, ce2 = tid + 1024;
  const int ct0 = ce0 / 24, ct1 = ce1 / 24, ct2 = ce2 / 24;
  const int cc0 = 8 * (ce0 - 24 * ct0), cc1 = 8 * (ce1 - 24 * ct1), cc2 = 8 * (ce2 - 24 * ct2);
  auto copy_load = [&](int wg) {
    cp0 = wb_win_pix(wg, ct0, H, W, nwx, nwimg, shift);
    cp1 = wb_win_pix(wg, ct1, H, W, nwx, nwimg, shift);
    cp2 = wb_win_pix(wg, ct2, H, W, nwx, nwimg, shift);
    cv0 = *reinterpret_cast<const uint4*>(a.x + cp0 * a.ldx + cc0);
    cv1 = *reinterpret_cast<const uint4*>(a.x + cp1 * a.ldx + cc1);
    cv2 = *reinterpret_cast<const uint4*>(a.x + cp2 * a.ldx + cc2);
  };
  auto copy_store = [&]() {
    *reinterpret_cast<uint4*>(a.out + cp0 * a.ldo + cc0) = cv0;
    *reinterpret_cast<uint4*>(a.out + cp1 * a.ldo + cc1) = cv1;
    *reinterpret_cast<uint4*>(a.out + cp2 * a.ldo + cc2) = cv2;
  };

  for (int i = 0; i < npair; ++i) {
    const bool two = 2 * i + 1 < nmine;               // wave-uniform
    const int wa = a.w0 + la[2 * i], wb = two ? a.w0 + la[2 * i + 1] : wa;
    if (two) gemm(std::integral_constant<int, 2>{});
    else gemm(std::integral_constant<int, 1>{});
    WB_T(3 + 4 * (i < 2 ? i : 2));
    __syncthreads();                                   // K / V^T / q^T visible; x free
    WB_T(4 + 4 * (i < 2 ? i : 2));
    if (i + 1 < npair) {
      const int nb = 2 * i + 3 < nmine ? 2 * i + 3 : 2 * i + 2;
      dma_x(a.w0 + la[2 * i + 2], a.w0 + la[nb]);
    }
    const bool cp = i < ncopy;                         // wave-uniform
    if (cp) copy_load(a.w0 + lc[i]);
    if (two) attend(std::integral_constant<int, 2>{}, wa, wb);
    else attend(std::integral_constant<int, 1>{}, wa, wa);
    if (cp) copy_store();
    WB_T(5 + 4 * (i < 2 ? i : 2));
    // the next windows' x landed (the O^T stores issued after it may still be in flight:
    // two store instructions per window)
    if (two) wb_wait_vm<4>();
    else wb_wait_vm<2>();
    __syncthreads();                                   // exchange free; x visible
    WB_T(6 + 4 * (i < 2 ? i : 2));
  }
  WB_T(15);

  // the inactive windows left: two at a time (six loads in flight per thread)
  for (int c = npair; c < ncopy; c += 2) {
    copy_load(a.w0 + lc[c]);
    if (c + 1 < ncopy) {
      const uint4 a0 = cv0, a1 = cv1, a2 = cv2;
      const long long q0 = cp0, q1 = cp1, q2 = cp2;
      copy_load(a.w0 + lc[c + 1]);
      *reinterpret_cast<uint4*>(a.out + q0 * a.ldo + cc0) = a0;
      *reinterpret_cast<uint4*>(a.out + q1 * a.ldo + cc1) = a1;
      *reinterpret_cast<uint4*>(a.out + q2 * a.ldo + cc2) = a2;
    }
    copy_store();
  }
  wb_wait_all();                                       // no LDS-DMA in flight at exit
  WB_T(17);
}

// out = x + Wp O^T + b over the launch's active windows (winblock_kernel's compacted list),
// the proj panel resident; 8 waves: token tiles 2tp, 2tp + 1 (tp = w & 1) x output channel
// tiles 3mg .. 3mg + 2 (mg = w >> 1), 36 MFMAs each, k-steps in winblock_v2_kernel's order
__global__ void __launch_bounds__(512, 1) winproj_kernel(const WinBlock3Args a) {
  using namespace wb3;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, qq = lane >> 4;
  const int H = a.H, W = a.W, shift = a.shift;
  const int nwx = W >> 3, nwimg = nwx * (H >> 3);
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) void*)sm;
  const int tp = w & 1, mg = w >> 1;
  const int nact = a.acount[a.chunk];
  const int G = gridDim.x;
  // O^T of window wg into buffer b: 24 pieces [tt][ks], 3 per wave
  auto dma_o = [&](int wg, int b) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int k = w + 8 * i;
      wb_dma16(a.oscr + (size_t)wg * OSLOT + (size_t)(k * 64 + lane) * 2, lds0 + P_O + (b * 24 + k) * 1024);
    }
  };
  uint2 xr[2][3];
  auto load_res = [&](int wg) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16_t* xrow = a.x + (long long)wb_win_pix(wg, 16 * (2 * tp + u) + n, H, W, nwx, nwimg, shift) * a.ldx;
#pragma unroll
      for (int mi = 0; mi < 3; ++mi)
        xr[u][mi] = *reinterpret_cast<const uint2*>(xrow + 16 * (3 * mg + mi) + 4 * qq);
    }
  };
  int r = blockIdx.x;
  int wg = r < nact ? a.alist[a.w0 + r] : 0;
  if (r < nact) dma_o(wg, 0);
  const int rot = ((blockIdx.x >> 3) * 5) % WPF;       // per-workgroup start (see winblock_kernel)
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    int f = w + 8 * i + rot;
    if (f >= WPF) f -= WPF;
    wb_dma16(a.wp + ((size_t)f * 64 + lane) * 8, lds0 + P_WP + f * 1024);
  }
  wb_dma16(a.bias + lane * 4, lds0 + P_BP);
  if (r < nact) load_res(wg);
  wb_wait_all();
  __syncthreads();
  const float* bp = reinterpret_cast<const float*>(sm + P_BP);
  for (int it = 0; r < nact; ++it, r += G) {
    const int b = it & 1;
    const int rn = r + G;
    const int wgn = rn < nact ? a.alist[a.w0 + rn] : 0;
    if (rn < nact) dma_o(wgn, b ^ 1);                 // the next window's O^T, in flight
    f32x4 acc[2][3];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int mi = 0; mi < 3; ++mi) acc[u][mi] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 6; ++ks) {
      uint4 ob[2];
#pragma unroll
      for (int u = 0; u < 2; ++u)
        ob[u] = *reinterpret_cast<const uint4*>(sm + P_O + (b * 24 + (2 * tp + u) * 6 + ks) * 1024 + lane * 16);
#pragma unroll
      for (int mi = 0; mi < 3; ++mi) {
        const int f = ((ks / 3) * 12 + 3 * mg + mi) * 3 + ks % 3;
        const uint4 wf = *reinterpret_cast<const uint4*>(sm + P_WP + f * 1024 + lane * 16);
#pragma unroll
        for (int u = 0; u < 2; ++u) mma_step<bf16_t>(acc[u][mi], wf, ob[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      bf16_t* orow = a.out + (long long)wb_win_pix(wg, 16 * (2 * tp + u) + n, H, W, nwx, nwimg, shift) * a.ldo;
#pragma unroll
      for (int mi = 0; mi < 3; ++mi) {
        const int c0 = 16 * (3 * mg + mi) + 4 * qq;
        const uint2 xv = xr[u][mi];
        float v[4] = {bf2f(xv.x & 0xFFFF), bf2f(xv.x >> 16), bf2f(xv.y & 0xFFFF), bf2f(xv.y >> 16)};
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) v[rr] += acc[u][mi][rr] + bp[c0 + rr];
        *reinterpret_cast<uint2*>(orow + c0) = make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      }
    }
    if (rn < nact) load_res(wgn);
    wg = wgn;
    wb_wait_all();                                     // next O^T and x landed, stores drained
    __syncthreads();                                   // buffer b free, b ^ 1 visible
  }
}

// ---------------------------------------------------------------------------------------
// The same block at ws 4, C 80, 8 heads of 10 (the 1/16-resolution attention blocks,
// TransformRGB.py:63,80): a window is 16 tokens = ONE 16-token tile, so each wave owns a
// whole window and nothing crosses waves.  q^T, k^T (channels x tokens) and v (tokens x
// channels) come from 16x16x32 MFMAs over x; every later product sums over 16 keys or over
// one 16-channel accumulator tile, so it takes its operands straight from the accumulators
// with v_mfma_f32_16x16x16_bf16 (lane l: row l & 15, k = 4(l >> 4) + j = the accumulator's
// rows 4(l >> 4) + r):
//   S^T  = sum over the 1-2 channel tiles a head touches of K_t Q_t^T  (q masked to the head's
//          10 channels)
//   P^T  = softmax over the 16 keys (4 lanes apart: two xor-shuffles)
//   O^T_t += V_t^T P^T  (rows of tile t outside the head masked)
//   out^T = Wp O^T  (5 x 5 fragments)
// One workgroup = NW windows; weights (46 KiB qkv + 12.5 KiB proj, fragment-major) are
// LDS-DMA'd once per workgroup; one barrier.
namespace wb4 {
constexpr int WS = 4, C = 80, HEADS = 8, DH = 10;
constexpr int WQF = 45;                                // 15 m-tiles x 3 k-steps, 1 KiB each
constexpr int WPP = 13;                                // proj: 25 x 512 B, DMA'd as 13 KiB
constexpr int NPIECE = WQF + WPP;
constexpr int L_WQ = 0;
constexpr int L_WP = WQF * 1024;                       // 46080
constexpr int L_TB = L_WP + WPP * 1024;                // 59392: bias [2][8 heads][49] fp32
constexpr int LDS = L_TB + 2 * 8 * 49 * 4;             // 62528
}  // namespace wb4

typedef __attribute__((ext_vector_type(4))) short s16x4;
__device__ __forceinline__ void mma16(f32x4& acc, uint2 a, uint2 b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, a),
                                                  __builtin_bit_cast(s16x4, b), acc, 0, 0, 0);
}

template <int NW>
__global__ void __launch_bounds__(64 * NW) winblock4_kernel(const WinBlockArgs a) {
  using namespace wb4;
  constexpr float LOG2E = 1.4426950408889634f;
  extern __shared__ __attribute__((aligned(16))) unsigned char sm[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = lane & 15, qq = lane >> 4;
  const int H = a.H, W = a.W, shift = a.shift;
  const int nwx = W / WS, nwy = H / WS;
  const int total = a.batch * nwx * nwy;
  const uint32_t lds0 = (uint32_t)(size_t)(__attribute__((address_space(3))) void*)sm;

  // ---- weights: NPIECE 1-KiB LDS-DMA pieces dealt over the waves
  for (int f = w; f < NPIECE; f += NW) {
    const bf16_t* src = f < WQF ? a.wq + ((size_t)f * 64 + lane) * 8
                                : a.wp + ((size_t)(f - WQF) * 64 + lane) * 8;
    wb_dma16(src, lds0 + f * 1024);
  }
  float* tb = reinterpret_cast<float*>(sm + L_TB);
  for (int e = tid; e < 49 * 8; e += 64 * NW) {        // table [49][8] -> [var][8][49]
    const int idx = e >> 3, hd = e & 7;
    const float v = a.table[e];
    tb[hd * 49 + idx] = v * LOG2E;
    tb[8 * 49 + hd * 49 + idx] = (v + -100.0f) * LOG2E;
  }

  // ---- this wave's window: token n -> pixel (cyclic shift folded in)
  const int gw = blockIdx.x * NW + w;
  const bool live = gw < total;
  int wy = 0, wx = 0, b = 0;
  if (live) {
    b = gw / (nwx * nwy);
    const int rem = gw - b * nwx * nwy;
    wy = rem / nwx; wx = rem - wy * nwx;
  }
  auto rid_of = [&](int t) {
    const int r = wy * WS + (t >> 2), c = wx * WS + (t & 3);
    return 3 * (r < H - WS ? 0 : (r < H - shift ? 1 : 2)) + (c < W - WS ? 0 : (c < W - shift ? 1 : 2));
  };
  int pix = 0;
  {
    int oy = wy * WS + (n >> 2) + shift; if (oy >= H) oy -= H;
    int ox = wx * WS + (n & 3) + shift; if (ox >= W) ox -= W;
    pix = (b * H + oy) * W + ox;
  }
  // remove_zero_windows (:38-47): the window's 16 alpha values, wave-uniform verdict
  const bool act = live && (!a.masked || __any(a.alpha[pix] != 0.0f));
  const bf16_t* xr = a.x + (long long)pix * a.ldx;
  uint4 X[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks)
    X[ks] = (act && (ks < 2 || qq < 2)) ? *reinterpret_cast<const uint4*>(xr + 32 * ks + 8 * qq)
                                       : make_uint4(0, 0, 0, 0);
  // relative-position-bias offsets of this lane's S^T elements (key 4qq + r, query n)
  int toff[4];
  {
    const int qrid = rid_of(n);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int jk = 4 * qq + r;
      const int idx = ((n >> 2) - (jk >> 2) + 3) * 7 + ((n & 3) - (jk & 3) + 3);
      const bool cut = shift > 0 && rid_of(jk) != qrid;
      toff[r] = L_TB + (cut ? 8 * 49 * 4 : 0) + idx * 4;
    }
  }
  wb_wait_all();
  __syncthreads();
  if (!live) return;
  bf16_t* orow = a.out + (long long)pix * a.ldo;
  if (!act) {                                          // transparent window: out = x
    if (qq < 2) {
#pragma unroll
      for (int k = 0; k < 5; ++k)
        *reinterpret_cast<uint4*>(orow + 40 * qq + 8 * k) = *reinterpret_cast<const uint4*>(xr + 40 * qq + 8 * k);
    }
    return;
  }

  // ================= q^T, k^T (channels x tokens), v (tokens x channels)
  f32x4 aq[5], ak[5], av[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) aq[t] = ak[t] = av[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      const uint4 fq = *reinterpret_cast<const uint4*>(sm + L_WQ + (t * 3 + ks) * 1024 + lane * 16);
      const uint4 fk = *reinterpret_cast<const uint4*>(sm + L_WQ + ((5 + t) * 3 + ks) * 1024 + lane * 16);
      const uint4 fv = *reinterpret_cast<const uint4*>(sm + L_WQ + ((10 + t) * 3 + ks) * 1024 + lane * 16);
      mma_step<bf16_t>(aq[t], fq, X[ks]);
      mma_step<bf16_t>(ak[t], fk, X[ks]);
      mma_step<bf16_t>(av[t], X[ks], fv);
    }
  }
  const float qscale = a.scale * LOG2E;
  uint2 k2[5], v2[5];
  float qv[5][4];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const float4 bq4 = *reinterpret_cast<const float4*>(a.bqkv + 16 * t + 4 * qq);
    const float4 bk4 = *reinterpret_cast<const float4*>(a.bqkv + 80 + 16 * t + 4 * qq);
    const float bv = a.bqkv[160 + 16 * t + n];
    qv[t][0] = (aq[t][0] + bq4.x) * qscale; qv[t][1] = (aq[t][1] + bq4.y) * qscale;
    qv[t][2] = (aq[t][2] + bq4.z) * qscale; qv[t][3] = (aq[t][3] + bq4.w) * qscale;
    k2[t] = make_uint2(pack_bf16x2(ak[t][0] + bk4.x, ak[t][1] + bk4.y),
                       pack_bf16x2(ak[t][2] + bk4.z, ak[t][3] + bk4.w));
    v2[t] = make_uint2(pack_bf16x2(av[t][0] + bv, av[t][1] + bv), pack_bf16x2(av[t][2] + bv, av[t][3] + bv));
  }

  f32x4 o[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) o[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < HEADS; ++h) {
    const int c0 = DH * h, c1 = DH * h + DH;           // the head's channels [c0, c1)
    const int t0 = c0 >> 4, t1 = (c1 - 1) >> 4;
    f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = t0; t <= t1; ++t) {
      float m4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = 16 * t + 4 * qq + j;
        m4[j] = (ch >= c0 && ch < c1) ? qv[t][j] : 0.0f;
      }
      mma16(s, k2[t], make_uint2(pack_bf16x2(m4[0], m4[1]), pack_bf16x2(m4[2], m4[3])));
    }
    float mx = -INFINITY;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] += *reinterpret_cast<const float*>(sm + toff[r] + 196 * h);
      mx = fmaxf(mx, s[r]);
    }
    mx = pair16_max(mx);
    mx = pair32_max(mx);
    float sum = 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s[r] = __builtin_amdgcn_exp2f(s[r] - mx);
      sum += s[r];
    }
    sum = pair16_sum(sum);
    sum = pair32_sum(sum);
    const float inv = __builtin_amdgcn_rcpf(sum);
    const uint2 pf = make_uint2(pack_bf16x2(s[0] * inv, s[1] * inv), pack_bf16x2(s[2] * inv, s[3] * inv));
#pragma unroll
    for (int t = t0; t <= t1; ++t) {
      const int ch = 16 * t + n;                       // V^T row of this lane
      const uint32_t keep = (ch >= c0 && ch < c1) ? 0xFFFFFFFFu : 0u;
      mma16(o[t], make_uint2(v2[t].x & keep, v2[t].y & keep), pf);
    }
  }
  // ================= out^T = Wp O^T, + b + x
  uint2 ob[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) ob[t] = pk4(o[t]);
#pragma unroll
  for (int m = 0; m < 5; ++m) {
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kt = 0; kt < 5; ++kt)
      mma16(acc, *reinterpret_cast<const uint2*>(sm + L_WP + (m * 5 + kt) * 512 + lane * 8), ob[kt]);
    const int c0 = 16 * m + 4 * qq;
    const float4 bp = *reinterpret_cast<const float4*>(a.bproj + c0);
    const uint2 xv = *reinterpret_cast<const uint2*>(xr + c0);
    const float v0 = bf2f(xv.x & 0xFFFF) + acc[0] + bp.x, v1 = bf2f(xv.x >> 16) + acc[1] + bp.y;
    const float v2_ = bf2f(xv.y & 0xFFFF) + acc[2] + bp.z, v3 = bf2f(xv.y >> 16) + acc[3] + bp.w;
    *reinterpret_cast<uint2*>(orow + c0) = make_uint2(pack_bf16x2(v0, v1), pack_bf16x2(v2_, v3));
  }
}

}  // namespace rgbac

using namespace rgbac;

#ifdef RGBAC_WB_TIMING
extern "C" int rgbac_debug_wb_times(unsigned long long* host, int nblocks) {
  if (nblocks > 8192) nblocks = 8192;
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wb_t), (size_t)nblocks * 18 * 8) != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host + (size_t)nblocks * 18, HIP_SYMBOL(g_wb_w), (size_t)nblocks * 2 * 8) ==
                 hipSuccess ? 0 : 1;
}
#endif


// the round-3 single-kernel form (winblock_v2_kernel) over the same packs: one workgroup per
// window pair streaming all four head pairs' weights; the faster form while one round of
// workgroups covers the windows
static int launch_winblock_v2(const WinBlockArgs& d, long long windows, hipStream_t st) {
  static unsigned long long attr = 0;
  lds_optin(reinterpret_cast<const void*>(winblock_v2_kernel), wb::LDS, &attr);
  hipLaunchKernelGGL(winblock_v2_kernel, dim3((unsigned)((windows + 1) / 2)), dim3(512), wb::LDS, st, d);
  return check_launch("winblock_v2_kernel");
}

namespace {
struct Wb3Layout {
  long long flags, alist, acount, oscr, total;
};
Wb3Layout wb3_layout(long long nwin) {
  auto up = [](long long v, long long m) { return (v + m - 1) / m * m; };
  Wb3Layout l;
  l.flags = 0;
  l.alist = up(nwin, wb3::CHUNK);
  l.acount = l.alist + up(nwin * 4, 256);
  l.oscr = l.acount + up((nwin + wb3::CHUNK - 1) / wb3::CHUNK * 4, 256);
  l.total = l.oscr + nwin * (long long)wb3::OSLOT * 8;
  return l;
}
}  // namespace

extern "C" int64_t rgbac_winattn_block_workspace(int batch, int h, int w) {
  if (batch <= 0 || h <= 0 || w <= 0 || h % 8 || w % 8) return -1;
  return wb3_layout((long long)batch * (h / 8) * (w / 8)).total;
}

extern "C" int rgbac_winattn_block(int batch, int h, int w, int shift, int masked, float scale,
                                   const void* x, int64_t ldx, const float* alpha,
                                   const void* wq_packed, const float* bias_pack,
                                   const void* wp_packed, const float* table_pad, void* out,
                                   int64_t ldo, void* work, int64_t work_bytes, void* stream) {
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && h % 8 == 0 && w % 8 == 0,
                "H and W must be positive multiples of the window size 8");
  RGBAC_REQUIRE(shift >= 0 && shift < 8, "0 <= shift < 8");
  RGBAC_REQUIRE(x && out && wq_packed && bias_pack && wp_packed && table_pad && work, "null pointer");
  RGBAC_REQUIRE(!masked || alpha, "masked attention needs alpha");
  RGBAC_REQUIRE(ldx >= 192 && ldo >= 192 && ldx % 8 == 0 && ldo % 8 == 0, "strides");
  RGBAC_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0 &&
                    ((uintptr_t)wq_packed % 16) == 0 && ((uintptr_t)wp_packed % 16) == 0 &&
                    ((uintptr_t)bias_pack % 16) == 0 && ((uintptr_t)table_pad % 16) == 0 &&
                    ((uintptr_t)work % 256) == 0,
                "16-byte aligned operands, 256-byte aligned workspace");
  RGBAC_REQUIRE(x != out, "out must not alias x");
  const long long nwin = (long long)batch * (h / 8) * (w / 8);
  RGBAC_REQUIRE((long long)batch * h * w < (1LL << 31), "pixel index must fit in 31 bits");
  const Wb3Layout lay = wb3_layout(nwin);
  RGBAC_REQUIRE(work_bytes >= lay.total, "workspace smaller than rgbac_winattn_block_workspace()");
  unsigned char* wk = static_cast<unsigned char*>(work);
  WinBlock3Args d;
  d.batch = batch; d.H = h; d.W = w; d.shift = shift; d.masked = masked; d.scale = scale;
  d.x = reinterpret_cast<const bf16_t*>(x); d.ldx = ldx; d.alpha = alpha;
  d.flags = wk + lay.flags;
  d.wq = reinterpret_cast<const bf16_t*>(wq_packed); d.bias = bias_pack;
  d.wp = reinterpret_cast<const bf16_t*>(wp_packed); d.table = table_pad;
  d.out = reinterpret_cast<bf16_t*>(out); d.ldo = ldo;
  d.oscr = reinterpret_cast<unsigned long long*>(wk + lay.oscr);
  d.alist = reinterpret_cast<int*>(wk + lay.alist);
  d.acount = reinterpret_cast<int*>(wk + lay.acount);
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  // form: the round-3 kernel below 2,048 windows (one round of workgroups, whose chain the
  // persistent pair is not shorter than), the head-pair kernels above; RGBAC_WINBLOCK_FORM=2|3
  // forces one (A/B and the bit-identity tests; read per call, host side only)
  const char* fe = getenv("RGBAC_WINBLOCK_FORM");
  const int form = (fe && fe[0] == '2') ? 2 : (fe && fe[0] == '3') ? 3 : (nwin < 2048 ? 2 : 3);
  if (form == 2) {
    RGBAC_REQUIRE(nwin < (1LL << 30), "too many windows");
    WinBlockArgs v;
    v.batch = batch; v.H = h; v.W = w; v.shift = shift; v.masked = masked; v.scale = scale;
    v.x = d.x; v.ldx = ldx; v.alpha = alpha; v.wq = d.wq; v.bqkv = bias_pack;
    v.wp = d.wp; v.bproj = bias_pack; v.table = table_pad; v.out = d.out; v.ldo = ldo;
    return launch_winblock_v2(v, nwin, st);
  }
  if (masked) {
    const long long blocks = (nwin + 3) / 4;
    RGBAC_REQUIRE(blocks < (1LL << 31), "too many windows");
    hipLaunchKernelGGL(winflag_kernel, dim3((unsigned)blocks), dim3(256), 0, st, d);
    const int rc = check_launch("winflag_kernel");
    if (rc) return rc;
  }
  static unsigned long long attr_a = 0, attr_b = 0;
  lds_optin(reinterpret_cast<const void*>(winblock_kernel), wb3::LDS_A, &attr_a);
  lds_optin(reinterpret_cast<const void*>(winproj_kernel), wb3::LDS_B, &attr_b);
  // slots per head pair: a quarter of the CUs (one workgroup per CU), a multiple of 8 so a
  // slot's four pair workgroups share blockIdx & 7
  const int ncu = device_cus();
  int slots = (ncu / 4) & ~7;
  if (slots < 8) slots = 8;
  int chunk = 0;
  for (long long w0 = 0; w0 < nwin; w0 += wb3::CHUNK, ++chunk) {
    const int nwc = (int)std::min<long long>(wb3::CHUNK, nwin - w0);
    const int s = std::min(slots, (nwc + 7) / 8 * 8);
    // list capacities: ceil(nwc / s) active and ceil(nwc / 4s) inactive windows per workgroup
    RGBAC_REQUIRE((nwc + s - 1) / s <= wb3::MAXA && (nwc + 4 * s - 1) / (4 * s) <= wb3::MAXC,
                  "window lists exceed the workgroup's capacity");
    d.w0 = (int)w0; d.nwc = nwc; d.slots = s; d.chunk = chunk;
    hipLaunchKernelGGL(winblock_kernel, dim3(4 * s), dim3(512), wb3::LDS_A, st, d);
    int rc = check_launch("winblock_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(winproj_kernel, dim3(std::min(ncu, nwc)), dim3(512), wb3::LDS_B, st, d);
    rc = check_launch("winproj_kernel");
    if (rc) return rc;
  }
  return RGBAC_OK;
}

extern "C" int rgbac_winattn_block_ws4(int batch, int h, int w, int shift, int masked, float scale,
                                       const void* x, int64_t ldx, const float* alpha,
                                       const void* wq_packed, const float* bqkv,
                                       const void* wp_packed, const float* bproj,
                                       const float* table, void* out, int64_t ldo, void* stream) {
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && h % 4 == 0 && w % 4 == 0,
                "H and W must be positive multiples of the window size 4");
  RGBAC_REQUIRE(shift >= 0 && shift < 4, "0 <= shift < 4");
  RGBAC_REQUIRE(x && out && wq_packed && bqkv && wp_packed && bproj && table, "null pointer");
  RGBAC_REQUIRE(!masked || alpha, "masked attention needs alpha");
  RGBAC_REQUIRE(ldx >= 80 && ldo >= 80 && ldx % 8 == 0 && ldo % 8 == 0, "strides");
  RGBAC_REQUIRE(((uintptr_t)x % 16) == 0 && ((uintptr_t)out % 16) == 0 &&
                    ((uintptr_t)bqkv % 16) == 0 && ((uintptr_t)bproj % 16) == 0, "16-byte alignment");
  RGBAC_REQUIRE(x != out, "out must not alias x");
  RGBAC_REQUIRE((long long)batch * h * w < (1LL << 31), "pixel index must fit in 31 bits");
  const long long windows = (long long)batch * (h / 4) * (w / 4);
  WinBlockArgs d;
  d.batch = batch; d.H = h; d.W = w; d.shift = shift; d.masked = masked; d.scale = scale;
  d.x = reinterpret_cast<const bf16_t*>(x); d.ldx = ldx; d.alpha = alpha;
  d.wq = reinterpret_cast<const bf16_t*>(wq_packed); d.bqkv = bqkv;
  d.wp = reinterpret_cast<const bf16_t*>(wp_packed); d.bproj = bproj; d.table = table;
  d.out = reinterpret_cast<bf16_t*>(out); d.ldo = ldo;
  static const int nw_env = [] {
    const char* e = getenv("RGBAC_WINBLOCK4_NW");        // windows (waves) per workgroup
    const int v = e ? atoi(e) : 0;
    return v == 1 || v == 2 || v == 4 || v == 8 ? v : 0;
  }();
  // enough workgroups for every CU before more windows per weight fetch
  const int nw = nw_env ? nw_env : (windows >= 2048 ? 4 : 2);
  static unsigned long long attr[4] = {0, 0, 0, 0};      // per device (lds_optin)
  lds_optin(reinterpret_cast<const void*>(winblock4_kernel<1>), wb4::LDS, &attr[0]);
  lds_optin(reinterpret_cast<const void*>(winblock4_kernel<2>), wb4::LDS, &attr[1]);
  lds_optin(reinterpret_cast<const void*>(winblock4_kernel<4>), wb4::LDS, &attr[2]);
  lds_optin(reinterpret_cast<const void*>(winblock4_kernel<8>), wb4::LDS, &attr[3]);
  const long long grid = (windows + nw - 1) / nw;
  RGBAC_REQUIRE(grid < (1LL << 31), "too many windows");
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  switch (nw) {
    case 1: hipLaunchKernelGGL(winblock4_kernel<1>, dim3((unsigned)grid), dim3(64), wb4::LDS, st, d); break;
    case 2: hipLaunchKernelGGL(winblock4_kernel<2>, dim3((unsigned)grid), dim3(128), wb4::LDS, st, d); break;
    case 4: hipLaunchKernelGGL(winblock4_kernel<4>, dim3((unsigned)grid), dim3(256), wb4::LDS, st, d); break;
    default: hipLaunchKernelGGL(winblock4_kernel<8>, dim3((unsigned)grid), dim3(512), wb4::LDS, st, d); break;
  }
  return check_launch("winblock4_kernel");
}
