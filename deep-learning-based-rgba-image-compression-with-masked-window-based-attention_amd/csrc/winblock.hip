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
// One workgroup = 2 windows = 128 tokens, 8 waves of 16 tokens (or 4 of 32; a wave's tokens
// lie in one window).  Per head pair (48 qkv channels of each kind):
//   QKV   q^T, k^T = Wq|Wk (LDS) x X^T (registers); v = X x Wv^T   -> LDS (bf16, padded to 32)
//   per head:  S^T = K Q^T (keys on the MFMA row axis), + B_rel (LDS table) + shift mask,
//              softmax (rows in 4 lanes: two xor-shuffles) -> P (wave-private LDS),
//              O^T = V^T P^T -> O (aliases P), out^T += Wproj[:, head] (LDS) x O^T (registers)
// The x tile stays in registers as MFMA fragments for all four pairs; the proj output
// (192 x 32 per wave) accumulates in registers over the 8 heads; the MASKSEL residual is
// the epilogue.  Weights are pre-packed fragment-major (1 KiB per 16 rows x 32 k) and
// streamed into LDS by LDS-DMA one pair / head ahead, waited on with counted vmcnt.
//
// MFMA v_mfma_f32_16x16x32_bf16 throughout (acc[row][col] += A[row][k] B[col][k]);
// per 32 tokens: 4 x 108 (QKV) + 8 x (8 + 8 + 24) = 752 MFMAs.  Softmax on exp2 with log2 e
// folded into the q scale and the bias tables.
//
// LDS (bytes): WQ 54 KiB | WP 2 x 12 KiB | QK [2 heads][q,k][128 tok][64 B] 32 KiB |
// VT [2 heads][32 ch][128 tok] 16 KiB | P/O [4 waves][4 KiB] | relative-position bias
// [table, table - 100 (the shift mask folded in)][8 heads][225] fp32 (head-major: the
// per-lane gathers spread over the banks) | proj bias -> 161,616 B: one workgroup per CU.
// Swizzles (all conflict-free for the ds_read_b128 lane groups): 64-B token rows
// chunk ^ ((tok >> 1) & 3); V^T 256-B rows chunk ^ (ch & 15); P 128-B rows chunk ^ (q & 7).
#include <cstdlib>

#include "common.h"

namespace rgbac {

namespace wb {
constexpr int WS = 8, NT = 64, C = 192, HEADS = 8, DH = 24, TOK = 128;
constexpr int WQF = 54;                                // qkv fragments per head pair
constexpr int WPF = 12;                                // proj fragments per head
constexpr int L_WQ = 0;
constexpr int L_WP = L_WQ + WQF * 1024;                // 55296
constexpr int L_QK = L_WP + 2 * WPF * 1024;            // 79872
constexpr int L_VT = L_QK + 2 * 2 * TOK * 64;          // 112640
constexpr int L_P = L_VT + 2 * 32 * TOK * 2;           // 129024
constexpr int L_TB = L_P + 4 * 4096;                   // 145408: bias [2][8 heads][225]
constexpr int L_BQ = L_TB + 2 * 8 * 225 * 4;           // 159808: bproj[192]
constexpr int LDS = L_BQ + 192 * 4;                    // 160576
}  // namespace wb

struct WinBlockArgs {
  int batch, H, W, shift, masked;
  float scale;
  const bf16_t* x; long long ldx;
  const float* alpha;                    // (B, H, W) fp32 when masked
  const bf16_t* wq;                      // [4 pairs][54][64 lanes][8]
  const float* bqkv;                     // [576]
  const bf16_t* wp;                      // [8 heads][12][64][8]
  const float* bproj;                    // [192]
  const float* table;                    // relative_position_bias_table [225][8]
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
template <int N>
__device__ __forceinline__ void wb_wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// NQT 16-token tiles per wave: NQT = 1 -> 8 waves (2 per SIMD: one wave's softmax VALU
// overlaps the other's MFMAs), NQT = 2 -> 4 waves (twice the weight-fragment reuse).
template <int NQT>
__global__ void __launch_bounds__(64 * 8 / NQT, 1) winblock_kernel(const WinBlockArgs a) {
  using namespace wb;
  constexpr int NWAVE = 8 / NQT, NTHR = 64 * NWAVE, TPW = 16 * NQT;
  constexpr int WQ_W = (WQF + NWAVE - 1) / NWAVE;      // DMA pieces per wave (7 or 14)
  constexpr int WP_W = (WPF + NWAVE - 1) / NWAVE;      // (2 or 3)
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
  const int tok0 = TPW * w;                            // this wave's first token (of 128)
  const int win = tok0 >> 6;                           // its window (0 or 1)
  const int lq0 = tok0 & 63;                           // ... and first query within it

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
    // both windows transparent: out = x on their tokens
    for (int e = tid; e < TOK * (C / 8); e += NTHR) {
      const int t = e / (C / 8), c8 = e - t * (C / 8);
      const int pix = pix_s[t];
      if (pix >= 0)
        *reinterpret_cast<uint4*>(a.out + (long long)pix * a.ldo + 8 * c8) =
            *reinterpret_cast<const uint4*>(a.x + (long long)pix * a.ldx + 8 * c8);
    }
    return;
  }

  // ---- weight streams: pair p's qkv fragments, head h's proj fragments (pieces past the
  // end repeat the last one: same bytes to the same place, so every wave issues as many)
  auto dma_wq = [&](int p) {
#pragma unroll
    for (int i = 0; i < WQ_W; ++i) {
      int f = w + NWAVE * i;
      if (f >= WQF) f = WQF - 1;
      wb_dma16(a.wq + ((size_t)(p * WQF + f) * 64 + lane) * 8, lds0 + L_WQ + f * 1024);
    }
  };
  auto dma_wp = [&](int h) {
#pragma unroll
    for (int i = 0; i < WP_W; ++i) {
      int f = w + NWAVE * i;
      if (f >= WPF) f = WPF - 1;
      wb_dma16(a.wp + ((size_t)(h * WPF + f) * 64 + lane) * 8,
               lds0 + L_WP + (h & 1) * WPF * 1024 + f * 1024);
    }
  };
  dma_wq(0);
  dma_wp(0);

  // ---- tables (in log2 units: softmax runs on exp2) and zero padding (q/k channels 24..31:
  // chunk 3; V^T rows 24..31)
  float* tb = reinterpret_cast<float*>(sm + L_TB);
  for (int e = tid; e < 225 * 8; e += NTHR) {          // table [225][8] -> [var][8][225]
    const int idx = e >> 3, hd = e & 7;
    const float v = a.table[e];
    tb[hd * 225 + idx] = v * LOG2E;
    tb[8 * 225 + hd * 225 + idx] = (v + -100.0f) * LOG2E;   // the shift mask's -100 folded in
  }
  float* bq = reinterpret_cast<float*>(sm + L_BQ);
  for (int e = tid; e < 192; e += NTHR) bq[e] = a.bproj[e];
  for (int e = tid; e < 2 * 2 * TOK; e += NTHR) {
    const int t = e & (TOK - 1);
    *reinterpret_cast<uint4*>(sm + L_QK + e * 64 + ((3 ^ ((t >> 1) & 3)) << 4)) = make_uint4(0, 0, 0, 0);
  }
  for (int e = tid; e < 2 * 8 * 16; e += NTHR) {       // [head][row 24..31][16 chunks]
    const int hh = e >> 7, r = 24 + ((e >> 4) & 7), c = e & 15;
    *reinterpret_cast<uint4*>(sm + L_VT + (hh * 32 + r) * 256 + (c << 4)) = make_uint4(0, 0, 0, 0);
  }

  // ---- this wave's x tile as MFMA fragments: X[j][ks] = tokens tok0+16j+n, k-chunk 4ks+qq
  uint4 X[NQT][6];
#pragma unroll
  for (int j = 0; j < NQT; ++j) {
    const int pix = pix_s[tok0 + 16 * j + n];
    const bf16_t* row = a.x + (long long)(pix < 0 ? 0 : pix) * a.ldx;
#pragma unroll
    for (int ks = 0; ks < 6; ++ks)
      X[j][ks] = pix < 0 ? make_uint4(0, 0, 0, 0)
                         : *reinterpret_cast<const uint4*>(row + 32 * ks + 8 * qq);
  }

  // ---- per-lane relative-position-bias offsets (head-invariant; +900 h per head), into the
  // "- 100" copy where the shift mask separates query and key:
  // S element (qt, kt, r) = (query lq0+16qt+n, key 16kt+4qq+r) of the window
  int toff[NQT][4][4];
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    const int iq = lq0 + 16 * qt + n;
    const int qrid = rid_s[64 * win + iq];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int jk = 16 * kt + 4 * qq + r;
        const int idx = ((iq >> 3) - (jk >> 3) + 7) * 15 + ((iq & 7) - (jk & 7) + 7);
        const bool cut = shift > 0 && rid_s[64 * win + jk] != qrid;
        toff[qt][kt][r] = L_TB + (cut ? 8 * 225 * 4 : 0) + idx * 4;
      }
  }

  f32x4 acc[12][NQT];                                  // proj output: [16-ch tile][token tile]
#pragma unroll
  for (int m = 0; m < 12; ++m)
#pragma unroll
    for (int j = 0; j < NQT; ++j) acc[m][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int swz64 = ((qq ^ ((n >> 1) & 3)) << 4);      // 64-B token rows, base % 16 == 0
  const float qscale = a.scale * LOG2E;                // q * scale, in log2 units
  wb_wait_vm<0>();
  __syncthreads();

  for (int p = 0; p < 4; ++p) {
    if (p > 0) {
      wb_wait_vm<WP_W>();                              // WQ(p) landed (WP(2p) may be in flight)
      __syncthreads();
    }
    // ================= QKV of heads 2p, 2p+1 for this wave's tokens
    if (act) {
      f32x4 aq[3][NQT], ak[3][NQT], av[NQT][3];
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int j = 0; j < NQT; ++j)
          aq[t][j] = ak[t][j] = av[j][t] = f32x4{0.f, 0.f, 0.f, 0.f};
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
        for (int t = 0; t < 3; ++t)
#pragma unroll
          for (int j = 0; j < NQT; ++j) {
            mma_step<bf16_t>(aq[t][j], fq[t], X[j][ks]);
            mma_step<bf16_t>(ak[t][j], fk[t], X[j][ks]);
            mma_step<bf16_t>(av[j][t], X[j][ks], fv[t]);
          }
      }
      // q (x scale), k -> token rows; v -> V^T rows.  Pair channel cp = 16t + 4qq + r.
#pragma unroll
      for (int t = 0; t < 3; ++t) {
        const int cp = 16 * t + 4 * qq;
        const int hh = cp >= DH ? 1 : 0, hc = cp - DH * hh;   // 4 channels, one head
        const float4 bq4 = *reinterpret_cast<const float4*>(a.bqkv + 48 * p + cp);
        const float4 bk4 = *reinterpret_cast<const float4*>(a.bqkv + 192 + 48 * p + cp);
#pragma unroll
        for (int j = 0; j < NQT; ++j) {
          const int tok = tok0 + 16 * j + n;
          const int off = tok * 64 + (((hc >> 3) ^ ((tok >> 1) & 3)) << 4) + 2 * (hc & 7);
          *reinterpret_cast<uint2*>(sm + L_QK + (hh * 2 + 0) * TOK * 64 + off) = make_uint2(
              pack_bf16x2((aq[t][j][0] + bq4.x) * qscale, (aq[t][j][1] + bq4.y) * qscale),
              pack_bf16x2((aq[t][j][2] + bq4.z) * qscale, (aq[t][j][3] + bq4.w) * qscale));
          *reinterpret_cast<uint2*>(sm + L_QK + (hh * 2 + 1) * TOK * 64 + off) = make_uint2(
              pack_bf16x2(ak[t][j][0] + bk4.x, ak[t][j][1] + bk4.y),
              pack_bf16x2(ak[t][j][2] + bk4.z, ak[t][j][3] + bk4.w));
        }
        // v: D[token][channel] -> lane holds tokens 16j+4qq+r of channel 16t+n
        const int cv = 16 * t + n;
        const int vh = cv >= DH ? 1 : 0, vc = cv - DH * vh;
        const float bv = a.bqkv[384 + 48 * p + cv];
#pragma unroll
        for (int j = 0; j < NQT; ++j) {
          const int tok = tok0 + 16 * j + 4 * qq;
          const int off = (vh * 32 + vc) * 256 + (((tok >> 3) ^ (vc & 15)) << 4) + 2 * (tok & 7);
          *reinterpret_cast<uint2*>(sm + L_VT + off) =
              make_uint2(pack_bf16x2(av[j][t][0] + bv, av[j][t][1] + bv),
                         pack_bf16x2(av[j][t][2] + bv, av[j][t][3] + bv));
        }
      }
    }
    __syncthreads();                                   // q/k/v of the pair visible; WQ free
    if (p < 3) dma_wq(p + 1);

#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int h = 2 * p + hh;
      unsigned char* const Pw = sm + L_P + w * (2048 * NQT);   // this wave's P, then O
      if (act) {
        // ---- S^T = K Q^T: keys (rows) of this window x this wave's queries
        f32x4 s[NQT][4];
        uint4 fqv[NQT], fkv[4];
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt)
          fqv[qt] = *reinterpret_cast<const uint4*>(
              sm + L_QK + (hh * 2 + 0) * TOK * 64 + (tok0 + 16 * qt + n) * 64 + swz64);
#pragma unroll
        for (int kt = 0; kt < 4; ++kt)
          fkv[kt] = *reinterpret_cast<const uint4*>(
              sm + L_QK + (hh * 2 + 1) * TOK * 64 + (64 * win + 16 * kt + n) * 64 + swz64);
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt)
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) {
            s[qt][kt] = f32x4{0.f, 0.f, 0.f, 0.f};
            mma_step<bf16_t>(s[qt][kt], fkv[kt], fqv[qt]);
          }
        // ---- + B_rel + shift mask, softmax (exp2: log2 e folded into q and the tables)
        // over the 64 keys (lane + lanes ^16, ^32, ^48)
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt) {
          float mx = -INFINITY;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float v = s[qt][kt][r] + *reinterpret_cast<const float*>(sm + toff[qt][kt][r] + 900 * h);
              s[qt][kt][r] = v;
              mx = fmaxf(mx, v);
            }
          mx = fmaxf(mx, __shfl_xor(mx, 16));
          mx = fmaxf(mx, __shfl_xor(mx, 32));
          float sum = 0.f;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float ex = __builtin_amdgcn_exp2f(s[qt][kt][r] - mx);
              s[qt][kt][r] = ex;
              sum += ex;
            }
          sum += __shfl_xor(sum, 16);
          sum += __shfl_xor(sum, 32);
          const float inv = __builtin_amdgcn_rcpf(sum);
          const int qi = 16 * qt + n;
#pragma unroll
          for (int kt = 0; kt < 4; ++kt) {
            const int k0 = 16 * kt + 4 * qq;
            *reinterpret_cast<uint2*>(Pw + qi * 128 + (((k0 >> 3) ^ (qi & 7)) << 4) + 2 * (k0 & 7)) =
                make_uint2(pack_bf16x2(s[qt][kt][0] * inv, s[qt][kt][1] * inv),
                           pack_bf16x2(s[qt][kt][2] * inv, s[qt][kt][3] * inv));
          }
        }
        // ---- O^T = V^T P^T: head channels (rows, 24..31 zero) x this wave's queries
        f32x4 o[2][NQT];
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt) o[ct][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          uint4 fa[2], fb[NQT];
#pragma unroll
          for (int ct = 0; ct < 2; ++ct) {
            const int ch = 16 * ct + n;
            fa[ct] = *reinterpret_cast<const uint4*>(
                sm + L_VT + (hh * 32 + ch) * 256 + (((8 * win + 4 * ks + qq) ^ (ch & 15)) << 4));
          }
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt) {
            const int qi = 16 * qt + n;
            fb[qt] = *reinterpret_cast<const uint4*>(Pw + qi * 128 + (((4 * ks + qq) ^ (qi & 7)) << 4));
          }
#pragma unroll
          for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int qt = 0; qt < NQT; ++qt) mma_step<bf16_t>(o[ct][qt], fa[ct], fb[qt]);
        }
        // O (token rows of 32 channels, bf16) over this wave's P: every P read above has
        // completed (its MFMAs produced o)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt) {
            const int tok = 16 * qt + n, c0 = 16 * ct + 4 * qq;
            *reinterpret_cast<uint2*>(Pw + tok * 64 + (((c0 >> 3) ^ ((tok >> 1) & 3)) << 4) + 2 * (c0 & 7)) =
                make_uint2(pack_bf16x2(o[ct][qt][0], o[ct][qt][1]),
                           pack_bf16x2(o[ct][qt][2], o[ct][qt][3]));
          }
      }
      // ---- WP(h) landed everywhere (WQ(p+1), issued after it, may still be in flight)
      if (hh == 0 && p < 3) wb_wait_vm<WQ_W>();
      else wb_wait_vm<0>();
      __syncthreads();
      if (h < HEADS - 1) dma_wp(h + 1);                // buffer (h+1)&1: proj(h-1) is done
      if (act) {
        // ---- out^T += Wproj[:, head h] O^T
        uint4 fo[NQT];
#pragma unroll
        for (int qt = 0; qt < NQT; ++qt)
          fo[qt] = *reinterpret_cast<const uint4*>(Pw + (16 * qt + n) * 64 + swz64);
#pragma unroll
        for (int m = 0; m < 12; ++m) {
          const uint4 fw = *reinterpret_cast<const uint4*>(
              sm + L_WP + (h & 1) * WPF * 1024 + m * 1024 + lane * 16);
#pragma unroll
          for (int qt = 0; qt < NQT; ++qt) mma_step<bf16_t>(acc[m][qt], fw, fo[qt]);
        }
      }
    }
  }

  // ---- epilogue: out = x + proj + b (active window) or x (MASKSEL, :236-240)
  const float* bp = reinterpret_cast<const float*>(sm + L_BQ);
#pragma unroll
  for (int qt = 0; qt < NQT; ++qt) {
    const int pix = pix_s[tok0 + 16 * qt + n];
    if (pix < 0) continue;
    const bf16_t* xr = a.x + (long long)pix * a.ldx;
    bf16_t* orow = a.out + (long long)pix * a.ldo;
#pragma unroll
    for (int m = 0; m < 12; ++m) {
      const int c0 = 16 * m + 4 * qq;
      const uint2 xv = *reinterpret_cast<const uint2*>(xr + c0);
      float v[4] = {bf2f(xv.x & 0xFFFF), bf2f(xv.x >> 16), bf2f(xv.y & 0xFFFF), bf2f(xv.y >> 16)};
      if (act) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += acc[m][qt][r] + bp[c0 + r];
      }
      *reinterpret_cast<uint2*>(orow + c0) =
          make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
    }
  }
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_winattn_block(int batch, int h, int w, int shift, int masked, float scale,
                                   const void* x, int64_t ldx, const float* alpha,
                                   const void* wq_packed, const float* bqkv,
                                   const void* wp_packed, const float* bproj, const float* table,
                                   void* out, int64_t ldo, void* stream) {
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && h % 8 == 0 && w % 8 == 0,
                "H and W must be positive multiples of the window size 8");
  RGBAC_REQUIRE(shift >= 0 && shift < 8, "0 <= shift < 8");
  RGBAC_REQUIRE(x && out && wq_packed && bqkv && wp_packed && bproj && table, "null pointer");
  RGBAC_REQUIRE(!masked || alpha, "masked attention needs alpha");
  RGBAC_REQUIRE(ldx >= 192 && ldo >= 192 && ldx % 8 == 0 && ldo % 8 == 0, "strides");
  RGBAC_REQUIRE(x != out, "out must not alias x");
  const long long windows = (long long)batch * (h / 8) * (w / 8);
  RGBAC_REQUIRE(windows < (1LL << 30), "too many windows");
  WinBlockArgs d;
  d.batch = batch; d.H = h; d.W = w; d.shift = shift; d.masked = masked; d.scale = scale;
  d.x = reinterpret_cast<const bf16_t*>(x); d.ldx = ldx; d.alpha = alpha;
  d.wq = reinterpret_cast<const bf16_t*>(wq_packed); d.bqkv = bqkv;
  d.wp = reinterpret_cast<const bf16_t*>(wp_packed); d.bproj = bproj; d.table = table;
  d.out = reinterpret_cast<bf16_t*>(out); d.ldo = ldo;
  static const int nqt = [] {
    const char* e = getenv("RGBAC_WINBLOCK_NQT");      // 1: 8 waves (default), 2: 4 waves
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(winblock_kernel<1>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, wb::LDS);
    hipFuncSetAttribute(reinterpret_cast<const void*>(winblock_kernel<2>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, wb::LDS);
    attr = true;
  }
  const dim3 grid((int)((windows + 1) / 2));
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (nqt == 2) hipLaunchKernelGGL(winblock_kernel<2>, grid, dim3(256), wb::LDS, st, d);
  else hipLaunchKernelGGL(winblock_kernel<1>, grid, dim3(512), wb::LDS, st, d);
  return check_launch("winblock_kernel");
}
