// Fused DSE EnhancementBlock (reference: layers/TransformRGB.py:16-49, and the alpha
// codec's DSE, models/AutoEncoderMask_Journal.py:39-48)
//
//   block(t) = conv2( ReLU( conv1(t) ) ) + t          (3x3, 32 -> 32, zero padding;
//                                                      LeakyReLU in the alpha codec)
//   DSE(x)   = out_conv( block3(block2(block1(f))) + f ) + x,   f = in_conv(x)  (1x1)
//
// One launch per block instead of two 3x3 conv passes (plus the two 1x1 passes): the
// ReLU intermediate never leaves LDS.  mode FIRST also evaluates f = in_conv(x) on the
// block's input halo (from the 1/3-channel DSE input, never materialising f in HBM);
// mode LAST adds f (recomputed from x at the output pixels), rounds the block output to
// bf16 (where the unfused path stores it) and runs out_conv + identity, writing the
// 1/3-channel DSE output.  So one DSE is 3 launches moving ~10 + 67 + 10 B per pixel
// instead of 8 launches moving ~480 B per pixel.
//
// Persistent workgroups (one per CU, 8 waves) loop over 16x32 output tiles:
//   In : the block input on the 20x36 halo                               (47.1 KB)
//   U  : act(conv1) on 18 rows x 36 (34 needed; zero outside the image)   (42.0 KB)
//   W  : conv1 / conv2 weights as MFMA A fragments (1 KiB per tap/16 rows) (36.9 KB)
// In and U share the row stride 36, so a U pixel's tap pixel in In is p + 36 dy + dx and
// conv1 runs over U flattened into 41 16-pixel fragments.  Chunk c of pixel p sits at
// slot c ^ ((p >> 1) & 3): conflict-free for the ds_read_b128 lane groups over any 16
// consecutive pixels, and -- every fragment starting at a multiple of 8 pixels (or 4 more,
// on odd conv2 rows) -- the swizzle of a lane depends only on its tap, so each fragment
// read is one precomputed lane offset + an immediate: no address VALU in the MFMA loops.
// The next tile's In is loaded into registers while this tile computes.
//
// MFMA v_mfma_f32_16x16x32_bf16 with A = weights (16 output channels x one tap's 32
// input channels), B = 16 pixels x 32 channels: each lane ends with 4 consecutive
// channels of one pixel.  Per 16x32 tile: conv1 40.5 fragments x 2 x 9, conv2 32 x 2 x 9.
#include <cstdlib>

#include "common.h"

namespace rgbac {

namespace dse {
constexpr int TY = 16, TX = 32;
constexpr int RS = TX + 4;                                   // In and U row stride (36 px)
constexpr int IH = TY + 4, UH = TY + 2;                      // In / U rows
constexpr int NIV = IH * RS;                                 // 720 In pixels
constexpr int NUF = (UH * RS + 15) / 16;                     // 41 conv1 fragments (648 px)
constexpr int NI = NUF * 16 + 2 * RS + 2 + 6;                // In slots incl. conv1 overrun
constexpr int WBYTES = 2 * 2 * 9 * 64 * 16;                  // 36864
constexpr int IBASE = WBYTES;
constexpr int UBASE = IBASE + NI * 64;                       // In: 47104 B
constexpr int LDS = UBASE + NUF * 16 * 64;                   // U: 41984 B -> 125952 B
enum { FIRST = 0, MID = 1, LAST = 2 };
}  // namespace dse

struct DseArgsDev {
  int batch, H, W, cin, mode;
  float slope;                           // block activation: ReLU (0) or LeakyReLU slope
  const bf16_t* x; long long ldx;        // DSE input (cin channels)       FIRST / LAST
  const bf16_t* t; long long ldt;        // block input (32 channels)      MID / LAST
  const bf16_t* w_in; int kp_in; const float* b_in;
  const bf16_t* w1; int kp1; const float* b1;
  const bf16_t* w2; int kp2; const float* b2;
  const bf16_t* w_out; int kp_out; const float* b_out;
  bf16_t* out; long long ldo;            // 32-channel block output, or the DSE output (LAST)
};

__device__ __forceinline__ uint4 lds16(const unsigned char* base, int off) {
  return *reinterpret_cast<const uint4*>(base + off);
}

// 8 waves, two per SIMD; conv1 / conv2 weight fragments read from LDS per tap.  (A 4-wave form
// holding conv1's weights in registers measured 20-40 % slower and was removed)
template <int MODE, int CIN>
__global__ void __launch_bounds__(512) dse_block_kernel(const DseArgsDev a) {
  using namespace dse;
  constexpr int NW = 8;
  constexpr int NTH = 64 * NW;
  constexpr int PRE = (NIV * 4 + NTH - 1) / NTH;             // In chunks per thread (6 / 12)
  constexpr int FST = 1024 * NW;                              // byte step between a wave's fragments
  constexpr int RPW = 16 / NW;                                // conv2 output rows per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float bb1[32], bb2[32];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n16 = lane & 15, q = lane >> 4;
  const int H = a.H, W = a.W;
  const int tx_n = (W + TX - 1) / TX, ty_n = (H + TY - 1) / TY;
  const int ntiles = a.batch * tx_n * ty_n;
  const float slope = a.slope;

  // ---- weights: conv1 / conv2 as A fragments (1 KiB per (conv, 16 rows, tap))
  for (int e = tid; e < 2 * 2 * 9 * 64; e += NTH) {
    const int l = e & 63, f = e >> 6;               // f = (conv*2 + j)*9 + tap
    const int tap = f % 9, j = (f / 9) & 1, cv = f / 18;
    const bf16_t* w = cv ? a.w2 : a.w1;
    const int kp = cv ? a.kp2 : a.kp1;
    *reinterpret_cast<uint4*>(smem + e * 16) = *reinterpret_cast<const uint4*>(
        w + (size_t)(16 * j + (l & 15)) * kp + tap * 32 + 8 * (l >> 4));
  }
  if (tid < 32) {
    bb1[tid] = a.b1[tid];
    bb2[tid] = a.b2[tid];
  }
  // 1x1 weights in registers, for the 8 channels this thread produces: FIRST -- chunk
  // tid & 3 of every In pixel it fills; LAST -- 16j + 4q + r of its output fragments
  constexpr int NC = CIN > 0 ? CIN : 1;
  float wi[8][NC], bi[8], wo[NC][8], bo[NC];
  if (MODE != MID) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ch = MODE == FIRST ? 8 * (tid & 3) + i : 16 * (i >> 2) + 4 * q + (i & 3);
      bi[i] = a.b_in[ch];
#pragma unroll
      for (int k = 0; k < NC; ++k) wi[i][k] = bf2f(a.w_in[(size_t)ch * a.kp_in + k].u);
      if (MODE == LAST) {
#pragma unroll
        for (int c = 0; c < NC; ++c) wo[c][i] = bf2f(a.w_out[(size_t)c * a.kp_out + ch].u);
      }
    }
    if (MODE == LAST) {
#pragma unroll
      for (int c = 0; c < NC; ++c) bo[c] = a.b_out[c];
    }
  }

  // ---- LDS byte offsets, tile-invariant.  Pixel p chunk c lives at p*64 + 16*(c ^ ((p>>1)&3)).
  // Every fragment of this wave starts at a pixel whose (p>>1)&3 contribution is known
  // (multiples of 8, or 36*odd rows: +2), so each read below is ONE lane offset + an
  // immediate: conv1 fragment i of tap t at o1[t] + 8192 i; conv2 fragment i at
  // o2[i>>1][t] + 64*(36*(i>>1) + 16*(i&1)).
  int o1[9], o2[2][9], ow[2], orr[2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    const int toff = (t / 3) * RS + t % 3;
    const int x = n16 + toff;
    o1[t] = IBASE + (16 * wave + x) * 64 + ((q ^ ((x >> 1) & 3)) << 4);
#pragma unroll
    for (int par = 0; par < 2; ++par)
      o2[par][t] = UBASE + (RPW * RS * wave + x) * 64 + ((q ^ ((2 * par + (x >> 1)) & 3)) << 4);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = 2 * j + (q >> 1);
    ow[j] = UBASE + (16 * wave + n16) * 64 + ((c ^ ((n16 >> 1) & 3)) << 4) + 8 * (q & 1);
#pragma unroll
    for (int par = 0; par < 2; ++par)
      orr[par][j] = IBASE + (RPW * RS * wave + 2 * RS + n16 + 2) * 64 +
                    ((c ^ ((2 * par + ((n16 + 2) >> 1)) & 3)) << 4) + 8 * (q & 1);
  }
  // In fill: chunk c = tid & 3 of pixels p = tid/4 + (NTH/4) r -> LDS at ofill + 16 NTH r
  const int ofill = IBASE + (tid >> 2) * 64 + (((tid & 3) ^ ((tid >> 3) & 3)) << 4);
  // conv1 extra fragment 40 (pixels 640..655): waves 0 and 1, one 16-channel half each;
  // its offsets are this wave's fragment-0 offsets moved from pixel 16*wave to 640
  const int xoff = (NUF - 1) * 1024 - 1024 * wave;

  auto load_in = [&](int t, uint4 (&pre)[PRE]) {
    int tt = t;
    const int tx = tt % tx_n; tt /= tx_n;
    const int ty = tt % ty_n;
    const int b = tt / ty_n;
#pragma unroll
    for (int r = 0; r < PRE; ++r) {
      const int p = (tid >> 2) + (NTH / 4) * r;
      const int py = p / RS, px = p - py * RS;
      const int gy = ty * TY - 2 + py, gx = tx * TX - 2 + px;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (p < NIV && (unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W) {
        const long long pix = (long long)(b * H + gy) * W + gx;
        if (MODE == FIRST) {
          v = *reinterpret_cast<const uint4*>(a.x + pix * a.ldx);
          v.w |= 0x80000000u;                           // "inside" mark (channel 7 unused)
        } else {
          v = *reinterpret_cast<const uint4*>(a.t + pix * a.ldt + 8 * (tid & 3));
        }
      }
      pre[r] = v;
    }
  };
  auto store_in = [&](const uint4 (&pre)[PRE]) {
#pragma unroll
    for (int r = 0; r < PRE; ++r) {
      if ((tid >> 2) + (NTH / 4) * r >= NIV) continue;
      uint4 v = pre[r];
      if (MODE == FIRST) {
        // f = in_conv(x) (bf16 weights and input, fp32 sum, + bias, stored bf16); 0 outside
        const bool inside = (v.w & 0x80000000u) != 0;
        v.w &= 0x7FFFFFFFu;
        const float xv[8] = {bf2f(v.x & 0xFFFF), bf2f(v.x >> 16), bf2f(v.y & 0xFFFF),
                             bf2f(v.y >> 16), bf2f(v.z & 0xFFFF), bf2f(v.z >> 16),
                             bf2f(v.w & 0xFFFF), bf2f(v.w >> 16)};
        float f[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          float s = 0.f;
#pragma unroll
          for (int k = 0; k < NC; ++k) s = fmaf(wi[i][k], xv[k], s);
          f[i] = inside ? s + bi[i] : 0.f;
        }
        v = make_uint4(pack_bf16x2(f[0], f[1]), pack_bf16x2(f[2], f[3]),
                       pack_bf16x2(f[4], f[5]), pack_bf16x2(f[6], f[7]));
      }
      *reinterpret_cast<uint4*>(smem + ofill + 16 * NTH * r) = v;
    }
  };

  int t = blockIdx.x;
  if (t >= ntiles) return;
  uint4 pre[PRE];
  load_in(t, pre);
  __syncthreads();                                     // weights + biases visible
  store_in(pre);

  for (; t < ntiles; t += gridDim.x) {
    int tt = t;
    const int tx = tt % tx_n; tt /= tx_n;
    const int ty = tt % ty_n;
    const int b = tt / ty_n;
    const int y0 = ty * TY, x0 = tx * TX;
    __syncthreads();                                   // In of this tile complete
    if (t + (int)gridDim.x < ntiles) load_in(t + gridDim.x, pre);   // next tile, in flight

    // ================= conv1 + act -> U (zero outside the image)
    {
      constexpr int NF = 40 / NW;                      // + fragment 40 (half) on waves 0, 1
      const bool extra = wave < 2;
      f32x4 acc[NF][2], accx;
#pragma unroll
      for (int i = 0; i < NF; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      accx = f32x4{0.f, 0.f, 0.f, 0.f};
      const int ax = extra ? wave : 0;                 // the extra fragment's channel half
      uint4 A[2][2], B[2][NF], BX[2], AX[2];
      auto load = [&](int tp, int sb) {
        A[sb][0] = lds16(smem, ((0 * 9 + tp) * 64 + lane) * 16);
        A[sb][1] = lds16(smem, ((1 * 9 + tp) * 64 + lane) * 16);
#pragma unroll
        for (int i = 0; i < NF; ++i) B[sb][i] = lds16(smem, o1[tp] + FST * i);
        if (extra) {
          BX[sb] = lds16(smem, o1[tp] + xoff);
          AX[sb] = ax ? A[sb][1] : A[sb][0];
        }
      };
      load(0, 0);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int sb = tp & 1;
        if (tp < 8) load(tp + 1, sb ^ 1);
#pragma unroll
        for (int i = 0; i < NF; ++i) {
          mma_step<bf16_t>(acc[i][0], A[sb][0], B[sb][i]);
          mma_step<bf16_t>(acc[i][1], A[sb][1], B[sb][i]);
        }
        if (extra) mma_step<bf16_t>(accx, AX[sb], BX[sb]);
        __builtin_amdgcn_sched_barrier(0);
      }
      // bias + act -> bf16 U; outside the image the 3x3 sees zero padding
      const bool interior = y0 >= 1 && x0 >= 1 && y0 + UH - 1 <= H && x0 + TX + 1 <= W;
      auto emit = [&](const f32x4& ac, int j, int f, int off) {
        const int c0 = 16 * j + 4 * q;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float s = ac[r] + bb1[c0 + r];
          v[r] = fmaxf(s, s * slope);                 // ReLU / LeakyReLU, 0 <= slope <= 1
        }
        if (!interior) {
          const int pu = 16 * f + n16;
          const int uy = pu / RS, ux = pu - uy * RS;
          const int gy = y0 - 1 + uy, gx = x0 - 1 + ux;
          if (!((unsigned)gy < (unsigned)H && (unsigned)gx < (unsigned)W))
            v[0] = v[1] = v[2] = v[3] = 0.f;
        }
        *reinterpret_cast<uint2*>(smem + off) =
            make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3]));
      };
#pragma unroll
      for (int i = 0; i < NF; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) emit(acc[i][j], j, wave + NW * i, ow[j] + FST * i);
      if (extra) emit(accx, ax, NUF - 1, (ax ? ow[1] : ow[0]) + xoff);
    }
    __syncthreads();                                   // U complete

    // ================= conv2 + bias + residual (+ f, out_conv, identity) -> HBM
    {
      constexpr int NF2 = 2 * RPW;                     // output fragments per wave (4 / 8)
      f32x4 acc[NF2][2];
#pragma unroll
      for (int i = 0; i < NF2; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      uint4 A[2][2], B[2][NF2];
      auto load = [&](int tp, int sb) {
        A[sb][0] = lds16(smem, ((2 * 9 + tp) * 64 + lane) * 16);
        A[sb][1] = lds16(smem, ((3 * 9 + tp) * 64 + lane) * 16);
#pragma unroll
        for (int i = 0; i < NF2; ++i)
          B[sb][i] = lds16(smem, o2[(i >> 1) & 1][tp] + 64 * (RS * (i >> 1) + 16 * (i & 1)));
      };
      load(0, 0);
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int sb = tp & 1;
        if (tp < 8) load(tp + 1, sb ^ 1);
#pragma unroll
        for (int i = 0; i < NF2; ++i) {
          mma_step<bf16_t>(acc[i][0], A[sb][0], B[sb][i]);
          mma_step<bf16_t>(acc[i][1], A[sb][1], B[sb][i]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      const long long pix0 = (long long)(b * H + y0) * W + x0;
#pragma unroll
      for (int i = 0; i < NF2; ++i) {
        const int oy = RPW * wave + (i >> 1), ox = 16 * (i & 1) + n16;
        const bool inside = y0 + oy < H && x0 + ox < W;
        const long long pix = pix0 + (long long)oy * W + ox;
        float v[2][4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int c0 = 16 * j + 4 * q;
          const uint2 rv = *reinterpret_cast<const uint2*>(
              smem + orr[(i >> 1) & 1][j] + 64 * (RS * (i >> 1) + 16 * (i & 1)));
          const float r4[4] = {bf2f(rv.x & 0xFFFF), bf2f(rv.x >> 16), bf2f(rv.y & 0xFFFF),
                               bf2f(rv.y >> 16)};
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] = acc[i][j][r] + bb2[c0 + r] + r4[r];
        }
        if (MODE != LAST) {
          if (inside) {
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              const int c0 = 16 * j + 4 * q;
              *reinterpret_cast<uint2*>(a.out + pix * a.ldo + c0) =
                  make_uint2(pack_bf16x2(v[j][0], v[j][1]), pack_bf16x2(v[j][2], v[j][3]));
            }
          }
        } else {
          // + f = in_conv(x) at this pixel, rounded to bf16 as the unfused path stores it
          uint4 xr = make_uint4(0, 0, 0, 0);
          if (inside) xr = *reinterpret_cast<const uint4*>(a.x + pix * a.ldx);
          const float xv[8] = {bf2f(xr.x & 0xFFFF), bf2f(xr.x >> 16), bf2f(xr.y & 0xFFFF),
                               bf2f(xr.y >> 16), bf2f(xr.z & 0xFFFF), bf2f(xr.z >> 16),
                               bf2f(xr.w & 0xFFFF), bf2f(xr.w >> 16)};
          float o[NC];
#pragma unroll
          for (int c = 0; c < NC; ++c) o[c] = 0.f;
#pragma unroll
          for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int i8 = 4 * j + r;
              float s = 0.f;
#pragma unroll
              for (int k = 0; k < NC; ++k) s = fmaf(wi[i8][k], xv[k], s);
              const float f = bf2f(f2bf(s + bi[i8]));
              const float vb = bf2f(f2bf(v[j][r] + f));       // block3 + x_first, stored bf16
#pragma unroll
              for (int c = 0; c < NC; ++c) o[c] = fmaf(wo[c][i8], vb, o[c]);
            }
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            o[c] = sum16_f(o[c]);
            o[c] = sum32_f(o[c]);
          }
          if (inside && q == 0) {
            bf16_t* dst = a.out + pix * a.ldo;
#pragma unroll
            for (int c = 0; c < NC; ++c) dst[c].u = f2bf(o[c] + bo[c] + xv[c]);
          }
        }
      }
    }
    if (t + (int)gridDim.x < ntiles) {
      __syncthreads();                                 // every read of In / U done
      store_in(pre);
    }
  }
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_dse_block(int mode, int batch, int h, int w, int cin, float slope, const void* x,
                               int64_t ldx, const void* t, int64_t ldt, const void* w_in,
                               int kp_in, const float* b_in, const void* w1, int kp1,
                               const float* b1, const void* w2, int kp2, const float* b2,
                               const void* w_out, int kp_out, const float* b_out, void* out,
                               int64_t ldo, void* stream) {
  RGBAC_REQUIRE(mode >= 0 && mode <= 2, "mode must be 0 (first), 1 (mid) or 2 (last)");
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0, "empty input");
  RGBAC_REQUIRE(w1 && w2 && b1 && b2 && out, "null conv1/conv2 operand");
  RGBAC_REQUIRE(kp1 >= 288 && kp2 >= 288, "conv1/conv2 must be 3x3 32->32 packs (k_pad >= 288)");
  RGBAC_REQUIRE(slope >= 0.f && slope <= 1.f, "activation slope must be in [0, 1]");
  if (mode != 1) {
    RGBAC_REQUIRE(x && w_in && b_in, "first/last block needs the DSE input and in_conv");
    RGBAC_REQUIRE(cin == 1 || cin == 3, "DSE input channels must be 1 or 3");
    RGBAC_REQUIRE(ldx >= 8 && ldx % 8 == 0, "DSE input ldc must be a multiple of 8");
    RGBAC_REQUIRE(kp_in >= cin, "in_conv pack too narrow");
  }
  if (mode != 0) RGBAC_REQUIRE(t && ldt >= 32 && ldt % 8 == 0, "block input must be 32 channels, ldc % 8 == 0");
  if (mode == 2) RGBAC_REQUIRE(w_out && b_out && kp_out >= 32 && ldo >= cin, "last block needs out_conv");
  else RGBAC_REQUIRE(ldo >= 32 && ldo % 4 == 0, "block output must be 32 channels");
  DseArgsDev d;
  d.batch = batch; d.H = h; d.W = w; d.cin = cin; d.mode = mode; d.slope = slope;
  d.x = reinterpret_cast<const bf16_t*>(x); d.ldx = ldx;
  d.t = reinterpret_cast<const bf16_t*>(t); d.ldt = ldt;
  d.w_in = reinterpret_cast<const bf16_t*>(w_in); d.kp_in = kp_in; d.b_in = b_in;
  d.w1 = reinterpret_cast<const bf16_t*>(w1); d.kp1 = kp1; d.b1 = b1;
  d.w2 = reinterpret_cast<const bf16_t*>(w2); d.kp2 = kp2; d.b2 = b2;
  d.w_out = reinterpret_cast<const bf16_t*>(w_out); d.kp_out = kp_out; d.b_out = b_out;
  d.out = reinterpret_cast<bf16_t*>(out); d.ldo = ldo;
  const int ncu = device_cus();
  const long long ntiles = (long long)batch * ((h + dse::TY - 1) / dse::TY) * ((w + dse::TX - 1) / dse::TX);
  RGBAC_REQUIRE(ntiles < (1LL << 30), "too many tiles");
  const int grid = (int)(ntiles < ncu ? ntiles : ncu);
  const size_t lds = dse::LDS;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int key = mode == 1 ? 10 : mode * 100 + cin;
  switch (key) {
#define RGBAC_DSE(M_, C_)                                                                       \
  case (M_ == 1 ? 10 : M_ * 100 + C_): {                                                      \
    static unsigned long long attr = 0;                                                         \
    lds_optin(reinterpret_cast<const void*>(dse_block_kernel<M_, C_>), (int)lds, &attr);       \
    hipLaunchKernelGGL((dse_block_kernel<M_, C_>), dim3(grid), dim3(512), lds, st, d);          \
    break;                                                                                      \
  }
    RGBAC_DSE(0, 1)
    RGBAC_DSE(0, 3)
    RGBAC_DSE(1, 0)
    RGBAC_DSE(2, 1)
    RGBAC_DSE(2, 3)
#undef RGBAC_DSE
    default:
      RGBAC_REQUIRE(false, "DSE input channels must be 1 or 3");
  }
  return check_launch("dse_block_kernel");
}
