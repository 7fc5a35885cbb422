// Implicit-GEMM convolution family on CDNA4 MFMA with fused epilogues.
//
// GEMM view (output-stationary, NHWC):   D[n][m] = sum_k W[n][k] * X[m][k]
//   n = output channel, m = output pixel of the "M grid", k = (tap, cin).
// A operand = packed weights [cout_pad][k_pad] (K contiguous), B operand =
// im2col rows gathered on the fly from up to three NHWC sources (fused
// channel concat).  Putting the channel on the MFMA row axis makes every lane
// own 4 consecutive channels of one pixel in the accumulator, so epilogue
// loads/stores are 16-byte (f32) / 8-byte (bf16) channel vectors.
//
// Tile: 256 threads = 4 waves, BM = 128 pixels (32 per wave), BN = 16*WN
// channels, K staged 128 bytes per row per step (64 bf16 / 32 f32) through a
// double-buffered, XOR-swizzled LDS image (chunk c of row r at c ^ (r & 7):
// conflict-free ds_read_b128 for the 16-lane fragment groups).
//   bf16: v_mfma_f32_16x16x32_bf16, one per 16x16 tile per 32-deep k-step.
//   f32 : v_mfma_f32_16x16x4_f32 x4 per 16-deep k-step (exact f32 FMA chain;
//         parity mode).  Lane l feeds k = 4*(l>>4)+e to MFMA e for both
//         operands, which is a permutation of k and so the same sum.
//
// Modes (rgbac_conv_mode): plain conv (stride 1/2), ConvTranspose2d(5, s2,
// p2, op1) split into 4 output-parity phases (blockIdx.z) each of which is a
// stride-1 conv with 3x3/3x2/2x3/2x2 taps, and subpel conv3x3 + PixelShuffle(2)
// folded into the store.
#include "common.h"

namespace rgbac {

struct ConvParams {
  int mode, batch, in_h, in_w, Hm, Wm, out_h, out_w, M, sy;
  int ksize, pad;
  int nsrc;
  const void* sp0; const void* sp1; const void* sp2;
  long long sld0, sld1, sld2;
  int send0, send1, send2;          // cumulative channel ends
  int cin_pad, k_pad;
  int cout, cout_pad;
  const void* w;
  const float* bias;
  void* out; long long out_ldc; int out_coff;
  int act; float act_param; int square;
  const void* res0; long long ld0;
  const void* res1; long long ld1;
  const void* res2; long long ld2;
  const uint8_t* sel;
};

__device__ __forceinline__ float gelu_f(float v) {
  return 0.5f * v * (1.0f + erff(v * 0.70710678118654752440f));
}
__device__ __forceinline__ float sigmoid_f(float v) { return 1.0f / (1.0f + expf(-v)); }

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

template <typename T>
__device__ __forceinline__ void epi_store(const ConvParams& p, int opix, int n, float (&v)[4]) {
  T* out = reinterpret_cast<T*>(p.out);
  const long long base = (long long)opix * p.out_ldc + p.out_coff + n;
  if (n + 3 < p.cout) {
    Elem<T>::st4(out + base, v);
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < p.cout) Elem<T>::st(out + base + r, v[r]);
  }
}

template <typename T>
__device__ __forceinline__ void load_res(const void* ptr, long long ld, int opix, int n,
                                         int cout, float (&v)[4]) {
  const T* r = reinterpret_cast<const T*>(ptr) + (long long)opix * ld + n;
  if (n + 3 < cout) {
    Elem<T>::ld4(r, v);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = (n + q < cout) ? Elem<T>::ld(r + q) : 0.0f;
  }
}

template <typename T, int WN>
__global__ void __launch_bounds__(256) conv_kernel(const ConvParams p) {
  constexpr int EPV = Elem<T>::EPV;
  constexpr int KB = 8 * EPV;       // elements of K per stage (128 bytes/row)
  constexpr int BN = 16 * WN;
  constexpr int BM = 128;
  constexpr int WM = 2;
  constexpr int A_ITERS = (BN * 8 + 255) / 256;
  __shared__ uint4 As[2][BN * 8];
  __shared__ uint4 Bs[2][BM * 8];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int phase = blockIdx.z;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int py = phase >> 1, px = phase & 1;
  int ntaps, tw;  // taps and taps per row for this phase
  if (p.mode == RGBAC_CONVT_S2) {
    tw = 3 - px;
    ntaps = (3 - py) * tw;
  } else {
    tw = p.ksize;
    ntaps = p.ksize * p.ksize;
  }
  const int ktot = ntaps * p.cin_pad;
  const int nk = (ktot + KB - 1) / KB;
  const T* wbase = reinterpret_cast<const T*>(p.w) + (size_t)phase * p.cout_pad * p.k_pad;

  // ---- per-thread im2col row state (rows fixed across the K loop)
  const int c = tid & 7;
  int rb[4], riy[4], rix[4];
  bool rv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    rv[i] = m < p.M;
    const int mm = rv[i] ? m : 0;
    const int mx = mm % p.Wm;
    const int t = mm / p.Wm;
    const int my = t % p.Hm;
    rb[i] = t / p.Hm;
    riy[i] = my * p.sy;
    rix[i] = mx * p.sy;
  }

  uint4 ra[A_ITERS], rbv[4];

  auto load_stage = [&](int kb) {
    // weights
#pragma unroll
    for (int i = 0; i < A_ITERS; ++i) {
      const int q = tid + 256 * i;
      if (q < BN * 8) {
        const int row = q >> 3;
        ra[i] = *reinterpret_cast<const uint4*>(wbase + (size_t)(n0 + row) * p.k_pad + kb * KB +
                                                (q & 7) * EPV);
      }
    }
    // activations (im2col gather)
    const int k = kb * KB + c * EPV;
    const int tap = k / p.cin_pad;
    const int ci = k - tap * p.cin_pad;
    bool kval = tap < ntaps;
    int dy, dx;
    {
      const int ty = tap / tw, tx = tap - ty * tw;
      if (p.mode == RGBAC_CONVT_S2) {
        dy = 1 - ty;
        dx = 1 - tx;
      } else {
        dy = ty - p.pad;
        dx = tx - p.pad;
      }
    }
    const void* sp;
    long long sld;
    int cs;
    if (ci < p.send0) {
      sp = p.sp0; sld = p.sld0; cs = ci;
    } else if (ci < p.send1) {
      sp = p.sp1; sld = p.sld1; cs = ci - p.send0;
    } else {
      sp = p.sp2; sld = p.sld2; cs = ci - p.send1;
      kval = kval && (ci < p.send2);
    }
    const T* src = reinterpret_cast<const T*>(sp);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int iy = riy[i] + dy, ix = rix[i] + dx;
      const bool ok = kval && rv[i] && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ok) {
        const long long off = ((long long)(rb[i] * p.in_h + iy) * p.in_w + ix) * sld + cs;
        v = *reinterpret_cast<const uint4*>(src + off);
        if (p.square) v = square_chunk<T>(v);
      }
      rbv[i] = v;
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_ITERS; ++i) {
      const int q = tid + 256 * i;
      if (q < BN * 8) {
        const int row = q >> 3;
        As[buf][row * 8 + ((q & 7) ^ (row & 7))] = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = (tid >> 3) + 32 * i;
      Bs[buf][row * 8 + (c ^ (row & 7))] = rbv[i];
    }
  };

  f32x4 acc[WN][WM];
#pragma unroll
  for (int j = 0; j < WN; ++j)
#pragma unroll
    for (int i = 0; i < WM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4, sw = lane & 7;
  for (int kb = 0; kb < nk; ++kb) {
    const int cur = kb & 1;
    if (kb + 1 < nk) load_stage(kb + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int chunk = (4 * s + fq) ^ sw;
      uint4 a[WN], b[WM];
#pragma unroll
      for (int j = 0; j < WN; ++j) a[j] = As[cur][(j * 16 + fr) * 8 + chunk];
#pragma unroll
      for (int i = 0; i < WM; ++i) b[i] = Bs[cur][(wave * 32 + i * 16 + fr) * 8 + chunk];
#pragma unroll
      for (int j = 0; j < WN; ++j)
#pragma unroll
        for (int i = 0; i < WM; ++i) mma_step<T>(acc[j][i], a[j], b[i]);
    }
    if (kb + 1 < nk) store_stage(cur ^ 1);
    __syncthreads();
  }

  // ---- fused epilogue: lane owns channels n..n+3 of pixel m per tile
#pragma unroll
  for (int i = 0; i < WM; ++i) {
    const int m = m0 + wave * 32 + i * 16 + fr;
    if (m >= p.M) continue;
    const int mx = m % p.Wm;
    const int t = m / p.Wm;
    const int my = t % p.Hm;
    const int b = t / p.Hm;
#pragma unroll
    for (int j = 0; j < WN; ++j) {
      const int n = n0 + j * 16 + fq * 4;
      if (n >= p.cout) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[j][i][r] + (p.bias ? p.bias[n + r] : 0.0f);
      if (p.mode == RGBAC_SUBPEL2) {
        // conv channel n+r = 4*cc + 2*ii + jj -> pixel (2my+ii, 2mx+jj), channel cc
        const int cc = n >> 2;
        T* out = reinterpret_cast<T*>(p.out);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float x = v[r];
          if (p.act == RGBAC_ACT_GELU) x = gelu_f(x);
          const int oy = 2 * my + (r >> 1), ox = 2 * mx + (r & 1);
          const long long o = ((long long)(b * p.out_h + oy) * p.out_w + ox) * p.out_ldc + p.out_coff + cc;
          Elem<T>::st(out + o, x);
        }
        continue;
      }
      int opix;
      if (p.mode == RGBAC_CONVT_S2)
        opix = (b * p.out_h + 2 * my + py) * p.out_w + 2 * mx + px;
      else
        opix = (b * p.out_h + my) * p.out_w + mx;
      if (p.res0) {
        float r0[4];
        load_res<T>(p.res0, p.ld0, opix, n, p.cout, r0);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += r0[r];
      }
      float r1[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.res1) load_res<T>(p.res1, p.ld1, opix, n, p.cout, r1);
      switch (p.act) {
        case RGBAC_ACT_GELU:
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = gelu_f(v[r]);
          break;
        case RGBAC_ACT_RELU:
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : 0.f;
          break;
        case RGBAC_ACT_LRELU:
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] > 0.f ? v[r] : v[r] * p.act_param;
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
          for (int r = 0; r < 4; ++r) v[r] = r1[r] / sqrtf(v[r]);
          break;
        case RGBAC_ACT_IGDN:
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = r1[r] * sqrtf(v[r]);
          break;
        case RGBAC_ACT_MASKSEL: {
          const bool on = p.sel[opix] != 0;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = on ? r1[r] + v[r] : r1[r];
          break;
        }
        default:
          break;
      }
      if (p.res2) {
        float r2[4];
        load_res<T>(p.res2, p.ld2, opix, n, p.cout, r2);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += r2[r];
      }
      epi_store<T>(p, opix, n, v);
    }
  }
}

template <typename T>
static int launch_conv(const ConvParams& p, int nphase, hipStream_t st) {
  const int wn = (p.cout_pad % 64 == 0) ? 4 : (p.cout_pad % 32 == 0) ? 2 : 1;
  dim3 grid((p.M + 127) / 128, p.cout_pad / (16 * wn), nphase);
  if (wn == 4)
    hipLaunchKernelGGL((conv_kernel<T, 4>), grid, dim3(256), 0, st, p);
  else if (wn == 2)
    hipLaunchKernelGGL((conv_kernel<T, 2>), grid, dim3(256), 0, st, p);
  else
    hipLaunchKernelGGL((conv_kernel<T, 1>), grid, dim3(256), 0, st, p);
  return check_launch("conv_kernel");
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_conv2d(const rgbac_conv_args* a, void* stream) {
  RGBAC_REQUIRE(a != nullptr, "null args");
  RGBAC_REQUIRE(a->dtype == RGBAC_F32 || a->dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(a->nsrc >= 1 && a->nsrc <= 3, "nsrc must be 1..3");
  RGBAC_REQUIRE(a->batch > 0 && a->in_h > 0 && a->in_w > 0, "bad input shape");
  RGBAC_REQUIRE(a->weight && a->out, "null weight/out");
  RGBAC_REQUIRE(a->cout > 0 && a->cout_pad >= a->cout && a->cout_pad % 16 == 0,
                "cout_pad must be >= cout and a multiple of 16");
  RGBAC_REQUIRE(a->cin_pad % 8 == 0 && a->cin_pad > 0, "cin_pad must be a multiple of 8");
  RGBAC_REQUIRE(a->k_pad % 64 == 0, "k_pad must be a multiple of 64");
  int csum = 0;
  for (int i = 0; i < a->nsrc; ++i) {
    RGBAC_REQUIRE(a->src[i].ptr != nullptr, "null source");
    RGBAC_REQUIRE(a->src[i].channels % 8 == 0 && a->src[i].channels > 0,
                  "source channels must be a positive multiple of 8");
    RGBAC_REQUIRE(a->src[i].ldc % 8 == 0 && a->src[i].ldc >= a->src[i].channels,
                  "source ldc must be a multiple of 8 and >= channels");
    csum += a->src[i].channels;
  }
  RGBAC_REQUIRE(csum <= a->cin_pad, "sum of source channels exceeds cin_pad");
  RGBAC_REQUIRE(a->out_ldc % 4 == 0 && a->out_coff % 4 == 0, "out_ldc/out_coff must be multiples of 4");
  RGBAC_REQUIRE(a->act >= RGBAC_ACT_NONE && a->act <= RGBAC_ACT_MASKSEL, "act");
  RGBAC_REQUIRE(a->act != RGBAC_ACT_MASKSEL || (a->sel && a->res1), "MASKSEL needs sel and res1");
  RGBAC_REQUIRE(!(a->act == RGBAC_ACT_TANH_HALF || a->act == RGBAC_ACT_GATE ||
                  a->act == RGBAC_ACT_GDN || a->act == RGBAC_ACT_IGDN) || a->res1,
                "act needs res1");

  ConvParams p{};
  p.mode = a->mode;
  p.batch = a->batch;
  p.in_h = a->in_h;
  p.in_w = a->in_w;
  int nphase = 1;
  if (a->mode == RGBAC_CONV) {
    RGBAC_REQUIRE(a->ksize == 1 || a->ksize == 3 || a->ksize == 5, "ksize must be 1/3/5");
    RGBAC_REQUIRE(a->stride == 1 || a->stride == 2, "stride must be 1/2");
    const int pad = a->ksize / 2;
    const int oh = (a->in_h + 2 * pad - a->ksize) / a->stride + 1;
    const int ow = (a->in_w + 2 * pad - a->ksize) / a->stride + 1;
    RGBAC_REQUIRE(a->out_h == oh && a->out_w == ow, "out size mismatch for conv");
    p.Hm = oh; p.Wm = ow; p.sy = a->stride; p.ksize = a->ksize; p.pad = pad;
    RGBAC_REQUIRE(a->ksize * a->ksize * a->cin_pad <= a->k_pad, "k_pad too small");
  } else if (a->mode == RGBAC_CONVT_S2) {
    RGBAC_REQUIRE(a->ksize == 5 && a->stride == 2, "CONVT_S2 supports k=5, s=2, p=2, op=1 only");
    RGBAC_REQUIRE(a->out_h == 2 * a->in_h && a->out_w == 2 * a->in_w, "out size mismatch for convT");
    RGBAC_REQUIRE(9 * a->cin_pad <= a->k_pad, "k_pad too small");
    p.Hm = a->in_h; p.Wm = a->in_w; p.sy = 1; p.ksize = 5; p.pad = 2;
    nphase = 4;
  } else if (a->mode == RGBAC_SUBPEL2) {
    RGBAC_REQUIRE(a->ksize == 3 && a->stride == 1, "SUBPEL2 is conv3x3 s1");
    RGBAC_REQUIRE(a->out_h == 2 * a->in_h && a->out_w == 2 * a->in_w, "out size mismatch for subpel");
    RGBAC_REQUIRE(a->cout % 4 == 0, "subpel cout must be a multiple of 4");
    RGBAC_REQUIRE(a->act == RGBAC_ACT_NONE || a->act == RGBAC_ACT_GELU, "subpel supports NONE/GELU");
    RGBAC_REQUIRE(!a->res0 && !a->res1 && !a->res2, "subpel has no residual epilogue");
    RGBAC_REQUIRE(9 * a->cin_pad <= a->k_pad, "k_pad too small");
    p.Hm = a->in_h; p.Wm = a->in_w; p.sy = 1; p.ksize = 3; p.pad = 1;
  } else {
    RGBAC_REQUIRE(false, "unknown conv mode");
  }
  const long long M = (long long)a->batch * p.Hm * p.Wm;
  RGBAC_REQUIRE(M < (1ll << 31), "too many output pixels");
  p.M = (int)M;
  p.out_h = a->out_h;
  p.out_w = a->out_w;
  p.nsrc = a->nsrc;
  p.sp0 = a->src[0].ptr; p.sld0 = a->src[0].ldc; p.send0 = a->src[0].channels;
  p.sp1 = a->nsrc > 1 ? a->src[1].ptr : a->src[0].ptr;
  p.sld1 = a->nsrc > 1 ? a->src[1].ldc : a->src[0].ldc;
  p.send1 = p.send0 + (a->nsrc > 1 ? a->src[1].channels : 0);
  p.sp2 = a->nsrc > 2 ? a->src[2].ptr : p.sp1;
  p.sld2 = a->nsrc > 2 ? a->src[2].ldc : p.sld1;
  p.send2 = p.send1 + (a->nsrc > 2 ? a->src[2].channels : 0);
  p.cin_pad = a->cin_pad;
  p.k_pad = a->k_pad;
  p.cout = a->cout;
  p.cout_pad = a->cout_pad;
  p.w = a->weight;
  p.bias = a->bias;
  p.out = a->out;
  p.out_ldc = a->out_ldc;
  p.out_coff = a->out_coff;
  p.act = a->act;
  p.act_param = a->act_param;
  p.square = a->square_input;
  p.res0 = a->res0; p.ld0 = a->res0_ldc;
  p.res1 = a->res1; p.ld1 = a->res1_ldc;
  p.res2 = a->res2; p.ld2 = a->res2_ldc;
  p.sel = a->sel;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a->dtype == RGBAC_F32) return launch_conv<float>(p, nphase, st);
  return launch_conv<bf16_t>(p, nphase, st);
}
