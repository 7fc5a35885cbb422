// Masked shifted-window attention core (per-window softmax(QK^T + B + M) V).
//
// The two dense projections of the block (qkv = Linear(C,3C), proj =
// Linear(C,C)) are per-pixel 1x1 GEMMs and run on the MFMA conv engine: the
// qkv GEMM produces an NHWC [B,H,W,3C] tensor in the ORIGINAL pixel frame, and
// the proj GEMM's MASKSEL epilogue adds the result back onto x only for pixels
// of active windows.  Because roll/partition/reverse are pure index
// permutations, this kernel folds the cyclic shift, window partition, window
// drop (remove_zero_windows) and scatter-back into its gather/store index
// math: no permuted copy of x is ever materialised and no host sync is needed
// to compact windows (reference: masked_win_attention.py:169-251 does ~8
// full-tensor copies and two device->host syncs per call).
//
// One workgroup = 64 tokens = 64/(ws*ws) windows (1 for ws=8, 4 for ws=4).
// Heads are processed one after another; q,k,v of a head are staged in LDS as
// fp32 and the two small products (64 x ws^2 x d) run on the VALU in fp32.
#include "common.h"
#include <cstdlib>

namespace rgbac {

template <typename T, int WS>
__global__ void __launch_bounds__(256)
winattn_core_kernel(int batch, int H, int W, int C, int heads, int shift, int masked,
                    float scale, const T* __restrict__ qkv, long long ldq,
                    const float* __restrict__ alpha, const float* __restrict__ bias,
                    T* __restrict__ out, long long ldo, uint8_t* __restrict__ sel,
                    const float* __restrict__ amask, int amask_nw) {
  constexpr int N = WS * WS;
  constexpr int NWIN = 64 / N;
  constexpr int DMAX = 24;
  constexpr int DP = DMAX + 1;
  __shared__ float qs[64 * DP];
  __shared__ float ks[64 * DP];
  __shared__ float vs[64 * DP];
  __shared__ float S[64 * (N + 1)];
  __shared__ int pix_s[64];
  __shared__ int act_s[NWIN];

  const int tid = threadIdx.x;
  const int nwx = W / WS, nwy = H / WS;
  const int total = batch * nwx * nwy;
  const int d = C / heads;

  if (tid < NWIN) act_s[tid] = masked ? 0 : 1;
  __syncthreads();
  if (tid < 64) {
    const int wi = tid / N, lt = tid % N;
    const int gw = blockIdx.x * NWIN + wi;
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
  if (tid < 64) {
    const int pix = pix_s[tid];
    if (pix >= 0 && sel) sel[pix] = (uint8_t)act_s[tid / N];
  }
  bool any = false;
#pragma unroll
  for (int w = 0; w < NWIN; ++w) any |= act_s[w] != 0;
  if (!any) {
    // every window of this group is transparent: attention output is 0
    for (int e = tid; e < 64 * C; e += 256) {
      const int t = e / C, ch = e - t * C;
      const int pix = pix_s[t];
      if (pix >= 0) Elem<T>::st(out + (long long)pix * ldo + ch, 0.0f);
    }
    return;
  }

  for (int h = 0; h < heads; ++h) {
    // ---- stage q (pre-scaled, as q = q * self.scale), k, v of head h
    for (int e = tid; e < 64 * d; e += 256) {
      const int t = e / d, j = e - t * d;
      const int pix = pix_s[t];
      float q = 0.f, k = 0.f, v = 0.f;
      if (pix >= 0) {
        const T* row = qkv + (long long)pix * ldq + h * d + j;
        q = Elem<T>::ld(row) * scale;
        k = Elem<T>::ld(row + C);
        v = Elem<T>::ld(row + 2 * C);
      }
      qs[t * DP + j] = q;
      ks[t * DP + j] = k;
      vs[t * DP + j] = v;
    }
    __syncthreads();
    // ---- scores: token i attends keys of its own window
    const float* bh = bias + (size_t)h * N * N;
    for (int e = tid; e < 64 * N; e += 256) {
      const int i = e / N, j = e - i * N;
      const int wbase = (i / N) * N;
      const int li = i - wbase;
      float s = 0.f;
      for (int q = 0; q < d; ++q) s = fmaf(qs[i * DP + q], ks[(wbase + j) * DP + q], s);
      s += bh[li * N + j];
      if (shift > 0) {
        // region id of each token in the shifted frame (masked_win_attention.py:196-216)
        const int wi = i / N;
        const int gw = blockIdx.x * NWIN + wi;
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
      if (amask) {
        // WindowAttention.forward(x, mask): window gw adds mask[gw % nW] (:114-122)
        const int gw = blockIdx.x * NWIN + i / N;
        s += amask[((size_t)(gw % amask_nw) * N + li) * N + j];
      }
      S[i * (N + 1) + j] = s;
    }
    __syncthreads();
    // ---- softmax over keys, 4 lanes per query row
    {
      const int i = tid >> 2, part = tid & 3;
      float mx = -INFINITY;
      for (int j = part; j < N; j += 4) mx = fmaxf(mx, S[i * (N + 1) + j]);
      mx = fmaxf(mx, __shfl_xor(mx, 1));
      mx = fmaxf(mx, __shfl_xor(mx, 2));
      float sum = 0.f;
      for (int j = part; j < N; j += 4) {
        const float ex = expf(S[i * (N + 1) + j] - mx);
        S[i * (N + 1) + j] = ex;
        sum += ex;
      }
      sum += __shfl_xor(sum, 1);
      sum += __shfl_xor(sum, 2);
      const float inv = 1.0f / sum;
      for (int j = part; j < N; j += 4) S[i * (N + 1) + j] *= inv;
    }
    __syncthreads();
    // ---- o = P v, written at the token's original pixel
    for (int e = tid; e < 64 * d; e += 256) {
      const int i = e / d, q = e - i * d;
      const int wbase = (i / N) * N;
      float o = 0.f;
#pragma unroll 8
      for (int j = 0; j < N; ++j) o = fmaf(S[i * (N + 1) + j], vs[(wbase + j) * DP + q], o);
      const int pix = pix_s[i];
      if (pix >= 0) {
        if (!act_s[i / N]) o = 0.f;
        Elem<T>::st(out + (long long)pix * ldo + h * d + q, o);
      }
    }
    __syncthreads();
  }
}


// ---------------------------------------------------------------------------
// MFMA variant for the model's two shapes: (ws 8, head dim 24, C 192) and
// (ws 4, head dim 10, C 80).  Per head h, in LDS:
//   Qs[64][DP] = q_h * scale, Ks[64][DP] = k_h     (DP = head dim padded to a k-step, zeros)
//   Vt[16*CT][64] = v_h^T                          (key index contiguous)
//   Ps[64][64]   = softmax probabilities          (zero outside a token's window)
// S^T = K Q^T on MFMA puts one query per lane column, its keys in the lane's
// accumulator registers + 3 partner lanes (l^16, l^32, l^48): the softmax row
// reductions are two xor-shuffles.  O = P V on MFMA leaves 4 consecutive
// channels of one query per lane -> channel-vector stores.
template <typename T, int WS, int DH>
__global__ void __launch_bounds__(256)
winattn_mfma_kernel(int batch, int H, int W, int C, int heads, int shift, int masked,
                    float scale, const T* __restrict__ qkv, long long ldq,
                    const float* __restrict__ alpha, const float* __restrict__ bias,
                    T* __restrict__ out, long long ldo, uint8_t* __restrict__ sel, int hpb,
                    const float* __restrict__ amask, int amask_nw) {
  constexpr int N = WS * WS;
  constexpr int NWIN = 64 / N;
  constexpr int EPV = Elem<T>::EPV;
  constexpr int KSTEP = 4 * EPV;
  constexpr int DP = (DH + KSTEP - 1) / KSTEP * KSTEP;
  constexpr int QRS = DP / EPV + 1;            // Q/K row stride in 16-B chunks (+1 pad)
  constexpr int PRS = 64 / EPV + 1;            // P / V^T row stride in chunks
  constexpr int CT = (DH + 15) / 16;           // 16-channel output tiles
  constexpr int ROWB = DH * (int)sizeof(T);
  constexpr int VEC = (ROWB % 16 == 0) ? 16 : (ROWB % 8 == 0 ? 8 : 4);
  constexpr int NP = ROWB / VEC;
  constexpr int KT = (WS == 8) ? 4 : 1;        // key tiles per query tile
  __shared__ __attribute__((aligned(16))) uint4 Qs[64 * QRS];
  __shared__ __attribute__((aligned(16))) uint4 Ks[64 * QRS];
  __shared__ __attribute__((aligned(16))) uint4 Vt[CT * 16 * PRS];
  __shared__ __attribute__((aligned(16))) uint4 Ps[64 * PRS];
  __shared__ int pix_s[64];
  __shared__ int rid_s[64];
  __shared__ int act_s[NWIN];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int nwx = W / WS, nwy = H / WS;
  const int total = batch * nwx * nwy;
  // Block -> (window group, head group), XCD-aware: blocks are dealt round-robin over the 8
  // XCDs (block i -> XCD i % 8), so all head groups of one window group get block ids with
  // the same residue and share that XCD's L2 for the window's qkv rows.
  const int hgroups = heads / hpb;
  const int xcd = blockIdx.x & 7, seq = blockIdx.x >> 3;
  const int hg = seq % hgroups;
  const int wgrp = (seq / hgroups) * 8 + xcd;
  const int h0 = hg * hpb, h1 = h0 + hpb;

  // zero only what the staging never writes but the MFMAs read: the q/k chunks past the head
  // dim (K padding to the MFMA k-step), the V^T rows past it, and for ws 4 the off-window
  // P entries (ws 8 writes every P column of every row each head)
  constexpr int QC0 = DH / EPV, QC1 = DP / EPV;   // chunks [QC0, QC1) hold padding
  for (int e = tid; e < 64 * (QC1 - QC0); e += 256) {
    const int t = e / (QC1 - QC0), c = QC0 + e % (QC1 - QC0);
    Qs[t * QRS + c] = Ks[t * QRS + c] = make_uint4(0, 0, 0, 0);
  }
  for (int e = tid; e < (CT * 16 - DH) * PRS; e += 256) Vt[DH * PRS + e] = make_uint4(0, 0, 0, 0);
  if constexpr (WS == 4)
    for (int e = tid; e < 64 * PRS; e += 256) Ps[e] = make_uint4(0, 0, 0, 0);
  if (tid < NWIN) act_s[tid] = masked ? 0 : 1;
  __syncthreads();
  if (tid < 64) {
    const int wi = tid / N, lt = tid % N;
    const int gw = wgrp * NWIN + wi;
    int pix = -1, rid = 0;
    if (gw < total) {
      const int b = gw / (nwx * nwy);
      const int rem = gw - b * nwx * nwy;
      const int wy = rem / nwx, wx = rem - (rem / nwx) * nwx;
      const int r = wy * WS + lt / WS, c = wx * WS + lt % WS;
      int oy = r + shift; if (oy >= H) oy -= H;
      int ox = c + shift; if (ox >= W) ox -= W;
      pix = (b * H + oy) * W + ox;
      if (masked && alpha[pix] != 0.0f) act_s[wi] = 1;
      // region id in the shifted frame (masked_win_attention.py:196-207)
      rid = 3 * (r < H - WS ? 0 : (r < H - shift ? 1 : 2)) + (c < W - WS ? 0 : (c < W - shift ? 1 : 2));
    }
    pix_s[tid] = pix;
    rid_s[tid] = rid;
  }
  __syncthreads();
  if (tid < 64 && pix_s[tid] >= 0 && sel && hg == 0) sel[pix_s[tid]] = (uint8_t)act_s[tid / N];
  bool any = false;
#pragma unroll
  for (int w = 0; w < NWIN; ++w) any |= act_s[w] != 0;
  if (!any) {
    const int CH = hpb * DH;                     // this block's head slice only
    for (int e = tid; e < 64 * CH; e += 256) {
      const int t = e / CH, ch = h0 * DH + (e - t * CH);
      if (pix_s[t] >= 0) Elem<T>::st(out + (long long)pix_s[t] * ldo + ch, 0.0f);
    }
    return;
  }

  const int qi = wave * 16 + fr;                 // this lane's query (row of S^T cols)
  const int qwin = qi / N, qloc = qi % N;
  const bool qact = act_s[qwin] != 0;
  const int qpix = pix_s[qi];
  const int qrid = rid_s[qi];
  // explicit additive mask of WindowAttention.forward(x, mask): this query's row of
  // mask[gw % nW] (masked_win_attention.py:114-122)
  const float* qmask = amask ? amask + ((size_t)((wgrp * NWIN + qwin) % amask_nw) * N + qloc) * N
                             : nullptr;

  for (int h = h0; h < h1; ++h) {
    // ---- relative-position bias of this lane's (query, key) pairs: issued before the staging
    // loop so the scattered L2 reads overlap the q/k/v gathers and the barrier
    const float* bh = bias + (size_t)h * N * N;
    float bias_r[KT][4];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int ktile = (WS == 8) ? kt : wave;
#pragma unroll
      for (int r = 0; r < 4; ++r) bias_r[kt][r] = bh[qloc * N + (ktile * 16 + fq * 4 + r) % N];
    }
    // ---- stage q*scale, k (rows) and v^T (transposed) with VEC-byte loads
    for (int e = tid; e < 3 * 64 * NP; e += 256) {
      const int which = e / (64 * NP);
      const int rem = e - which * 64 * NP;
      const int t = rem / NP, pc = rem - t * NP;
      const int pix = pix_s[t];
      constexpr int EV = VEC / (int)sizeof(T);
      float v[EV];
      if (pix >= 0) {
        const T* src = qkv + (long long)pix * ldq + which * C + h * DH + pc * EV;
        if constexpr (VEC == 16) {
          const uint4 raw = *reinterpret_cast<const uint4*>(src);
          const T* el = reinterpret_cast<const T*>(&raw);
#pragma unroll
          for (int q = 0; q < EV; ++q) v[q] = Elem<T>::ld(el + q);
        } else if constexpr (VEC == 8) {
          const uint2 raw = *reinterpret_cast<const uint2*>(src);
          const T* el = reinterpret_cast<const T*>(&raw);
#pragma unroll
          for (int q = 0; q < EV; ++q) v[q] = Elem<T>::ld(el + q);
        } else {
          const uint32_t raw = *reinterpret_cast<const uint32_t*>(src);
          const T* el = reinterpret_cast<const T*>(&raw);
#pragma unroll
          for (int q = 0; q < EV; ++q) v[q] = Elem<T>::ld(el + q);
        }
      } else {
#pragma unroll
        for (int q = 0; q < EV; ++q) v[q] = 0.f;
      }
      if (which == 2) {
        T* vt = reinterpret_cast<T*>(Vt);
#pragma unroll
        for (int q = 0; q < EV; ++q) Elem<T>::st(vt + (pc * EV + q) * (PRS * EPV) + t, v[q]);
      } else {
        T* row = reinterpret_cast<T*>(which == 0 ? Qs : Ks) + t * (QRS * EPV) + pc * EV;
#pragma unroll
        for (int q = 0; q < EV; ++q) Elem<T>::st(row + q, which == 0 ? v[q] * scale : v[q]);
      }
    }
    __syncthreads();

    // ---- S^T tile(s): keys on the MFMA row axis, this wave's 16 queries on columns
    f32x4 s[KT];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int ktile = (WS == 8) ? kt : wave;   // ws 4: the query tile IS its window
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < DP / KSTEP; ++ks) {
        const uint4 a = Ks[(ktile * 16 + fr) * QRS + 4 * ks + fq];
        const uint4 b = Qs[(wave * 16 + fr) * QRS + 4 * ks + fq];
        mma_step<T>(s[kt], a, b);
      }
    }
    // ---- + relative position bias + shift mask, softmax over the window's keys
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
    mx = fmaxf(mx, __shfl_xor(mx, 16));
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    float sum = 0.f;
#pragma unroll
    for (int kt = 0; kt < KT; ++kt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float ex = expf(s[kt][r] - mx);
        s[kt][r] = ex;
        sum += ex;
      }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = 1.0f / sum;
    T* prow = reinterpret_cast<T*>(Ps) + qi * (PRS * EPV);
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
      const int ktile = (WS == 8) ? kt : wave;
      float pv[4] = {s[kt][0] * inv, s[kt][1] * inv, s[kt][2] * inv, s[kt][3] * inv};
      Elem<T>::st4(prow + ktile * 16 + fq * 4, pv);
    }
    __syncthreads();

    // ---- O^T = V^T P^T: channels on rows, this wave's queries on columns
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 64 / KSTEP; ++ks) {
        const uint4 a = Vt[(ct * 16 + fr) * PRS + 4 * ks + fq];
        const uint4 b = Ps[(wave * 16 + fr) * PRS + 4 * ks + fq];
        mma_step<T>(o, a, b);
      }
      const int c0 = ct * 16 + fq * 4;
      if (qpix >= 0 && c0 < DH) {
        float ov[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[r] = qact ? o[r] : 0.0f;
        T* dst = out + (long long)qpix * ldo + h * DH + c0;
        if constexpr (DH % 4 == 0) {
          Elem<T>::st4(dst, ov);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (c0 + r < DH) Elem<T>::st(dst + r, ov[r]);
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_winattn_core_ex(int dtype, int batch, int h, int w, int channels,
                                     int heads, int ws, int shift, int masked, float scale,
                                     const void* qkv, int64_t ldq, const float* alpha,
                                     const float* bias, void* out, int64_t ldo, uint8_t* sel,
                                     const float* amask, int amask_nw, int hpb, void* stream) {
  RGBAC_REQUIRE(dtype == RGBAC_F32 || dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(ws == 4 || ws == 8, "window size must be 4 or 8");
  RGBAC_REQUIRE(batch > 0 && h > 0 && w > 0 && h % ws == 0 && w % ws == 0,
                "H and W must be positive multiples of the window size");
  RGBAC_REQUIRE(heads > 0 && channels % heads == 0 && channels / heads <= 24,
                "head dim must divide C and be <= 24");
  RGBAC_REQUIRE(shift >= 0 && shift < ws, "0 <= shift < window_size");
  RGBAC_REQUIRE(qkv && out && bias, "null pointer");
  RGBAC_REQUIRE(!masked || (alpha && sel), "masked attention needs alpha and sel");
  RGBAC_REQUIRE(ldq >= 3 * channels && ldo >= channels, "strides");
  RGBAC_REQUIRE(!amask || amask_nw > 0, "an explicit mask needs nW > 0");
  const long long windows = (long long)batch * (h / ws) * (w / ws);
  const int nwin = 64 / (ws * ws);
  const int blocks = (int)((windows + nwin - 1) / nwin);
  // MFMA path: one block per (window group, head group) of hpb heads (1: 8x the blocks of
  // one-block-per-window, which left 2 blocks per CU walking 8 heads serially); an hpb that
  // does not divide heads falls back to 1.  Window groups padded to a multiple of 8
  // (XCD-aware order; padding groups have no valid window and write nothing).
  if (hpb < 1 || heads % hpb) hpb = 1;
  const long long mblocks_ll = (long long)((blocks + 7) / 8) * 8 * (heads / hpb);
  RGBAC_REQUIRE(mblocks_ll < (1LL << 31), "too many windows for one launch");
  const int mblocks = (int)mblocks_ll;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
#define RGBAC_WA(T, WS)                                                                    \
  hipLaunchKernelGGL((winattn_core_kernel<T, WS>), dim3(blocks), dim3(256), 0, st, batch, h, \
                     w, channels, heads, shift, masked, scale, (const T*)qkv, ldq, alpha,    \
                     bias, (T*)out, ldo, sel, amask, amask_nw)
#define RGBAC_WM(T, WS, DH)                                                                \
  hipLaunchKernelGGL((winattn_mfma_kernel<T, WS, DH>), dim3(mblocks), dim3(256), 0, st, batch, \
                     h, w, channels, heads, shift, masked, scale, (const T*)qkv, ldq, alpha,   \
                     bias, (T*)out, ldo, sel, hpb, amask, amask_nw)
  const int dh = channels / heads;
  const bool mfma_shape = (ws == 8 && dh == 24) || (ws == 4 && dh == 10);
  if (mfma_shape && dtype == RGBAC_F32) {
    if (ws == 8) RGBAC_WM(float, 8, 24); else RGBAC_WM(float, 4, 10);
  } else if (mfma_shape) {
    if (ws == 8) RGBAC_WM(bf16_t, 8, 24); else RGBAC_WM(bf16_t, 4, 10);
  } else if (dtype == RGBAC_F32) {
    if (ws == 8) RGBAC_WA(float, 8); else RGBAC_WA(float, 4);
  } else {
    if (ws == 8) RGBAC_WA(bf16_t, 8); else RGBAC_WA(bf16_t, 4);
  }
#undef RGBAC_WA
#undef RGBAC_WM
  return check_launch("winattn_core");
}

extern "C" int rgbac_winattn_core(int dtype, int batch, int h, int w, int channels, int heads,
                                  int ws, int shift, int masked, float scale, const void* qkv,
                                  int64_t ldq, const float* alpha, const float* bias, void* out,
                                  int64_t ldo, uint8_t* sel, void* stream) {
  return rgbac_winattn_core_ex(dtype, batch, h, w, channels, heads, ws, shift, masked, scale, qkv,
                               ldq, alpha, bias, out, ldo, sel, nullptr, 0, 1, stream);
}
