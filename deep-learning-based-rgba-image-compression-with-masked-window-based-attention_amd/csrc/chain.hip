// Slice-chain engine: the channel-conditional entropy model's dependent 3x3 conv stacks in ONE
// persistent launch (models/AutoEncoderRGB_Journal.py:240-266, AutoEncoderMask_Journal.py:
// 268-298: per slice cc_mean / cc_scale stacks -> (mu | sigma) + GaussianConditional + STE ->
// lrp stack -> y_hat += 0.5 tanh, the next slice reading y_hat).
//
// Why one launch.  At 256^2 x B8 the latent grid is 8 x 32 x 32: every stage of the chain is
// about one round of workgroups on 256 CUs, and 36 such stages run back to back.  As separate
// launches each paid a launch boundary, a cold operand-staging burst and a drain (the
// per-workgroup probe, DESIGN §12b: 3.4-4.8 us staging + 2-4 us epilogue around 1-6 us of K
// loop).  Here every workgroup walks the stage list itself:
//   * a stage's work items are (tile, output-channel chunk); a tile is 4 latent rows x 16
//     columns of one image; item i of a stage goes to workgroup i mod grid;
//   * an item waits only for the tiles its 3x3 patch reads: the previous stage's items on
//     row blocks ty-1 .. ty+1 of the same image (one monotonic counter per (stage, image,
//     row block)).  Every stage covers every tile, so by induction stage s-k is complete
//     within k row blocks -- which also covers the older sources (y_hat slices, the pre-lrp
//     slice) and every buffer a later stage overwrites;
//   * the weight ring of the next item is requested BEFORE its dependency wait (weights
//     depend on nothing), so the wait overlaps the weight latency;
//   * hand-offs follow MI355X_MICROARCH.md's validated write-through form (placement-
//     independent: no assumption on which XCD runs what): every byte produced inside the
//     launch is stored `sc1` (write-through) by 8- or 16-byte stores, every storing wave waits
//     vmcnt(0), a workgroup barrier, then ONE lane adds to the counter (agent-scope atomic);
//     the consumer's lane 0 polls the counters with `sc1` loads, a barrier releases the other
//     waves, and every load of produced bytes is an `sc1` buffer load into registers (then
//     LDS);
//   * every wait is bounded: after ~0.2 s without progress the workgroup sets the error word
//     and stops waiting (the launch then completes with wrong values; the host reports it) --
//     a dependency bug can never hang the GPU.
//
// Item bodies (bf16, fragment-major weights as conv_fpatch_kernel / conv_npatch_kernel):
//   wide   (GELU / no activation, cout > 16): 12 waves = 4 N waves x 3 kernel rows (K split),
//          BN = 64 * TN output channels, the K loop fully unrolled over CPT 32-channel chunks
//          per tap (CPT = 2, 3, 4, 7), row partials summed through LDS in a fixed order;
//   narrow (GAUSS: (mu | sigma) of 8 channels + GaussianConditional + STE + bits; TANH_HALF:
//          y_hat = pre + 0.5 tanh(v); cout <= 16): 12 waves split the k-steps, partials summed
//          in a fixed order, one wave per pixel row runs the epilogue; bits partial per tile.
// Arithmetic, operand order and epilogue formulas are those of the per-stage kernels, so the
// outputs are bit-identical to the launch-per-stage path.
#include <cstdlib>
#include <cstring>

#include "common.h"
#include "conv_common.h"

namespace rgbac {

namespace chain {
constexpr int TH = 4, TW = 16, PW = TW + 2, PR = (TH + 2) * PW;   // tile and patch geometry
constexpr int NW = 4, KS = 3, NWAVE = NW * KS, NT = 64 * NWAVE;  // 12 waves, 768 threads
constexpr int MAXCG = 64;                                         // (group, chunk) pairs
constexpr int MAX_STAGES = 64;
constexpr int KIND_WIDE = 0, KIND_NARROW = 1;
constexpr int SPIN_LIMIT = 200000;                                // ~0.2 s of polling
}  // namespace chain

struct ChainStage {
  int ngroups, kind, act, tn, cpt, ncg;
  int target;                       // items of THIS stage per (image, row block)
  int pad_;
  int cg[chain::MAXCG];             // (group << 8) | chunk, for c in [0, ncg)
  ConvGroup g[kMaxGroups];
};

struct ChainArgs {
  const ChainStage* st;
  int nstages, batch, H, W, tyn, txn;
  int* cnt;                         // [nstages][batch][tyn], zeroed before the launch
  int* err;                         // set to 1 by a workgroup whose wait gave up
};

// ---- write-through / L1-bypassing memory ops (cache policy aux 16 = sc1 on gfx950)
constexpr int kSC1 = 16;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}
// offset >= 2^31 is out of range: the load returns zeros (zero padding without a branch)
__device__ __forceinline__ uint4 ld16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kSC1));
}
__device__ __forceinline__ void st8_sc1(void* p, uint2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), rsrc_of(p), 0, 0, kSC1);
}

__device__ __forceinline__ int poll_sc1(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Lane 0 of wave 0 waits until the previous stage's counters of row blocks ty-1..ty+1 reach
// their targets; the caller's barrier releases the workgroup.
__device__ __forceinline__ void chain_wait(const ChainArgs& a, int s, int b, int ty,
                                           int target, bool& bail) {
  if (threadIdx.x != 0 || s == 0 || bail) return;
  const int* base = a.cnt + ((size_t)(s - 1) * a.batch + b) * a.tyn;
  const int r0 = ty > 0 ? ty - 1 : 0, r1 = ty + 1 < a.tyn ? ty + 1 : a.tyn - 1;
  for (int r = r0; r <= r1; ++r) {
    int spins = 0;
    while (poll_sc1(base + r) < target) {
      __builtin_amdgcn_s_sleep(2);
      if ((++spins & 1023) == 0 &&
          (spins > chain::SPIN_LIMIT || poll_sc1(a.err) != 0)) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bail = true;
        return;
      }
    }
  }
}

// Every storing wave has waited for its stores; one lane publishes the item.
__device__ __forceinline__ void chain_signal(const ChainArgs& a, int s, int b, int ty) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_fetch_add(a.cnt + ((size_t)s * a.batch + b) * a.tyn + ty, 1, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Stage the (TH+2) x 18 x cin32 input patch (rows of nch data chunks + 2 pad chunks) with sc1
// loads into registers, then LDS.  Pixels outside the image and padding channels are zeros.
template <int NCHT>
__device__ __forceinline__ void chain_stage_patch(const ConvGroup& g, uint4* patch, int b, int y0,
                                                  int x0, int in_h, int in_w, int nch) {
  constexpr int MAXL = (chain::PR * (NCHT + 2) + chain::NT - 1) / chain::NT;
  const int RSc = nch + 2;
  const int total = chain::PR * RSc;
  const __amdgpu_buffer_rsrc_t r0 = rsrc_of(g.sp0), r1 = rsrc_of(g.sp1), r2 = rsrc_of(g.sp2);
  const int send0 = g.send0, send1 = g.send1, send2 = g.send2;
  const int sld0 = (int)g.sld0, sld1 = (int)g.sld1, sld2 = (int)g.sld2;
  uint4 v[MAXL];
#pragma unroll
  for (int u = 0; u < MAXL; ++u) {
    const int f = threadIdx.x + u * chain::NT;
    const int row = f / RSc, c = f - (f / RSc) * RSc;
    const int py = row / chain::PW, px = row - (row / chain::PW) * chain::PW;
    const int iy = y0 - 1 + py, ix = x0 - 1 + px;
    const int ch = c << 3;
    const bool in0 = ch < send0, in1 = ch < send1;
    const int sld = in0 ? sld0 : (in1 ? sld1 : sld2);
    const int cs = ch - (in0 ? 0 : (in1 ? send0 : send1));
    const bool ok = f < total && c < nch && ch < send2 && (unsigned)iy < (unsigned)in_h &&
                    (unsigned)ix < (unsigned)in_w;
    const unsigned off = ok ? ((unsigned)((b * in_h + iy) * in_w + ix) * (unsigned)sld +
                               (unsigned)cs) * 2u : 0x80000000u;
    v[u] = in0 ? ld16_sc1(r0, off) : (in1 ? ld16_sc1(r1, off) : ld16_sc1(r2, off));
  }
#pragma unroll
  for (int u = 0; u < MAXL; ++u) {
    const int f = threadIdx.x + u * chain::NT;
    if (f < total) patch[f] = v[u];
  }
}

// ---------------------------------------------------------------------------------------
// Wide item: TH x 16 pixels x BN = 64 TN channels of group g, K split by kernel row.
template <int TN, int CPT>
__device__ __forceinline__ void chain_wide_item(const ChainArgs& a, const ChainStage& st,
                                                const ConvGroup& g, uint4* patch, int s, int b,
                                                int ty, int tx, int nb, bool& bail) {
  using T = bf16_t;
  using namespace chain;
  constexpr int TM = TH, NKSC = 9 * CPT, NKSP = NKSC / KS;
  constexpr int RC0 = TN == 1 ? RGBAC_CHAIN_RC1 : RGBAC_CHAIN_RC1 / 2;
  constexpr int RC1 = (RC0 + 1) / 2;
  constexpr int RC = RC1 < NKSP ? RC1 : NKSP;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave = wave_all % NW, kp = wave_all / NW;
  const int fr = lane & 15, fq = lane >> 4;
  const int n0 = nb * 64 * TN;
  const int y0 = ty * TH, x0 = tx * TW;
  const int ntile0 = (n0 >> 4) + wave * TN;
  const uint4* const wf = reinterpret_cast<const uint4*>(g.w);

  // weights and biases first: they depend on nothing
  float pbias[TN][4];
  const int nb0 = n0 + wave * TN * 16 + fq * 4;
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      pbias[j][r] = (g.bias && nb0 + j * 16 + r < g.cout) ? g.bias[nb0 + j * 16 + r] : 0.0f;
  const uint4* wj[TN];
  uint4 cring[RC][TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) wj[j] = wf + ((size_t)(ntile0 + j) * NKSC + kp * NKSP) * 64 + lane;
#pragma unroll
  for (int u = 0; u < RC; ++u)
#pragma unroll
    for (int j = 0; j < TN; ++j) cring[u][j] = wj[j][u * 64];

  chain_wait(a, s, b, ty, s > 0 ? a.st[s - 1].target : 0, bail);
  __syncthreads();                             // dependencies met; previous item's LDS free
  chain_stage_patch<CPT * 4>(g, patch, b, y0, x0, a.H, a.W, CPT * 4);
  __syncthreads();

  constexpr int RS = 4 * CPT + 2;
  int lb[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) lb[i] = ((i + kp) * PW + fr) * RS + fq;
  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKSP; ++ks) {
    const int tap = ks / CPT, cc = ks - (ks / CPT) * CPT;   // tap < 3: the row sits in lb
    const int off = (tap % 3) * RS + cc * 4;
    uint4 bb[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) bb[i] = patch[lb[i] + off];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], cring[ks % RC][j], bb[i]);
    if (ks + RC < NKSP) {
#pragma unroll
      for (int j = 0; j < TN; ++j) cring[ks % RC][j] = wj[j][(ks + RC) * 64];
    }
  }
  // row partials: dy 0 + dy 1 + dy 2 (fixed order), through LDS over the dead patch
  f32x4* const red = reinterpret_cast<f32x4*>(patch);
  __syncthreads();
  if (kp > 0) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) red[((((kp - 1) * NW + wave) * TN + j) * TM + i) * 64 + lane] = acc[j][i];
  }
  __syncthreads();
  if (kp == 0) {
#pragma unroll
    for (int q = 0; q < KS - 1; ++q)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const f32x4 t = red[(((q * NW + wave) * TN + j) * TM + i) * 64 + lane];
          acc[j][i] = f32x4{acc[j][i][0] + t[0], acc[j][i][1] + t[1], acc[j][i][2] + t[2],
                            acc[j][i][3] + t[3]};
        }
    // epilogue: bias (+ GELU), bf16 quads stored write-through
    T* const out = reinterpret_cast<T*>(g.out) + g.out_coff;
    const bool gelu = st.act == RGBAC_ACT_GELU;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const long long opix = (long long)(b * a.H + y0 + i) * a.W + x0 + fr;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = nb0 + j * 16;
        if (n < g.cout) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[j][i][r] + pbias[j][r];
            if (gelu) v[r] = gelu_t<T>(v[r]);
          }
          st8_sc1(out + opix * g.out_ldc + n,
                  make_uint2(pack_bf16x2(v[0], v[1]), pack_bf16x2(v[2], v[3])));
        }
      }
    }
  }
  chain_signal(a, s, b, ty);
}

// ---------------------------------------------------------------------------------------
// Narrow item: TH x 16 pixels x cout <= 16 * TN, the k-steps split over the 12 waves.
// GAUSS: (mu | sigma) of cout / 2 channels -- 8: mu in lanes fq < 2, sigma of the same
// channels in lanes fq ^ 2 (a lane ^ 32 shuffle); 16: mu in N tile 0, sigma in N tile 1.
template <int NCHT, int TN>
__device__ __forceinline__ void chain_narrow_item(const ChainArgs& a, const ChainStage& st,
                                                  const ConvGroup& g, uint4* patch, double* wsum,
                                                  int s, int b, int ty, int tx, bool& bail) {
  using T = bf16_t;
  using namespace chain;
  constexpr int TM = TH, R = 4;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int y0 = ty * TH, x0 = tx * TW;
  const int cin32 = (g.cin_pad + 31) & ~31;
  const int nch = cin32 >> 3, RSc = nch + 2, cpt = cin32 >> 5;
  const int nks = 9 * cpt;
  const int k0 = nks * wave / NWAVE, k1 = nks * (wave + 1) / NWAVE;
  const bool gauss = st.act == RGBAC_ACT_GAUSS;
  const int cout = g.cout, nho = cout >> 1;
  const int ei = wave < TM ? wave : 0;
  const int m_e = (b * a.H + y0 + ei) * a.W + x0 + fr;
  float pb[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * j + 4 * fq + r;
      pb[j][r] = (g.bias && n < cout) ? g.bias[n] : 0.0f;
    }
  const uint4* const wf = reinterpret_cast<const uint4*>(g.w);
  uint4 ring[R][TN];
  int lks = k0;
#pragma unroll
  for (int u = 0; u < R; ++u) {
    if (lks < k1) {
#pragma unroll
      for (int j = 0; j < TN; ++j) ring[u][j] = wf[((size_t)j * nks + lks) * 64 + lane];
    }
    ++lks;
  }

  chain_wait(a, s, b, ty, s > 0 ? a.st[s - 1].target : 0, bail);
  __syncthreads();
  // the epilogue's res1 quad (GAUSS: y; TANH_HALF: the pre-lrp slice; sc1 -- produced in this
  // launch), channels 4 fq .. + 3 of the lane's pixel, requested behind the dependency wait
  uint2 rq = make_uint2(0, 0);
  const bool rlane = wave < TM && 4 * fq < (gauss ? nho : cout);
  if (rlane) {
    const uint4 t = ld16_sc1(rsrc_of(g.res1), (unsigned)(((long long)m_e * g.ld1 + 4 * fq) * 2) & ~15u);
    rq = (fq & 1) ? make_uint2(t.z, t.w) : make_uint2(t.x, t.y);
  }
  chain_stage_patch<NCHT>(g, patch, b, y0, x0, a.H, a.W, nch);
  __syncthreads();

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  int tap = k0 / cpt, cc = k0 - (k0 / cpt) * cpt;
  for (int ks0 = k0; ks0 < k1; ks0 += R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (ks0 + u < k1) {
        const int dy = tap / 3, dx = tap - 3 * (tap / 3);
        uint4 bb[TM];
#pragma unroll
        for (int i = 0; i < TM; ++i) bb[i] = patch[((i + dy) * PW + fr + dx) * RSc + cc * 4 + fq];
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], ring[u][j], bb[i]);
        if (++cc == cpt) { cc = 0; ++tap; }
      }
      if (lks < k1) {
#pragma unroll
        for (int j = 0; j < TN; ++j) ring[u][j] = wf[((size_t)j * nks + lks) * 64 + lane];
      }
      ++lks;
    }
  }
  f32x4* const red = reinterpret_cast<f32x4*>(patch);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) red[((wave * TN + j) * TM + i) * 64 + lane] = acc[j][i];
  __syncthreads();
  double bits = 0.0;
  if (wave < TM) {
    float v[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] = 0.0f;
      for (int w = 0; w < NWAVE; ++w) {
        const f32x4 p = red[((w * TN + j) * TM + ei) * 64 + lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] += p[r];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] += pb[j][r];
    }
    const float yv[4] = {bf2f(rq.x & 0xFFFF), bf2f(rq.x >> 16), bf2f(rq.y & 0xFFFF), bf2f(rq.y >> 16)};
    if (gauss) {
      float sg[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) sg[r] = TN == 1 ? xor32_f(v[0][r]) : v[TN - 1][r];
      if (rlane) {
        float hat[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // gauss_elem_y's arithmetic, the y_hat store gathered into one 8-byte quad
          const float mu = v[0][r];
          hat[r] = rintf(yv[r] - mu) + mu;
          const float xin = g.aux0 ? yv[r] + g.aux0[(long long)m_e * nho + 4 * fq + r] : hat[r];
          const float d = fabsf(xin - mu);
          const float sc = fmaxf(sg[r], 0.11f);
          const float lik = fmaxf(std_cum_f((0.5f - d) / sc) - std_cum_f((-0.5f - d) / sc), 1e-9f);
          if (g.aux1) g.aux1[(long long)m_e * nho + 4 * fq + r] = lik;
          const float bt = (-1.0f * logf(lik + 1e-10f)) / 0.69314718055994530942f;
          bits += (double)fminf(fmaxf(bt, 0.0f), 50.0f);
        }
        st8_sc1(reinterpret_cast<T*>(g.out) + (long long)m_e * g.out_ldc + g.out_coff + 4 * fq,
                make_uint2(pack_bf16x2(hat[0], hat[1]), pack_bf16x2(hat[2], hat[3])));
      }
    } else if (rlane) {                        // TANH_HALF: y_hat = pre + 0.5 tanh(v)
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = yv[r] + 0.5f * tanhf(v[0][r]);
      st8_sc1(reinterpret_cast<T*>(g.out) + (long long)m_e * g.out_ldc + g.out_coff + 4 * fq,
              make_uint2(pack_bf16x2(o[0], o[1]), pack_bf16x2(o[2], o[3])));
    }
  }
  if (gauss) {
    for (int o = 32; o > 0; o >>= 1) bits += __shfl_xor(bits, o);
    if (wave < TM && lane == 0) wsum[wave] = bits;
    __syncthreads();
    if (tid == 0)
      g.partial[(b * a.tyn + ty) * a.txn + tx] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
  }
  chain_signal(a, s, b, ty);
}

template <int TN>
__device__ __forceinline__ void chain_wide_dispatch(const ChainArgs& a, const ChainStage& st,
                                                    const ConvGroup& g, uint4* patch, int s,
                                                    int b, int ty, int tx, int nb, bool& bail) {
  switch (st.cpt) {
    case 2: chain_wide_item<TN, 2>(a, st, g, patch, s, b, ty, tx, nb, bail); break;
    case 3: chain_wide_item<TN, 3>(a, st, g, patch, s, b, ty, tx, nb, bail); break;
    case 4: chain_wide_item<TN, 4>(a, st, g, patch, s, b, ty, tx, nb, bail); break;
    default: chain_wide_item<TN, 7>(a, st, g, patch, s, b, ty, tx, nb, bail); break;
  }
}

__global__ void __launch_bounds__(chain::NT, 1) chain_kernel(const ChainArgs a) {
  using namespace chain;
  extern __shared__ __attribute__((aligned(16))) uint4 patch[];
  __shared__ double wsum[TH];
  bool bail = false;
  const int ntile = a.batch * a.tyn * a.txn;
  for (int s = 0; s < a.nstages; ++s) {
    const ChainStage& st = a.st[s];
    const int ncg = st.ncg;
    const int items = ntile * ncg;
    for (int it = blockIdx.x; it < items; it += gridDim.x) {
      // tile-major: the items of one tile are consecutive, tiles run in (image, row, column)
      // order, so early row blocks of every image are produced first
      const int tile = it / ncg, c = it - (it / ncg) * ncg;
      const int tx = tile % a.txn, t2 = tile / a.txn;
      const int ty = t2 % a.tyn, b = t2 / a.tyn;
      const int cgv = st.cg[c];
      const ConvGroup& g = st.g[cgv >> 8];
      if (st.kind == KIND_NARROW) {
        if (st.tn == 1) {
          if (st.cpt <= 4) chain_narrow_item<16, 1>(a, st, g, patch, wsum, s, b, ty, tx, bail);
          else chain_narrow_item<32, 1>(a, st, g, patch, wsum, s, b, ty, tx, bail);
        } else {
          if (st.cpt <= 4) chain_narrow_item<16, 2>(a, st, g, patch, wsum, s, b, ty, tx, bail);
          else chain_narrow_item<32, 2>(a, st, g, patch, wsum, s, b, ty, tx, bail);
        }
      } else if (st.tn == 1) {
        chain_wide_dispatch<1>(a, st, g, patch, s, b, ty, tx, cgv & 255, bail);
      } else {
        chain_wide_dispatch<2>(a, st, g, patch, s, b, ty, tx, cgv & 255, bail);
      }
    }
  }
}

// LDS: the patch (cin32 <= 256: 108 rows x 34 chunks) and the K-split partials (wide TN 2:
// 2 x 4 x 2 x 4 KiB; narrow: 12 x TN x 4 KiB) share one buffer
constexpr size_t kChainLds = 96 * 1024;

static int chain_ncu() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    if (ncu < 1) ncu = 256;
    (void)hipFuncSetAttribute((const void*)chain_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kChainLds);
    (void)hipGetLastError();
  }
  return ncu;
}

}  // namespace rgbac

using namespace rgbac;

extern "C" int rgbac_chain_desc_size(void) { return (int)sizeof(ChainStage); }

extern "C" int64_t rgbac_chain_counter_words(int32_t nstages, int32_t batch, int32_t h) {
  return (int64_t)nstages * batch * (h / chain::TH) + 1;     // + the error word
}

extern "C" int rgbac_chain_build(const rgbac_conv_args* args, const int32_t* stage_ngroups,
                                 int32_t nstages, void* host_table) {
  using namespace chain;
  RGBAC_REQUIRE(args && stage_ngroups && host_table, "null pointer");
  RGBAC_REQUIRE(nstages >= 1 && nstages <= MAX_STAGES, "nstages must be 1..64");
  const int ncu = chain_ncu();
  const rgbac_conv_args* a0 = &args[0];
  const int B = a0->batch, H = a0->in_h, W = a0->in_w;
  RGBAC_REQUIRE(H % TH == 0 && W % TW == 0, "latent grid must be a multiple of 4 x 16");
  ChainStage* out = reinterpret_cast<ChainStage*>(host_table);
  int k = 0;
  for (int s = 0; s < nstages; ++s) {
    ChainStage st;
    memset(&st, 0, sizeof(st));
    const int ng = stage_ngroups[s];
    RGBAC_REQUIRE(ng >= 1 && ng <= kMaxGroups, "stage groups must be 1..10");
    const rgbac_conv_args* a = &args[k];
    st.ngroups = ng;
    st.act = a->act;
    int cpt = -1, cmax = 0;
    for (int i = 0; i < ng; ++i) {
      const rgbac_conv_args* c = &args[k + i];
      RGBAC_REQUIRE(c->dtype == RGBAC_BF16 && c->mode == RGBAC_CONV && c->ksize == 3 &&
                        c->stride == 1 && c->batch == B && c->in_h == H && c->in_w == W &&
                        c->out_h == H && c->out_w == W && c->act == a->act && c->ksplit == 1,
                    "chain stages: bf16 3x3 stride-1 convs on one latent grid, one activation "
                    "per stage, no split-K");
      RGBAC_REQUIRE(c->act == RGBAC_ACT_NONE || c->act == RGBAC_ACT_GELU ||
                        c->act == RGBAC_ACT_GAUSS || c->act == RGBAC_ACT_TANH_HALF,
                    "chain stage activation must be none / GELU / GAUSS / TANH_HALF");
      RGBAC_REQUIRE(!c->res0 && !c->res2 && !c->zout && !c->sel && !c->square_input,
                    "chain stages take no res0 / res2 / zout / sel / squared input");
      RGBAC_REQUIRE(c->out_ldc % 4 == 0 && c->out_coff % 4 == 0, "out_ldc / out_coff % 4");
      const int rc = fill_group(c, 9, st.g[i]);
      if (rc != RGBAC_OK) return rc;
      const int cp = ((c->cin_pad + 31) & ~31) >> 5;
      RGBAC_REQUIRE(cpt < 0 || cp == cpt, "a stage's groups must share cin rounded to 32");
      cpt = cp;
      cmax = c->cout > cmax ? c->cout : cmax;
      if (c->act == RGBAC_ACT_GAUSS || c->act == RGBAC_ACT_TANH_HALF)
        RGBAC_REQUIRE(c->res1 && c->res1_ldc % 8 == 0 && c->cout <= 32 && c->cout % 8 == 0 &&
                          (c->act != RGBAC_ACT_GAUSS ||
                           ((c->cout == 16 || c->cout == 32) && c->partial)) &&
                          (c->act != RGBAC_ACT_TANH_HALF || c->cout <= 16),
                      "GAUSS needs (mu | sigma) of 8 or 16 channels, y and a bits partial; "
                      "TANH_HALF the pre-lrp slice (res1, ldc % 8) and cout <= 16");
    }
    st.cpt = cpt;
    const bool narrow = st.act == RGBAC_ACT_GAUSS || st.act == RGBAC_ACT_TANH_HALF;
    if (narrow) {
      RGBAC_REQUIRE(cpt <= 8, "narrow chain stages: cin <= 256");
      st.kind = KIND_NARROW;
      st.tn = cmax > 16 ? 2 : 1;
      st.ncg = ng;
      for (int i = 0; i < ng; ++i) st.cg[i] = i << 8;
    } else {
      RGBAC_REQUIRE(cpt == 2 || cpt == 3 || cpt == 4 || cpt == 7,
                    "wide chain stages: cin rounded to 32 must be 64, 96, 128 or 224");
      st.kind = KIND_WIDE;
      // BN 128 while that still fills every CU, else 64
      const long long tiles = (long long)B * (H / TH) * (W / TW);
      int n128 = 0;
      for (int i = 0; i < ng; ++i) n128 += (args[k + i].cout + 127) / 128;
      st.tn = tiles * n128 >= ncu ? 2 : 1;
      const int bn = 64 * st.tn;
      st.ncg = 0;
      for (int i = 0; i < ng; ++i) {
        RGBAC_REQUIRE(args[k + i].cout_pad >= (args[k + i].cout + bn - 1) / bn * bn,
                      "packed rows must cover the last chunk");
        for (int nb = 0; nb * bn < args[k + i].cout; ++nb) {
          RGBAC_REQUIRE(st.ncg < MAXCG, "too many (group, chunk) pairs in a stage");
          st.cg[st.ncg++] = (i << 8) | nb;
        }
      }
    }
    st.target = (W / TW) * st.ncg;
    out[s] = st;
    k += ng;
  }
  return RGBAC_OK;
}

extern "C" int rgbac_chain_launch(const void* dev_table, int32_t nstages, int32_t batch, int32_t h,
                                  int32_t w, int32_t* counters, void* stream) {
  using namespace chain;
  RGBAC_REQUIRE(dev_table && counters, "null pointer");
  RGBAC_REQUIRE(nstages >= 1 && nstages <= MAX_STAGES, "nstages must be 1..64");
  RGBAC_REQUIRE(batch > 0 && h % TH == 0 && w % TW == 0 && h > 0 && w > 0, "latent grid");
  const hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int ncu = chain_ncu();
  const int64_t words = rgbac_chain_counter_words(nstages, batch, h);
  if (hipMemsetAsync(counters, 0, (size_t)words * 4, st) != hipSuccess) {
    set_error("rgbac_chain_launch: counter reset failed");
    return RGBAC_E_LAUNCH;
  }
  ChainArgs a;
  a.st = reinterpret_cast<const ChainStage*>(dev_table);
  a.nstages = nstages;
  a.batch = batch;
  a.H = h;
  a.W = w;
  a.tyn = h / TH;
  a.txn = w / TW;
  a.cnt = counters;
  a.err = counters + words - 1;
  // one workgroup per CU: every workgroup resident, so no wait can depend on an unscheduled one
  hipLaunchKernelGGL(chain_kernel, dim3(ncu), dim3(NT), kChainLds, st, a);
  return check_launch("chain_kernel");
}
