// Implicit-GEMM convolution family on CDNA4 MFMA with fused epilogues.
//
// GEMM view (output-stationary, NHWC):   D[n][m] = sum_k W[n][k] * X[m][k]
//   n = output channel, m = output pixel of the "M grid", k = (tap, cin).
// A operand = packed weights [rows][k_pad] (K contiguous); B operand = im2col
// rows gathered on the fly from up to three NHWC sources (fused channel
// concat).  Putting channels on the MFMA row axis gives every lane 4
// consecutive channels of one pixel in the accumulator, so epilogue
// loads/stores are channel vectors.
//
// Staging: both operands go HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4,
// one 1-KiB piece per wave-instruction) into an NBUF-deep ring of K stages
// (128 or 256 bytes of K per row per stage: 64/128 bf16, 32/64 f32).  The 16-byte
// chunk c of row r lives at slot c ^ (r & 7) (conflict-free ds_read_b128 for the
// 16-lane fragment groups); because the DMA destination is lane-linear, the XOR is
// applied to the per-lane SOURCE chunk.  Weight pieces use the SADDR form (fixed
// per-lane offset, scalar stage base); im2col pieces test a per-lane tap-validity
// bitmask.  Padding taps / out-of-image pixels read a zero page.  (Measured and
// dropped: a chunk-major image with 64-row pieces, whose K decode is scalar -- its
// 64 cache lines per DMA instruction cost more than the VALU it saves.)  Stage s+NBUF-1 is issued while
// stage s is consumed; a counted s_waitcnt vmcnt + raw s_barrier retires one
// stage per iteration (no vmcnt(0) drain in the loop).
//   bf16: v_mfma_f32_16x16x32_bf16 per 16x16 tile per 32-deep k-step.
//   f32 : v_mfma_f32_16x16x4_f32 x4 per 16-deep k-step (exact f32 FMA chains,
//         parity mode); lane l feeds k = 4*(l>>4)+e to MFMA e for both
//         operands (a permutation of k: the same sum).
//
// Modes (rgbac_conv_mode): plain conv (stride 1/2), ConvTranspose2d(5, s2,
// p2, op1) as four output-parity phases (stride-1 convs with 3x3/3x2/2x3/2x2
// taps) in one launch, and subpel conv3x3 + PixelShuffle(2) folded into the
// store.  Split-K (ksplit > 1) writes fp32 partial slabs that
// conv_splitk_epilogue sums in a fixed order (deterministic).
//
// Groups: one launch runs up to kMaxGroups independent convs that share the
// geometry (mode, input/output size, kernel, stride, tile, split, activation)
// but have their own weights, sources, outputs and residuals (blockIdx.z =
// group, split, phase).  The model uses it for the cc_mean/cc_scale stacks,
// the conv_a/conv_b residual units and h_mean_s/h_scale_s, which are
// independent chains of identical shape.
#include <cstdlib>

#include "common.h"
#include "conv_common.h"

namespace rgbac {

#ifdef RGBAC_WG_TIMING
// probe builds only (tools/wg_probe.py): per-workgroup 100-MHz wall-clock stamps at phase
// boundaries of the slice-chain conv kernels (0 start, 1 operands staged / K loop entered,
// 2 K loop done, 3 end), recorded by thread 0
__device__ unsigned long long g_wg_t[16384][4];
#define WG_T(k)                                                                              \
  do {                                                                                       \
    if (threadIdx.x == 0) {                                                                  \
      const unsigned b_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);    \
      if (b_ < 16384) g_wg_t[b_][k] = wall_clock64();                                        \
    }                                                                                        \
  } while (0)
#else
#define WG_T(k) do {} while (0)
#endif

// BM x BN tile, 4 waves laid out WGM (along m) x WGN (along n), NBUF-stage ring of
// K stages of KSM x 128 bytes per row (KSM = 2: half the barriers and ring bookkeeping per
// MFMA, for the issue-bound small-M convs).
template <typename T, int BM, int BN, int WGM, int WGN, int NBUF, int KSM = 1>
__global__ void __launch_bounds__(256) conv_kernel(const ConvArgsDev args) {
  constexpr int EPV = Elem<T>::EPV;
  constexpr int CPR = 8 * KSM;                // 16-byte chunks per row per stage
  constexpr int KS = CPR * EPV;               // K elements per stage
  constexpr int RPP = 64 / CPR;               // rows per DMA piece
  constexpr int TM = BM / WGM / 16;           // 16-pixel tiles per wave
  constexpr int TN = BN / WGN / 16;           // 16-channel tiles per wave
  constexpr int IA = BN / RPP, IB = BM / RPP; // DMA pieces per stage
  constexpr int LW = (IA + 3) / 4 + IB / 4;  // pieces per wave per stage (uniform)
  constexpr int STAGE = (BN + BM) * CPR;      // uint4 per stage
  static_assert(KSM == 1 || KSM == 2, "stage width");
  static_assert(WGM * WGN == 4, "4 waves");
  static_assert(TM >= 1 && TN >= 1, "tile");
  static_assert(NBUF * STAGE * 4 >= BM * BN, "GAUSS epilogue reuses the ring as a [BM][BN] fp32 tile");
  __shared__ __attribute__((aligned(16))) uint4 smem[NBUF * STAGE];
  __shared__ double red[4];

  const ConvShared& s = args.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Block order.  The dispatcher deals consecutive workgroup ids round-robin to the
  // 8 XCDs (each with its own 4 MiB L2); with remap, XCD x gets one contiguous run of
  // (group, split, M-tile, phase, N-tile) ids, N fastest, so the N-tiles and phases
  // sharing an M-tile's im2col rows -- and neighbouring M-tiles sharing halo rows --
  // run on the same L2 (bijective for any grid size).
  int mblk, nblk, phase, split, gi;
  {
    const int Mb = gridDim.x, Nb = gridDim.y;
    const int lin = blockIdx.x + Mb * (blockIdx.y + Nb * blockIdx.z);
    int t;
    if (s.remap) {
      const int nwg = Mb * Nb * gridDim.z;
      const int xcd = lin & 7, q = nwg >> 3, r = nwg & 7;
      t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (lin >> 3);
      nblk = t % Nb; t /= Nb;
      phase = t % s.nphase; t /= s.nphase;
      mblk = t % Mb; t /= Mb;
    } else {
      mblk = blockIdx.x; nblk = blockIdx.y;
      t = blockIdx.z;
      phase = t % s.nphase; t /= s.nphase;
    }
    split = t % s.ksplit;
    gi = t / s.ksplit;
  }
  const ConvGroup& g = args.g[gi];
  const int m0 = mblk * BM, n0 = nblk * BN;
  if (n0 >= g.cout) return;                    // groups may differ in cout
  const int py = phase >> 1, px = phase & 1;
  int ntaps, tw;
  if (s.mode == RGBAC_CONVT_S2) {
    tw = 3 - px;
    ntaps = (3 - py) * tw;
  } else {
    tw = s.ksize;
    ntaps = s.ksize * s.ksize;
  }
  const int ktot = ntaps * g.cin_pad;
  const int nst = (ktot + KS - 1) / KS;
  const int s_beg = (int)((long long)nst * split / s.ksplit);
  const int s_end = (int)((long long)nst * (split + 1) / s.ksplit);
  const int ns = s_end - s_beg;

  // Kernel arguments the K loop reads, held in registers: the DMA statement clobbers
  // "memory", which would otherwise force a scalar reload of every field per stage.
  const int in_h = s.in_h, in_w = s.in_w, cin_pad = g.cin_pad, Mtot = s.M;
  const int send0 = g.send0, send1 = g.send1, send2 = g.send2;
  const char* const sp0 = reinterpret_cast<const char*>(g.sp0);
  const char* const sp1 = reinterpret_cast<const char*>(g.sp1);
  const char* const sp2 = reinterpret_cast<const char*>(g.sp2);
  const int sld0 = (int)g.sld0, sld1 = (int)g.sld1, sld2 = (int)g.sld2;
  const bool convt = s.mode == RGBAC_CONVT_S2;
  const int pad = s.pad;
  const bool sq_in = s.square != 0;

  // ---- stage image, row-major: A region (BN rows) then B region (BM rows), CPR slots per
  //      row; chunk c of row r lives at slot r*CPR + (c ^ (r & 7)) (conflict-free fragment
  //      reads: 8 consecutive rows of one chunk hit 8 distinct 16-byte bank groups).  One DMA
  //      piece = 64 consecutive slots = RPP rows x CPR chunks; the DMA destination is
  //      lane-linear, so the XOR goes on each lane's SOURCE chunk.  Wave w issues A pieces
  //      w, w+4, .. (a surplus slot re-issues the last piece, so every wave retires the same
  //      count per stage) and B pieces w, w+4, ..: all of a wave's pieces have the parity of
  //      w, so with 4-row pieces too a lane's source chunk -- and its K decode -- is one
  //      value for all its pieces.
  constexpr int NAW = (IA + 3) / 4;             // A pieces per wave
  constexpr int NBW = IB / 4;                   // B pieces per wave
  static_assert(IB % 4 == 0 && LW == NAW + NBW, "piece geometry");
  const int lrow = lane / CPR;
  const int rsw = (RPP * wave + lrow) & 7;      // (row & 7) of every piece row this lane fills
  const int c = (lane % CPR) ^ rsw;             // the lane's source chunk
  uint32_t aoff[NAW];                           // byte offset of the lane's A chunk (stage 0)
  int alds[NAW];                                // uint4 slot of the A piece in a stage
  const char* const wbase =
      reinterpret_cast<const char*>(g.w) + (size_t)phase * g.rows * g.k_pad * sizeof(T);
#pragma unroll
  for (int i = 0; i < NAW; ++i) {
    const int q = min(wave + 4 * i, IA - 1);
    const int row = RPP * q + lrow;
    alds[i] = q * 64;
    aoff[i] = (uint32_t)(((n0 + row) * g.k_pad + ((lane % CPR) ^ (row & 7)) * EPV) *
                         (int)sizeof(T));
  }
  // per B piece: the lane's input pixel of tap (0, 0) and its per-tap validity bits
  // (bit t set when tap t reads inside the image; bit 31 is never set)
  int pb[NBW];
  uint32_t vmask[NBW];
#pragma unroll
  for (int r = 0; r < NBW; ++r) {
    const int m = m0 + RPP * (wave + 4 * r) + lrow;
    const bool mval = m < Mtot;
    const int mm = mval ? m : 0;
    const int t = udiv(mm, s.Wm, s.rWm);
    const int mx = mm - t * s.Wm;
    const int b = udiv(t, s.Hm, s.rHm);
    const int biy = (t - b * s.Hm) * s.sy, bix = mx * s.sy;
    pb[r] = (b * in_h + biy) * in_w + bix;
    uint32_t vm = 0;
    for (int tap = 0, ty = 0, tx = 0; tap < ntaps; ++tap) {
      const int iy = biy + (convt ? 1 - ty : ty - pad), ix = bix + (convt ? 1 - tx : tx - pad);
      if (mval && (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w) vm |= 1u << tap;
      if (++tx == tw) { tx = 0; ++ty; }
    }
    vmask[r] = vm;
  }

  // ---- incremental k -> (tap, ci) decode of this lane's source chunk
  KDec dec;
  {
    const int k0 = s_beg * KS + c * EPV;
    dec.tap = k0 / cin_pad;
    dec.ci = k0 - dec.tap * cin_pad;
    dec.ty = dec.tap / tw;
    dec.tx = dec.tap - dec.ty * tw;
  }

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wm = wave % WGM, wn = wave / WGM;
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)smem);

  // Staging code for stage `st_issue` (used by the prologue and the steady-state loop).
  // A macro, not a lambda: captured locals would be address-taken, and the DMA
  // statement's "memory" clobber then pins them to scratch; and a merged prologue /
  // steady-state loop makes the accumulators a loop-carried VGPR/AGPR copy pair.
  // Per B piece the lane does: tap-bit test, pixel + tap offset, mul24 by the source's
  // row pitch, 64-bit add and the zero-page select (the host keeps sources < 2^24 pixels).
#define CONV_ISSUE_STAGE(st_issue)                                                            \
  do {                                                                                        \
    const uint32_t lst = lbase + (uint32_t)(((st_issue) % NBUF) * STAGE * 16);               \
    const char* wst = wbase + (size_t)(s_beg + (st_issue)) * KS * sizeof(T);                  \
_Pragma("unroll")                                                                             \
    for (int i = 0; i < NAW; ++i) dma16_s(wst, aoff[i], lst + alds[i] * 16);                 \
    const int dy = convt ? 1 - dec.ty : dec.ty - pad;                                         \
    const int dx = convt ? 1 - dec.tx : dec.tx - pad;                                         \
    const int ci = dec.ci;                                                                    \
    const bool in0 = ci < send0, in1 = ci < send1;                                            \
    const char* src = in0 ? sp0 : (in1 ? sp1 : sp2);                                          \
    const int sldb = (in0 ? sld0 : (in1 ? sld1 : sld2)) * (int)sizeof(T);                     \
    const int csb = (ci - (in0 ? 0 : (in1 ? send0 : send1))) * (int)sizeof(T);               \
    const int bit = ((dec.tap < ntaps) & (ci < send2)) ? dec.tap : 31;                        \
    const int doff = dy * in_w + dx;                                                          \
_Pragma("unroll")                                                                             \
    for (int r = 0; r < NBW; ++r) {                                                           \
      const bool ok = (vmask[r] >> bit) & 1u;                                                 \
      const unsigned off = (unsigned)__umul24((unsigned)(pb[r] + doff), (unsigned)sldb) +     \
                           (unsigned)csb;                                                     \
      const void* gp = ok ? (const void*)(src + off) : (const void*)g_zero_page;              \
      dma16_l(gp, lst + (IA + wave + 4 * r) * 64 * 16);                                       \
    }                                                                                         \
    /* advance this lane's decode to the next stage */                                        \
    dec.ci += KS;                                                                             \
    while (dec.ci >= cin_pad) {                                                               \
      dec.ci -= cin_pad;                                                                      \
      ++dec.tap;                                                                              \
      if (++dec.tx == tw) { dec.tx = 0; ++dec.ty; }                                           \
    }                                                                                         \
  } while (0)

#pragma unroll
  for (int st = 0; st < NBUF - 1; ++st)
    if (st < ns) CONV_ISSUE_STAGE(st);

  for (int it = 0; it < ns; ++it) {
    // retire stage `it`: leave the stages issued after it in flight
    wait_ring<LW, NBUF - 2>(ns - 1 - it);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (it + NBUF - 1 < ns) CONV_ISSUE_STAGE(it + NBUF - 1);
    const uint4* As = smem + (it % NBUF) * STAGE;
    const uint4* Bs = As + BN * CPR;
#pragma unroll
    for (int ks = 0; ks < 2 * KSM; ++ks) {
      const int chunk = (4 * ks + fq) ^ (fr & 7);
      uint4 a[TN], b[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) a[j] = As[(wn * TN * 16 + j * 16 + fr) * CPR + chunk];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        b[i] = Bs[(wm * TM * 16 + i * 16 + fr) * CPR + chunk];
        if (sq_in) b[i] = square_chunk<T>(b[i]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], a[j], b[i]);
    }
  }

#undef CONV_ISSUE_STAGE

  if (s.act == RGBAC_ACT_GAUSS) {
    // (mu | sigma) tile -> LDS [BM][BN] fp32, then one (pixel, channel) per thread
    float* tilef = reinterpret_cast<float*>(smem);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ml = wm * TM * 16 + i * 16 + fr;
          const int nl = wn * TN * 16 + j * 16 + fq * 4 + r;
          tilef[ml * BN + nl] = acc[j][i][r] + (g.bias ? g.bias[nl] : 0.0f);
        }
    __syncthreads();
    const int nch = g.cout >> 1;
    double bits = 0.0;
    for (int e = tid; e < BM * nch; e += 256) {
      const int ml = e / nch, ch = e - ml * nch;
      const int m = m0 + ml;
      if (m < s.M) bits += (double)gauss_elem<T>(g, m, ch, nch, tilef[ml * BN + ch],
                                                 tilef[ml * BN + nch + ch]);
    }
    const double tot = block_sum_f64(bits, red);
    if (tid == 0) g.partial[mblk] = tot;
    return;
  }

  // ---- epilogue: lane owns channels n..n+3 of pixel m for every (j, i) tile
  int nn[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) nn[j] = n0 + wn * TN * 16 + j * 16 + fq * 4;
  if (s.ksplit > 1 && g.cnt) {
    // split-K slab, then an in-launch reduction by the tile's last-arriving split block
    // (agent-scope release / relaxed ticket / agent-scope acquire; cdna_hip_programming.md
    // "In-launch split-K reduction"), so no separate reduce launch is needed
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * TM * 16 + i * 16 + fr;
      if (m >= s.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (nn[j] >= g.cout) continue;
        float* w = g.ws + (((size_t)split * s.nphase + phase) * s.M + m) * g.cout16 + nn[j];
        *reinterpret_cast<float4*>(w) =
            make_float4(acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = reinterpret_cast<int*>(red);
    if (tid == 0) {
      const int tix = ((gi * s.nphase + phase) * (int)gridDim.x + mblk) * (int)gridDim.y + nblk;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int old = __hip_atomic_fetch_add(&g.cnt[tix], 1, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == s.ksplit - 1;
      if (last) {
        __hip_atomic_store(&g.cnt[tix], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    // R quads per thread per pass; every slab and residual load of a pass is issued before
    // any math (the reducer pays ~one memory latency per pass, not one per load)
    constexpr int NQ = BN / 4;
    constexpr int R = (BM * NQ / 256) < 4 ? (BM * NQ / 256) : 4;
    static_assert(R >= 1 && (BM * NQ) % (256 * R) == 0, "reducer geometry");
    const size_t sstride = (size_t)s.nphase * s.M * g.cout16;
    for (int e0 = tid; e0 < BM * NQ; e0 += 256 * R) {
      int mq[R], nq4[R];
      bool ok[R];
      float v[R][4];
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int e = e0 + 256 * q;
        const int ml = e / NQ;
        mq[q] = m0 + ml;
        nq4[q] = n0 + 4 * (e - ml * NQ);
        ok[q] = mq[q] < s.M && nq4[q] < g.cout;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[q][r] = 0.f;
      }
      const float* base = g.ws + (size_t)phase * s.M * g.cout16;
      for (int sp = 0; sp < s.ksplit; ++sp) {
        float4 t[R];
#pragma unroll
        for (int q = 0; q < R; ++q)
          t[q] = ok[q] ? *reinterpret_cast<const float4*>(base + sp * sstride +
                                                          (size_t)mq[q] * g.cout16 + nq4[q])
                       : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int q = 0; q < R; ++q) {
          v[q][0] += t[q].x; v[q][1] += t[q].y; v[q][2] += t[q].z; v[q][3] += t[q].w;
        }
      }
#pragma unroll
      for (int q = 0; q < R; ++q)
        if (ok[q]) epilogue4<T>(s, g, phase, mq[q], nq4[q], v[q]);
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wm * TM * 16 + i * 16 + fr;
    if (m >= s.M) continue;
    if (s.ksplit > 1) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if (nn[j] >= g.cout) continue;
        float* w = g.ws + (((size_t)split * s.nphase + phase) * s.M + m) * g.cout16 + nn[j];
        *reinterpret_cast<float4*>(w) =
            make_float4(acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]);
      }
      continue;
    }
    // the row's residual loads are issued together, then the math and stores (one
    // memory latency per 16-pixel row instead of one per 16x16 tile)
    epilogue_tile_row<T, TN>(s, g, phase, m, nn, acc, i);
  }
}

// ---------------------------------------------------------------------------
// Persistent variant of conv_kernel (no GAUSS epilogue).  grid = (G, 1, Z): block x of
// z-slice (group, split, phase) walks the slice's output tiles f = x, x + G, ...
// (N-tile fastest) and streams ONE flattened sequence of (tile, K-stage) pieces through
// the NBUF ring, so the next tile's first stages load while the current tile's last
// stages compute and its epilogue stores -- the prologue/epilogue latency of short-K
// convs (1x1, GDN, qkv/proj, x1, DSE) is hidden instead of paid once per tile.
template <typename T, int BM, int BN, int WGM, int WGN, int NBUF>
__global__ void __launch_bounds__(256) conv_pers_kernel(const ConvArgsDev args) {
  constexpr int EPV = Elem<T>::EPV;
  constexpr int KS = 8 * EPV;
  constexpr int TM = BM / WGM / 16;
  constexpr int TN = BN / WGN / 16;
  constexpr int IA = BN / 8, IB = BM / 8;
  constexpr int LW = (IA + IB + 3) / 4;
  constexpr int STAGE = (BN + BM) * 8;
  static_assert(WGM * WGN == 4, "4 waves");
  static_assert(TM >= 1 && TN >= 1, "tile");
  __shared__ __attribute__((aligned(16))) uint4 smem[NBUF * STAGE];

  const ConvShared& s = args.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int t = blockIdx.z;
  const int phase = t % s.nphase; t /= s.nphase;
  const int split = t % s.ksplit;
  const int gi = t / s.ksplit;
  const ConvGroup& g = args.g[gi];
  const int Mb = (s.M + BM - 1) / BM;
  const int Nb = (g.cout + BN - 1) / BN;
  const int ntile = Mb * Nb;
  const int G = gridDim.x;
  if ((int)blockIdx.x >= ntile) return;
  const int mytiles = (ntile - 1 - (int)blockIdx.x) / G + 1;

  const int py = phase >> 1, px = phase & 1;
  int ntaps, tw;
  if (s.mode == RGBAC_CONVT_S2) {
    tw = 3 - px;
    ntaps = (3 - py) * tw;
  } else {
    tw = s.ksize;
    ntaps = s.ksize * s.ksize;
  }
  const int ktot = ntaps * g.cin_pad;
  const int nst = (ktot + KS - 1) / KS;
  const int s_beg = (int)((long long)nst * split / s.ksplit);
  const int s_end = (int)((long long)nst * (split + 1) / s.ksplit);
  const int ns = s_end - s_beg;
  const int nq = mytiles * ns;

  const int in_h = s.in_h, in_w = s.in_w, cin_pad = g.cin_pad, Mtot = s.M;
  const int Wm = s.Wm, Hm = s.Hm, sy = s.sy;
  const double rWm = s.rWm, rHm = s.rHm;
  const int send0 = g.send0, send1 = g.send1, send2 = g.send2;
  const char* const sp0 = reinterpret_cast<const char*>(g.sp0);
  const char* const sp1 = reinterpret_cast<const char*>(g.sp1);
  const char* const sp2 = reinterpret_cast<const char*>(g.sp2);
  const int sld0 = (int)g.sld0, sld1 = (int)g.sld1, sld2 = (int)g.sld2;
  const bool convt = s.mode == RGBAC_CONVT_S2;
  const int pad = s.pad;
  const bool sq_in = s.square != 0;
  const int kpad = g.k_pad;

  const int lrow = lane >> 3;
  const int c = (lane & 7) ^ lrow;
  int jpc[LW];
  bool isA[LW];
  int lofs[LW];
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    int j = wave + 4 * i;
    if (j >= IA + IB) j = IA + IB - 1;
    jpc[i] = j;
    isA[i] = j < IA;
    lofs[i] = j * 64;
  }
  const T* wbase = reinterpret_cast<const T*>(g.w) + (size_t)phase * g.rows * kpad + c * EPV;
  // per-piece state of the tile currently being ISSUED
  const T* wrow[LW];
  int pbase[LW], biy[LW], bix[LW];
  bool bval[LW];
  KDec dec;
  const int k0 = s_beg * KS + c * EPV;

#define PERS_SETUP_TILE(ti)                                                                   \
  do {                                                                                        \
    const int f_ = (int)blockIdx.x + (ti) * G;                                                \
    const int n0_ = (f_ % Nb) * BN, m0_ = (f_ / Nb) * BM;                                     \
    _Pragma("unroll")                                                                         \
    for (int i = 0; i < LW; ++i) {                                                            \
      wrow[i] = wbase + (size_t)(n0_ + (isA[i] ? 8 * jpc[i] + lrow : 0)) * kpad;              \
      const int m = m0_ + 8 * (jpc[i] - IA) + lrow;                                           \
      bval[i] = !isA[i] && m < Mtot;                                                          \
      const int mm = bval[i] ? m : 0;                                                         \
      const int t_ = udiv(mm, Wm, rWm);                                                       \
      const int mx = mm - t_ * Wm;                                                            \
      const int b_ = udiv(t_, Hm, rHm);                                                       \
      biy[i] = (t_ - b_ * Hm) * sy;                                                           \
      bix[i] = mx * sy;                                                                       \
      pbase[i] = (b_ * in_h + biy[i]) * in_w + bix[i];                                        \
    }                                                                                         \
    dec.tap = k0 / cin_pad;                                                                   \
    dec.ci = k0 - dec.tap * cin_pad;                                                          \
    dec.ty = dec.tap / tw;                                                                    \
    dec.tx = dec.tap - dec.ty * tw;                                                           \
  } while (0)

#define PERS_ISSUE(q_)                                                                        \
  do {                                                                                        \
    const int qq_ = (q_);                                                                     \
    const int sti_ = qq_ % ns;                                                                \
    if (sti_ == 0) PERS_SETUP_TILE(qq_ / ns);                                                 \
    const int dy = convt ? 1 - dec.ty : dec.ty - pad;                                         \
    const int dx = convt ? 1 - dec.tx : dec.tx - pad;                                         \
    const int ci = dec.ci;                                                                    \
    const bool in0 = ci < send0, in1 = ci < send1;                                            \
    const char* src = in0 ? sp0 : (in1 ? sp1 : sp2);                                          \
    const int sld = in0 ? sld0 : (in1 ? sld1 : sld2);                                         \
    const int cs = ci - (in0 ? 0 : (in1 ? send0 : send1));                                    \
    const bool kval = (dec.tap < ntaps) & (ci < send2);                                       \
    const int doff = dy * in_w + dx;                                                          \
    const int kk = (s_beg + sti_) * KS;                                                       \
    uint4* stage = smem + (qq_ % NBUF) * STAGE;                                               \
    _Pragma("unroll")                                                                         \
    for (int i = 0; i < LW; ++i) {                                                            \
      const void* gp;                                                                         \
      if (isA[i]) {                                                                           \
        gp = wrow[i] + kk;                                                                    \
      } else {                                                                                \
        const int iy = biy[i] + dy, ix = bix[i] + dx;                                         \
        const bool ok = kval & bval[i] & ((unsigned)iy < (unsigned)in_h) &                    \
                        ((unsigned)ix < (unsigned)in_w);                                      \
        const unsigned off = ((unsigned)((pbase[i] + doff) * sld + cs)) * (unsigned)sizeof(T); \
        gp = ok ? (const void*)(src + off) : (const void*)g_zero_page;                        \
      }                                                                                       \
      dma16(gp, stage + lofs[i]);                                                             \
    }                                                                                         \
    dec.ci += KS;                                                                             \
    while (dec.ci >= cin_pad) {                                                               \
      dec.ci -= cin_pad;                                                                      \
      ++dec.tap;                                                                              \
      if (++dec.tx == tw) { dec.tx = 0; ++dec.ty; }                                           \
    }                                                                                         \
  } while (0)

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int wm = wave % WGM, wn = wave / WGM;
  const int fr = lane & 15, fq = lane >> 4, sw = lane & 7;

#pragma unroll
  for (int st = 0; st < NBUF - 1; ++st)
    if (st < nq) PERS_ISSUE(st);

  int ktile = 0, kst = 0;                      // tile / stage being consumed
  for (int q = 0; q < nq; ++q) {
    wait_ring<LW, NBUF - 2>(nq - 1 - q);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (q + NBUF - 1 < nq) PERS_ISSUE(q + NBUF - 1);
    const uint4* As = smem + (q % NBUF) * STAGE;
    const uint4* Bs = As + BN * 8;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = (4 * ks + fq) ^ sw;
      uint4 a[TN], b[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) a[j] = As[(wn * TN * 16 + j * 16 + fr) * 8 + chunk];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        b[i] = Bs[(wm * TM * 16 + i * 16 + fr) * 8 + chunk];
        if (sq_in) b[i] = square_chunk<T>(b[i]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], a[j], b[i]);
    }
    if (++kst < ns) continue;
    // ---- tile `ktile` complete: fused epilogue, then reset the accumulators
    {
      const int f = (int)blockIdx.x + ktile * G;
      const int n0 = (f % Nb) * BN, m0 = (f / Nb) * BM;
      int nn[TN];
#pragma unroll
      for (int j = 0; j < TN; ++j) nn[j] = n0 + wn * TN * 16 + j * 16 + fq * 4;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * TM * 16 + i * 16 + fr;
        if (m < Mtot) {
          if (s.ksplit > 1) {
#pragma unroll
            for (int j = 0; j < TN; ++j) {
              if (nn[j] >= g.cout) continue;
              float* w = g.ws + (((size_t)split * s.nphase + phase) * s.M + m) * g.cout16 + nn[j];
              *reinterpret_cast<float4*>(w) =
                  make_float4(acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]);
            }
          } else {
            epilogue_tile_row<T, TN>(s, g, phase, m, nn, acc, i);
          }
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    kst = 0;
    ++ktile;
  }
#undef PERS_ISSUE
#undef PERS_SETUP_TILE
}

template <typename T>
__global__ void __launch_bounds__(256) conv_splitk_epilogue(const ConvArgsDev args, int gi) {
  const ConvShared& s = args.s;
  const ConvGroup& g = args.g[gi];
  const int nq = g.cout16 / 4;
  const long long total = (long long)s.nphase * s.M * nq;
  for (long long e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const int q = (int)(e % nq);
    const long long pm = e / nq;
    const int m = (int)(pm % s.M);
    const int ph = (int)(pm / s.M);
    const int n = 4 * q;
    if (n >= g.cout) continue;
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    // up to 8 slabs' loads in flight before the first add (the adds keep slab order: the
    // sums are the one-load-at-a-time loop's, bit for bit)
    const size_t slab = (size_t)s.nphase * s.M * g.cout16;
    const float* wp = g.ws + ((size_t)ph * s.M + m) * g.cout16 + n;
    for (int sp0 = 0; sp0 < s.ksplit; sp0 += 8) {
      float4 t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (sp0 + u < s.ksplit) t[u] = *reinterpret_cast<const float4*>(wp + (sp0 + u) * slab);
#pragma unroll
      for (int u = 0; u < 8; ++u)
        if (sp0 + u < s.ksplit) { v[0] += t[u].x; v[1] += t[u].y; v[2] += t[u].z; v[3] += t[u].w; }
    }
    epilogue4<T>(s, g, ph, m, n, v);
  }
}

// ---------------------------------------------------------------------------
// Weight-resident persistent variant (small K: 1x1 convs, GDN, qkv/proj,
// DSE 3x3 at 32 channels, ...).  Each workgroup DMAs its BN x K weight panel
// into LDS ONCE, then streams pixel tiles t = blockIdx.x + i*gridDim.x through
// a 3-deep B ring.  Stages are numbered by one flat counter across tiles, so
// the next tile's loads are in flight while the current tile's epilogue runs.
// Requires nst <= NSA stages of K, ksplit == 1, no GAUSS epilogue.
template <typename T, int BM, int BN, int WGM, int WGN, int NSA>
__global__ void __launch_bounds__(256) conv_wres_kernel(const ConvArgsDev args) {
  constexpr int EPV = Elem<T>::EPV;
  constexpr int KS = 8 * EPV;
  constexpr int TM = BM / WGM / 16;
  constexpr int TN = BN / WGN / 16;
  constexpr int IA = BN / 8, IB = BM / 8;
  constexpr int LWA = (IA + 3) / 4, LWB = (IB + 3) / 4;
  constexpr int NB = 3;
  static_assert(WGM * WGN == 4 && TM >= 1 && TN >= 1, "tile");
  __shared__ __attribute__((aligned(16))) uint4 smem[NSA * BN * 8 + NB * BM * 8];
  uint4* const Ares = smem;
  uint4* const Bring = smem + NSA * BN * 8;

  const ConvShared& s = args.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int phase = blockIdx.z % s.nphase;
  const int gi = blockIdx.z / s.nphase;
  const ConvGroup& g = args.g[gi];
  const int n0 = blockIdx.y * BN;
  if (n0 >= g.cout) return;
  const int py = phase >> 1, px = phase & 1;
  int ntaps, tw;
  if (s.mode == RGBAC_CONVT_S2) {
    tw = 3 - px;
    ntaps = (3 - py) * tw;
  } else {
    tw = s.ksize;
    ntaps = s.ksize * s.ksize;
  }
  const int nst = (ntaps * g.cin_pad + KS - 1) / KS;
  const int mtiles = (s.M + BM - 1) / BM;
  const int mine = blockIdx.x < mtiles ? (mtiles - 1 - blockIdx.x) / gridDim.x + 1 : 0;
  const int Q = mine * nst;
  const int lrow = lane >> 3;
  const int c = (lane & 7) ^ lrow;

  // ---- resident weight panel: all nst stages of rows n0..n0+BN-1
  const T* wbase = reinterpret_cast<const T*>(g.w) + (size_t)phase * g.rows * g.k_pad;
  for (int st = 0; st < nst; ++st) {
#pragma unroll
    for (int i = 0; i < LWA; ++i) {
      int j = wave + 4 * i;
      if (j >= IA) j = IA - 1;
      dma16(wbase + (size_t)(n0 + 8 * j + lrow) * g.k_pad + st * KS + c * EPV,
            Ares + st * BN * 8 + j * 64);
    }
  }

  auto issueB = [&](int q) {
    const int tl = q / nst;
    const int st = q - tl * nst;
    const int m0 = (blockIdx.x + tl * gridDim.x) * BM;
    const int k = st * KS + c * EPV;
    const int tap = k / g.cin_pad;
    const int ci = k - tap * g.cin_pad;
    const int ty = tap / tw, tx = tap - ty * tw;
    int dy, dx;
    if (s.mode == RGBAC_CONVT_S2) {
      dy = 1 - ty; dx = 1 - tx;
    } else {
      dy = ty - s.pad; dx = tx - s.pad;
    }
    const void* sp;
    long long sld;
    int cs;
    bool kval = tap < ntaps;
    if (ci < g.send0) {
      sp = g.sp0; sld = g.sld0; cs = ci;
    } else if (ci < g.send1) {
      sp = g.sp1; sld = g.sld1; cs = ci - g.send0;
    } else {
      sp = g.sp2; sld = g.sld2; cs = ci - g.send1;
      kval = kval && ci < g.send2;
    }
    const T* src = reinterpret_cast<const T*>(sp);
    uint4* buf = Bring + (q % NB) * BM * 8;
#pragma unroll
    for (int i = 0; i < LWB; ++i) {
      int j = wave + 4 * i;
      if (j >= IB) j = IB - 1;
      const int m = m0 + 8 * j + lrow;
      const void* gp = (const void*)g_zero_page;
      if (kval && m < s.M) {
        const int t = udiv(m, s.Wm, s.rWm);
        const int mx = m - t * s.Wm;
        const int b = udiv(t, s.Hm, s.rHm);
        const int iy = (t - b * s.Hm) * s.sy + dy, ix = mx * s.sy + dx;
        if (iy >= 0 && iy < s.in_h && ix >= 0 && ix < s.in_w)
          gp = (const void*)(src + ((long long)(b * s.in_h + iy) * s.in_w + ix) * sld + cs);
      }
      dma16(gp, buf + j * 64);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = wave % WGM, wn = wave / WGM;
  const int fr = lane & 15, fq = lane >> 4, sw = lane & 7;
  int nn[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) nn[j] = n0 + wn * TN * 16 + j * 16 + fq * 4;

  if (Q > 0) issueB(0);
  if (Q > 1) issueB(1);
  for (int q = 0; q < Q; ++q) {
    if (q + 1 < Q) wait_vm<LWB>(); else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (q + 2 < Q) issueB(q + 2);
    const int tl = q / nst;
    const int st = q - tl * nst;
    const uint4* As = Ares + st * BN * 8;
    const uint4* Bs = Bring + (q % NB) * BM * 8;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = (4 * ks + fq) ^ sw;
      uint4 a[TN], b[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) a[j] = As[(wn * TN * 16 + j * 16 + fr) * 8 + chunk];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        b[i] = Bs[(wm * TM * 16 + i * 16 + fr) * 8 + chunk];
        if (s.square) b[i] = square_chunk<T>(b[i]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], a[j], b[i]);
    }
    if (st == nst - 1) {
      const int m0 = (blockIdx.x + tl * gridDim.x) * BM;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wm * TM * 16 + i * 16 + fr;
        float v[TN][4];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] = acc[j][i][r];
          acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        if (m < s.M) epilogue_row<T, TN>(s, g, phase, m, nn, v);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Direct small-K variant (CONV mode, K <= NKS k-steps).  The workgroup's weight
// panel (16*NT rows x K) is loaded into LDS once; then every WAVE walks its own
// 16-pixel tiles (tile = (blockIdx.x*4 + wave) + i*gridDim.x*4): the im2col row
// of pixel (lane&15), chunk (lane>>4) of every k-step, is loaded straight into
// VGPRs (one 16-byte load per k-step; zero for padding), the NT x nks MFMAs run
// from LDS weight fragments, and the fused epilogue stores the tile.  No
// barrier after the weight load: latency is hidden by the other resident waves.
template <typename T, int NT, int NKS>
__global__ void __launch_bounds__(256) conv_direct_kernel(const ConvArgsDev args, int rs) {
  constexpr int EPV = Elem<T>::EPV;
  constexpr int KSTEP = 4 * EPV;
  constexpr int BN = 16 * NT;
  extern __shared__ __attribute__((aligned(16))) uint4 Wl[];   // [BN][rs] chunks
  __shared__ int ktab[NKS * 4];   // per (k-step, chunk): valid | src | dx | dy | channel

  const ConvShared& s = args.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const ConvGroup& g = args.g[blockIdx.z];
  const int n0 = blockIdx.y * BN;
  if (n0 >= g.cout) return;
  const int ntaps = s.ksize * s.ksize;
  const int nks = (ntaps * g.cin_pad + KSTEP - 1) / KSTEP;
  const T* wbase = reinterpret_cast<const T*>(g.w);
  for (int e = tid; e < BN * nks * 4; e += 256) {
    const int row = e / (nks * 4), ch = e - row * (nks * 4);
    Wl[row * rs + ch] = n0 + row < g.rows
        ? *reinterpret_cast<const uint4*>(wbase + (size_t)(n0 + row) * g.k_pad + ch * EPV)
        : make_uint4(0, 0, 0, 0);   // panel rows past the packed cout_pad
  }
  if (tid < NKS * 4) {
    const int st = tid >> 2, q = tid & 3;
    const int k = st * KSTEP + q * EPV;
    const int tap = k / g.cin_pad;
    const int ci = k - tap * g.cin_pad;
    const int ty = tap / s.ksize, tx = tap - ty * s.ksize;
    int src, cs;
    bool ok = st < nks && tap < ntaps;
    if (ci < g.send0) { src = 0; cs = ci; }
    else if (ci < g.send1) { src = 1; cs = ci - g.send0; }
    else { src = 2; cs = ci - g.send1; ok = ok && ci < g.send2; }
    ktab[tid] = cs | ((ty - s.pad + 4) << 12) | ((tx - s.pad + 4) << 15) | (src << 18) | ((int)ok << 20);
  }
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  const int ntile = (s.M + 15) / 16;
  for (int tile = blockIdx.x * 4 + wave; tile < ntile; tile += gridDim.x * 4) {
    const int m = tile * 16 + fr;
    const int mm = m < s.M ? m : s.M - 1;
    const int t = udiv(mm, s.Wm, s.rWm);
    const int x = mm - t * s.Wm;
    const int b = udiv(t, s.Hm, s.rHm);
    const int y = t - b * s.Hm;
    uint4 bv[NKS];
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      bv[st] = make_uint4(0, 0, 0, 0);
      if (st < nks) {
        const int e = ktab[st * 4 + fq];
        const int iy = y * s.sy + ((e >> 12) & 7) - 4, ix = x * s.sy + ((e >> 15) & 7) - 4;
        const int src = (e >> 18) & 3;
        if ((e >> 20) && iy >= 0 && iy < s.in_h && ix >= 0 && ix < s.in_w) {
          const T* base = reinterpret_cast<const T*>(src == 0 ? g.sp0 : (src == 1 ? g.sp1 : g.sp2));
          const long long ld = src == 0 ? g.sld0 : (src == 1 ? g.sld1 : g.sld2);
          bv[st] = *reinterpret_cast<const uint4*>(
              base + ((long long)(b * s.in_h + iy) * s.in_w + ix) * ld + (e & 0xFFF));
        }
        if (s.square) bv[st] = square_chunk<T>(bv[st]);
      }
    }
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      if (st < nks) {
#pragma unroll
        for (int j = 0; j < NT; ++j) mma_step<T>(acc[j], Wl[(j * 16 + fr) * rs + st * 4 + fq], bv[st]);
      }
    }
    if (m < s.M) {
      constexpr int CH = NT < 4 ? NT : 4;          // epilogue in chunks of <= 4 tiles
#pragma unroll
      for (int j0 = 0; j0 < NT; j0 += CH) {
        int nn[CH];
        float v[CH][4];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          nn[j] = n0 + (j0 + j) * 16 + fq * 4;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] = acc[j0 + j][r];
        }
        epilogue_row<T, CH>(s, g, 0, m, nn, v);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Spatial-tile variant for 3x3 stride-1 convs with Cin = 32 and Cout <= 32
// (the DSE EnhancementBlocks at full resolution): one workgroup per 16x16 output
// tile stages its 18x18x32 input halo (20.7 KB) and the whole 32 x 288 weight
// panel (18.4 KB) in LDS once, then each wave runs 4 rows x 2 channel tiles x
// 9 taps = 72 MFMAs straight from LDS (the k-step of 32 channels is one tap).
// Both LDS images use slot = chunk ^ ((row >> 1) & 3), conflict-free for the
// ds_read_b128 lane groups of the fragment reads.  bf16 only.
template <typename T>
__global__ void __launch_bounds__(256, 4) conv3x3_c32_kernel(const ConvArgsDev args) {
  constexpr int TS = 16, HS = TS + 2, NH = HS * HS;
  __shared__ __attribute__((aligned(16))) uint4 Xs[NH * 4];
  __shared__ __attribute__((aligned(16))) uint4 Ws[32 * 36];
  const ConvShared& s = args.s;
  const ConvGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int tx_n = s.Wm / TS, ty_n = s.Hm / TS;
  int t = blockIdx.x;
  const int tx = t % tx_n; t /= tx_n;
  const int ty = t % ty_n;
  const int b = t / ty_n;
  const int y0 = ty * TS, x0 = tx * TS;
  // every global load of the staging is issued before the first LDS store (fully unrolled
  // register staging): one memory latency per workgroup, not one per loop iteration (the
  // strided loops compiled to load / vmcnt(0) / ds_write chains)
  constexpr int NWL = (32 * 36 + 255) / 256, NXL = (NH * 4 + 255) / 256;
  const T* wsrc = reinterpret_cast<const T*>(g.w);
  const T* xsrc = reinterpret_cast<const T*>(g.sp0);
  uint4 wv[NWL], xv[NXL];
  // (branch-free: a thread past the end takes the last slot's clamped index, loading and
  // storing the same value as its owner -- no exec-masked block for the compiler to sink the
  // loads into, which would split them into separately waited groups again)
#pragma unroll
  for (int u = 0; u < NWL; ++u) {
    const int e = min(tid + 256 * u, 32 * 36 - 1);
    const int r = e / 36, c = e - r * 36;
    wv[u] = *reinterpret_cast<const uint4*>(wsrc + (size_t)r * g.k_pad + c * 8);
  }
  bool xin[NXL];
#pragma unroll
  for (int u = 0; u < NXL; ++u) {
    const int e = min(tid + 256 * u, NH * 4 - 1);
    const int hr = e >> 2, c = e & 3;
    const int hy = hr / HS, hx = hr - hy * HS;
    const int iy = y0 + hy - 1, ix = x0 + hx - 1;
    xin[u] = iy >= 0 && iy < s.in_h && ix >= 0 && ix < s.in_w;
    const int cy = min(max(iy, 0), s.in_h - 1), cx = min(max(ix, 0), s.in_w - 1);
    xv[u] = *reinterpret_cast<const uint4*>(xsrc + ((long long)(b * s.in_h + cy) * s.in_w + cx) * g.sld0 + c * 8);
  }
#pragma unroll
  for (int u = 0; u < NWL; ++u) {
    const int e = min(tid + 256 * u, 32 * 36 - 1);
    const int r = e / 36, c = e - r * 36;
    Ws[r * 36 + (c ^ ((r >> 1) & 3))] = wv[u];
  }
  const bool sq = s.square;
#pragma unroll
  for (int u = 0; u < NXL; ++u) {
    const int e = min(tid + 256 * u, NH * 4 - 1);
    const int hr = e >> 2, c = e & 3;
    uint4 v = xin[u] ? xv[u] : make_uint4(0, 0, 0, 0);
    if (sq) v = square_chunk<T>(v);
    Xs[hr * 4 + (c ^ ((hr >> 1) & 3))] = v;
  }
  __syncthreads();
  f32x4 acc[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int dy = tap / 3, dx = tap % 3;
    uint4 A[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = 16 * j + fr;
      A[j] = Ws[r * 36 + ((4 * tap + fq) ^ ((r >> 1) & 3))];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int hr = (wave * 4 + i + dy) * HS + fr + dx;
      const uint4 B = Xs[hr * 4 + (fq ^ ((hr >> 1) & 3))];
#pragma unroll
      for (int j = 0; j < 2; ++j) mma_step<T>(acc[j][i], A[j], B);
    }
  }
  // stride-1 CONV: output pixel = m.  The residual / bias operands of two rows' quads are
  // requested before their stores (the output may alias a residual -- the training path's
  // in-place gradient accumulation -- and a load issued behind a store waits for it)
  float bias[2][4];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = 16 * j + fq * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) bias[j][r] = (g.bias && n < g.cout) ? g.bias[n + r] : 0.0f;
  }
#pragma unroll
  for (int i0 = 0; i0 < 4; i0 += 2) {
    EpiIn in[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = (b * s.Hm + y0 + wave * 4 + i0 + i) * s.Wm + x0 + fr;
#pragma unroll
      for (int j = 0; j < 2; ++j)
        if (16 * j + fq * 4 < g.cout) in[i][j].template load<T>(g, s.act, (long long)m, 16 * j + fq * 4);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int m = (b * s.Hm + y0 + wave * 4 + i0 + i) * s.Wm + x0 + fr;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = 16 * j + fq * 4;
        if (n >= g.cout) continue;
        float v[4] = {acc[j][i0 + i][0], acc[j][i0 + i][1], acc[j][i0 + i][2], acc[j][i0 + i][3]};
        epilogue4_fin<T>(s, g, (long long)m, n, v, bias[j], in[i][j]);
      }
    }
  }
}

template <typename T, int NT>
static void launch_direct(const ConvArgsDev& d, dim3 grid, int rs, int nks_max, hipStream_t st) {
  constexpr int NKS = 12;
  const size_t lds = (size_t)16 * NT * rs * 16;
  (void)nks_max;
  hipLaunchKernelGGL((conv_direct_kernel<T, NT, NKS>), grid, dim3(256), lds, st, d, rs);
}

struct TileCfg { int bm, bn; };
// 0..6: streaming K-ring kernel; 7..12: weight-resident persistent kernel (kWresStages)
static const TileCfg kTiles[] = {
    {128, 128}, {128, 64}, {64, 64}, {128, 32}, {64, 32}, {128, 16}, {64, 16},
    {128, 64}, {64, 64}, {128, 32}, {64, 32}, {128, 128}, {128, 16},
    {16, 16}, {16, 32}, {16, 48}, {16, 64}, {16, 96}, {16, 192},
    {256, 32},
    // 20..26: the streaming shapes of 0..6 with a deeper LDS ring (more K stages in flight)
    {128, 128}, {128, 64}, {64, 64}, {128, 32}, {64, 32}, {128, 16}, {64, 16},
    // 27..33: the streaming shapes of 0..6, persistent over output tiles (conv_pers_kernel)
    {128, 128}, {128, 64}, {64, 64}, {128, 32}, {64, 32}, {128, 16}, {64, 16},
    // 34: small-K wave-streaming kernel (32-pixel wave tiles x up to 192 channels)
    {32, 96},
    // 35: narrow-output wave-streaming kernel (32-pixel wave tiles x <= 32 channels, full K)
    {32, 32},
    // 36..41: patch-resident kernel (TH x 16 M-grid pixels x BN channels, 8 waves)
    {128, 192}, {128, 128}, {128, 96}, {128, 256}, {128, 192}, {128, 64},
    // 42..47: fragment-streamed patch kernel (TH x 16 pixels x BN channels)
    {128, 192}, {64, 192}, {128, 128}, {64, 128}, {128, 256}, {128, 64},
    // 48, 49: patch-resident kernel with a 4-deep weight ring
    {128, 64}, {128, 128},
    // 50: fragment-streamed patch kernel, 4 x 16 pixels x 64 channels
    {64, 64},
    // 51..53: fragment-streamed patch kernel, unrolled K split by kernel row (KS = 3)
    {64, 64}, {64, 128}, {64, 192},
    // 54: full-width pointwise kernel (32-pixel wave tiles x all 192 output channels)
    {32, 192},
    // 55: narrow-output patch kernel (4 x 16 pixels x <= 32 channels, K split over 8 waves)
    {64, 32},
    // 56..58: K-split fragment-patch kernel on taller tiles (TH x 16 pixels: the weight
    // panel, most of a workgroup's bytes, amortised over 2-4x the pixels)
    {128, 64}, {128, 128}, {256, 32}};
constexpr int kNumTiles = sizeof(kTiles) / sizeof(kTiles[0]);
constexpr int kFirstWres = 7;
constexpr int kWresStages = 6;
constexpr int kFirstDirect = 13;   // 13..18: direct kernel with NT = bn/16
constexpr int kDirectSteps = 12;
constexpr int kTileSpatial = 19;   // conv3x3_c32_kernel (16x16 pixels x 32 channels)
constexpr int kFirstDeep = 20;     // 20..26: deep-ring streaming tiles
constexpr int kFirstPers = 27;     // 27..33: persistent streaming tiles
constexpr int kTileSmallK = 34;    // conv_smallk_kernel (bf16, plain conv, K <= 256)
constexpr int kTileWStream = 35;   // conv_wstream_kernel (bf16, stride 1, k 1/3, cout <= 32)
constexpr int kFirstPatch = 36;    // 36..41: conv_patch_kernel (bf16; k3 s1 conv/subpel, convT)
constexpr int kFirstFPatch = 42;   // 42..47: conv_fpatch_kernel (fragment-major weights)
constexpr int kFirstPatch2 = 48;   // 48, 49: conv_patch_kernel with NBUF = 4
constexpr int kTileFPatch464 = 50; // conv_fpatch_kernel<4, 64>
constexpr int kFirstFPatchKS = 51; // 51..53: conv_fpatch_kernel<4, 64|128|192, ..., KS = 3>
constexpr int kTilePW = 54;        // conv_pw_kernel (bf16 1x1, one source, cin/cout <= 192)
constexpr int kTileNPatch = 55;    // conv_npatch_kernel (bf16 3x3 s1, cout <= 32, fragment-major)
constexpr int kFirstFPatchKS2 = 56; // 56..58: conv_fpatch_kernel<8,64|8,128|16,32, ..., KS = 3>
__host__ __device__ constexpr bool patch_tile(int t) {   // conv_patch_kernel tiles
  return (t >= 36 && t <= 41) || t == 48 || t == 49;
}
__host__ __device__ constexpr bool fpatch_tile(int t) {
  return (t >= 42 && t <= 47) || (t >= 50 && t <= 53) || (t >= 56 && t <= 58);
}
__host__ __device__ constexpr bool fpatch_ks_tile(int t) {
  return (t >= 51 && t <= 53) || (t >= 56 && t <= 58);
}
#ifndef RGBAC_RC1
#define RGBAC_RC1 24   // unrolled-K fragment-patch weight ring depth at TN 1 (TN 2: half)
#endif
// RGBAC_FPATCH_CPT=0 disables the unrolled-K fragment-patch variants (A/B switch)
static bool fpatch_cpt_enabled() {
  static const bool on = [] {
    const char* e = getenv("RGBAC_FPATCH_CPT");
    return !(e && e[0] == '0');
  }();
  return on;
}
constexpr int kSmallKMax = 256;

// ---------------------------------------------------------------------------
// Pointwise (1x1, stride 1, one source, K = cin_pad <= 16 * NKS) wave-streaming kernel,
// bf16: the HBM-bound 1x1 convs at full resolution -- GDN/IGDN norm pools, qkv/proj,
// gates, the DSE in/out projections.  The block's weight panel (BN = 32*NT rows x K) is
// staged in LDS once; then each WAVE streams 32-pixel tiles on its own (no barrier):
// per 16-deep k-step ONE 16-byte load per lane (pixel lane&31, channels 8*(lane>>5)..+7,
// straight into VGPRs at an immediate offset from the pixel's row) feeds NT
// v_mfma_f32_32x32x16_bf16 whose A fragments come from the LDS panel.  Each k-step's
// fragment is reloaded for the wave's NEXT tile right after its MFMAs issue (a register
// ring), so the next tile's HBM reads overlap this tile's MFMAs and epilogue.
typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int NT, int NKS>
__global__ void __launch_bounds__(256, 2) conv_smallk_kernel(const ConvArgsDev args) {
  constexpr int BN = 32 * NT;
  constexpr int RS = 2 * NKS + 1;               // uint4 per panel row (odd: spreads banks)
  __shared__ __attribute__((aligned(16))) uint4 Wl[BN * RS];
  __shared__ float bl[BN];

  const ConvShared& s = args.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const ConvGroup& g = args.g[blockIdx.z];
  const int n0 = blockIdx.y * BN;
  if (n0 >= g.cout) return;
  const int act = s.act;
  for (int e = tid; e < BN; e += 256) bl[e] = (g.bias && n0 + e < g.rows) ? g.bias[n0 + e] : 0.0f;
  const int nchunk = g.cin_pad / 8;              // 8-channel chunks of K
  {
    const bf16_t* wbase = reinterpret_cast<const bf16_t*>(g.w);
    for (int e = tid; e < BN * 2 * NKS; e += 256) {
      const int row = e / (2 * NKS), ch = e - row * (2 * NKS);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n0 + row < g.rows && ch < nchunk)
        v = *reinterpret_cast<const uint4*>(wbase + (size_t)(n0 + row) * g.k_pad + ch * 8);
      Wl[row * RS + ch] = v;
    }
  }
  __syncthreads();

  const int Mtot = s.M;
  const int ld = (int)g.sld0;
  const bool sq_in = s.square != 0;
  const int r32 = lane & 31, h = lane >> 5;
  const char* const src = reinterpret_cast<const char*>(g.sp0) + 16 * h;
  // chunk 2*st+h of a pixel exists iff 16*st + 8*h < cin_pad
  const int ntile = (Mtot + 31) / 32;
  const int tstride = gridDim.x * 4;
  int tile = blockIdx.x * 4 + wave;
  if (tile >= ntile) return;

#define PW_LOAD(dst, st, rowp_, valid_)                                                       \
  do {                                                                                        \
    const bool ok_ = (valid_) & (2 * (st) + h < nchunk);                                      \
    const uint4* p_ = ok_ ? reinterpret_cast<const uint4*>((rowp_) + 32 * (st)) : g_zero_page; \
    dst = *p_;                                                                                \
  } while (0)

  uint4 bv[NKS];
  {
    const int m = tile * 32 + r32;
    const bool valid = m < Mtot;
    const char* rowp = src + (size_t)(valid ? m : 0) * ld * 2;
#pragma unroll
    for (int st = 0; st < NKS; ++st) PW_LOAD(bv[st], st, rowp, valid);
  }
  for (; tile < ntile; tile += tstride) {
    const int mn = (tile + tstride) * 32 + r32;
    const bool nvalid = mn < Mtot;
    const char* nrowp = src + (size_t)(nvalid ? mn : 0) * ld * 2;
    f32x16 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][r] = 0.0f;
    // (NKS is the launch's exact k-step count: no runtime guard between k-steps, so the
    // compiler can run the LDS fragment reads ahead of the MFMAs)
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      uint4 b = bv[st];
      if (sq_in) b = square_chunk<bf16_t>(b);
      const bf16x8 bb = __builtin_bit_cast(bf16x8, b);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint4 a = Wl[(j * 32 + r32) * RS + 2 * st + h];
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a), bb,
                                                         acc[j], 0, 0, 0);
      }
      PW_LOAD(bv[st], st, nrowp, nvalid);
    }
    const int m = tile * 32 + r32;
    if (m < Mtot) {
      // per 32-channel column: the 4 quads' residual loads are issued together, then
      // the math and stores (one memory latency per column, not per quad)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        EpiIn in[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = n0 + j * 32 + 8 * q + 4 * h;
          if (n < g.cout) in[q].load<bf16_t>(g, act, (long long)m, n);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int nl = j * 32 + 8 * q + 4 * h;
          if (n0 + nl < g.cout) {
            float v[4] = {acc[j][4 * q], acc[j][4 * q + 1], acc[j][4 * q + 2], acc[j][4 * q + 3]};
            const float bias[4] = {bl[nl], bl[nl + 1], bl[nl + 2], bl[nl + 3]};
            epilogue4_fin<bf16_t>(s, g, (long long)m, n0 + nl, v, bias, in[q]);
          }
        }
      }
    }
  }
#undef PW_LOAD
}

template <int NT, int NKS>
static void launch_smallk_nt(const ConvArgsDev& d, int ny, int nz, hipStream_t st) {
  static int per_cu = -1;                            // a property of the kernel
  auto kern = conv_smallk_kernel<NT, NKS>;
  if (per_cu < 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
  }
  const int ncu = device_cus();
  const int ntile = (d.s.M + 31) / 32;
  int gx = (ncu * per_cu + ny * nz - 1) / (ny * nz);
  const int need = (ntile + 3) / 4;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(kern, dim3(gx, ny, nz), dim3(256), 0, st, d);
}

template <int NKS>
static void launch_smallk_k(const ConvArgsDev& d, int max_cout, hipStream_t st) {
  const int nz = d.s.ngroups;
  if (max_cout <= 32) launch_smallk_nt<1, NKS>(d, 1, nz, st);
  else if (max_cout <= 64) launch_smallk_nt<2, NKS>(d, 1, nz, st);
  else launch_smallk_nt<3, NKS>(d, (max_cout + 95) / 96, nz, st);
}

static void launch_smallk(const ConvArgsDev& d, int nks16, int max_cout, hipStream_t st) {
  switch (nks16) {
    case 1: launch_smallk_k<1>(d, max_cout, st); break;
    case 2: launch_smallk_k<2>(d, max_cout, st); break;
    case 3: launch_smallk_k<3>(d, max_cout, st); break;
    case 4: launch_smallk_k<4>(d, max_cout, st); break;
    case 5: launch_smallk_k<5>(d, max_cout, st); break;
    case 6: launch_smallk_k<6>(d, max_cout, st); break;
    case 7: case 8: launch_smallk_k<8>(d, max_cout, st); break;
    case 9: case 10: case 11: case 12: launch_smallk_k<12>(d, max_cout, st); break;
    default: launch_smallk_k<16>(d, max_cout, st); break;
  }
}

// ---------------------------------------------------------------------------
// Full-width pointwise kernel (bf16; 1x1 stride-1 conv, one source, cin_pad <= 32 * NKS,
// cout <= 192): the HBM-bound 1x1 convs at full resolution -- GDN / IGDN norm pools, the
// attention block's output gate, ... .  conv_smallk_kernel holds 96 output rows per
// workgroup (two column blocks re-read the input: 1.5x the algorithmic bytes on the 128^2
// IGDN) and pays one memory round trip per 32-channel column of the epilogue.  Here:
//   * a 512-thread workgroup holds all 192 rows of the weight panel in LDS (LDS-DMA, 16-byte
//     chunk c of row r at slot c ^ (r & 7): conflict-free ds_read_b128 for the 8-lane
//     groups), so every input pixel is read from HBM once; two workgroups per CU (16 waves,
//     <= 128 VGPRs) keep enough loads in flight for HBM;
//   * each wave streams 16-pixel tiles: per 32-deep k-step ONE 16-byte load per lane
//     straight into VGPRs feeds 12 v_mfma_f32_16x16x32_bf16 (all 192 output channels), and
//     is reloaded with the NEXT tile's fragment right behind its MFMAs (a register ring);
//   * the tile's res1 operand (GDN / IGDN x, the gate's a, MASKSEL's x: 12 raw quads per
//     lane) is requested as one batch before the epilogue math: one memory latency per
//     tile, not per column (<= 128 VGPRs: four waves per SIMD hide it).
// Persistent grid; no barrier after the weight panel.
template <int NKS, bool DACT>
__global__ void __launch_bounds__(512, 4) conv_pw_kernel(const ConvArgsDev args) {
  constexpr int NT = 12, BN = 192, NCH = 4 * NKS;  // 16-byte chunks per weight row
  static_assert(NCH % 8 == 0, "swizzle groups of 8 chunks");
  constexpr int NPIECE = BN * NCH / 64;            // 1-KiB LDS-DMA pieces of the panel
  constexpr int NW = 8;
  extern __shared__ __attribute__((aligned(16))) uint4 Wl[];
  __shared__ float bl[BN];
  const ConvShared& s = args.s;
  const ConvGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nchunk = g.cin_pad >> 3;               // real 8-channel chunks of K
  {
    // weight panel: LDS slot d = 64 p + lane -> (row, slot), source chunk slot ^ (row & 7)
    const bf16_t* wbase = reinterpret_cast<const bf16_t*>(g.w);
    const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)Wl);
    for (int p = wave; p < NPIECE; p += NW) {
      const int d = p * 64 + lane;
      const int row = d / NCH, slot = d - (d / NCH) * NCH;
      const int ch = slot ^ (row & 7);
      const bool ok = row < g.rows && ch < nchunk;
      dma16_l(ok ? (const void*)(wbase + (size_t)row * g.k_pad + ch * 8) : (const void*)g_zero_page,
              lbase + p * 1024);
    }
  }
  for (int e = tid; e < BN; e += 64 * NW) bl[e] = (g.bias && e < g.cout) ? g.bias[e] : 0.0f;

  const int Mtot = s.M, act = s.act;
  const int ld = (int)g.sld0;
  const bool sq_in = s.square != 0;
  const int fr = lane & 15, fq = lane >> 4;
  const char* const src = reinterpret_cast<const char*>(g.sp0) + 16 * fq;
  const int ntile = (Mtot + 15) / 16;
  const int tstride = gridDim.x * NW;
  int tile = blockIdx.x * NW + wave;

#define PWW_LOAD(dst, st, rowp_, valid_)                                                      \
  do {                                                                                        \
    const bool ok_ = (valid_) & (4 * (st) + fq < nchunk);                                     \
    const uint4* p_ = ok_ ? reinterpret_cast<const uint4*>((rowp_) + 64 * (st)) : g_zero_page; \
    dst = *p_;                                                                                \
  } while (0)

  // the first tile's input fragments are requested beside the weight panel, so the two
  // memory latencies overlap (one wait for both)
  uint4 bv[NKS];
  {
    const int m = tile * 16 + fr;
    const bool valid = m < Mtot;
    const char* rowp = src + (size_t)(valid ? m : 0) * ld * 2;
#pragma unroll
    for (int st = 0; st < NKS; ++st) PWW_LOAD(bv[st], st, rowp, valid);
  }
  wait_vm<0>();
  __syncthreads();
  if (tile >= ntile) return;
  const bf16_t* const R1 = reinterpret_cast<const bf16_t*>(g.res1);
  const int cout = g.cout;
  for (; tile < ntile; tile += tstride) {
    const int m = tile * 16 + fr;
    const bool valid = m < Mtot;
    const long long mm = valid ? m : 0;
    const bool sel_on = act == RGBAC_ACT_MASKSEL ? (valid && g.sel[mm] != 0) : true;
    const int mn = (tile + tstride) * 16 + fr;
    const bool nvalid = mn < Mtot;
    const char* nrowp = src + (size_t)(nvalid ? mn : 0) * ld * 2;
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      uint4 b = bv[st];
      if (sq_in) b = square_chunk<bf16_t>(b);
      const int slot = (4 * st + fq) ^ (fr & 7);
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const uint4 a = Wl[(16 * j + fr) * NCH + slot];
        mma_step<bf16_t>(acc[j], a, b);
      }
      PWW_LOAD(bv[st], st, nrowp, nvalid);
    }
    if (valid && !g.res0 && !g.res2) {
      // res1 quads of the whole tile (raw bf16), all requested before any epilogue math
      uint2 e1[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = 16 * j + 4 * fq;
        e1[j] = (R1 && n < cout) ? *reinterpret_cast<const uint2*>(R1 + mm * g.ld1 + n)
                                 : make_uint2(0, 0);
      }
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int n = 16 * j + 4 * fq;
        if (n < cout) {
          EpiIn in;
#pragma unroll
          for (int r = 0; r < 4; ++r) { in.r0[r] = 0.f; in.r2[r] = 0.f; }
          in.r1[0] = bf2f(e1[j].x & 0xFFFF); in.r1[1] = bf2f(e1[j].x >> 16);
          in.r1[2] = bf2f(e1[j].y & 0xFFFF); in.r1[3] = bf2f(e1[j].y >> 16);
          in.on = sel_on;
          float v[4] = {acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
          const float bias[4] = {bl[n], bl[n + 1], bl[n + 2], bl[n + 3]};
          epilogue4_fin<bf16_t, DACT>(s, g, (long long)m, n, v, bias, in);
        }
      }
    } else if (valid) {
      // with res0 / res2 (the gate's x, the training step's in-place gradient accumulation):
      // every residual quad of a third of the tile requested before that third's math and
      // stores -- the output may alias a residual, so a load behind a store waits for it, and
      // loading per quad serialised one memory latency per quad (12 per tile)
      const bf16_t* const R0 = reinterpret_cast<const bf16_t*>(g.res0);
      const bf16_t* const R2 = reinterpret_cast<const bf16_t*>(g.res2);
#pragma unroll
      for (int h = 0; h < 3; ++h) {
        constexpr int NH = NT / 3;
        uint2 e0[NH], e1[NH], e2[NH];
#pragma unroll
        for (int jj = 0; jj < NH; ++jj) {
          const int n = 16 * (NH * h + jj) + 4 * fq;
          const bool on = n < cout;
          e0[jj] = (R0 && on) ? *reinterpret_cast<const uint2*>(R0 + mm * g.ld0 + n) : make_uint2(0, 0);
          e1[jj] = (R1 && on) ? *reinterpret_cast<const uint2*>(R1 + mm * g.ld1 + n) : make_uint2(0, 0);
          e2[jj] = (R2 && on) ? *reinterpret_cast<const uint2*>(R2 + mm * g.ld2 + n) : make_uint2(0, 0);
        }
#pragma unroll
        for (int jj = 0; jj < NH; ++jj) {
          const int j = NH * h + jj;
          const int n = 16 * j + 4 * fq;
          if (n < cout) {
            EpiIn in;
            in.r0[0] = bf2f(e0[jj].x & 0xFFFF); in.r0[1] = bf2f(e0[jj].x >> 16);
            in.r0[2] = bf2f(e0[jj].y & 0xFFFF); in.r0[3] = bf2f(e0[jj].y >> 16);
            in.r1[0] = bf2f(e1[jj].x & 0xFFFF); in.r1[1] = bf2f(e1[jj].x >> 16);
            in.r1[2] = bf2f(e1[jj].y & 0xFFFF); in.r1[3] = bf2f(e1[jj].y >> 16);
            in.r2[0] = bf2f(e2[jj].x & 0xFFFF); in.r2[1] = bf2f(e2[jj].x >> 16);
            in.r2[2] = bf2f(e2[jj].y & 0xFFFF); in.r2[3] = bf2f(e2[jj].y >> 16);
            in.on = sel_on;
            float v[4] = {acc[j][0], acc[j][1], acc[j][2], acc[j][3]};
            const float bias[4] = {bl[n], bl[n + 1], bl[n + 2], bl[n + 3]};
            epilogue4_fin<bf16_t, DACT>(s, g, (long long)m, n, v, bias, in);
          }
        }
      }
    }
  }
#undef PWW_LOAD
}

// Pointwise kernel, forward form (bf16; 1x1 stride-1 conv, one source, cin_pad <= 32 * NKS,
// cout <= 192, cout % 8 == 0; epilogues without zout / folded activation backward): the
// GDN / IGDN norm pools and the attention blocks' output gate (layers/GDN.py:64-94,
// layers/Masked_Attention.py:182-189).  At 64^2 x B8 the whole launch is 128 pixels per CU:
// conv_pw_kernel spent it in three dependent memory round trips per wave (weight panel +
// input, then the epilogue's res1 quads after the MFMAs, then the stores), ~21 us for ~25 MB
// (PMC: 62 % of wave cycles waiting).  Here:
//   * each wave's 16-pixel input tile lands in its own LDS slot by LDS-DMA (16-byte chunk c
//     of pixel row r at slot c ^ (r & 7)), in the same request burst as the weight panel and
//     the tile's residual quads (res0 / res2, and res1 unless it IS the input): one memory
//     latency before the MFMAs, none after them;
//   * GDN / IGDN (res1 == the input, square_input): the x quads of the epilogue are read from
//     the LDS tile the MFMAs consumed -- the input is read from memory once, not twice;
//   * the next tile's input DMA and residual loads are issued right after this tile's
//     fragments have been consumed, so they overlap its epilogue and stores.
// One 512-thread workgroup per CU (weights 72 KiB + 8 x 6 KiB tiles), persistent over tiles.
// conv_pw2_kernel's epilogue for one pixel row (channels 16 j + 4 fq .. + 3), ACT fixed at
// compile time (-1: no activation), epilogue4_fin's order: v = acc + bias; the folded
// activation backward (DGELU / DLRELU: v * act'(res0)) or v = SQBWD ? res0 + 2 res1 v :
// v + res0; the pre-activation to zout (training forward); act; + res2; bf16 store.
template <int NT, int ACT>
__device__ __forceinline__ void pw2_epi(bf16_t* orow, bf16_t* zrow, const f32x4 (&acc)[NT],
                                        const float* bl, const uint2 (&c0)[NT],
                                        const uint2 (&c1)[NT], const uint2 (&c2)[NT], int fq,
                                        int cout, bool sel_on, float act_param) {
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = 16 * j + 4 * fq;
    if (n >= cout) continue;
    const float r0[4] = {bf2f(c0[j].x & 0xFFFF), bf2f(c0[j].x >> 16), bf2f(c0[j].y & 0xFFFF),
                         bf2f(c0[j].y >> 16)};
    const float r1[4] = {bf2f(c1[j].x & 0xFFFF), bf2f(c1[j].x >> 16), bf2f(c1[j].y & 0xFFFF),
                         bf2f(c1[j].y >> 16)};
    const float r2[4] = {bf2f(c2[j].x & 0xFFFF), bf2f(c2[j].x >> 16), bf2f(c2[j].y & 0xFFFF),
                         bf2f(c2[j].y >> 16)};
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = acc[j][r] + bl[n + r];
      if constexpr (ACT == RGBAC_ACT_DGELU || ACT == RGBAC_ACT_DLRELU)
        x = dact_apply<bf16_t>(ACT, act_param, x, r0[r]);
      else if constexpr (ACT == RGBAC_ACT_SQBWD)
        x = r0[r] + 2.0f * r1[r] * x;
      else
        x = x + r0[r];
      v[r] = x;
    }
    if (zrow) Elem<bf16_t>::st4(zrow + n, v);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x = v[r];
      if constexpr (ACT == RGBAC_ACT_GDN) x = gdn_t<bf16_t>(r1[r], x);
      else if constexpr (ACT == RGBAC_ACT_IGDN) x = igdn_t<bf16_t>(r1[r], x);
      else if constexpr (ACT == RGBAC_ACT_GATE) x = r1[r] * sigmoid_f(x);
      else if constexpr (ACT == RGBAC_ACT_GELU) x = gelu_fast(x);
      else if constexpr (ACT == RGBAC_ACT_MASKSEL) x = sel_on ? r1[r] + x : r1[r];
      else if constexpr (ACT == RGBAC_ACT_RELU) x = x > 0.f ? x : 0.f;
      else if constexpr (ACT == RGBAC_ACT_LRELU) x = x > 0.f ? x : x * act_param;
      v[r] = x + r2[r];
    }
    Elem<bf16_t>::st4(orow + n, v);
  }
}

template <int NKS>
__global__ void __launch_bounds__(512, 2) conv_pw2_kernel(const ConvArgsDev args) {
  constexpr int NT = 12, BN = 192, NCH = 4 * NKS, NW = 8, TS = 24;   // TS: tile row chunks
  static_assert(NCH % 8 == 0 && NCH <= TS, "swizzle groups of 8 chunks");
  constexpr int NPIECE = BN * NCH / 64;            // 1-KiB LDS-DMA pieces of the panel
  constexpr int XP = 16 * TS / 64;                 // pieces of one 16-pixel tile (6)
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  __shared__ float bl[BN];
  const ConvShared& s = args.s;
  const ConvGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int nchunk = g.cin_pad >> 3;               // real 8-channel chunks of K
  const int Mtot = s.M, act = s.act, cout = g.cout;
  const int ld = (int)g.sld0;
  const bool sq_in = s.square != 0;
  const bool xl = g.res1 == g.sp0 && g.ld1 == g.sld0;   // epilogue x from the LDS tile
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)lds);
  const uint32_t xbase = lbase + (uint32_t)(BN * NCH + wave * 16 * TS) * 16u;
  const uint4* const Xl = lds + BN * NCH + wave * 16 * TS;
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
  for (int e = tid; e < BN; e += 64 * NW) bl[e] = (g.bias && e < cout) ? g.bias[e] : 0.0f;

  const char* const src = reinterpret_cast<const char*>(g.sp0);
  const bf16_t* const R0 = reinterpret_cast<const bf16_t*>(g.res0);
  const bf16_t* const R1 = xl ? nullptr : reinterpret_cast<const bf16_t*>(g.res1);
  const bf16_t* const R2 = reinterpret_cast<const bf16_t*>(g.res2);
  const int ntile = (Mtot + 15) / 16;
  const int tstride = gridDim.x * NW;
  int tile = blockIdx.x * NW + wave;

  // input tile -> this wave's LDS slot (rows past M and padding chunks read the zero page)
#define PW2_DMA(t_)                                                                           \
  do {                                                                                        \
    _Pragma("unroll")                                                                         \
    for (int p_ = 0; p_ < XP; ++p_) {                                                         \
      const int d_ = p_ * 64 + lane;                                                          \
      const int row_ = d_ / TS, slot_ = d_ - (d_ / TS) * TS;                                  \
      const int ch_ = slot_ ^ (row_ & 7);                                                     \
      const int m_ = (t_) * 16 + row_;                                                        \
      const bool ok_ = m_ < Mtot && ch_ < nchunk;                                             \
      dma16_l(ok_ ? (const void*)(src + ((size_t)m_ * ld + ch_ * 8) * 2)                      \
                  : (const void*)g_zero_page, xbase + p_ * 1024);                             \
    }                                                                                         \
  } while (0)
  // the tile's residual quads (channels 16 j + 4 fq .. + 3 of pixel fr), raw bf16
#define PW2_RES(t_, e0_, e1_, e2_)                                                            \
  do {                                                                                        \
    const int m_ = (t_) * 16 + fr;                                                            \
    const bool v_ = m_ < Mtot;                                                                \
    const long long mm_ = v_ ? m_ : 0;                                                        \
    _Pragma("unroll")                                                                         \
    for (int j_ = 0; j_ < NT; ++j_) {                                                         \
      const int n_ = 16 * j_ + 4 * fq;                                                        \
      const bool on_ = v_ && n_ < cout;                                                       \
      e0_[j_] = (R0 && on_) ? *reinterpret_cast<const uint2*>(R0 + mm_ * g.ld0 + n_) : make_uint2(0, 0); \
      e1_[j_] = (R1 && on_) ? *reinterpret_cast<const uint2*>(R1 + mm_ * g.ld1 + n_) : make_uint2(0, 0); \
      e2_[j_] = (R2 && on_) ? *reinterpret_cast<const uint2*>(R2 + mm_ * g.ld2 + n_) : make_uint2(0, 0); \
    }                                                                                         \
  } while (0)

  uint2 e0[NT], e1[NT], e2[NT];
  if (tile < ntile) {
    PW2_DMA(tile);
    PW2_RES(tile, e0, e1, e2);
  }
  wait_vm<0>();
  __syncthreads();
  bf16_t* const out = reinterpret_cast<bf16_t*>(g.out);
  for (; tile < ntile; tile += tstride) {
    f32x4 acc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < NKS; ++st) {
      uint4 b = Xl[fr * TS + ((4 * st + fq) ^ (fr & 7))];
      if (sq_in) b = square_chunk<bf16_t>(b);
      const int slot = (4 * st + fq) ^ (fr & 7);
#pragma unroll
      for (int j = 0; j < NT; ++j) mma_step<bf16_t>(acc[j], lds[(16 * j + fr) * NCH + slot], b);
    }
    if (xl) {                                      // GDN / IGDN: x quads from the LDS tile
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int c = 2 * j + (fq >> 1);
        e1[j] = *reinterpret_cast<const uint2*>(
            reinterpret_cast<const char*>(Xl + fr * TS + (c ^ (fr & 7))) + 8 * (fq & 1));
      }
    }
    // this tile's operands are in registers: the next tile's requests go out now
    const int m = tile * 16 + fr;
    const bool valid = m < Mtot;
    const bool sel_on = act == RGBAC_ACT_MASKSEL ? (valid && g.sel[m] != 0) : true;
    uint2 c0[NT], c1[NT], c2[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) { c0[j] = e0[j]; c1[j] = e1[j]; c2[j] = e2[j]; }
    const int nt = tile + tstride;
    if (nt < ntile) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // tile reads done before the DMA
      PW2_DMA(nt);
      PW2_RES(nt, e0, e1, e2);
    }
    if (valid) {
      bf16_t* const orow = out + (long long)m * g.out_ldc + g.out_coff;
      bf16_t* const zrow = g.zout ? reinterpret_cast<bf16_t*>(g.zout) + (long long)m * g.zld +
                                        g.out_coff : nullptr;
      // one compile-time epilogue per activation (a per-element switch compiled to scalar
      // compare-and-branch chains: ~3,000 SALU per wave)
#define PW2_EPI(A) pw2_epi<NT, A>(orow, zrow, acc, bl, c0, c1, c2, fq, cout, sel_on, s.act_param)
      switch (act) {
        case RGBAC_ACT_GDN: PW2_EPI(RGBAC_ACT_GDN); break;
        case RGBAC_ACT_IGDN: PW2_EPI(RGBAC_ACT_IGDN); break;
        case RGBAC_ACT_GATE: PW2_EPI(RGBAC_ACT_GATE); break;
        case RGBAC_ACT_GELU: PW2_EPI(RGBAC_ACT_GELU); break;
        case RGBAC_ACT_MASKSEL: PW2_EPI(RGBAC_ACT_MASKSEL); break;
        case RGBAC_ACT_RELU: PW2_EPI(RGBAC_ACT_RELU); break;
        case RGBAC_ACT_LRELU: PW2_EPI(RGBAC_ACT_LRELU); break;
        case RGBAC_ACT_SQBWD: PW2_EPI(RGBAC_ACT_SQBWD); break;
        case RGBAC_ACT_DGELU: PW2_EPI(RGBAC_ACT_DGELU); break;
        case RGBAC_ACT_DLRELU: PW2_EPI(RGBAC_ACT_DLRELU); break;
        default: PW2_EPI(-1); break;
      }
#undef PW2_EPI
    }
    if (nt < ntile) wait_vm<0>();
  }
#undef PW2_DMA
#undef PW2_RES
}

// DACT: the instance with the folded activation backward (training input gradients); the
// forward's instance leaves that epilogue out (the kernel sits at its 128-VGPR limit)
template <int NKS, bool DACT>
static void launch_pw_k(const ConvArgsDev& d, hipStream_t st) {
  auto kern = conv_pw_kernel<NKS, DACT>;
  constexpr size_t lds = (size_t)192 * 4 * NKS * 16;
  static unsigned long long attr = 0;                 // per device
  lds_optin((const void*)kern, (int)lds, &attr);
  const int ncu = device_cus();
  const int nz = d.s.ngroups;
  const int ntile = (d.s.M + 15) / 16;
  int gx = (2 * ncu + nz - 1) / nz;
  const int need = (ntile + 7) / 8;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(kern, dim3(gx, 1, nz), dim3(512), lds, st, d);
}

template <int NKS>
static void launch_pw2_k(const ConvArgsDev& d, hipStream_t st) {
  auto kern = conv_pw2_kernel<NKS>;
  constexpr size_t lds = ((size_t)192 * 4 * NKS + 8 * 16 * 24) * 16;
  static unsigned long long attr = 0;                 // per device
  lds_optin((const void*)kern, (int)lds, &attr);
  const int ncu = device_cus();
  const int nz = d.s.ngroups;
  const int ntile = (d.s.M + 15) / 16;
  int gx = (ncu + nz - 1) / nz;
  const int need = (ntile + 7) / 8;
  if (gx > need) gx = need;
  if (gx < 1) gx = 1;
  hipLaunchKernelGGL(kern, dim3(gx, 1, nz), dim3(512), lds, st, d);
}

// conv_pw2_kernel's preconditions (the rest -- one source, 1x1, cin/cout <= 192 -- are the
// pointwise tile's own); RGBAC_PW2=0 keeps conv_pw_kernel (A/B switch)
static bool pw2_ok(const ConvArgsDev& d) {
  static const bool on = [] {
    const char* e = getenv("RGBAC_PW2");
    return !(e && e[0] == '0');
  }();
  if (!on || d.s.act == RGBAC_ACT_TANH_HALF || d.s.act == RGBAC_ACT_GAUSS ||
      d.s.mode != RGBAC_CONV)
    return false;
  // (multi-tile launches too: with the compile-time epilogue the 128^2 IGDN takes 38.0 us
  // here vs 44.5 us on conv_pw_kernel, same box; RGBAC_PW2_ALL=0 keeps those on the old one)
  static const bool all = [] {
    const char* e = getenv("RGBAC_PW2_ALL");
    return !(e && e[0] == '0');
  }();
  if (!all && (long long)(d.s.M + 15) / 16 * d.s.ngroups > 8LL * 256) return false;
  for (int i = 0; i < d.s.ngroups; ++i) {
    const ConvGroup& g = d.g[i];
    if ((g.zout && g.zld % 4) || g.cout % 8 || g.out_coff % 8 || g.out_ldc % 8 || g.cout > 192 ||
        (g.res0 && g.ld0 % 4) || (g.res1 && g.ld1 % 4) || (g.res2 && g.ld2 % 4))
      return false;
  }
  return true;
}

static void launch_pw(const ConvArgsDev& d, int cin_max, hipStream_t st) {
  if (pw3_ok(d, cin_max)) {                        // GDN / IGDN forward: pw3.hip
    launch_pw3(d, st);
    return;
  }
  if (pw2_ok(d)) {
    if (cin_max <= 64) launch_pw2_k<2>(d, st);
    else if (cin_max <= 128) launch_pw2_k<4>(d, st);
    else launch_pw2_k<6>(d, st);
    return;
  }
  if (is_dact(d.s.act)) {
    if (cin_max <= 64) launch_pw_k<2, true>(d, st);
    else if (cin_max <= 128) launch_pw_k<4, true>(d, st);
    else launch_pw_k<6, true>(d, st);
    return;
  }
  if (cin_max <= 64) launch_pw_k<2, false>(d, st);
  else if (cin_max <= 128) launch_pw_k<4, false>(d, st);
  else launch_pw_k<6, false>(d, st);
}

// ---------------------------------------------------------------------------
// Narrow-output patch kernel (bf16; 3x3 stride-1 conv, up to three concatenated sources,
// cout <= 32): the slice chain's tail convs -- (mu | sigma) + GaussianConditional (256 -> 16)
// and the lrp output conv (128 -> 8, y_hat = pre + tanh / 2).  conv_wstream_kernel gathers
// every im2col fragment from L2 (9 x the input bytes per 32-pixel tile) and re-streams the
// whole weight panel per 32 pixels; a per-workgroup timestamp probe showed its loads, not its
// MFMAs, set the time (10.6 of 13.5 us per workgroup at 8192 pixels).  Here a workgroup owns a
// 4 x 16-pixel tile: its (4+2) x 18-pixel input patch is staged in LDS ONCE by LDS-DMA (as
// conv_fpatch_kernel), its 8 waves split K (each streams only its own k-steps of the
// fragment-major weights into a register ring: every weight byte is read once per tile), the
// wave partials are summed through LDS in a fixed order, and waves 0..3 run the epilogue of
// one pixel row each, with the biases and the GAUSS input y requested before the K loop.
// GAUSS: (mu | sigma) of 8 channels sit in lanes fq < 2 / fq >= 2 of one 16-row N tile (the
// sigma quad arrives by a lane ^ 32 shuffle); of 16 channels in N tiles 0 / 1 of one lane.
template <int TN>
__global__ void __launch_bounds__(512) conv_npatch_kernel(const ConvArgsDev args) {
  using T = bf16_t;
  constexpr int TH = 4, TM = 4, TW = 16, PW = TW + 2, PR = (TH + 2) * PW, NW = 8, R = 4;
  extern __shared__ __attribute__((aligned(16))) uint4 patch[];
  __shared__ double wsum[TM];
  WG_T(0);
  const ConvShared& s = args.s;
  const int tsp = blockIdx.x, gi = blockIdx.z;   // spatial tile (the GAUSS partial's slot), group
  const ConvGroup& g = args.g[gi];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int txn = s.Wm / TW, tyn = s.Hm / TH;
  int t = tsp;
  const int txi = t % txn; t /= txn;
  const int tyi = t % tyn;
  const int b = t / tyn;
  const int y0 = tyi * TH, x0 = txi * TW;
  const int in_h = s.in_h, in_w = s.in_w, cin_pad = g.cin_pad;
  const int cin32 = (cin_pad + 31) & ~31;
  const int nch = cin32 >> 3, RSc = nch + 2, cpt = cin32 >> 5;
  const int nks = 9 * cpt;
  const int k0 = nks * wave / NW, k1 = nks * (wave + 1) / NW;
  const bool gauss = s.act == RGBAC_ACT_GAUSS;
  const int cout = g.cout, nho = cout >> 1;       // GAUSS: mu / sigma channels

  // ---- operands of this wave's epilogue row (waves 0..TM-1), requested first
  const int ei = wave < TM ? wave : 0;
  const int m_e = (b * s.Hm + y0 + ei) * s.Wm + x0 + fr;
  float pb[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int n = 16 * j + 4 * fq + r;
      pb[j][r] = (g.bias && n < cout) ? g.bias[n] : 0.0f;
    }
  float yv[4] = {0.f, 0.f, 0.f, 0.f};
  const bool ylane = gauss && wave < TM && 4 * fq < nho;  // lanes holding mu channels 4fq..+3
  if (ylane) {
    const T* yr = reinterpret_cast<const T*>(g.res1) + (long long)m_e * g.ld1 + 4 * fq;
#pragma unroll
    for (int r = 0; r < 4; ++r) yv[r] = Elem<T>::ld(yr + r);
  }

  const uint4* const wf = reinterpret_cast<const uint4*>(g.w);
  uint4 ring[R][TN];
  int lks = k0;

  // ---- stage the input patch (as conv_fpatch_kernel): flat uint4 f -> (row, chunk)
  {
    const int send0 = g.send0, send1 = g.send1, send2 = g.send2;
    const char* const sp0 = reinterpret_cast<const char*>(g.sp0);
    const char* const sp1 = reinterpret_cast<const char*>(g.sp1);
    const char* const sp2 = reinterpret_cast<const char*>(g.sp2);
    const int sld0 = (int)g.sld0, sld1 = (int)g.sld1, sld2 = (int)g.sld2;
    const int total = PR * RSc;
    const int npiece = (total + 63) >> 6;
    const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)patch);
    for (int pc = wave; pc < npiece; pc += NW) {
      const int f = (pc << 6) + lane;
      const int row = f / RSc, c = f - (f / RSc) * RSc;
      const int py = row / PW, px = row - (row / PW) * PW;
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const int ch = c << 3;
      const bool in0 = ch < send0, in1 = ch < send1;
      const char* src = in0 ? sp0 : (in1 ? sp1 : sp2);
      const int sld = in0 ? sld0 : (in1 ? sld1 : sld2);
      const int cs = ch - (in0 ? 0 : (in1 ? send0 : send1));
      const bool ok = row < PR && c < nch && ch < send2 && (unsigned)iy < (unsigned)in_h &&
                      (unsigned)ix < (unsigned)in_w;
      const unsigned off = ok ? ((unsigned)((b * in_h + iy) * in_w + ix) * (unsigned)sld +
                                 (unsigned)cs) * 2u : 0u;
      dma16_l(ok ? (const void*)(src + off) : (const void*)g_zero_page, lbase + (pc << 10));
    }
    // weight ring prologue (this wave's k-steps [k0, k1) of the fragment-major copy) behind
    // the patch pieces, left in flight: the counted wait retires only the patch (in-order
    // returns), not the ring
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (lks < k1) {
#pragma unroll
        for (int j = 0; j < TN; ++j) ring[u][j] = wf[((size_t)j * nks + lks) * 64 + lane];
      }
      ++lks;
    }
    const int nring = (k1 - k0 < R ? k1 - k0 : R) * TN;    // loads just issued (wave-uniform)
    switch (nring) {
      case 8: wait_vm<8>(); break;
      case 6: wait_vm<6>(); break;
      case 4: wait_vm<4>(); break;
      case 3: wait_vm<3>(); break;
      case 2: wait_vm<2>(); break;
      case 1: wait_vm<1>(); break;
      default: wait_vm<0>(); break;
    }
    __syncthreads();
  }
  WG_T(1);

  // ---- this wave's share of K: k-step ks = tap * cpt + cc
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
  WG_T(2);

  // ---- wave partials -> LDS (over the dead patch) -> fixed-order sum per epilogue row
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
      for (int w = 0; w < NW; ++w) {
        const f32x4 p = red[((w * TN + j) * TM + ei) * 64 + lane];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] += p[r];
      }
    }
    if (gauss) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] += pb[j][r];
      float sg[4];
#pragma unroll
      for (int r = 0; r < 4; ++r)
        sg[r] = TN == 1 ? xor32_f(v[0][r]) : v[TN - 1][r];          // nho 8: lane ^ 32
      if (ylane) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          bits += (double)gauss_elem_y<T>(g, m_e, 4 * fq + r, nho, v[0][r], sg[r], yv[r]);
      }
    } else if (s.mode == RGBAC_SUBPEL2) {
      // subpel conv (the decoder's last ConvTranspose as conv3x3 + PixelShuffle): bias,
      // optional GELU and the shuffled store of epilogue4 (no residual operands, host-checked)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = 16 * j + 4 * fq;
        if (n < cout) epilogue4<T, false>(s, g, 0, m_e, n, v[j]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = 16 * j + 4 * fq;
        if (n < cout) {
          EpiIn in;
          in.template load<T>(g, s.act, (long long)m_e, n);
          epilogue4_fin<T, false>(s, g, (long long)m_e, n, v[j], pb[j], in);
        }
      }
    }
  }
  if (gauss) {
    for (int o = 32; o > 0; o >>= 1) bits += __shfl_xor(bits, o);
    if (wave < TM && lane == 0) wsum[wave] = bits;
    __syncthreads();
    if (tid == 0) g.partial[tsp] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
  }
  WG_T(3);
}

static void launch_npatch(const ConvArgsDev& d, int max_cout, hipStream_t st) {
  int cmax = 0;
  for (int i = 0; i < d.s.ngroups; ++i) cmax = d.g[i].cin_pad > cmax ? d.g[i].cin_pad : cmax;
  const size_t patch = (size_t)6 * 18 * (((cmax + 31) & ~31) / 8 + 2) * 16;
  const int tn = max_cout > 16 ? 2 : 1;
  const size_t red = (size_t)8 * tn * 4 * 64 * 16;
  const size_t lds = ((patch > red ? patch : red) + 1023) & ~(size_t)1023;
  const dim3 grid((unsigned)((long long)d.s.batch * (d.s.Hm / 4) * (d.s.Wm / 16)), 1, d.s.ngroups);
  // (below 160 KiB: the kernel also holds a few static LDS words); per device
  static unsigned long long attr1 = 0, attr2 = 0;
  lds_optin((const void*)conv_npatch_kernel<1>, 128 * 1024, &attr1);
  lds_optin((const void*)conv_npatch_kernel<2>, 128 * 1024, &attr2);
  if (tn == 2) hipLaunchKernelGGL(conv_npatch_kernel<2>, grid, dim3(512), lds, st, d);
  else hipLaunchKernelGGL(conv_npatch_kernel<1>, grid, dim3(512), lds, st, d);
}

// ---------------------------------------------------------------------------
// Narrow-output K-split kernel (bf16, plain conv, stride 1, k = 1 or 3, up to three
// concatenated sources, cout <= 32, K = taps * cin_pad <= 16 * kWsMaxSteps): the slice
// chain's (mu | sigma) + GaussianConditional convs (256 -> 16, K = 2304) and lrp output
// convs (128 -> 8, tanh update).  In the LDS-ring kernel they are a 36-stage serial K loop
// over only 128 workgroups.  Here one workgroup owns a 32-pixel tile and its 4 waves split
// K four ways: per 16-deep k-step each lane loads one 16-byte weight fragment (row lane&31)
// and one 16-byte im2col fragment (pixel lane&31; tap / channel from a per-chunk LDS table)
// straight into an R-deep register ring -- no LDS staging of either operand -- for one
// v_mfma_f32_32x32x16_bf16.  The four partial tiles are summed through LDS and wave 0 runs
// the epilogue; the GAUSS epilogue works in the accumulator layout (mu channel c and sigma
// channel c + nch of a pixel sit in the same lane) and writes one fp64 bits partial per tile.
constexpr int kWsMaxSteps = 146;

template <int R, int NW>
__global__ void __launch_bounds__(64 * NW) conv_wstream_kernel(const ConvArgsDev args) {
  __shared__ int ktab[2 * kWsMaxSteps];
  __shared__ float bl[32];
  __shared__ __attribute__((aligned(16))) float part[NW - 1][16][64];
  WG_T(0);
  const ConvShared& s = args.s;
  const ConvGroup& g = args.g[blockIdx.z];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntaps = s.ksize * s.ksize;
  const int kused = ntaps * g.cin_pad;
  const int nks = (kused + 15) / 16;
  for (int kc = tid; kc < 2 * nks; kc += 64 * NW) {
    const int k = kc * 8;
    const int tap = k / g.cin_pad;
    const int ci = k - tap * g.cin_pad;
    const int ty = tap / s.ksize, tx = tap - ty * s.ksize;
    int src, cs;
    bool ok = k < kused && tap < ntaps;
    if (ci < g.send0) { src = 0; cs = ci; }
    else if (ci < g.send1) { src = 1; cs = ci - g.send0; }
    else { src = 2; cs = ci - g.send1; ok = ok && ci < g.send2; }
    ktab[kc] = cs | ((ty - s.pad + 4) << 12) | ((tx - s.pad + 4) << 15) | (src << 18) |
               ((int)ok << 20);
  }
  if (tid < 32) bl[tid] = (g.bias && tid < g.rows) ? g.bias[tid] : 0.0f;
  __syncthreads();

  const int in_h = s.in_h, in_w = s.in_w, Mtot = s.M;
  const char* const sp0 = reinterpret_cast<const char*>(g.sp0);
  const char* const sp1 = reinterpret_cast<const char*>(g.sp1);
  const char* const sp2 = reinterpret_cast<const char*>(g.sp2);
  const int sld0 = (int)g.sld0, sld1 = (int)g.sld1, sld2 = (int)g.sld2;
  const int r32 = lane & 31, h = lane >> 5;
  const int tile = blockIdx.x;
  const int m = tile * 32 + r32;
  const bool valid = m < Mtot;
  const int mm = valid ? m : 0;
  const int t_ = udiv(mm, s.Wm, s.rWm);
  const int px = mm - t_ * s.Wm;
  const int pb = udiv(t_, s.Hm, s.rHm);
  const int py = t_ - pb * s.Hm;
  // this wave's k-steps [k0, k1)
  const int k0 = (nks * wave) / NW, k1 = (nks * (wave + 1)) / NW;
  const bf16_t* wrow = reinterpret_cast<const bf16_t*>(g.w) + (size_t)r32 * g.k_pad + 8 * h;

#define WS_LOAD(da, db, ks_)                                                                  \
  do {                                                                                        \
    const int e_ = ktab[2 * (ks_) + h];                                                       \
    const int iy_ = py + ((e_ >> 12) & 7) - 4, ix_ = px + ((e_ >> 15) & 7) - 4;              \
    const int sr_ = (e_ >> 18) & 3;                                                           \
    const bool ok_ = valid & ((e_ >> 20) != 0) & ((unsigned)iy_ < (unsigned)in_h) &           \
                     ((unsigned)ix_ < (unsigned)in_w);                                        \
    const char* base_ = sr_ == 0 ? sp0 : (sr_ == 1 ? sp1 : sp2);                              \
    const int ld_ = sr_ == 0 ? sld0 : (sr_ == 1 ? sld1 : sld2);                               \
    const unsigned off_ =                                                                     \
        ((unsigned)(((pb * in_h + iy_) * in_w + ix_) * ld_ + (e_ & 0xFFF))) * 2u;             \
    const uint4* p_ = ok_ ? reinterpret_cast<const uint4*>(base_ + off_) : g_zero_page;       \
    db = *p_;                                                                                 \
    da = *reinterpret_cast<const uint4*>(wrow + 16 * (ks_));                                  \
  } while (0)

  uint4 av[R], bv[R];
#pragma unroll
  for (int u = 0; u < R; ++u) {
    av[u] = make_uint4(0, 0, 0, 0);
    bv[u] = make_uint4(0, 0, 0, 0);
    if (k0 + u < k1) WS_LOAD(av[u], bv[u], k0 + u);
  }
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
  for (int c = k0; c < k1; c += R) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int ks = c + u;
      if (ks < k1) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, av[u]),
                                                      __builtin_bit_cast(bf16x8, bv[u]), acc,
                                                      0, 0, 0);
        if (ks + R < k1) WS_LOAD(av[u], bv[u], ks + R);
      }
    }
  }
#undef WS_LOAD
  WG_T(1);
  // ---- sum the waves' partial tiles (waves 1..NW-1 -> LDS -> wave 0)
  if (wave > 0) {
#pragma unroll
    for (int r = 0; r < 16; ++r) part[wave - 1][r][lane] = acc[r];
  }
  __syncthreads();
  if (wave > 0) return;
  WG_T(2);
#pragma unroll
  for (int w = 0; w < NW - 1; ++w)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += part[w][r][lane];

  // accumulator layout: lane (pixel r32, half h) holds channel 8q + 4h + r in acc[4q + r]
  if (s.act == RGBAC_ACT_GAUSS) {
    const int nch = g.cout >> 1;                   // 8 or 16
    double bits = 0.0;
    if (valid) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 8 * q + 4 * h + r;
          if (c < nch) {
            // sigma channel c + nch sits in accumulator quad q + nch/8 (static indices)
            const float mu = acc[4 * q + r] + bl[c];
            const float sg = (nch == 8 ? acc[4 * (q + 1) + r] : acc[4 * ((q + 2) & 3) + r]) +
                             bl[c + nch];
            bits += (double)gauss_elem<bf16_t>(g, m, c, nch, mu, sg);
          }
        }
    }
    for (int o = 32; o > 0; o >>= 1) bits += __shfl_xor(bits, o);
    if (lane == 0) g.partial[tile] = bits;
  } else if (valid) {
    EpiIn in[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 8 * q + 4 * h;
      if (n < g.cout) in[q].template load<bf16_t>(g, s.act, (long long)m, n);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int n = 8 * q + 4 * h;
      if (n < g.cout) {
        float v[4] = {acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
        const float bias[4] = {bl[n], bl[n + 1], bl[n + 2], bl[n + 3]};
        epilogue4_fin<bf16_t>(s, g, (long long)m, n, v, bias, in[q]);
      }
    }
  }
  WG_T(3);
}

// 8 waves split K when every wave still gets >= 8 k-steps (the latency-bound chain convs:
// K = 2304 / 1152 -> 18 / 9 steps per wave instead of 36 / 18).
static void launch_wstream(const ConvArgsDev& d, hipStream_t st) {
  const int ntile = (d.s.M + 31) / 32;
  int nks = 0;
  for (int i = 0; i < d.s.ngroups; ++i) {
    const int n = (d.s.ksize * d.s.ksize * d.g[i].cin_pad + 15) / 16;
    if (n > nks) nks = n;
  }
  static const int nw_env = [] {
    const char* e = getenv("RGBAC_WSTREAM_WAVES");
    return e ? atoi(e) : 0;
  }();
  const int nw = nw_env == 4 || nw_env == 8 ? nw_env : (nks >= 64 ? 8 : 4);
  if (nw == 8)
    hipLaunchKernelGGL((conv_wstream_kernel<8, 8>), dim3(ntile, 1, d.s.ngroups), dim3(512), 0, st, d);
  else
    hipLaunchKernelGGL((conv_wstream_kernel<8, 4>), dim3(ntile, 1, d.s.ngroups), dim3(256), 0, st, d);
}

// Persistent grid: as many blocks per z-slice as fit on the chip at once (occupancy query,
// cached per kernel), evened out so every block gets the same number of tiles (+-1).
template <typename T, int BM, int BN, int WGM, int WGN, int NBUF>
static void launch_pers(const ConvArgsDev& d, int ntile, int nz, hipStream_t st) {
  static int per_cu = -1;                            // a property of the kernel
  auto kern = conv_pers_kernel<T, BM, BN, WGM, WGN, NBUF>;
  if (per_cu < 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, 256, 0) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
  }
  const int ncu = device_cus();
  int cap = (ncu * per_cu + nz - 1) / nz;
  if (cap < 1) cap = 1;
  const int rounds = (ntile + cap - 1) / cap;
  const int G = (ntile + rounds - 1) / rounds;
  hipLaunchKernelGGL(kern, dim3(G, 1, nz), dim3(256), 0, st, d);
}



// Lean phase epilogue of the patch kernels (CONV / CONVT_S2 modes): the lane's TM rows x TN
// quads of 4 channels; bias loaded once per phase, the activation a template parameter and
// the residual choice one wave-uniform branch per phase (the generic epilogue_tile_row
// re-tests act / residual pointers / bounds per element, which measured ~1.7k VALU +
// 1.1k SALU per wave per phase on the 192-channel convT -- more issue time than the
// phase's MFMAs).  Needs cout % 4 == 0, no zout, no res1 (callers check).
template <int TN, int TM, int ACT>
__device__ __forceinline__ void patch_epi(const ConvShared& s, const ConvGroup& g, int ph, int b,
                                          int yrow0, int x, const int (&nn)[TN],
                                          const f32x4 (&acc)[TN][TM],
                                          const float (*pbias)[4] = nullptr) {
  using T = bf16_t;
  float bias[TN][4];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r)
      bias[j][r] = pbias ? pbias[j][r] : (g.bias ? g.bias[nn[j] + r] : 0.0f);
  const bool convt = s.mode == RGBAC_CONVT_S2;
  const int py = convt ? ph >> 1 : 0, px = convt ? ph & 1 : 0, sc = convt ? 2 : 1;
  const int cout = g.cout;
  T* const out = reinterpret_cast<T*>(g.out) + g.out_coff;
  const T* const r0 = reinterpret_cast<const T*>(g.res0);
  const T* const r2 = reinterpret_cast<const T*>(g.res2);
  const long long ldo = g.out_ldc, ld0 = g.ld0, ld2 = g.ld2;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const long long opix = (long long)(b * s.out_h + sc * (yrow0 + i) + py) * s.out_w +
                           sc * x + px;
    float v[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j][r] = acc[j][i][r] + bias[j][r];
    if (r0) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        if (nn[j] < cout) {
          float t[4];
          Elem<T>::ld4(r0 + opix * ld0 + nn[j], t);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            v[j][r] = ACT == RGBAC_ACT_DGELU ? dact_apply<T>(s.act, s.act_param, v[j][r], t[r])
                                             : v[j][r] + t[r];
        }
    }
    if constexpr (ACT == RGBAC_ACT_GELU) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] = gelu_t<T>(v[j][r]);
    } else if constexpr (ACT == RGBAC_ACT_RELU) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) v[j][r] = v[j][r] > 0.f ? v[j][r] : 0.f;
    }
    if (r2) {
#pragma unroll
      for (int j = 0; j < TN; ++j)
        if (nn[j] < cout) {
          float t[4];
          Elem<T>::ld4(r2 + opix * ld2 + nn[j], t);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[j][r] += t[r];
        }
    }
#pragma unroll
    for (int j = 0; j < TN; ++j)
      if (nn[j] < cout) Elem<T>::st4(out + opix * ldo + nn[j], v[j]);
  }
}

// Dispatch of a patch kernel's phase epilogue: the lean form where it applies, else the
// generic per-row epilogue (SUBPEL2 stores, zout, res1 activations, ragged cout).
// ``pbias``: the lane's biases (bias[nn[j] + r]) loaded up front by the caller, or nullptr.
// DACT = false: no folded activation backward (the forward instances; their register
// allocation is the one measured before the training epilogues existed)
template <int TN, int TM, bool DACT>
__device__ __forceinline__ void patch_epilogue(const ConvShared& s, const ConvGroup& g, int ph,
                                               int b, int yrow0, int x0, int fr,
                                               const int (&nn)[TN], const f32x4 (&acc)[TN][TM],
                                               const float (*pbias)[4] = nullptr) {
  const bool lean = s.mode != RGBAC_SUBPEL2 && !g.zout && !g.res1 && (g.cout & 3) == 0;
  if (lean && s.act == RGBAC_ACT_NONE) {
    patch_epi<TN, TM, RGBAC_ACT_NONE>(s, g, ph, b, yrow0, x0 + fr, nn, acc, pbias);
  } else if (lean && s.act == RGBAC_ACT_GELU) {
    patch_epi<TN, TM, RGBAC_ACT_GELU>(s, g, ph, b, yrow0, x0 + fr, nn, acc, pbias);
  } else if (lean && s.act == RGBAC_ACT_RELU) {
    patch_epi<TN, TM, RGBAC_ACT_RELU>(s, g, ph, b, yrow0, x0 + fr, nn, acc, pbias);
  } else if (DACT && lean && is_dact(s.act)) {     // both folded activation backwards
    patch_epi<TN, TM, RGBAC_ACT_DGELU>(s, g, ph, b, yrow0, x0 + fr, nn, acc, pbias);
  } else {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = (b * s.Hm + yrow0 + i) * s.Wm + x0 + fr;
      epilogue_tile_row<bf16_t, TN, TM, DACT>(s, g, ph, m, nn, acc, i);
    }
  }
}

// ---------------------------------------------------------------------------
// Patch-resident implicit GEMM (bf16), for the 3x3 stride-1 convs (slice stacks, hyper
// convs, subpel convs) and the 5x5/s2 ConvTranspose (all four output phases).
//
// The im2col-staging conv_kernel stages every input pixel once per tap (9x / 25x the input
// bytes), and -- measured with PMC counters on the 192-channel convT -- spends ~11 SALU +
// 15 VALU instructions per MFMA on its per-stage gather decode: it is instruction-issue
// bound at ~14 % of the matrix pipe.  Here a workgroup owns a TH x 16 tile of the M grid
// (the output grid, or for CONVT_S2 the input grid shared by the four phases) and BN
// output channels:
//   * per 64-channel chunk the (TH+2) x 18 input patch (halo 1) is staged ONCE by LDS-DMA
//     into a double buffer; every tap reads its B fragments from it at a shifted row;
//   * patch rows are 8 data chunks + 2 pad chunks of 16 bytes (160 B): the 16 consecutive
//     rows of a fragment read are bank-conflict-free for any tap shift, and a fragment
//     address is a per-lane constant + a wave-uniform tap offset (one v_add per row
//     segment per stage, the k-step in the instruction's immediate offset);
//   * the weights stream through a 3-deep ring of (tap, chunk) stages of BN x 64 (16-byte
//     chunk c of row r at slot c ^ (r & 7)), one counted s_waitcnt + barrier per stage;
//     the next chunk's patch pieces ride with the third stage of the current chunk (its
//     buffer was last read a chunk ago);
//   * 8 waves (2 per SIMD) as WGM x WGN; per stage a wave runs 2 k-steps of TN x TM
//     v_mfma_f32_16x16x32_bf16 from (TN + TM) ds_read_b128 per k-step;
//   * every per-stage index is carried incrementally (no integer division in the loop);
//   * CONVT_S2: phases run one after another (9, 6, 6, 4 taps); the epilogue of a phase
//     runs while the next phase's first stages are already in flight;
//   * the 5x5 stride-2 conv (Analysis x2 / x3, TransformRGB.py:55-58): polyphase -- with
//     u = 2y + ky - 2 = 2(y + dy) + qy, the conv is the sum over the four input phases
//     P_q[i][j] = in[2i + qy][2j + qx] of stride-1 convs with (3 - qy) x (3 - qx) taps
//     (dy, dx in -1..1, kernel tap (2 dy + qy + 2, 2 dx + qx + 2)), so the M grid is the
//     output grid and a group (phase, chunk) stages the phase image's (TH+2) x 18 patch --
//     every input pixel is fetched once per tile (plus the halo) instead of once per tap,
//     the im2col tiles' 3.3x fetch.  The weights are the plain CONV packing (k = tap *
//     cin_pad + ci over the 25 taps), walked phase by phase; the four phases accumulate
//     into one tile and the epilogue runs once.
template <int TH, int BN, int WGM, int WGN, int NBUF, bool DACT>
__global__ void __launch_bounds__(512) conv_patch_kernel(const ConvArgsDev args) {
  using T = bf16_t;
  constexpr int NW = 8;
  static_assert(WGM * WGN == NW, "8 waves");
  constexpr int TW = 16, PW = TW + 2, PH = TH + 2, PR = PH * PW;
  constexpr int RSC = 10;                         // uint4 per patch row: 8 data + 2 pad
  constexpr int PPIECE = (PR * RSC + 63) / 64;    // 1-KiB DMA pieces per patch chunk
  constexpr int PQ = (PPIECE + NW - 1) / NW;      // patch pieces per wave
  constexpr int TM = TH / WGM, TN = BN / WGN / 16;
  static_assert(TM >= 1 && TN >= 1 && TM * WGM == TH && TN * WGN * 16 == BN, "tile");
  constexpr int IA = BN / 8;                      // weight pieces per stage
  constexpr int NAW = (IA + NW - 1) / NW;         // per wave (a surplus slot re-issues)
  static_assert(NBUF == 3 || NBUF == 4, "ring depth (the patch rider sits at tap NBUF-1 of "
                                        "a group; groups have >= 4 taps)");
  constexpr int RT = NBUF - 1;                    // tap of a group that carries the rider
  constexpr int WSTAGE = BN * 8;                  // uint4 per weight stage
  constexpr int PSTAGE = PPIECE * 64;             // uint4 per patch buffer
  __shared__ __attribute__((aligned(16))) uint4 smem[NBUF * WSTAGE + 2 * PSTAGE];

  const ConvShared& s = args.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int txn = s.Wm / TW, tyn = s.Hm / TH;
  int nblk, txi, tyi, b, gi;
  {
    const int nwg = gridDim.x * gridDim.y;
    int t = blockIdx.x + gridDim.x * blockIdx.y;
    if (s.remap) {                               // XCD-contiguous runs, N tile fastest
      const int xcd = t & 7, q = nwg >> 3, r = nwg & 7;
      t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (t >> 3);
    }
    nblk = t % gridDim.y; t /= gridDim.y;
    txi = t % txn; t /= txn;
    tyi = t % tyn; t /= tyn;
    b = t % s.batch;
    gi = t / s.batch;
  }
  const ConvGroup& g = args.g[gi];
  const int n0 = nblk * BN;
  if (n0 >= g.cout) return;
  const int y0 = tyi * TH, x0 = txi * TW;
  const bool convt = s.mode == RGBAC_CONVT_S2;
  const bool s2 = s.mode == RGBAC_CONV && s.sy == 2;     // polyphase 5x5 stride-2 conv
  const int nph = (convt || s2) ? 4 : 1;
  // phase split (grid z = 4, ksplit 4): this workgroup runs phase blockIdx.z only -- a convT
  // phase writes its own output pixels; a strided-conv phase writes its fp32 partial slab,
  // summed in phase order by conv_splitk_epilogue
  const int pz = gridDim.z > 1 ? (int)blockIdx.z : -1;
  const int ph0 = pz >= 0 ? pz : 0;
  const int in_h = s.in_h, in_w = s.in_w, cin_pad = g.cin_pad;
  const int nck = (cin_pad + 63) >> 6;
  const int send0 = g.send0, send1 = g.send1, send2 = g.send2;
  const char* const sp0 = reinterpret_cast<const char*>(g.sp0);
  const char* const sp1 = reinterpret_cast<const char*>(g.sp1);
  const char* const sp2 = reinterpret_cast<const char*>(g.sp2);
  const int sld0 = (int)g.sld0, sld1 = (int)g.sld1, sld2 = (int)g.sld2;
  // groups (phase, chunk); group sizes 9 (conv) or 9, 6, 6, 4 (convT phases)
  const int ntap0 = (3 - (ph0 >> 1)) * (3 - (ph0 & 1));   // taps of phase ph0 (9 when nph 1)
  const int ngroups = pz >= 0 ? nck : nph * nck;
  const int ns = pz >= 0 ? nck * ntap0 : (nph == 4 ? nck * 25 : nck * 9);

  // ---- per-lane DMA geometry (constant through the K loop)
  const int lrow = lane >> 3;
  uint32_t aoff[NAW];
  int alds[NAW];
#pragma unroll
  for (int i = 0; i < NAW; ++i) {
    const int q = min(wave + NW * i, IA - 1);
    const int row = 8 * q + lrow;
    alds[i] = q * 64;
    aoff[i] = (uint32_t)(((n0 + row) * g.k_pad + ((lane & 7) ^ (row & 7)) * 8) * 2);
  }
  // patch piece of a lane: pixel (r / PW, r % PW) of the (TH+2) x 18 patch, channel chunk c;
  // pmask bit q: the pixel exists in phase q (s2; bit 0 only otherwise), ppix: its pixel
  // index in phase 0 (s2: the phase-q pixel is ppix + qy * in_w + qx)
  int ppix[PQ], plds[PQ], pch[PQ];
  unsigned pmask[PQ];
#pragma unroll
  for (int i = 0; i < PQ; ++i) {
    const int q = min(wave + NW * i, PPIECE - 1);
    const int f = q * 64 + lane;
    const int r = f / RSC, c = f - (f / RSC) * RSC;
    plds[i] = q * 64;
    pch[i] = c * 8;
    const int py = r / PW, px = r - (r / PW) * PW;
    const bool rc_ok = r < PR && c < 8;
    if (s2) {
      const int iy = 2 * (y0 - 1 + py), ix = 2 * (x0 - 1 + px);
      unsigned m = 0;
#pragma unroll
      for (int ph = 0; ph < 4; ++ph)
        if (rc_ok && (unsigned)(iy + (ph >> 1)) < (unsigned)in_h &&
            (unsigned)(ix + (ph & 1)) < (unsigned)in_w)
          m |= 1u << ph;
      pmask[i] = m;
      ppix[i] = m ? (b * in_h + iy) * in_w + ix : 0;
    } else {
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const bool ok = rc_ok && (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w;
      pmask[i] = ok ? 1u : 0u;
      ppix[i] = ok ? (b * in_h + iy) * in_w + ix : 0;
    }
  }
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)smem);
  const uint32_t lpatch = lbase + NBUF * WSTAGE * 16;
  const size_t phstride = (size_t)g.rows * g.k_pad * 2;     // bytes per convT phase
  const char* const wbase = reinterpret_cast<const char*>(g.w);

#define PATCH_ISSUE(grp_, ck_, ph_)                                                           \
  do {                                                                                        \
    const uint32_t lpb = lpatch + (uint32_t)(((grp_) & 1) * PSTAGE * 16);                     \
    const int pbit = s2 ? (ph_) : 0;                                                          \
    const int pdel = s2 ? ((ph_) >> 1) * in_w + ((ph_) & 1) : 0;                              \
_Pragma("unroll")                                                                             \
    for (int i = 0; i < PQ; ++i) {                                                            \
      const int ch = ((ck_) << 6) + pch[i];                                                   \
      const bool in0 = ch < send0, in1 = ch < send1;                                          \
      const char* src = in0 ? sp0 : (in1 ? sp1 : sp2);                                        \
      const int sld = in0 ? sld0 : (in1 ? sld1 : sld2);                                       \
      const int cs = ch - (in0 ? 0 : (in1 ? send0 : send1));                                  \
      const bool ok = ((pmask[i] >> pbit) & 1u) && (ch < send2);                              \
      const unsigned off = ((unsigned)(ppix[i] + pdel) * (unsigned)sld + (unsigned)cs) * 2u;  \
      const void* gp = ok ? (const void*)(src + off) : (const void*)g_zero_page;              \
      dma16_l(gp, lpb + plds[i] * 16);                                                        \
    }                                                                                         \
  } while (0)

  // issue-side state: stage weight address, tap / chunk / phase counters, group index
  int itap = 0, intap = ntap0, ick = 0, iph = ph0, igrp = 0, itx = 0, itw = 3 - (ph0 & 1);
  const int tapstep = cin_pad * 2;                // bytes from one tap's column to the next
  // current phase's packed weights / current stage's weight column
  const char* wph = convt ? wbase + ph0 * phstride : wbase;
  const char* wst = s2 ? wbase + ((ph0 >> 1) * 5 + (ph0 & 1)) * tapstep : wph;

  // s2: the group's taps (ty, tx) are kernel taps (2 ty + qy, 2 tx + qx) of the plain 5x5
  // packing: +2 taps along a row, +10 - 2 (tw - 1) taps to the next row's first
#define STAGE_ISSUE(st_)                                                                      \
  do {                                                                                        \
    const uint32_t lst = lbase + (uint32_t)(((st_) % NBUF) * WSTAGE * 16);                    \
_Pragma("unroll")                                                                             \
    for (int i = 0; i < NAW; ++i) dma16_s(wst, aoff[i], lst + alds[i] * 16);                  \
    if (itap == RT && igrp + 1 < ngroups) {      /* the next group's patch rides here */     \
      const bool last_ck = ick + 1 == nck;                                                    \
      PATCH_ISSUE(igrp + 1, last_ck ? 0 : ick + 1, last_ck ? iph + 1 : iph);                 \
    }                                                                                         \
    if (s2) {                                                                                 \
      if (++itx == itw) { itx = 0; wst += (10 - 2 * (itw - 1)) * tapstep; }                   \
      else wst += 2 * tapstep;                                                                \
    } else {                                                                                  \
      wst += tapstep;                                                                         \
    }                                                                                         \
    if (++itap == intap) {                                                                    \
      itap = 0; itx = 0; ++igrp;                                                              \
      if (++ick == nck) {                                                                     \
        ick = 0; ++iph;                                                                       \
        if (!s2) wph += phstride;                                                             \
        itw = 3 - (iph & 1);                                                                  \
        intap = (3 - (iph >> 1)) * itw;                                                       \
      }                                                                                       \
      wst = s2 ? wbase + (((iph >> 1) * 5 + (iph & 1)) * tapstep) + (ick << 7)                \
               : wph + (ick << 7);                                                            \
    }                                                                                         \
  } while (0)

  PATCH_ISSUE(0, 0, ph0);
#pragma unroll
  for (int st = 0; st < NBUF - 1; ++st)
    if (st < ns) STAGE_ISSUE(st);

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int wm = wave % WGM, wn = wave / WGM;
  const int fr = lane & 15, fq = lane >> 4;
  // per-lane LDS element offsets (uint4 units): A rows of k-step 0 / 1, B row-segment bases
  const int arow = (wn * TN * 16 + fr) * 8;
  const int a0 = arow + ((0 + fq) ^ (fr & 7)), a1 = arow + ((4 + fq) ^ (fr & 7));
  int bbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) bbase[i] = ((wm * TM + i) * PW + fr) * RSC + fq;
  // compute-side state: tap within the group, tap offset (uint4), group parity, phase
  int ctap = 0, cntap = ntap0, ctx = 0, ctw = 3 - (ph0 & 1), cck = 0, cph = ph0, cgrp = 0;
  int toff = convt ? (2 * PW + 2) * RSC : 0;      // (oy * PW + ox) * RSC of the group's tap 0

  for (int it = 0; it < ns; ++it) {
    // retire stage `it`; the ops issued after its weight pieces may stay in flight: the
    // stages it+1 .. it+NBUF-2 already issued, and a patch rider carried by one of stages
    // it .. it+NBUF-2 (tap RT of this group, if it is not the last group)
    {
      const bool rider = ctap >= RT - (NBUF - 2) && ctap <= RT && cgrp + 1 < ngroups;
      const int after = min(NBUF - 2, ns - 1 - it);
      if constexpr (NBUF == 4) {
        if (after >= 2) { if (rider) wait_vm<2 * NAW + PQ>(); else wait_vm<2 * NAW>(); }
        else if (after == 1) { if (rider) wait_vm<NAW + PQ>(); else wait_vm<NAW>(); }
        else { if (rider) wait_vm<PQ>(); else wait_vm<0>(); }
      } else {
        if (after >= 1) { if (rider) wait_vm<NAW + PQ>(); else wait_vm<NAW>(); }
        else { if (rider) wait_vm<PQ>(); else wait_vm<0>(); }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    if (it + NBUF - 1 < ns) STAGE_ISSUE(it + NBUF - 1);
    const uint4* As = smem + (it % NBUF) * WSTAGE;
    const uint4* Ps = smem + NBUF * WSTAGE + (cgrp & 1) * PSTAGE + toff;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      uint4 a[TN], bb[TM];
#pragma unroll
      for (int j = 0; j < TN; ++j) a[j] = As[(ks ? a1 : a0) + j * 128];
#pragma unroll
      for (int i = 0; i < TM; ++i) bb[i] = Ps[bbase[i] + 4 * ks];
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], a[j], bb[i]);
    }
    // advance the compute-side tap: x fastest (convT taps step -1 in the patch, conv +1)
    ++ctap;
    if (++ctx == ctw) {                           // (ty, tw-1) -> (ty+1, 0)
      ctx = 0;
      toff += convt ? (-PW + ctw - 1) * RSC : (PW - ctw + 1) * RSC;
    } else {
      toff += convt ? -RSC : RSC;
    }
    if (ctap == cntap) {                          // end of a (phase, chunk) group
      ctap = 0; ctx = 0; ++cgrp;
      toff = convt ? (2 * PW + 2) * RSC : 0;
      if (++cck == nck) {                         // end of a phase: epilogue (s2: the last)
        cck = 0;
        if (!s2 || cph == 3 || pz >= 0) {
          int nn[TN];
#pragma unroll
          for (int j = 0; j < TN; ++j) nn[j] = n0 + wn * TN * 16 + j * 16 + fq * 4;
          if (s2 && pz >= 0) {                      // the phase's fp32 partial slab
#pragma unroll
            for (int i = 0; i < TM; ++i) {
              const int m = (b * s.Hm + y0 + wm * TM + i) * s.Wm + x0 + fr;
#pragma unroll
              for (int j = 0; j < TN; ++j)
                if (nn[j] < g.cout)
                  *reinterpret_cast<float4*>(g.ws + ((size_t)pz * s.M + m) * g.cout16 + nn[j]) =
                      make_float4(acc[j][i][0], acc[j][i][1], acc[j][i][2], acc[j][i][3]);
            }
          } else {
            patch_epilogue<TN, TM, DACT>(s, g, s2 ? 0 : cph, b, y0 + wm * TM, x0, fr, nn, acc);
          }
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
        ++cph;
        ctw = 3 - (cph & 1);
        cntap = (3 - (cph >> 1)) * ctw;
      }
    }
  }
#undef STAGE_ISSUE
#undef PATCH_ISSUE
}

// ---------------------------------------------------------------------------
// Fragment-streamed patch kernel (bf16): the same M-grid tiles as conv_patch_kernel (3x3
// stride-1 conv / subpel, 5x5/s2 convT with its four phases), but with NO barrier in the K
// loop: the block's whole input patch -- (TH+2) x 18 pixels x every input channel -- is
// staged in LDS once (LDS-DMA, rows padded by two 16-byte chunks: the 16 consecutive rows of
// a B-fragment read are then bank-conflict-free for any tap shift), and each wave streams
// its A fragments straight from a FRAGMENT-MAJOR weight copy into an R-deep register ring:
// one 1-KiB block per (phase, 16-row N tile, 32-deep k-step) holds the 64 lanes' 16-byte
// fragments in lane order, so every weight load is a fully coalesced global_load_dwordx4.
// K runs tap-major over channels padded to 32 per tap (k' = tap * cin32 + ci; zero weights
// and zero patch channels in the padding).  Waves: 1 (M) x NW (N); wave = TH rows of 16
// pixels x BN/NW channels.  Each phase's k-steps are padded to a multiple of R (idle steps)
// so the unrolled ring never straddles a phase's epilogue.
//
// KS = 3 (unrolled-K variants only): the K loop is split by kernel row -- 3 x NW waves, wave
// (kp, wn) runs the 3 taps of row dy = kp (3 x CPT k-steps) for N wave wn, so each SIMD holds
// three independent k-step chains instead of one (the 32x32-latent slice convs launch about
// one workgroup per CU: with one wave per SIMD every k-step paid its LDS / L2 latency in
// full).  The row partials are summed through LDS (over the dead patch) in the fixed order
// dy 0 + dy 1 + dy 2 and the dy-0 waves run the epilogue.
template <int TH, int BN, int NW, int R, int CPT = 0, int KS = 1>
__global__ void __launch_bounds__(64 * NW * KS) conv_fpatch_kernel(const ConvArgsDev args) {
  using T = bf16_t;
  constexpr int TW = 16, PW = TW + 2, PR = (TH + 2) * PW;
  constexpr int TM = TH, TN = BN / NW / 16;
  static_assert(TN * NW * 16 == BN, "tile");
  static_assert(KS == 1 || (KS == 3 && CPT > 0), "K split by kernel row: unrolled-K only");
  extern __shared__ __attribute__((aligned(16))) uint4 patch[];
  WG_T(0);

  const ConvShared& s = args.s;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave_all = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave = KS > 1 ? wave_all % NW : wave_all;       // N wave
  const int kp = KS > 1 ? wave_all / NW : 0;                // kernel row of this K part
  const int txn = s.Wm / TW, tyn = s.Hm / TH;
  int nblk, txi, tyi, b, gi;
  {
    const int nwg = gridDim.x * gridDim.y;
    int t = blockIdx.x + gridDim.x * blockIdx.y;
    if (s.remap) {                               // XCD-contiguous runs, N tile fastest
      const int xcd = t & 7, q = nwg >> 3, r = nwg & 7;
      t = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (t >> 3);
    }
    nblk = t % gridDim.y; t /= gridDim.y;
    txi = t % txn; t /= txn;
    tyi = t % tyn; t /= tyn;
    b = t % s.batch;
    gi = t / s.batch;
  }
  const ConvGroup& g = args.g[gi];
  const int n0 = nblk * BN;
  if (n0 >= g.cout) return;
  const int y0 = tyi * TH, x0 = txi * TW;
  const bool convt = s.mode == RGBAC_CONVT_S2;
  const int nph = convt ? 4 : 1;
  const int in_h = s.in_h, in_w = s.in_w, cin_pad = g.cin_pad;
  const int cin32 = (cin_pad + 31) & ~31;
  const int nch = cin32 >> 3;                    // 16-byte chunks of a patch row (real part)
  const int RSc = nch + 2;                       // + 2 pad chunks (bank spread)
  const int cpt = cin32 >> 5;                    // 32-deep k-steps per tap
  const int nks_max = (convt ? 9 : 9) * cpt;     // k-steps of the widest phase (layout stride)
  const uint4* const wf = reinterpret_cast<const uint4*>(g.w);
  const int ntile0 = (n0 >> 4) + wave * TN;      // this wave's first 16-row N tile

  // CPT > 0 (conv mode, every group's cin rounds up to 32*CPT, host-checked): the K loop is
  // fully unrolled -- 9 taps x CPT 32-deep k-steps -- so every patch read is a per-lane base +
  // a compile-time immediate and the weight ring is statically indexed: no per-k-step
  // division, tap bookkeeping or address arithmetic (the generic loop below spends ~14
  // SALU/VALU instructions per MFMA on them: issue-bound at 8 % of the matrix pipe on the
  // 32x32-latent slice convs).  The first R k-steps' weights are requested before the patch.
  // A k-step is only TN x TM MFMAs (64-128 cycles), so the weight ring runs RC steps ahead
  // (RC x the step >= an L2 round trip): 12 steps at TN 1, 8 at TN 2, 4 beyond.
  constexpr int NKSC = 9 * (CPT > 0 ? CPT : 1);
  constexpr int NKSP = NKSC / KS;                // k-steps of this wave's K part
  constexpr int RC0 = CPT > 0 ? (TN == 1 ? RGBAC_RC1 : (TN == 2 ? RGBAC_RC1 / 2 : 4)) : 1;
  constexpr int RC1 = KS > 1 ? (RC0 + 1) / 2 : RC0;   // three chains per SIMD share the latency
  constexpr int RC = RC1 < NKSP ? RC1 : NKSP;
  const uint4* wj[TN];
  uint4 cring[RC][TN];
  // the unrolled-K variants' epilogue biases, requested first (a cold bias read in the
  // epilogue cost a memory round trip at the end of the dependency chain)
  float pbias[TN][4];
  if constexpr (CPT > 0) {
    const int nb0 = n0 + wave * TN * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        pbias[j][r] = (g.bias && nb0 + j * 16 + r < g.cout) ? g.bias[nb0 + j * 16 + r] : 0.0f;
#pragma unroll
    for (int j = 0; j < TN; ++j)
      wj[j] = wf + ((size_t)(ntile0 + j) * NKSC + kp * NKSP) * 64 + lane;
  }

  // ---- stage the whole patch: flat uint4 index f -> (row, chunk), zero page outside
  {
    const int send0 = g.send0, send1 = g.send1, send2 = g.send2;
    const char* const sp0 = reinterpret_cast<const char*>(g.sp0);
    const char* const sp1 = reinterpret_cast<const char*>(g.sp1);
    const char* const sp2 = reinterpret_cast<const char*>(g.sp2);
    const int sld0 = (int)g.sld0, sld1 = (int)g.sld1, sld2 = (int)g.sld2;
    const int total = PR * RSc;
    const int npiece = (total + 63) >> 6;
    const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(size_t)(lptr_t)patch);
    for (int pc = wave_all; pc < npiece; pc += NW * KS) {
      const int f = (pc << 6) + lane;
      const int row = f / RSc, c = f - (f / RSc) * RSc;
      const int py = row / PW, px = row - (row / PW) * PW;
      const int iy = y0 - 1 + py, ix = x0 - 1 + px;
      const int ch = c << 3;
      const bool in0 = ch < send0, in1 = ch < send1;
      const char* src = in0 ? sp0 : (in1 ? sp1 : sp2);
      const int sld = in0 ? sld0 : (in1 ? sld1 : sld2);
      const int cs = ch - (in0 ? 0 : (in1 ? send0 : send1));
      const bool ok = row < PR && c < nch && ch < send2 && (unsigned)iy < (unsigned)in_h &&
                      (unsigned)ix < (unsigned)in_w;
      const unsigned off = ok ? ((unsigned)((b * in_h + iy) * in_w + ix) * (unsigned)sld +
                                 (unsigned)cs) * 2u : 0u;
      dma16_l(ok ? (const void*)(src + off) : (const void*)g_zero_page, lbase + (pc << 10));
    }
    if constexpr (CPT > 0) {
      // the weight ring is requested BEHIND the patch pieces and left in flight: the wait
      // below retires only the older requests (loads return in order), so the workgroup
      // waits for its patch, not for the whole ring prologue (the per-workgroup probe's
      // 3.4-4.8 us "stage" phase of the slice-chain convs was mostly that prologue)
#pragma unroll
      for (int u = 0; u < RC; ++u)
#pragma unroll
        for (int j = 0; j < TN; ++j) cring[u][j] = wj[j][u * 64];
      wait_vm<RC * TN>();
    } else {
      wait_vm<0>();
    }
    __syncthreads();
  }
  WG_T(1);

  if constexpr (CPT > 0) {
    constexpr int RS = 4 * CPT + 2;               // patch row stride (uint4) == RSc
    const int fr = lane & 15, fq = lane >> 4;
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
      // KS 3: ks < 3 * CPT, so tap / 3 == 0 and the row offset sits in lb
      const int tap = ks / CPT, cc = ks - (ks / CPT) * CPT;
      const int off = ((tap / 3) * PW + tap % 3) * RS + cc * 4;
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
    WG_T(2);
    if constexpr (KS > 1) {
      f32x4* const red = reinterpret_cast<f32x4*>(patch);
      __syncthreads();                            // every wave is done with the patch
      if (kp > 0) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
            red[((((kp - 1) * NW + wave) * TN + j) * TM + i) * 64 + lane] = acc[j][i];
      }
      __syncthreads();
      if (kp > 0) return;
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
    }
    int nn[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) nn[j] = n0 + wave * TN * 16 + j * 16 + fq * 4;
    patch_epilogue<TN, TM, false>(s, g, 0, b, y0, x0, fr, nn, acc, pbias);
    WG_T(3);
    return;
  }

  // ---- per-phase k-steps (padded to a multiple of R) and the weight fragment pointer
  const int nt16 = g.rows >> 4;
  auto phase_steps = [&](int ph) {
    return (convt ? (3 - (ph >> 1)) * (3 - (ph & 1)) : 9) * cpt;
  };
  // load-side iterator over the padded flat step sequence
  int lph = 0, lks = 0, lpad = (phase_steps(0) + R - 1) / R * R, lreal = phase_steps(0);
#define FP_LOAD(dst)                                                                          \
  do {                                                                                        \
    if (lph < nph && lks < lreal) {                                                           \
_Pragma("unroll")                                                                             \
      for (int j = 0; j < TN; ++j)                                                            \
        dst[j] = wf[((size_t)(lph * nt16 + ntile0 + j) * nks_max + lks) * 64 + lane];         \
    }                                                                                         \
    if (++lks == lpad) {                                                                      \
      lks = 0;                                                                                \
      if (++lph < nph) { lreal = phase_steps(lph); lpad = (lreal + R - 1) / R * R; }          \
    }                                                                                         \
  } while (0)

  uint4 ring[R][TN];
#pragma unroll
  for (int u = 0; u < R; ++u) FP_LOAD(ring[u]);

  f32x4 acc[TN][TM];
  const int fr = lane & 15, fq = lane >> 4;
  for (int ph = 0; ph < nph; ++ph) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int real = phase_steps(ph);
    const int tw = convt ? 3 - (ph & 1) : 3;
    int tap = 0, cc = 0;                         // k-step -> (tap, 32-channel chunk)
    for (int ks0 = 0; ks0 < real; ks0 += R) {
#pragma unroll
      for (int u = 0; u < R; ++u) {
        if (ks0 + u < real) {
          const int tyo = tap / tw, txo = tap - (tap / tw) * tw;
          const int oy = convt ? 2 - tyo : tyo, ox = convt ? 2 - txo : txo;
          uint4 bb[TM];
#pragma unroll
          for (int i = 0; i < TM; ++i) {
            const int pr = (i + oy) * PW + fr + ox;
            bb[i] = patch[pr * RSc + cc * 4 + fq];
          }
#pragma unroll
          for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int i = 0; i < TM; ++i) mma_step<T>(acc[j][i], ring[u][j], bb[i]);
          if (++cc == cpt) { cc = 0; ++tap; }
        }
        FP_LOAD(ring[u]);
      }
    }
    int nn[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) nn[j] = n0 + wave * TN * 16 + j * 16 + fq * 4;
    patch_epilogue<TN, TM, false>(s, g, ph, b, y0, x0, fr, nn, acc);
  }
#undef FP_LOAD
}

template <typename T>
static int launch_conv(const ConvArgsDev& d, int tile, int max_cout, hipStream_t st, int part) {
  const ConvShared& s = d.s;
  const TileCfg tc = kTiles[tile];
  const bool inlaunch = s.ksplit > 1 && d.g[0].cnt != nullptr &&
                        (tile < kFirstWres || (tile >= kFirstDeep && tile < kFirstPers));
  if (part == 2) {                         // split-K reduce + epilogue kernels only
    const bool patch_slabs = patch_tile(tile) && s.mode == RGBAC_CONV;   // strided-conv split
    if (s.ksplit == 1 || inlaunch || tile == kTileSpatial || tile == kTileSmallK ||
        tile == kTileWStream || (tile >= kFirstPatch && !patch_slabs) ||
        (tile >= kFirstWres && tile < kFirstDeep))
      return RGBAC_OK;
    goto splitk_epilogue;
  }
  if (tile == kTileSpatial) {
    if constexpr (sizeof(T) == 2) {
      dim3 grid((unsigned)((long long)s.batch * (s.Hm / 16) * (s.Wm / 16)), 1, s.ngroups);
      hipLaunchKernelGGL(conv3x3_c32_kernel<T>, grid, dim3(256), 0, st, d);
      return check_launch("conv3x3_c32_kernel");
    } else {
      set_error("the spatial 3x3 tile is bf16 only");
      return RGBAC_E_ARG;
    }
  }
  if (tile >= kFirstDirect && tile < kFirstDeep) {
    const int ny = (max_cout + tc.bn - 1) / tc.bn;
    const int nz = s.ngroups;
    const int ntile = (s.M + 15) / 16;
    int gx = (512 + ny * nz - 1) / (ny * nz);
    if (gx > (ntile + 3) / 4) gx = (ntile + 3) / 4;
    if (gx < 1) gx = 1;
    int nks_max = 0;
    const int kstep = sizeof(T) == 4 ? 16 : 32;
    for (int i = 0; i < s.ngroups; ++i) {
      const int nk = (s.ksize * s.ksize * d.g[i].cin_pad + kstep - 1) / kstep;
      if (nk > nks_max) nks_max = nk;
    }
    const int rs = nks_max * 4 + 1;
    if ((size_t)tc.bn * rs * 16 > 65536) {
      set_error("direct tile weight panel exceeds 64 KiB of LDS");
      return RGBAC_E_ARG;
    }
    dim3 grid(gx, ny, nz);
    switch (tc.bn / 16) {
      case 1: launch_direct<T, 1>(d, grid, rs, nks_max, st); break;
      case 2: launch_direct<T, 2>(d, grid, rs, nks_max, st); break;
      case 3: launch_direct<T, 3>(d, grid, rs, nks_max, st); break;
      case 4: launch_direct<T, 4>(d, grid, rs, nks_max, st); break;
      case 6: launch_direct<T, 6>(d, grid, rs, nks_max, st); break;
      default: launch_direct<T, 12>(d, grid, rs, nks_max, st); break;
    }
    return check_launch("conv_direct_kernel");
  }
  if (tile >= kFirstWres && tile < kFirstDeep) {
    const int mtiles = (s.M + tc.bm - 1) / tc.bm;
    const int ny = (max_cout + tc.bn - 1) / tc.bn;
    const int nz = s.nphase * s.ngroups;
    int gx = (512 + ny * nz - 1) / (ny * nz);
    if (gx > mtiles) gx = mtiles;
    if (gx < 1) gx = 1;
    dim3 grid(gx, ny, nz);
    constexpr int NS = kWresStages;
    switch (tile) {
      case 7: hipLaunchKernelGGL((conv_wres_kernel<T, 128, 64, 2, 2, NS>), grid, dim3(256), 0, st, d); break;
      case 8: hipLaunchKernelGGL((conv_wres_kernel<T, 64, 64, 2, 2, NS>), grid, dim3(256), 0, st, d); break;
      case 9: hipLaunchKernelGGL((conv_wres_kernel<T, 128, 32, 4, 1, NS>), grid, dim3(256), 0, st, d); break;
      case 10: hipLaunchKernelGGL((conv_wres_kernel<T, 64, 32, 2, 2, NS>), grid, dim3(256), 0, st, d); break;
      case 11: hipLaunchKernelGGL((conv_wres_kernel<T, 128, 128, 2, 2, NS>), grid, dim3(256), 0, st, d); break;
      default: hipLaunchKernelGGL((conv_wres_kernel<T, 128, 16, 4, 1, NS>), grid, dim3(256), 0, st, d); break;
    }
    return check_launch("conv_wres_kernel");
  }
  if (tile == kTileNPatch) {
    if constexpr (sizeof(T) == 2) {
      launch_npatch(d, max_cout, st);
      return check_launch("conv_npatch_kernel");
    } else {
      set_error("the narrow patch tile is bf16 only");
      return RGBAC_E_ARG;
    }
  }
  if (tile == kTilePW) {
    if constexpr (sizeof(T) == 2) {
      int cmax = 0;
      for (int i = 0; i < s.ngroups; ++i) cmax = d.g[i].cin_pad > cmax ? d.g[i].cin_pad : cmax;
      launch_pw(d, cmax, st);
      return check_launch("conv_pw_kernel");
    } else {
      set_error("the full-width pointwise tile is bf16 only");
      return RGBAC_E_ARG;
    }
  }
  if (fpatch_tile(tile)) {
    if constexpr (sizeof(T) == 2) {
      const int th = tc.bm / 16;
      const int nbn = (max_cout + tc.bn - 1) / tc.bn;
      const long long nsp = (long long)s.batch * (s.Hm / th) * (s.Wm / 16) * s.ngroups;
      int cmax = 0;
      for (int i = 0; i < s.ngroups; ++i) cmax = d.g[i].cin_pad > cmax ? d.g[i].cin_pad : cmax;
      size_t lds = ((size_t)(th + 2) * 18 * (((cmax + 31) & ~31) / 8 + 2) * 16 + 1023) &
                   ~(size_t)1023;                         // whole 1-KiB DMA pieces
      const bool ks3 = fpatch_ks_tile(tile);
      if (ks3) {                                          // row partials over the patch
        const size_t red = (size_t)2 * (tc.bn / 16) * th * 64 * 16;
        if (red > lds) lds = red;
      }
      if (lds > 160 * 1024) {
        set_error("fragment-patch tile: the input patch exceeds 160 KiB of LDS");
        return RGBAC_E_ARG;
      }
      dim3 grid((unsigned)nsp, (unsigned)nbn, 1);
      // the unrolled-K variant when it is a conv and every group has the same cin32 of 3, 4
      // or 7 k-steps per tap (the slice stacks: 80..128 and 224 input channels)
      int cpt = 0;
      if (s.mode == RGBAC_CONV || (ks3 && s.mode == RGBAC_SUBPEL2)) {
        cpt = ((d.g[0].cin_pad + 31) & ~31) >> 5;
        for (int i = 1; i < s.ngroups; ++i)
          if ((((d.g[i].cin_pad + 31) & ~31) >> 5) != cpt) cpt = 0;
        // 8..10 k-steps per tap (the hyperprior's 256..320-channel 3x3 convs / subpel convs
        // on the 16x16 grid): the K-split tiles 51 / 52 only
        const bool wide = ks3 && (tile == kFirstFPatchKS || tile == kFirstFPatchKS + 1);
        if (!(cpt == 3 || cpt == 4 || cpt == 7 || (wide && cpt >= 8 && cpt <= 10))) cpt = 0;
        if (!fpatch_cpt_enabled()) cpt = 0;
      }
      if (ks3 && cpt == 0) {
        set_error("K-split fragment-patch tiles: 3x3 conv with 96/128/224 (tiles 51/52 also "
                  "256/288/320)-channel inputs only");
        return RGBAC_E_ARG;
      }
#define RGBAC_FP1(TH_, BN_, C_)                                                               \
  do {                                                                                        \
    auto k_ = conv_fpatch_kernel<TH_, BN_, 4, 4, C_>;                                         \
    static unsigned long long attr_ = 0;                                                      \
    lds_optin((const void*)k_, 160 * 1024, &attr_);                                          \
    hipLaunchKernelGGL(k_, grid, dim3(256), lds, st, d);                                      \
  } while (0)
#define RGBAC_FPK(TH_, BN_, NW_, C_)                                                          \
  do {                                                                                        \
    auto k_ = conv_fpatch_kernel<TH_, BN_, NW_, 4, C_, 3>;                                    \
    static unsigned long long attr_ = 0;                                                      \
    lds_optin((const void*)k_, 160 * 1024, &attr_);                                          \
    hipLaunchKernelGGL(k_, grid, dim3(64 * NW_ * 3), lds, st, d);                             \
  } while (0)
#define RGBAC_FPKS(TH_, BN_, NW_)                                                             \
  do {                                                                                        \
    if (cpt == 3) RGBAC_FPK(TH_, BN_, NW_, 3);                                                \
    else if (cpt == 4) RGBAC_FPK(TH_, BN_, NW_, 4);                                           \
    else RGBAC_FPK(TH_, BN_, NW_, 7);                                                         \
  } while (0)
#define RGBAC_FPKW(BN_)                                                                       \
  do {                                                                                        \
    if (cpt == 8) RGBAC_FPK(4, BN_, 4, 8);                                                    \
    else if (cpt == 9) RGBAC_FPK(4, BN_, 4, 9);                                               \
    else if (cpt == 10) RGBAC_FPK(4, BN_, 4, 10);                                             \
    else RGBAC_FPKS(4, BN_, 4);                                                               \
  } while (0)
#define RGBAC_FP(TH_, BN_)                                                                    \
  do {                                                                                        \
    if (TH_ != 4) RGBAC_FP1(TH_, BN_, 0);  /* 8-row tiles: the generic loop is faster */     \
    else if (cpt == 3) RGBAC_FP1(TH_, BN_, 3);                                                \
    else if (cpt == 4) RGBAC_FP1(TH_, BN_, 4);                                                \
    else if (cpt == 7) RGBAC_FP1(TH_, BN_, 7);                                                \
    else RGBAC_FP1(TH_, BN_, 0);                                                              \
  } while (0)
      switch (tile) {
        case 42: RGBAC_FP(8, 192); break;
        case 43: RGBAC_FP(4, 192); break;
        case 44: RGBAC_FP(8, 128); break;
        case 45: RGBAC_FP(4, 128); break;
        case 46: RGBAC_FP(8, 256); break;
        case kTileFPatch464: RGBAC_FP(4, 64); break;
        case kFirstFPatchKS: RGBAC_FPKW(64); break;
        case kFirstFPatchKS + 1: RGBAC_FPKW(128); break;
        case kFirstFPatchKS + 2: RGBAC_FPKS(4, 192, 4); break;
        case kFirstFPatchKS2: RGBAC_FPKS(8, 64, 4); break;
        case kFirstFPatchKS2 + 1: RGBAC_FPKS(8, 128, 4); break;
        case kFirstFPatchKS2 + 2: RGBAC_FPKS(16, 32, 2); break;
        default: RGBAC_FP(8, 64); break;
      }
#undef RGBAC_FP
#undef RGBAC_FP1
#undef RGBAC_FPKW
#undef RGBAC_FPKS
#undef RGBAC_FPK
      return check_launch("conv_fpatch_kernel");
    } else {
      set_error("the fragment-patch tiles are bf16 only");
      return RGBAC_E_ARG;
    }
  }
  if (tile >= kFirstPatch) {
    if constexpr (sizeof(T) == 2) {
      const int th = tc.bm / 16;
      const long long nsp = (long long)s.batch * (s.Hm / th) * (s.Wm / 16) * s.ngroups;
      // ksplit 4: the phase split (grid z = the 5x5/s2 conv's / convT's four phases)
      dim3 grid((unsigned)nsp, (unsigned)((max_cout + tc.bn - 1) / tc.bn), s.ksplit > 1 ? 4 : 1);
      // the folded activation backward (training input gradients) in instances of their own:
      // the forward instances keep the register allocation they were tuned with (the shared
      // epilogue code cost the 5x5/s2 patch kernels 37 % when compiled into them)
#define PATCH_LAUNCH(DA)                                                                               \
      switch (tile) {                                                                                  \
        case 36: hipLaunchKernelGGL((conv_patch_kernel<8, 192, 2, 4, 3, DA>), grid, dim3(512), 0, st, d); break; \
        case 37: hipLaunchKernelGGL((conv_patch_kernel<8, 128, 2, 4, 3, DA>), grid, dim3(512), 0, st, d); break; \
        case 38: hipLaunchKernelGGL((conv_patch_kernel<8, 96, 4, 2, 3, DA>), grid, dim3(512), 0, st, d); break;  \
        case 39: hipLaunchKernelGGL((conv_patch_kernel<8, 256, 2, 4, 3, DA>), grid, dim3(512), 0, st, d); break; \
        case 40: hipLaunchKernelGGL((conv_patch_kernel<8, 192, 2, 4, 4, DA>), grid, dim3(512), 0, st, d); break; \
        case 48: hipLaunchKernelGGL((conv_patch_kernel<8, 64, 4, 2, 4, DA>), grid, dim3(512), 0, st, d); break;  \
        case 49: hipLaunchKernelGGL((conv_patch_kernel<8, 128, 2, 4, 4, DA>), grid, dim3(512), 0, st, d); break; \
        default: hipLaunchKernelGGL((conv_patch_kernel<8, 64, 4, 2, 3, DA>), grid, dim3(512), 0, st, d); break;  \
      }
      if (is_dact(s.act)) {
        PATCH_LAUNCH(true)
      } else {
        PATCH_LAUNCH(false)
      }
#undef PATCH_LAUNCH
      const int rc = check_launch("conv_patch_kernel");
      if (rc || s.ksplit == 1 || s.mode != RGBAC_CONV || part == 1) return rc;
      goto splitk_epilogue;
    } else {
      set_error("the patch tiles are bf16 only");
      return RGBAC_E_ARG;
    }
  }
  if (tile == kTileWStream) {
    if constexpr (sizeof(T) == 2) {
      launch_wstream(d, st);
      return check_launch("conv_wstream_kernel");
    } else {
      set_error("the narrow wave-streaming tile is bf16 only");
      return RGBAC_E_ARG;
    }
  }
  if (tile == kTileSmallK) {
    if constexpr (sizeof(T) == 2) {
      int nks16 = 0;
      for (int i = 0; i < s.ngroups; ++i) {
        const int k = (s.ksize * s.ksize * d.g[i].cin_pad + 15) / 16;
        if (k > nks16) nks16 = k;
      }
      launch_smallk(d, nks16, max_cout, st);
      return check_launch("conv_smallk_kernel");
    } else {
      set_error("the small-K tile is bf16 only");
      return RGBAC_E_ARG;
    }
  }
  if (tile >= kFirstPers) {
    const int ntile = ((s.M + tc.bm - 1) / tc.bm) * ((max_cout + tc.bn - 1) / tc.bn);
    const int nz = s.nphase * s.ksplit * s.ngroups;
    switch (tile) {
      case 27: launch_pers<T, 128, 128, 2, 2, 2>(d, ntile, nz, st); break;
      case 28: launch_pers<T, 128, 64, 4, 1, 3>(d, ntile, nz, st); break;
      case 29: launch_pers<T, 64, 64, 2, 2, 3>(d, ntile, nz, st); break;
      case 30: launch_pers<T, 128, 32, 4, 1, 3>(d, ntile, nz, st); break;
      case 31: launch_pers<T, 64, 32, 2, 2, 3>(d, ntile, nz, st); break;
      case 32: launch_pers<T, 128, 16, 4, 1, 3>(d, ntile, nz, st); break;
      default: launch_pers<T, 64, 16, 4, 1, 3>(d, ntile, nz, st); break;
    }
  } else {
  dim3 grid((s.M + tc.bm - 1) / tc.bm, (max_cout + tc.bn - 1) / tc.bn,
            s.nphase * s.ksplit * s.ngroups);
  switch (tile) {
    case 0: hipLaunchKernelGGL((conv_kernel<T, 128, 128, 2, 2, 2>), grid, dim3(256), 0, st, d); break;
    case 1: hipLaunchKernelGGL((conv_kernel<T, 128, 64, 4, 1, 3>), grid, dim3(256), 0, st, d); break;
    case 2: hipLaunchKernelGGL((conv_kernel<T, 64, 64, 2, 2, 3>), grid, dim3(256), 0, st, d); break;
    case 3: hipLaunchKernelGGL((conv_kernel<T, 128, 32, 4, 1, 3>), grid, dim3(256), 0, st, d); break;
    case 4: hipLaunchKernelGGL((conv_kernel<T, 64, 32, 2, 2, 3>), grid, dim3(256), 0, st, d); break;
    case 5: hipLaunchKernelGGL((conv_kernel<T, 128, 16, 4, 1, 3>), grid, dim3(256), 0, st, d); break;
    case 6: hipLaunchKernelGGL((conv_kernel<T, 64, 16, 4, 1, 3>), grid, dim3(256), 0, st, d); break;
    case 20: hipLaunchKernelGGL((conv_kernel<T, 128, 128, 2, 2, 2, 2>), grid, dim3(256), 0, st, d); break;
    case 21: hipLaunchKernelGGL((conv_kernel<T, 128, 64, 4, 1, 2, 2>), grid, dim3(256), 0, st, d); break;
    case 22: hipLaunchKernelGGL((conv_kernel<T, 64, 64, 2, 2, 2, 2>), grid, dim3(256), 0, st, d); break;
    case 23: hipLaunchKernelGGL((conv_kernel<T, 128, 32, 4, 1, 2, 2>), grid, dim3(256), 0, st, d); break;
    case 24: hipLaunchKernelGGL((conv_kernel<T, 64, 32, 2, 2, 3, 2>), grid, dim3(256), 0, st, d); break;
    case 25: hipLaunchKernelGGL((conv_kernel<T, 128, 16, 4, 1, 2, 2>), grid, dim3(256), 0, st, d); break;
    default: hipLaunchKernelGGL((conv_kernel<T, 64, 16, 4, 1, 3, 2>), grid, dim3(256), 0, st, d); break;
  }
  }
  {
    int rc = check_launch("conv_kernel");
    if (rc || s.ksplit == 1 || part == 1 || inlaunch) return rc;
  }
splitk_epilogue:
  for (int gi = 0; gi < s.ngroups; ++gi) {
    const long long total = (long long)s.nphase * s.M * (d.g[gi].cout16 / 4);
    long long gsz = (total + 255) / 256;
    if (gsz > 8192) gsz = 8192;
    hipLaunchKernelGGL((conv_splitk_epilogue<T>), dim3((int)gsz), dim3(256), 0, st, d, gi);
    const int rc = check_launch("conv_splitk_epilogue");
    if (rc) return rc;
  }
  return RGBAC_OK;
}

int fill_group(const rgbac_conv_args* a, int ntaps_max, ConvGroup& g) {
  RGBAC_REQUIRE(a->nsrc >= 1 && a->nsrc <= 3, "nsrc must be 1..3");
  RGBAC_REQUIRE(a->weight && a->out, "null weight/out");
  RGBAC_REQUIRE(a->ksplit == 1 || a->workspace ||
                    (patch_tile(a->tile) && a->mode == RGBAC_CONVT_S2),   // (phase split)
                "split-K needs a workspace");
  RGBAC_REQUIRE(a->cout > 0 && a->cout_pad % 128 == 0 && a->cout_pad >= a->cout,
                "cout_pad (packed weight rows) must be a multiple of 128 and >= cout");
  RGBAC_REQUIRE(a->cin_pad % 8 == 0 && a->cin_pad > 0, "cin_pad must be a multiple of 8");
  RGBAC_REQUIRE(a->k_pad % 64 == 0, "k_pad must be a multiple of 64");
  RGBAC_REQUIRE(ntaps_max * a->cin_pad <= a->k_pad, "k_pad too small for the taps");
  int csum = 0;
  for (int i = 0; i < a->nsrc; ++i) {
    RGBAC_REQUIRE(a->src[i].ptr != nullptr, "null source");
    RGBAC_REQUIRE(a->src[i].channels % 8 == 0 && a->src[i].channels > 0,
                  "source channels must be a positive multiple of 8");
    RGBAC_REQUIRE(a->src[i].ldc % 8 == 0 && a->src[i].ldc >= a->src[i].channels,
                  "source ldc must be a multiple of 8 and >= channels");
    RGBAC_REQUIRE(((uintptr_t)a->src[i].ptr) % 16 == 0, "source pointers must be 16-byte aligned");
    csum += a->src[i].channels;
  }
  RGBAC_REQUIRE(csum == a->cin_pad, "sum of source channels must equal cin_pad");
  RGBAC_REQUIRE(a->out_ldc % 4 == 0 && a->out_coff % 4 == 0, "out_ldc/out_coff must be multiples of 4");
  RGBAC_REQUIRE(a->act != RGBAC_ACT_MASKSEL || (a->sel && a->res1), "MASKSEL needs sel and res1");
  RGBAC_REQUIRE(!(a->act == RGBAC_ACT_TANH_HALF || a->act == RGBAC_ACT_GATE ||
                  a->act == RGBAC_ACT_GDN || a->act == RGBAC_ACT_IGDN ||
                  a->act == RGBAC_ACT_GAUSS) || a->res1,
                "act needs res1");
  g.sp0 = a->src[0].ptr; g.sld0 = a->src[0].ldc; g.send0 = a->src[0].channels;
  g.sp1 = a->nsrc > 1 ? a->src[1].ptr : a->src[0].ptr;
  g.sld1 = a->nsrc > 1 ? a->src[1].ldc : a->src[0].ldc;
  g.send1 = g.send0 + (a->nsrc > 1 ? a->src[1].channels : 0);
  g.sp2 = a->nsrc > 2 ? a->src[2].ptr : g.sp1;
  g.sld2 = a->nsrc > 2 ? a->src[2].ldc : g.sld1;
  g.send2 = g.send1 + (a->nsrc > 2 ? a->src[2].channels : 0);
  RGBAC_REQUIRE(!a->zout || (a->zout_ldc % 4 == 0 && a->act != RGBAC_ACT_GAUSS),
                "zout needs zout_ldc % 4 == 0 and no GAUSS epilogue");
  RGBAC_REQUIRE(a->act != RGBAC_ACT_SQBWD || (a->res0 && a->res1 && !a->bias),
                "SQBWD needs res0 (direct gradient), res1 (x) and no bias");
  RGBAC_REQUIRE(!is_dact(a->act) || (a->res0 && !a->res1 && !a->res2 && !a->bias && !a->zout &&
                                      a->mode != RGBAC_SUBPEL2 && !a->square_input &&
                                      !fpatch_tile(a->tile) && a->tile != kTileNPatch),
                "DGELU / DLRELU need res0 (the producer's pre-activation) and no bias, res1, res2, "
                "zout, subpel store, squared input or fragment-major (forward-only) tile");
  g.zout = a->zout;
  g.zld = a->zout_ldc;
  g.cnt = a->tile_counters;
  g.cin_pad = a->cin_pad;
  g.k_pad = a->k_pad;
  g.cout = a->cout;
  g.rows = a->cout_pad;
  g.cout16 = (a->cout + 15) / 16 * 16;
  g.w = a->weight;
  g.bias = a->bias;
  g.out = a->out;
  g.out_ldc = a->out_ldc;
  g.out_coff = a->out_coff;
  g.res0 = a->res0; g.ld0 = a->res0_ldc;
  g.res1 = a->res1; g.ld1 = a->res1_ldc;
  g.res2 = a->res2; g.ld2 = a->res2_ldc;
  g.sel = a->sel;
  g.ws = reinterpret_cast<float*>(a->workspace);
  g.aux0 = a->aux0;
  g.aux1 = a->aux1;
  g.partial = a->partial;
  return RGBAC_OK;
}

}  // namespace rgbac

using namespace rgbac;

#ifdef RGBAC_WG_TIMING
extern "C" int rgbac_debug_wg_times(unsigned long long* host, int nblocks) {
  if (nblocks > 16384) nblocks = 16384;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wg_t), (size_t)nblocks * 4 * 8) == hipSuccess ? 0 : 1;
}
extern "C" int rgbac_debug_wg_reset(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_wg_t)) != hipSuccess) return 1;
  return hipMemset(p, 0, sizeof(g_wg_t)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int rgbac_conv_num_tiles(void) { return kNumTiles; }
// 1 for the fragment-streamed patch tiles (42..47, 50..53), whose `weight` must be the
// fragment-major copy documented in rgbac.h; 0 for the plain packed layout; -1 out of range.
extern "C" int rgbac_conv_tile_weight_layout(int tile) {
  if (tile < 0 || tile >= kNumTiles) return -1;
  return (fpatch_tile(tile) || tile == kTileNPatch) ? 1 : 0;
}
extern "C" int rgbac_conv_max_groups(void) { return kMaxGroups; }

extern "C" int rgbac_conv2d_grouped(const rgbac_conv_args* args, int ngroups, void* stream) {
  return rgbac_conv2d_grouped_part(args, ngroups, 0, stream);
}

extern "C" int rgbac_conv2d_grouped_part(const rgbac_conv_args* args, int ngroups, int part,
                                         void* stream) {
  RGBAC_REQUIRE(part >= 0 && part <= 2, "part must be 0 (all), 1 (main) or 2 (split-K epilogue)");
  RGBAC_REQUIRE(args != nullptr, "null args");
  RGBAC_REQUIRE(ngroups >= 1 && ngroups <= kMaxGroups, "ngroups must be 1..10");
  const rgbac_conv_args* a = &args[0];
  RGBAC_REQUIRE(a->dtype == RGBAC_F32 || a->dtype == RGBAC_BF16, "dtype");
  RGBAC_REQUIRE(a->batch > 0 && a->in_h > 0 && a->in_w > 0, "bad input shape");
  RGBAC_REQUIRE(a->tile >= 0 && a->tile < kNumTiles, "tile index out of range");
  RGBAC_REQUIRE(a->ksplit >= 1 && a->ksplit <= 64, "ksplit must be 1..64");
  RGBAC_REQUIRE(a->act >= RGBAC_ACT_NONE && a->act <= RGBAC_ACT_DLRELU, "act");
  for (int i = 1; i < ngroups; ++i) {
    const rgbac_conv_args* b = &args[i];
    RGBAC_REQUIRE(b->dtype == a->dtype && b->mode == a->mode && b->batch == a->batch &&
                      b->in_h == a->in_h && b->in_w == a->in_w && b->ksize == a->ksize &&
                      b->stride == a->stride && b->out_h == a->out_h && b->out_w == a->out_w &&
                      b->tile == a->tile && b->ksplit == a->ksplit && b->act == a->act &&
                      b->act_param == a->act_param && b->square_input == a->square_input,
                  "grouped convs must share geometry, tile, split and activation");
  }
  ConvArgsDev d{};
  ConvShared& s = d.s;
  s.mode = a->mode;
  s.batch = a->batch;
  s.in_h = a->in_h;
  s.in_w = a->in_w;
  s.nphase = 1;
  int ntaps_max;
  if (a->mode == RGBAC_CONV) {
    RGBAC_REQUIRE(a->ksize == 1 || a->ksize == 3 || a->ksize == 5, "ksize must be 1/3/5");
    RGBAC_REQUIRE(a->stride == 1 || a->stride == 2, "stride must be 1/2");
    const int pad = a->ksize / 2;
    const int oh = (a->in_h + 2 * pad - a->ksize) / a->stride + 1;
    const int ow = (a->in_w + 2 * pad - a->ksize) / a->stride + 1;
    RGBAC_REQUIRE(a->out_h == oh && a->out_w == ow, "out size mismatch for conv");
    s.Hm = oh; s.Wm = ow; s.sy = a->stride; s.ksize = a->ksize; s.pad = pad;
    ntaps_max = a->ksize * a->ksize;
  } else if (a->mode == RGBAC_CONVT_S2) {
    RGBAC_REQUIRE(a->ksize == 5 && a->stride == 2, "CONVT_S2 supports k=5, s=2, p=2, op=1 only");
    RGBAC_REQUIRE(a->out_h == 2 * a->in_h && a->out_w == 2 * a->in_w, "out size mismatch for convT");
    s.Hm = a->in_h; s.Wm = a->in_w; s.sy = 1; s.ksize = 5; s.pad = 2;
    s.nphase = 4;
    ntaps_max = 9;
  } else if (a->mode == RGBAC_SUBPEL2) {
    RGBAC_REQUIRE(a->ksize == 3 && a->stride == 1, "SUBPEL2 is conv3x3 s1");
    RGBAC_REQUIRE(a->out_h == 2 * a->in_h && a->out_w == 2 * a->in_w, "out size mismatch for subpel");
    RGBAC_REQUIRE(a->act == RGBAC_ACT_NONE || a->act == RGBAC_ACT_GELU, "subpel supports NONE/GELU");
    s.Hm = a->in_h; s.Wm = a->in_w; s.sy = 1; s.ksize = 3; s.pad = 1;
    ntaps_max = 9;
  } else {
    RGBAC_REQUIRE(false, "unknown conv mode");
  }
  s.rWm = 1.0 / s.Wm;
  s.rHm = 1.0 / s.Hm;
  RGBAC_REQUIRE(!(a->tile < kFirstWres || (a->tile >= kFirstDeep && a->tile < kFirstPers)) ||
                    (long long)a->batch * a->in_h * a->in_w < (1ll << 24),
                "streaming conv tiles address sources of < 2^24 pixels (24-bit gather multiply)");
  const long long M = (long long)a->batch * s.Hm * s.Wm;
  RGBAC_REQUIRE(M < (1ll << 31), "too many output pixels");
  s.M = (int)M;
  s.out_h = a->out_h;
  s.out_w = a->out_w;
  s.act = a->act;
  s.act_param = a->act_param;
  s.square = a->square_input;
  s.ksplit = a->ksplit;
  s.ngroups = ngroups;
  static const int remap_env = [] {
    const char* e = getenv("RGBAC_XCD_REMAP");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  s.remap = remap_env;
  if (a->tile == kTileNPatch) {
    RGBAC_REQUIRE(a->dtype == RGBAC_BF16 &&
                      (a->mode == RGBAC_CONV ||
                       (a->mode == RGBAC_SUBPEL2 && !a->res0 && !a->res1 && !a->res2 &&
                        (a->act == RGBAC_ACT_NONE || a->act == RGBAC_ACT_GELU))) &&
                      a->ksplit == 1 && a->ksize == 3 && a->stride == 1 && s.Wm % 16 == 0 &&
                      s.Hm % 4 == 0,
                  "the narrow patch tile needs bf16, a 3x3 stride-1 conv (or subpel conv with "
                  "no residual, act none / GELU), ksplit 1, the grid a multiple of 16 wide "
                  "and 4 high");
    RGBAC_REQUIRE((long long)a->batch * a->in_h * a->in_w < (1ll << 24),
                  "the narrow patch tile addresses sources of < 2^24 pixels");
    for (int i = 0; i < ngroups; ++i) {
      RGBAC_REQUIRE(args[i].cout <= 32 && args[i].cout_pad % 16 == 0 &&
                        args[i].cout_pad >= (args[i].cout > 16 ? 32 : 16) &&
                        (size_t)6 * 18 * (((args[i].cin_pad + 31) & ~31) / 8 + 2) * 16 <=
                            128 * 1024,
                    "the narrow patch tile needs cout <= 32 and the input patch within 128 KiB");
      RGBAC_REQUIRE(a->act != RGBAC_ACT_GAUSS || args[i].cout == 16 || args[i].cout == 32,
                    "GAUSS on the narrow patch tile needs (mu|sigma) halves of 8 or 16 channels");
    }
  } else if (a->tile == kTilePW) {
    RGBAC_REQUIRE(a->dtype == RGBAC_BF16 && a->mode == RGBAC_CONV && a->ksplit == 1 &&
                      a->ksize == 1 && a->stride == 1 && a->act != RGBAC_ACT_GAUSS,
                  "the full-width pointwise tile needs bf16, a 1x1 stride-1 conv, ksplit 1 and "
                  "no GAUSS epilogue");
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE(args[i].nsrc == 1 && args[i].cin_pad <= 192 && args[i].cout <= 192,
                    "the full-width pointwise tile needs one source, cin_pad <= 192, cout <= 192");
  } else if (a->tile == kTileSpatial) {
    RGBAC_REQUIRE(a->dtype == RGBAC_BF16 && a->mode == RGBAC_CONV && a->ksize == 3 &&
                      a->stride == 1 && a->ksplit == 1 && a->act != RGBAC_ACT_GAUSS &&
                      s.Hm % 16 == 0 && s.Wm % 16 == 0,
                  "the spatial 3x3 tile needs bf16, 3x3 stride 1, H/W multiples of 16, ksplit 1");
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE(args[i].nsrc == 1 && args[i].cin_pad == 32 && args[i].src[0].channels == 32 &&
                        args[i].cout <= 32 && args[i].k_pad >= 288,
                    "the spatial 3x3 tile needs one 32-channel source and cout <= 32");
  } else if (a->tile >= kFirstPatch) {
    const int th = kTiles[a->tile].bm / 16;
    // ksplit 4 on conv_patch_kernel tiles: the phase split of the 5x5/s2 conv / convT
    const bool psplit = a->ksplit == 4 && patch_tile(a->tile) &&
                        (a->mode == RGBAC_CONVT_S2 ||
                         (a->mode == RGBAC_CONV && a->ksize == 5 && a->stride == 2));
    RGBAC_REQUIRE(a->dtype == RGBAC_BF16 && (a->ksplit == 1 || psplit) && !a->square_input &&
                      a->act != RGBAC_ACT_GAUSS &&
                      (a->mode == RGBAC_CONVT_S2 ||
                       (a->ksize == 3 && a->stride == 1 &&
                        (a->mode == RGBAC_CONV || a->mode == RGBAC_SUBPEL2)) ||
                       (a->mode == RGBAC_CONV && a->ksize == 5 && a->stride == 2 &&
                        !fpatch_tile(a->tile))) &&
                      s.Wm % 16 == 0 && s.Hm % th == 0,
                  "the patch tiles need bf16, ksplit 1, a 3x3 stride-1 conv/subpel, the 5x5/s2 "
                  "convT or (conv_patch_kernel tiles) the 5x5/s2 conv, the M grid a multiple of "
                  "16 wide and of the tile height high");
    RGBAC_REQUIRE((long long)a->batch * a->in_h * a->in_w < (1ll << 24),
                  "patch tiles address sources of < 2^24 pixels");
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE(args[i].cout_pad >= ((args[i].cout + kTiles[a->tile].bn - 1) /
                                         kTiles[a->tile].bn) * kTiles[a->tile].bn &&
                        args[i].k_pad >= ntaps_max * args[i].cin_pad &&
                        (!fpatch_tile(a->tile) ||
                         args[i].cout_pad % 16 == 0),
                    "patch tiles read whole BN-row weight tiles");
  } else if (a->tile == kTileWStream) {
    RGBAC_REQUIRE(a->dtype == RGBAC_BF16 && a->mode == RGBAC_CONV && a->ksplit == 1 &&
                      a->stride == 1 && (a->ksize == 1 || a->ksize == 3),
                  "the narrow wave-streaming tile needs bf16, a stride-1 1x1/3x3 conv, ksplit 1");
    for (int i = 0; i < ngroups; ++i) {
      RGBAC_REQUIRE(args[i].cout <= 32 && args[i].cin_pad < 4096 &&
                        (ntaps_max * args[i].cin_pad + 15) / 16 <= kWsMaxSteps,
                    "the narrow wave-streaming tile needs cout <= 32 and K <= 2336");
      RGBAC_REQUIRE(a->act != RGBAC_ACT_GAUSS ||
                        (args[i].cout % 16 == 0 && args[i].cout <= 32),
                    "GAUSS on the narrow tile needs (mu|sigma) halves of 8 or 16 channels");
    }
  } else if (a->tile == kTileSmallK) {
    RGBAC_REQUIRE(a->dtype == RGBAC_BF16 && a->mode == RGBAC_CONV && a->ksplit == 1 &&
                      a->act != RGBAC_ACT_GAUSS,
                  "the small-K tile needs bf16, a plain conv, ksplit 1 and no GAUSS epilogue");
    RGBAC_REQUIRE(a->ksize == 1 && a->stride == 1, "the small-K tile is a 1x1 stride-1 conv");
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE(args[i].cin_pad <= kSmallKMax && args[i].nsrc == 1,
                    "the small-K tile needs one source with cin_pad <= 256");
  } else if (a->tile >= kFirstDirect && a->tile < kFirstDeep) {
    RGBAC_REQUIRE(a->mode == RGBAC_CONV && a->ksplit == 1 && a->act != RGBAC_ACT_GAUSS,
                  "direct tiles need a plain conv, ksplit 1 and no GAUSS epilogue");
    const int ks_elems = a->dtype == RGBAC_F32 ? 16 : 32;
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE((ntaps_max * args[i].cin_pad + ks_elems - 1) / ks_elems <= kDirectSteps,
                    "K too large for a direct tile");
  } else if (a->tile >= kFirstWres && a->tile < kFirstDeep) {
    RGBAC_REQUIRE(a->ksplit == 1 && a->act != RGBAC_ACT_GAUSS,
                  "weight-resident tiles need ksplit 1 and no GAUSS epilogue");
    const int ks_elems = a->dtype == RGBAC_F32 ? 32 : 64;
    for (int i = 0; i < ngroups; ++i)
      RGBAC_REQUIRE((ntaps_max * args[i].cin_pad + ks_elems - 1) / ks_elems <= kWresStages,
                    "K too large for a weight-resident tile");
  }
  int max_cout = 0;
  for (int i = 0; i < ngroups; ++i) {
    const rgbac_conv_args* b = &args[i];
    if (a->mode == RGBAC_SUBPEL2) {
      RGBAC_REQUIRE(b->cout % 4 == 0, "subpel cout must be a multiple of 4");
      RGBAC_REQUIRE(!b->res0 && !b->res1 && !b->res2, "subpel has no residual epilogue");
    }
    if (a->act == RGBAC_ACT_GAUSS) {
      RGBAC_REQUIRE(a->mode == RGBAC_CONV && a->ksplit == 1, "GAUSS needs a plain conv, ksplit 1");
      RGBAC_REQUIRE(a->tile < kFirstPers || a->tile == kTileWStream || a->tile == kTileNPatch,
                    "GAUSS needs a non-persistent tile");
      RGBAC_REQUIRE(b->cout % 2 == 0 && b->cout <= kTiles[a->tile].bn,
                    "GAUSS needs (mu|sigma) channels in one N tile");
      RGBAC_REQUIRE(b->partial, "GAUSS needs a partial-sum buffer");
    }
    for (int j = 0; j < b->nsrc; ++j)
      RGBAC_REQUIRE((long long)a->batch * a->in_h * a->in_w * b->src[j].ldc *
                            (a->dtype == RGBAC_F32 ? 4 : 2) < (1ll << 31),
                    "each conv source must span < 2 GiB (32-bit gather offsets)");
    int rc = fill_group(b, ntaps_max, d.g[i]);
    if (rc) return rc;
    if (b->cout > max_cout) max_cout = b->cout;
  }
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  if (a->dtype == RGBAC_F32) return launch_conv<float>(d, a->tile, max_cout, st, part);
  return launch_conv<bf16_t>(d, a->tile, max_cout, st, part);
}

extern "C" int rgbac_conv2d(const rgbac_conv_args* a, void* stream) {
  return rgbac_conv2d_grouped(a, 1, stream);
}
