// Fused model-fit step: forward + heteroscedastic NLL + backward-data of the dynamics
// ensemble (BatchedGaussianEnsemble.fit's per-step compute_loss + loss.backward(),
// src/dynamics.py:112-122,136-153,236-253) in ONE launch, one 512-thread workgroup per
// (16-row tile, head, member) -- the decomposition of the split-heads forward and
// backward it replaces (csrc/mlp.hip mlp_fwd_kernel + mlp_bwd_ens_kernel).
//
// A workgroup of head h keeps everything between the forward and the backward in LDS:
//   x -> trunk L1 -> trunk L2 -> both heads' hidden layers (waves 0, 1, 2, 7 the diff
//   head, waves 3-6 the log-var head: pair_wave_code), each wave forming its split-K share of its head's
//   output layer from the columns it produced) -> D, log-var -> the NLL element
//   gradients -> dZ of head h's output layer -> head h's hidden dZ -> its share of the
//   trunk dZ (dz for h = 0, dz2 for h = 1; the trunk gradient is linear in the heads')
// The pre-activations z of the trunk layers and of head h's hidden layer stay in LDS for
// the backward's act'(z) (fused into the backward products' epilogues); only what the
// weight-gradient launch reads leaves the CU: the layer inputs (x, trunk y's, head h's
// hidden y; head 0's workgroup saves the trunk side) and every dZ. No z, D or log-var
// round trip through HBM, no second launch, no elementwise backward phases.
//
// Both heads' forwards run in every workgroup (the NLL of an element needs the diff
// and the log-var outputs): one 200x200 layer more per workgroup than the two launches,
// in one phase with the output layers (SIMD-balanced 7/6/6/7 blocks).
#include "common.hpp"
#include "critic_rows.hpp"

using namespace drpo;

namespace {
constexpr int FF_NW = 8;
constexpr int FF_NT = FF_NW * 64;
constexpr int FF_ROWS = 16;
constexpr int FF_LDH = 264;   // == 8 (mod 64): conflict-free A-fragment reads
}  // namespace

#ifdef DRPO_STAMPS
// profiling builds only (profiles/fit_stamps.py): per-workgroup s_memtime phase stamps
__device__ unsigned long long g_fit_stamps[4096][16];
#define FSTAMP(i)                                                                                 \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long _t;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    const unsigned _w = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);          \
    if (threadIdx.x == 0 && _w < 4096u) g_fit_stamps[_w][(i)] = _t;                               \
  } while (0)
DRPO_API int drpo_debug_stamps_fit(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fit_stamps), sizeof(unsigned long long) * 16 * (size_t)n);
}
#else
#define FSTAMP(i) \
  do {            \
  } while (0)
#endif

struct FitFbArgs {
  drpo_mlp_fwd_t f;      // forward mirrors, biases, y saves, input sources / normalizer
  drpo_mlp_bwd_t b;      // transposed mirrors, dz (trunk: dz | dz2 by head), nets as in f
  drpo_ens_upstream_t u; // NLL: states, targets, bounds, loss workspace
};
typedef const __attribute__((address_space(4))) FitFbArgs FitK;   // read in place (scalar loads)

// forward epilogue (swish): y -> out (LDS), z -> zb (LDS, the backward's act'), y -> gy
// (the weight gradient's input; rows < nrows)
template <int MAXC>
__device__ __forceinline__ void ff_epi_fwd(const f32x4 (&acc)[1][MAXC], const float (&bvs)[MAXC], int N, float* out,
                                           float* zb, float* gy, int ldg, int nrows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l15 = lane & 15, g = lane >> 4;
  const int NB = (N + 15) >> 4;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int cb = wave + FF_NW * c;
    if (cb >= NB) continue;
    const int col = cb * 16 + l15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g + r;
      const float z = acc[0][c][r] + bvs[c];
      const float y = act_fn<ACT_SILU>(z);
      out[row * FF_LDH + col] = col < N ? y : 0.f;
      zb[row * FF_LDH + col] = col < N ? z : 0.f;
      if (gy && col < N && row < nrows) gstore(gy + (size_t)row * ldg + col, y);
    }
  }
}

// backward epilogue: dZ = (dZ_next W) * act'(z) (swish, z from LDS) -> out (LDS, the
// next product's input; padding rows and columns zero) and -> gdz (rows < nrows)
template <int MAXC>
__device__ __forceinline__ void ff_epi_bwd(const f32x4 (&acc)[1][MAXC], int N, float* out, const float* zb, float* gdz,
                                           int ldg, int nrows) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l15 = lane & 15, g = lane >> 4;
  const int NB = (N + 15) >> 4;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int cb = wave + FF_NW * c;
    if (cb >= NB) continue;
    const int col = cb * 16 + l15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g + r;
      const float z = zb[row * FF_LDH + col];
      const float s = fast_sigmoid(z);
      const bool in = col < N && row < nrows;
      const float d = in ? acc[0][c][r] * (s * (1.f + z * (1.f - s))) : 0.f;
      if (out) out[row * FF_LDH + col] = d;
      if (gdz && in) gstore(gdz + (size_t)row * ldg + col, d);
    }
  }
}

// Weight rings. Every layer's first FPT-1 (heads: FPH-1) k-steps of packed-mirror
// fragments are issued by the PREVIOUS phase, right after its last MFMA and before its
// epilogue and barrier, so the cold first touch of a layer's weights (the mirrors were
// rewritten by the previous step's Adam) overlaps that epilogue instead of stalling the
// layer's first MFMA; the ring then streams the rest of the layer as tile_dense_mma does.
constexpr int FPT = 3;   // ring depth of the trunk-width (2 blocks per wave) layers (6: +1 %,
                         // profiles/r06/ring_ab2/fit)
constexpr int FPH = 4;   // ring depth of the heads phase (3-4 blocks per wave)
constexpr int FP1 = 5;   // the first layer's ring: K <= 64 (4 k-steps) preloaded whole

// Trunk-width layers: wave w owns column blocks w and w + 8 (clamped to a valid block:
// a wave with one valid block computes a discarded copy of it, which costs nothing -- the
// phase is bounded by SIMD 0's 4 blocks at N = 200, 2 per wave at N = 256)
template <int NK, int R = FPT>
__device__ __forceinline__ void ff_pre2(const float* __restrict__ P, int NCB, f32x4 (&bq)[R][2]) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int u = 0; u < R - 1; ++u)
    if (u < NK)
#pragma unroll
      for (int c = 0; c < 2; ++c) bq[u][c] = load_pk(P, min(wave + FF_NW * c, NCB - 1), u, NK);
}

template <int NK, int R = FPT>
__device__ __forceinline__ void ff_mma2(const float* in, const float* __restrict__ P, int NCB, f32x4 (&bq)[R][2],
                                        f32x4 (&acc)[1][2]) {
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int cbs[2] = {min(wave, NCB - 1), min(wave + FF_NW, NCB - 1)};
#pragma unroll
  for (int c = 0; c < 2; ++c) acc[0][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 an = *reinterpret_cast<const f32x4*>(in + l15 * FF_LDH + 4 * g), ac;
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    if (s + R - 1 < NK) {
#pragma unroll
      for (int c = 0; c < 2; ++c) bq[(s + R - 1) % R][c] = load_pk(P, cbs[c], s + R - 1, NK);
    }
    ac = an;
    if (s + 1 < NK) an = *reinterpret_cast<const f32x4*>(in + l15 * FF_LDH + 16 * (s + 1) + 4 * g);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        acc[0][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[m], bq[s % R][c][m], acc[0][c], 0, 0, 0);
  }
}

__device__ __forceinline__ void ff_bias2(const float* __restrict__ bias, int N, float (&bv)[2]) {
  const int wave = threadIdx.x >> 6, l15 = threadIdx.x & 15;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int col = (wave + FF_NW * c) * 16 + l15;
    bv[c] = col < N ? gload(bias + col) : 0.f;
  }
}

// the heads phase (rollout.hip pair_split_core's schedule): a wave owns blocks base,
// base + 4, ... (3-4) of its head's hidden layer, then its split-K share of the head's
// output layer from exactly those columns. Ring, output-layer fragments and biases are
// preloaded for 4 blocks (a 4th past the layer clamped and unused).
template <int NK>
__device__ __forceinline__ void ff_pre_heads(int base, int NCB, const float* __restrict__ P,
                                             const float* __restrict__ bias, int N, const float* __restrict__ Pn,
                                             f32x4 (&bq)[FPH][4], f32x4 (&nb)[4], float (&bv)[4]) {
  const int l15 = threadIdx.x & 15;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int cb = min(base + 4 * c, NCB - 1);
#pragma unroll
    for (int u = 0; u < FPH - 1; ++u) bq[u][c] = load_pk(P, cb, u, NK);
    nb[c] = load_pk(Pn, 0, cb, NK);
    const int col = (base + 4 * c) * 16 + l15;
    bv[c] = col < N ? gload(bias + col) : 0.f;
  }
}

template <int NC, int NK>
__device__ __forceinline__ void ff_heads_core(int base, const float* in, const float* __restrict__ P, int N,
                                              f32x4 (&bq)[FPH][4], const f32x4 (&nb)[4], const float (&bvs)[4],
                                              float* out, float* zb, float* gy, int nrows, float* red_slot,
                                              const float* __restrict__ Pnext, f32x4 (&bqn)[FPT][2]) {
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  int cbs[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) cbs[c] = base + 4 * c;
  f32x4 acc[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 an = *reinterpret_cast<const f32x4*>(in + l15 * FF_LDH + 4 * g), ac;
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    if (s + FPH - 1 < NK) {
#pragma unroll
      for (int c = 0; c < NC; ++c) bq[(s + FPH - 1) % FPH][c] = load_pk(P, cbs[c], s + FPH - 1, NK);
    }
    ac = an;
    if (s + 1 < NK) an = *reinterpret_cast<const f32x4*>(in + l15 * FF_LDH + 16 * (s + 1) + 4 * g);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[m], bq[s % FPH][c][m], acc[c], 0, 0, 0);
  }
  ff_pre2<1>(Pnext, (N + 15) >> 4, bqn);   // the backward's first product (K = S + 1: one k-step)
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = cbs[c] * 16 + l15;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = 4 * g + r;
      const float z = acc[c][r] + bvs[c];
      const float y = act_fn<ACT_SILU>(z);
      out[row * FF_LDH + col] = col < N ? y : 0.f;
      if (zb) zb[row * FF_LDH + col] = col < N ? z : 0.f;
      if (gy && col < N && row < nrows) gstore(gy + (size_t)row * N + col, y);
    }
  }
  wave_lds_sync();
  f32x4 pacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(out + l15 * FF_LDH + 16 * cbs[c] + 4 * g);
#pragma unroll
    for (int m = 0; m < 4; ++m) pacc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], nb[c][m], pacc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red_slot[(4 * g + r) * 16 + l15] = pacc[r];
}

template <int NK>
__device__ __forceinline__ void fit_fb_body(FitK& k, float* smem) {
  auto& F = k.f;
  auto& Bd = k.b;
  auto& U = k.u;
  float* xin = smem;
  float* T1 = xin + FF_ROWS * FF_LDH;   // trunk L1 y
  float* T2 = T1 + FF_ROWS * FF_LDH;    // trunk L2 y; later the NLL bound partials
  float* HA = T2 + FF_ROWS * FF_LDH;    // diff head hidden y; later G, then trunk-L2 dZ
  float* HB = HA + FF_ROWS * FF_LDH;    // log-var head hidden y; later head-h hidden dZ
  float* Z1 = HB + FF_ROWS * FF_LDH;
  float* Z2 = Z1 + FF_ROWS * FF_LDH;
  float* ZH = Z2 + FF_ROWS * FF_LDH;
  float* red = ZH + FF_ROWS * FF_LDH;   // 8 x 256 head output partials
  __shared__ float s_mse[FF_NW];
  const int tid = threadIdx.x;
  const LogicalBlock lb = xcd_block();   // one member's tiles per XCD (shared weights in L2)
  const int bx = lb.x, h = lb.y, z = lb.z;
  const int64_t b = U.b;
  const int row0 = bx * FF_ROWS;
  if (row0 >= b) return;
  FSTAMP(0);
  const int nrows = (int)min((int64_t)FF_ROWS, b - row0);
  const int S = U.S, S1 = S + 1;
  const bool tsave = h == 0;   // the trunk side's saves: head 0's workgroup
  const size_t zr = (size_t)z * b + row0;   // this tile's first row of member z
  auto& t0 = F.net[0].L[0];
  auto& t1 = F.net[0].L[1];
  const int Hm = t1.dout;
  const int NCB = (Hm + 15) >> 4;
  const int c0 = F.cols[0], c1 = F.cols[1];
  const int din0 = c0 + c1;
  const int nk1 = round_up(din0, 16) >> 4;

  // the first layer's whole weight tile, then the NLL's per-element inputs, ahead of
  // the input staging (independent loads: one round trip for all of them)
  f32x4 bq1[FP1][2];
  float bvt[2];
  {
    const float* P = t0.W + (size_t)z * t0.wstride;
    switch (nk1) {
      case 1: ff_pre2<1, FP1>(P, NCB, bq1); break;
      case 2: ff_pre2<2, FP1>(P, NCB, bq1); break;
      case 3: ff_pre2<3, FP1>(P, NCB, bq1); break;
      default: ff_pre2<4, FP1>(P, NCB, bq1); break;
    }
    ff_bias2(t0.b + (size_t)z * t0.bstride, Hm, bvt);
  }
  const int nr = tid >> 4, nk = tid & 15;   // NLL element of threads < 256
  const bool nll = tid < FF_ROWS * 16 && nr < nrows && nk < S1;
  float n_s = 0.f, n_t = 0.f, n_hi = 0.f, n_lo = 0.f, n_bd = 0.f, n_bl = 0.f;
  if (nll) {
    const int64_t row = row0 + nr;
    n_hi = gload(U.maxlv + nk);
    n_lo = gload(U.minlv + nk);
    n_bd = gload(F.net[1].L[1].b + (size_t)z * F.net[1].L[1].bstride + nk);
    n_bl = gload(F.net[2].L[1].b + (size_t)z * F.net[2].L[1].bstride + nk);
    n_s = nk < S ? gload(U.s + (int64_t)z * U.s_zstride + row * S + nk) : 0.f;
    n_t = gload(U.t + (int64_t)z * U.t_zstride + row * S1 + nk);
  }

  FSTAMP(9);
  // ---- input x = [normalize(s), a] -------------------------------------------------
  const int kpad = nk1 * 16;
  stage_input_tile<FF_NT>(xin, FF_LDH, FF_ROWS, nrows, row0, kpad, F.src[0] + (size_t)z * F.sstride[0],
                         c1 ? F.src[1] + (size_t)z * F.sstride[1] : nullptr, nullptr, c0, c1, 0, F.ld[0], F.ld[1], 0,
                         F.nmean, F.nstd, false, tsave ? F.save_x : nullptr, (int64_t)zr);
  lds_barrier();
  FSTAMP(1);

  // Saves for the weight gradients (layer inputs y, every dZ) leave from the epilogues.
  // (Deferring them to 16-byte stores of the LDS tile after each barrier measured no
  // gain: profiles/r05/fit_defer.)
  // ---- trunk ------------------------------------------------------------------------
  float* sy0 = tsave && t0.sy ? t0.sy + zr * Hm : nullptr;
  float* sy1 = tsave && t1.sy ? t1.sy + zr * Hm : nullptr;
  f32x4 bqt[FPT][2];
  {
    f32x4 acc[1][2];
    switch (nk1) {
      case 1: ff_mma2<1, FP1>(xin, t0.W + (size_t)z * t0.wstride, NCB, bq1, acc); break;
      case 2: ff_mma2<2, FP1>(xin, t0.W + (size_t)z * t0.wstride, NCB, bq1, acc); break;
      case 3: ff_mma2<3, FP1>(xin, t0.W + (size_t)z * t0.wstride, NCB, bq1, acc); break;
      default: ff_mma2<4, FP1>(xin, t0.W + (size_t)z * t0.wstride, NCB, bq1, acc); break;
    }
    FSTAMP(10);
    float bv[2] = {bvt[0], bvt[1]};
    ff_pre2<NK>(t1.W + (size_t)z * t1.wstride, NCB, bqt);
    ff_bias2(t1.b + (size_t)z * t1.bstride, Hm, bvt);
    FSTAMP(11);
    ff_epi_fwd(acc, bv, Hm, T1, Z1, sy0, Hm, nrows);
    FSTAMP(12);
  }
  lds_barrier();
  FSTAMP(2);
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned pcode = pair_wave_code(wave);   // 7 / 6 / 6 / 7 blocks per SIMD (common.hpp)
  const bool second = pcode >> 2;
  const int base = pcode & 3;
  auto& Hn = F.net[second ? 2 : 1];
  auto& l0 = Hn.L[0];
  auto& l1 = Hn.L[1];
  f32x4 bqh[FPH][4], nbh[4];
  float bvh[4];
  {
    f32x4 acc[1][2];
    ff_mma2<NK>(T1, t1.W + (size_t)z * t1.wstride, NCB, bqt, acc);
    ff_pre_heads<NK>(base, NCB, l0.W + (size_t)z * l0.wstride, l0.b + (size_t)z * l0.bstride, Hm,
                     l1.W + (size_t)z * l1.wstride, bqh, nbh, bvh);
    ff_epi_fwd(acc, bvt, Hm, T2, Z2, sy1, Hm, nrows);
  }
  lds_barrier();
  FSTAMP(3);
  // ---- both heads: hidden + output layers, one phase ----------------------------------
  auto& Hb = Bd.net[1 + h];
  auto& o1 = Hb.L[1];
  auto& o0 = Hb.L[0];
  auto& lown = F.net[1 + h].L[0];
  float* syh = lown.sy ? lown.sy + zr * Hm : nullptr;   // this workgroup's head's hidden y
  {
    const bool own = (second ? 1 : 0) == h;
    const int nc = min(4, (NCB - base + 3) / 4);
    float* slot = red + (size_t)(second ? FF_NW / 2 + (FF_NW / 2 - 1 - base) : base) * 256;
    const float* P = l0.W + (size_t)z * l0.wstride;
    float* out = second ? HB : HA;
    float* zb = own ? ZH : nullptr;
    float* gy = own ? syh : nullptr;
    const float* Pb1 = o1.W + (size_t)z * o1.wstride;
    if (nc == 4) ff_heads_core<4, NK>(base, T2, P, Hm, bqh, nbh, bvh, out, zb, gy, nrows, slot, Pb1, bqt);
    else ff_heads_core<3, NK>(base, T2, P, Hm, bqh, nbh, bvh, out, zb, gy, nrows, slot, Pb1, bqt);
  }
  lds_barrier();
  FSTAMP(4);
  // ---- NLL (drpo_ens_loss's arithmetic; ens_upstream in csrc/mlp.hip) -------------------
  float* Gd = T1;   // head h's output gradient (T1, the trunk's first layer y, is dead)
  {
    const int64_t nbx = (b + FF_ROWS - 1) / FF_ROWS;
    const float inv_n = 1.f / (float)(b * S1);
    const float gsc = (U.gscale ? *U.gscale : 1.f) * inv_n;
    float lacc = 0.f;
    if (tid < FF_ROWS * 16) {
      float gd = 0.f, gl = 0.f, cmn = 0.f, cmx = 0.f;
      if (nll) {
        const int64_t o = ((int64_t)z * b + row0 + nr) * S1 + nk;
        const float D = narrow_pair_sum<FF_NW, 1>(red, 0, nr, nk) + n_bd;
        const float raw = narrow_pair_sum<FF_NW, 1>(red, 1, nr, nk) + n_bl;
        const float hi = n_hi, lo = n_lo;
        const float l1v = hi - softplusf(hi - raw);
        const float l = lo + softplusf(l1v - lo);
        const float m = D + n_s;
        const float diff = n_t - m;
        const float iv = expf(-l);
        lacc = diff * diff * iv + l;
        const float dl = (1.f - diff * diff * iv) * gsc;
        const float s1 = sp_grad(l1v - lo), s2 = sp_grad(hi - raw);
        gd = -2.f * diff * iv * gsc;
        gl = dl * s1 * s2;
        cmn = dl * (1.f - s1);
        cmx = dl * s1 * (1.f - s2);
        if (o1.dz) gstore(o1.dz + o, h == 0 ? gd : gl);
      }
      Gd[nr * FF_LDH + nk] = h == 0 ? gd : gl;
      T2[nr * FF_LDH + nk] = cmn;
      T2[nr * FF_LDH + 64 + nk] = cmx;
    }
    // mse partial: per-wave sums, then the waves in order (as ens_upstream)
    float v = lacc * inv_n;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((tid & 63) == 0) s_mse[tid >> 6] = v;
    lds_barrier();
    FSTAMP(5);
    if (h == 0) {
      float* part_mse = U.part;
      float* part_min = part_mse + (size_t)U.Z * nbx;
      float* part_max = part_min + (size_t)U.Z * nbx * S1;
      const size_t pb = (size_t)z * nbx + bx;
      if (tid == 0) {
        float t = 0.f;
        for (int w = 0; w < FF_NW; ++w) t += s_mse[w];
        part_mse[pb] = t;
      }
      if (tid < S1) {
        float a0 = 0.f, a1 = 0.f;
        for (int r = 0; r < FF_ROWS; ++r) {
          a0 += T2[r * FF_LDH + tid];
          a1 += T2[r * FF_LDH + 64 + tid];
        }
        part_min[pb * S1 + tid] = a0;
        part_max[pb * S1 + tid] = a1;
      }
    }
  }
  // ---- backward: head h's hidden dZ, its trunk-L2 share, its trunk-L1 share ------------
  auto& tb = Bd.net[0].L[1];
  auto& ta = Bd.net[0].L[0];
  float* dzh = o0.dz ? o0.dz + zr * Hm : nullptr;
  float* dz2p = h == 0 ? tb.dz : tb.dz2;
  float* dzt2 = dz2p ? dz2p + zr * Hm : nullptr;
  float* dz1p = h == 0 ? ta.dz : ta.dz2;
  float* dzt1 = dz1p ? dz1p + zr * Hm : nullptr;
  {
    f32x4 acc[1][2];
    ff_mma2<1>(Gd, o1.W + (size_t)z * o1.wstride, NCB, bqt, acc);   // K = S + 1 <= 16
    FSTAMP(13);
    ff_pre2<NK>(o0.W + (size_t)z * o0.wstride, NCB, bqt);
    FSTAMP(14);
    ff_epi_bwd(acc, Hm, HB, ZH, dzh, Hm, nrows);
    FSTAMP(15);
  }
  lds_barrier();
  FSTAMP(6);
  {
    f32x4 acc[1][2];
    ff_mma2<NK>(HB, o0.W + (size_t)z * o0.wstride, NCB, bqt, acc);
    ff_pre2<NK>(tb.W + (size_t)z * tb.wstride, NCB, bqt);
    ff_epi_bwd(acc, Hm, HA, Z2, dzt2, Hm, nrows);
  }
  lds_barrier();
  FSTAMP(7);
  {
    f32x4 acc[1][2];
    ff_mma2<NK>(HA, tb.W + (size_t)z * tb.wstride, NCB, bqt, acc);
    ff_epi_bwd(acc, Hm, nullptr, Z1, dzt1, Hm, nrows);
  }
  FSTAMP(8);
}

__global__ __launch_bounds__(FF_NT) void fit_fb_kernel(FitFbArgs args) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  FitK& k = *(FitK*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)args;
  if (k.f.net[0].L[1].dout == 200) fit_fb_body<13>(k, smem);
  else fit_fb_body<16>(k, smem);
}

static_assert(sizeof(FitFbArgs) <= 4096, "fused fit kernarg");

DRPO_API int drpo_ens_fit_fb(const drpo_mlp_fwd_t* f, const drpo_mlp_bwd_t* bd, const drpo_ens_upstream_t* up,
                             const drpo_ens_reduce_t* red_in, drpo_ens_reduce_t* reduce_out, drpo_stream_t stream) {
  DRPO_REQUIRE(f && bd && up && red_in && reduce_out, "drpo_ens_fit_fb: null argument");
  const drpo_mlp_net_t &tr = f->net[0], &h1 = f->net[1], &h2 = f->net[2];
  const int S1 = up->S + 1;
  const int din0 = f->cols[0] + f->cols[1];
  const int H = tr.nl == 2 ? tr.L[1].dout : -1;
  bool ok = f->trunk && f->nnets == 3 && tr.nl == 2 && h1.nl == 2 && h2.nl == 2 && f->cols[2] == 0 &&
            f->cols[0] == up->S && din0 >= 1 && din0 <= 64 && (H == 200 || H == 256) && tr.L[0].dout == H &&
            tr.L[0].din == din0 && tr.L[1].din == H && S1 <= 16 && f->nbatch == up->Z && f->rows == up->b &&
            bd->nbatch == up->Z && bd->rows == up->b && bd->trunk && bd->nnets == 3;
  for (const drpo_mlp_net_t* n : {&h1, &h2})
    ok = ok && n->L[0].din == H && n->L[0].dout == H && n->L[1].din == H && n->L[1].dout == S1 &&
         n->L[0].act == ACT_SILU && n->L[1].act == ACT_NONE;
  ok = ok && tr.L[0].act == ACT_SILU && tr.L[1].act == ACT_SILU;
  for (int j = 0; j < 3; ++j)
    for (int l = 0; l < 2; ++l)
      ok = ok && f->net[j].L[l].W && bd->net[j].L[l].W && bd->net[j].L[l].din == f->net[j].L[l].din &&
           bd->net[j].L[l].dout == f->net[j].L[l].dout;
  ok = ok && bd->net[0].L[0].dz && bd->net[0].L[0].dz2 && bd->net[0].L[1].dz && bd->net[0].L[1].dz2;
  DRPO_REQUIRE(ok, "drpo_ens_fit_fb: needs the ensemble trunk [S+A <= 64 -> H -> H] and two heads [H -> H -> S+1 <= 16] "
                   "(swish, H = 200 | 256) with the split-heads trunk dZ (dz | dz2)");
  DRPO_REQUIRE(up->s && up->t && up->minlv && up->maxlv && up->part && up->b >= 1 && up->Z >= 1 && up->Z <= 256,
               "drpo_ens_fit_fb: bad upstream");
  const int nbx = (int)((up->b + FF_ROWS - 1) / FF_ROWS);
  *reduce_out = *red_in;
  reduce_out->part = up->part;
  reduce_out->nbx = nbx;
  reduce_out->Z = up->Z;
  reduce_out->S1 = S1;
  reduce_out->minlv = up->minlv;
  reduce_out->maxlv = up->maxlv;
  reduce_out->gscale = up->gscale;
  FitFbArgs a{*f, *bd, *up};
  const size_t lds = sizeof(float) * ((size_t)8 * FF_ROWS * FF_LDH + FF_NW * 256);
  fit_fb_kernel<<<dim3((unsigned)nbx, 2, (unsigned)up->Z), FF_NT, lds, (hipStream_t)stream>>>(a);
  DRPO_LAUNCH_CHECK("ens_fit_fb");
  return DRPO_OK;
}
