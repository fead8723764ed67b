// Generic fused MLP kernels for the SAC update and the ensemble fit (mlp() nets of
// src/torch_util.py:190-211; BatchedLinear ensembles of src/dynamics.py:26-52).
//
//  mlp_fwd_kernel   one launch runs a whole net (or a trunk + its heads) for a
//                   16-row tile per 512-thread workgroup, activations kept in
//                   LDS, optional saves of every layer's post-(and pre-)activation
//                   for the backward pass. grid.y = independent nets on the same
//                   input (twin critics), grid.z = ensemble members.
//  mlp_bwd_kernel   fused backward-data: dZ_l = dY_l * act'(saved), dY_{l-1} =
//                   dZ_l W_l through every layer (heads -> summed trunk grad ->
//                   trunk), saving dZ_l for the weight gradients and the input
//                   gradient (e.g. dQ/da for the actor update).
// (the weight gradients dW = dZ^T Y of every layer run in csrc/wgrad.hip)

#include "common.hpp"
#include "critic_rows.hpp"
#include "ens_reduce.hpp"

using namespace drpo;

namespace {

constexpr int FW_NW = 8;              // waves per workgroup (fwd / bwd)
constexpr int FW_NT = FW_NW * 64;
constexpr int FW_ROWS = 16;
constexpr int FW_MAXC = 2;            // 16 column blocks / 8 waves
constexpr int LDH = 264;              // LDS stride for widths <= 256 (== 8 mod 64)
constexpr int MAXL = 3;
constexpr int MAXN = 3;

}  // namespace


// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
#ifdef DRPO_STAMPS
// profiling builds only (profiles/stamps.py): per-workgroup s_memtime stamps
__device__ unsigned long long g_stamps[1 << 16][16];
#define STAMP(i)                                                                                  \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long _t;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    const unsigned _w = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);          \
    if (threadIdx.x == 0 && _w < (1u << 16)) g_stamps[_w][(i)] = _t;                              \
  } while (0)
DRPO_API int drpo_debug_stamps(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16 * (size_t)n);
}
DRPO_API int drpo_debug_stamps_clear() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps)) != hipSuccess) return 1;
  return (int)hipMemset(p, 0, sizeof(g_stamps));
}
// backward stamps: rows 32768.. of the same buffer (the forward's slots stay intact)
#define STAMPW(i)                                                                                 \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long _t;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    const unsigned _w = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);          \
    if (threadIdx.x == 0 && _w < 32768u) g_stamps[32768 + _w][(i)] = _t;                          \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#define STAMPW(i) \
  do {            \
  } while (0)
#endif
template <int ACT, int RB>
__device__ __forceinline__ void run_layer_act(const float* in, int ldi, const drpo_mlp_layer_t& L, const float* W,
                                              const float* b, float* out, int ldo, float* red, const GSave& gs) {
  if (L.dout <= 16)
    tile_dense_narrow<FW_NW, RB, ACT>(in, ldi, L.din, W, b, L.dout, out, ldo, red, gs);
  else
    tile_dense<FW_NW, RB, FW_MAXC, ACT>(in, ldi, L.din, W, b, L.dout, out, ldo, gs);
}

// one layer of a (16*RB)-row tile: packed weights of batch item z, bias, activation,
// optional global saves of the post-/pre-activation for the backward pass
template <int RB = 1>
__device__ __forceinline__ void run_layer(const float* in, int ldi, const drpo_mlp_layer_t& __restrict__ L, int z, int64_t rows,
                                          int row0, int nrows, float* out, float* red, bool save = true) {
  const float* W = L.W + (size_t)z * L.wstride;
  const float* b = L.b + (size_t)z * L.bstride;
  const size_t so = ((size_t)z * rows + row0) * L.dout;
  GSave gs{save && L.sy ? L.sy + so : nullptr, save && L.sz ? L.sz + so : nullptr, L.dout, nrows};
  switch (L.act) {
    case ACT_RELU: run_layer_act<ACT_RELU, RB>(in, LDH, L, W, b, out, LDH, red, gs); break;
    case ACT_SILU: run_layer_act<ACT_SILU, RB>(in, LDH, L, W, b, out, LDH, red, gs); break;
    case ACT_TANH: run_layer_act<ACT_TANH, RB>(in, LDH, L, W, b, out, LDH, red, gs); break;
    default: run_layer_act<ACT_NONE, RB>(in, LDH, L, W, b, out, LDH, red, gs); break;
  }
  (void)ldi;
}

// Runs net NI's layers (compile-time net and layer indices: runtime indexing into
// the by-value kernarg struct would force a private-memory copy); returns the LDS
// buffer holding the final activation.
template <int NI>
__device__ __forceinline__ float* run_net(const drpo_mlp_fwd_t& a, float* in, float* bufA, float* bufB, int z, int row0, int nrows,
                          float* red, bool save = true) {
  float* cur = in;
#pragma unroll
  for (int l = 0; l < MAXL; ++l) {
    if (l < a.net[NI].nl) {
      float* out = (cur == bufA) ? bufB : bufA;
      run_layer(cur, LDH, a.net[NI].L[l], z, a.rows, row0, nrows, out, red, save);
      lds_barrier();
      STAMP(2 + 4 * NI + l);
      cur = out;
    }
  }
  return cur;
}

__global__ __launch_bounds__(FW_NT) void mlp_fwd_kernel(drpo_mlp_fwd_t a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* xin = smem;                       // ROWS x LDH
  float* bA = xin + FW_ROWS * LDH;
  float* bB = bA + FW_ROWS * LDH;
  float* T = bB + FW_ROWS * LDH;           // trunk output (trunk mode)
  float* red = T + FW_ROWS * LDH;          // FW_NW * 256
  const int tid = threadIdx.x;
  const LogicalBlock lb = xcd_block();   // one member's tiles per XCD (shared weights in L2)
  const int z = lb.z;
  const int row0 = lb.x * FW_ROWS;
  if (row0 >= a.rows) return;
  const int nrows = (int)min((int64_t)FW_ROWS, a.rows - row0);
  const int din0 = a.cols[0] + a.cols[1] + a.cols[2];
  const int kpad = round_up(din0, 16);
  // split heads: this workgroup runs the trunk and head lb.y + 1; only head 1's
  // workgroup writes the trunk-side saves
  const bool split = a.trunk && a.split_heads;
  const bool tsave = !split || lb.y == 0;
  STAMP(0);
  stage_input_tile<FW_NT>(xin, LDH, FW_ROWS, nrows, row0, kpad, a.src[0] + (size_t)z * a.sstride[0],
                          a.cols[1] ? a.src[1] + (size_t)z * a.sstride[1] : nullptr,
                          a.cols[2] ? a.src[2] + (size_t)z * a.sstride[2] : nullptr, a.cols[0], a.cols[1], a.cols[2],
                          a.ld[0], a.ld[1], a.ld[2], a.nmean, a.nstd, false, tsave ? a.save_x : nullptr,
                          (int64_t)z * a.rows + row0);
  lds_barrier();
  STAMP(1);
  if (!a.trunk) {
    if (lb.y == 0) run_net<0>(a, xin, bA, bB, z, row0, nrows, red);
    else if (lb.y == 1) run_net<1>(a, xin, bA, bB, z, row0, nrows, red);
    else run_net<2>(a, xin, bA, bB, z, row0, nrows, red);
  } else if (split) {
    // the trunk output buffer and the (consumed) input tile are the head's ping-pong pair
    float* t = run_net<0>(a, xin, bA, bB, z, row0, nrows, red, tsave);
    if (lb.y == 0) run_net<1>(a, t, t, xin, z, row0, nrows, red);
    else run_net<2>(a, t, t, xin, z, row0, nrows, red);
  } else {
    float* t = run_net<0>(a, xin, bA, bB, z, row0, nrows, red);
    // move the trunk output out of the ping-pong pair
    const int w = a.net[0].L[a.net[0].nl - 1].dout;
    const int wpad = round_up(w, 16);
    for (int e = tid; e < FW_ROWS * wpad; e += FW_NT) {
      const int r = e / wpad, k = e - r * wpad;
      T[r * LDH + k] = t[r * LDH + k];
    }
    lds_barrier();
    if (a.nnets > 1) run_net<1>(a, T, bA, bB, z, row0, nrows, red);
    if (a.nnets > 2) run_net<2>(a, T, bA, bB, z, row0, nrows, red);
  }
}

static size_t fwd_lds() { return sizeof(float) * ((size_t)4 * FW_ROWS * LDH + FW_NW * 256); }

static int check_net(const drpo_mlp_net_t& n, int din) {
  if (n.nl < 1 || n.nl > MAXL) return 0;
  for (int l = 0; l < n.nl; ++l) {
    if (n.L[l].din != din || n.L[l].dout < 1 || n.L[l].dout > 256 || !n.L[l].W) return 0;
    din = n.L[l].dout;
  }
  return 1;
}

// ---------------------------------------------------------------------------
// multi-job forward: several independent forwards in one launch
// ---------------------------------------------------------------------------
// Job descriptors live in device memory (built once per workspace layout and read
// with scalar loads), grid.y enumerates (job, net) slots, grid.x row tiles. The
// latency chain of one 16-row tile (stage -> layer -> layer -> ...) is serial, so
// running e.g. the actor, safe actor, twin critics and constraint critic of one
// SAC loss in one launch puts 4 such chains on every CU at once.
namespace {
constexpr int MJ_MAXSLOT = 16;
}
struct MultiArgs {
  const drpo_mlp_fwd_t* jobs;
  unsigned char slot_job[MJ_MAXSLOT], slot_net[MJ_MAXSLOT];
  uint64_t seed, ctr;
};

__device__ __forceinline__ GSave layer_save(const drpo_mlp_layer_t& L, int z, int64_t rows, int row0, int nrows) {
  const size_t so = ((size_t)z * rows + row0) * L.dout;
  return GSave{L.sy ? L.sy + so : nullptr, L.sz ? L.sz + so : nullptr, L.dout, nrows};
}

template <int RB>
__device__ __forceinline__ float* run_net_g(const drpo_mlp_net_t& __restrict__ n, int64_t rows, float* in, float* bufA,
                                            float* bufB, int z, int row0, int nrows, float* red) {
  float* cur = in;
  const int nl = n.nl;
  for (int l = 0; l < nl; ++l) {
    float* out = (cur == bufA) ? bufB : bufA;
    const drpo_mlp_layer_t& L = n.L[l];
    const GSave gs = layer_save(L, z, rows, row0, nrows);
    const bool defer = save_deferrable(gs.gy, gs.gz, L.dout);
    run_layer<RB>(cur, LDH, L, z, rows, row0, nrows, out, red, !defer);
    lds_barrier();
    if (defer) save_tile_lds<FW_NT, 16 * RB>(out, LDH, gs.gy, L.dout, nrows);
    STAMP(2 + l);
    cur = out;
  }
  return cur;
}

// Trunk-mode job whose two heads are [256 -> N, act0] -> [N -> n<=16, act1] each (the
// constraint critic's mean and log-std heads, src/ssac.py:46-92): both heads' hidden
// layers run as ONE paired layer over the trunk output (2N output columns, one
// k-loop) and both output layers as one split-K narrow pair, so the job's serial
// chain is 4 layers instead of 6.
__device__ __forceinline__ bool heads_pairable(const drpo_mlp_fwd_t* __restrict__ a) {
  if (a->nnets != 3) return false;
  const drpo_mlp_net_t& n1 = a->net[1];
  const drpo_mlp_net_t& n2 = a->net[2];
  return n1.nl == 2 && n2.nl == 2 && n1.L[0].din == 256 && n2.L[0].din == 256 && n1.L[0].dout == n2.L[0].dout &&
         n1.L[0].act == n2.L[0].act && n1.L[1].act == n2.L[1].act && n1.L[1].dout <= 16 && n2.L[1].dout <= 16;
}


template <int RB, int ACT0, int ACT1>
__device__ __forceinline__ void heads_pair_act(const drpo_mlp_fwd_t* __restrict__ a, const float* T, float* hA,
                                               float* hB, float* o, int z, int row0, int nrows, float* red) {
  const drpo_mlp_layer_t& A0 = a->net[1].L[0];
  const drpo_mlp_layer_t& B0 = a->net[2].L[0];
  const drpo_mlp_layer_t& A1 = a->net[1].L[1];
  const drpo_mlp_layer_t& B1 = a->net[2].L[1];
  // (saves from the epilogue: deferring them to 16-byte stores after the barrier, as
  // run_net_g does, spilled 60 VGPRs in this paired layer, profiles/r05/defer_saves)
  tile_dense_pair<FW_NW, RB, 4, ACT0, 16, 2>(T, LDH, 256, A0.W + (size_t)z * A0.wstride, A0.b + (size_t)z * A0.bstride,
                                          A0.dout, hA, B0.W + (size_t)z * B0.wstride, B0.b + (size_t)z * B0.bstride,
                                          B0.dout, hB, LDH, layer_save(A0, z, a->rows, row0, nrows),
                                          layer_save(B0, z, a->rows, row0, nrows));
  lds_barrier();
  STAMP(5);
  tile_dense_narrow_pair<FW_NW, RB, ACT1>(hA, hB, LDH, A0.dout, A1.W + (size_t)z * A1.wstride,
                                          A1.b + (size_t)z * A1.bstride, A1.dout, o, B1.W + (size_t)z * B1.wstride,
                                          B1.b + (size_t)z * B1.bstride, B1.dout, o + 16, LDH, red,
                                          layer_save(A1, z, a->rows, row0, nrows),
                                          layer_save(B1, z, a->rows, row0, nrows));
}

template <int RB, int ACT0>
__device__ __forceinline__ void heads_pair_act0(const drpo_mlp_fwd_t* __restrict__ a, const float* T, float* hA,
                                                float* hB, float* o, int z, int row0, int nrows, float* red) {
  switch (a->net[1].L[1].act) {
    case ACT_RELU: heads_pair_act<RB, ACT0, ACT_RELU>(a, T, hA, hB, o, z, row0, nrows, red); break;
    case ACT_SILU: heads_pair_act<RB, ACT0, ACT_SILU>(a, T, hA, hB, o, z, row0, nrows, red); break;
    case ACT_TANH: heads_pair_act<RB, ACT0, ACT_TANH>(a, T, hA, hB, o, z, row0, nrows, red); break;
    default: heads_pair_act<RB, ACT0, ACT_NONE>(a, T, hA, hB, o, z, row0, nrows, red); break;
  }
}

template <int RB>
__device__ __forceinline__ void heads_pair(const drpo_mlp_fwd_t* __restrict__ a, const float* T, float* hA, float* hB,
                                           float* o, int z, int row0, int nrows, float* red) {
  switch (a->net[1].L[0].act) {
    case ACT_RELU: heads_pair_act0<RB, ACT_RELU>(a, T, hA, hB, o, z, row0, nrows, red); break;
    case ACT_SILU: heads_pair_act0<RB, ACT_SILU>(a, T, hA, hB, o, z, row0, nrows, red); break;
    case ACT_TANH: heads_pair_act0<RB, ACT_TANH>(a, T, hA, hB, o, z, row0, nrows, red); break;
    default: heads_pair_act0<RB, ACT_NONE>(a, T, hA, hB, o, z, row0, nrows, red); break;
  }
}

// The fused squashed-Gaussian head of a policy job (squashed_gaussian_row's arithmetic,
// src/policy.py:88-97, src/squashed_gaussian.py): one thread per (row, action dim)
// instead of one per row, on the hardware transcendentals of critic_rows.hpp
// (~1e-6 relative), log(std) taken as the log-std itself (the
// reference's log(exp(log_std))); the per-dim log-prob terms are summed per row in
// dimension order through LDS (lpt). The per-row libm chain it replaces was 5.6-8 k
// cycles at the end of every policy workgroup (profiles/r05/sac_fwd_stamps).
template <int ROWS>
__device__ __forceinline__ void squash_head_tile(const float* outp, int row0, int nrows, const drpo_policy_head_t& hd,
                                                 uint64_t seed, uint64_t ctr, float* lpt, float* a_lds = nullptr) {
  const int A = hd.A, mode = hd.mode - 1;
  const int tid = threadIdx.x;
  if (tid < ROWS * A) {   // ROWS * A <= ROWS * 8 <= FW_NT
    const int r = tid / A, d = tid - r * A;
    float term = 0.f;
    if (r < nrows) {
      const int64_t i = row0 + r, k = i * A + d;
      const float* rrow = outp + r * LDH;
      const float mu = rrow[d];
      const float ls = -6.f + 10.f * cr_rcp(1.f + cr_exp(-rrow[A + d]));
      const float sd = cr_exp(ls) * 1.0f;
      if (hd.amean) gstore(hd.amean + k, fast_tanh(mu));
      if (mode != 2) {
        const float e = normal_at(hd.eps, k, seed, ctr, hd.site);
        const float u = (mode == 0) ? e * sd + mu : mu + e * sd;
        const float act = fast_tanh(u);
        if (hd.a) gstore(hd.a + k, act);
        if (a_lds) a_lds[r * LDH + d] = act;   // chain: the action as the next net's input columns
        if (hd.u) gstore(hd.u + k, u);
        if (hd.e) gstore(hd.e + k, e);
        const float ladj = 2.f * (0.69314718055994531f - u - cr_softplus(-2.f * u));
        const float base = -((u - mu) * (u - mu)) * cr_rcp(2.f * (sd * sd)) - ls - 0.91893853320467274f;
        term = (0.f - ladj) + base;
      }
    }
    lpt[tid] = term;
  }
  if (hd.logp && mode != 2) {
    lds_barrier();
    if (tid < nrows) {
      float lp = 0.f;
      for (int d = 0; d < A; ++d) lp += lpt[tid * A + d];
      gstore(hd.logp + row0 + tid, lp);
    }
  }
}

// A pair job (drpo_mlp_fwd_t.pair): two 3-layer ReLU nets of one shape on the same input
// -- the twin critics, the actor and the safe actor -- run by ONE workgroup: waves 0-3
// run net 0's layers, waves 4-7 net 1's (4 column blocks each of a 256-wide layer, so
// every SIMD carries one wave of each net: balanced), the narrow output layers as one
// split-K pair. One staging and one chain of three phases instead of two workgroups each
// staging the input and running three phases (forward stamps: staging + first layer +
// narrow layer are ~15-20 k cycles of each such workgroup, profiles/r05/sac_fwd_stamps).
// Buffers: in -> (bA, bB) -> (in, T) -> bA columns [0, 16) (net 0) and [16, 32) (net 1).
template <int RB, int NK0>
__device__ __forceinline__ void pair_nets_nk(const drpo_mlp_net_t& A, const drpo_mlp_net_t& B, int64_t rows, float* in,
                                             float* bA, float* bB, float* T, int z, int row0, int nrows, float* red) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool second = wave >= FW_NW / 2;
  const int wl = second ? wave - FW_NW / 2 : wave;
  const drpo_mlp_net_t& N = second ? B : A;
  auto W = [&](const drpo_mlp_layer_t& L) { return L.W + (size_t)z * L.wstride; };
  auto bb = [&](const drpo_mlp_layer_t& L) { return L.b + (size_t)z * L.bstride; };
  const drpo_mlp_layer_t &L0 = N.L[0], &L1 = N.L[1];
  // (saves from the epilogue: deferred 16-byte saves measured 2 us slower here,
  // profiles/r05/defer_saves)
  tile_dense_core<FW_NW / 2, RB, 4, ACT_RELU, NK0, 0, 2>(in, LDH, L0.din, W(L0), bb(L0), L0.dout, second ? bB : bA,
                                                         LDH, layer_save(L0, z, rows, row0, nrows), nullptr, wl);
  lds_barrier();
  STAMP(2);
  tile_dense_core<FW_NW / 2, RB, 4, ACT_RELU, 16, 0, 2>(second ? bB : bA, LDH, 256, W(L1), bb(L1), L1.dout,
                                                        second ? T : in, LDH, layer_save(L1, z, rows, row0, nrows),
                                                        nullptr, wl);
  lds_barrier();
  STAMP(3);
  const drpo_mlp_layer_t &A2 = A.L[2], &B2 = B.L[2];
  tile_dense_narrow_pair<FW_NW, RB, ACT_NONE>(in, T, LDH, A2.din, W(A2), bb(A2), A2.dout, bA, W(B2), bb(B2), B2.dout,
                                              bA + 16, LDH, red, layer_save(A2, z, rows, row0, nrows),
                                              layer_save(B2, z, rows, row0, nrows));
  lds_barrier();
  STAMP(4);
}

template <int RB>
__device__ __forceinline__ void pair_nets(const drpo_mlp_net_t& A, const drpo_mlp_net_t& B, int64_t rows, float* in,
                                          float* bA, float* bB, float* T, int z, int row0, int nrows, float* red) {
  if (A.L[0].din <= 16) pair_nets_nk<RB, 1>(A, B, rows, in, bA, bB, T, z, row0, nrows, red);
  else pair_nets_nk<RB, 4>(A, B, rows, in, bA, bB, T, z, row0, nrows, red);
}

// host-side shape check of a pair job (the kernel's pair_nets assumptions)
static int pair_ok(const drpo_mlp_fwd_t* a) {
  if (a->trunk || a->nnets != 2) return 0;
  const drpo_mlp_net_t &A = a->net[0], &B = a->net[1];
  if (A.nl != 3 || B.nl != 3) return 0;
  for (int l = 0; l < 3; ++l)
    if (A.L[l].din != B.L[l].din || A.L[l].dout != B.L[l].dout || A.L[l].act != B.L[l].act) return 0;
  const int k0 = (A.L[0].din + 15) >> 4;
  return (k0 == 1 || k0 == 4) && A.L[0].dout == 256 && A.L[1].din == 256 && A.L[1].dout == 256 &&
         A.L[2].dout <= 16 && A.L[0].act == ACT_RELU && A.L[1].act == ACT_RELU && A.L[2].act == ACT_NONE;
}

template <int RB>
__global__ __launch_bounds__(FW_NT) __attribute__((amdgpu_waves_per_eu(RB == 1 ? 4 : 2, RB == 1 ? 4 : 2))) void mlp_fwd_multi_kernel(MultiArgs m) {
  constexpr int ROWS = 16 * RB;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* xin = smem;
  float* bA = xin + ROWS * LDH;
  float* bB = bA + ROWS * LDH;
  float* T = bB + ROWS * LDH;
  float* red = T + ROWS * LDH;
  const drpo_mlp_fwd_t* __restrict__ a = m.jobs + m.slot_job[blockIdx.y];
  const int net = m.slot_net[blockIdx.y];
  const int tid = threadIdx.x;
  const int z = blockIdx.z;
  const int row0 = blockIdx.x * ROWS;
  if (row0 >= a->rows || z >= a->nbatch) return;
  const int nrows = (int)min((int64_t)ROWS, a->rows - row0);
  STAMP(0);
  const int c0 = a->cols[0], c1 = a->cols[1];
  const int din0 = c0 + c1 + a->cols[2];
  const int kpad = round_up(din0, 16);
  // chain jobs: the src[1] block (the action) comes from the pre net's head below
  const bool chain = a->pre.nl > 0;
  const int c2 = a->cols[2];
  stage_input_tile<FW_NT>(xin, LDH, ROWS, nrows, row0, kpad, a->src[0] + (size_t)z * a->sstride[0],
                          (c1 && !chain) ? a->src[1] + (size_t)z * a->sstride[1] : nullptr,
                          c2 ? a->src[2] + (size_t)z * a->sstride[2] : nullptr, c0, c1, c2, a->ld[0], a->ld[1],
                          a->ld[2], a->nmean, a->nstd, chain, a->save_x, (int64_t)z * a->rows + row0);
  lds_barrier();
  STAMP(1);
  if (chain) {
    // the policy on the src[0] columns (its first layer reads the input tile's first K
    // columns; the weights are zero beyond its own K), its sampled action into the input
    // tile's src[1] columns
    const float* po = run_net_g<RB>(a->pre, a->rows, xin, bA, bB, z, row0, nrows, red);
    squash_head_tile<ROWS>(po, row0, nrows, a->pre_head, m.seed, m.ctr, red, xin + c0);
    lds_barrier();
    STAMP(7);
  }
  float* outp;
  float* outp2 = nullptr;
  if (a->pair) {
    pair_nets<RB>(a->net[0], a->net[1], a->rows, xin, bA, bB, T, z, row0, nrows, red);
    outp = bA;
    outp2 = bA + 16;
  } else if (!a->trunk) {
    outp = run_net_g<RB>(a->net[net], a->rows, xin, bA, bB, z, row0, nrows, red);
  } else if (heads_pairable(a)) {
    // trunk output stays where the trunk left it; the paired heads use the two
    // other full buffers and write their narrow outputs into xin (consumed)
    float* t = run_net_g<RB>(a->net[0], a->rows, xin, bA, bB, z, row0, nrows, red);
    outp = nullptr;
    heads_pair<RB>(a, t, T, t == bA ? bB : bA, xin, z, row0, nrows, red);
    STAMP(6);
    if (a->ccb_out) {
      // the constraint critic's upper bound, max over C (drpo_cc_head), from the heads'
      // outputs in LDS (mean head: xin columns 0.., log-std head: columns 16..)
      lds_barrier();
      if (tid < nrows) {
        const int C = a->net[1].L[1].dout;
        const float* rowp = xin + tid * LDH;
        float best = 0.f;
        for (int c = 0; c < C; ++c) {
          float v = rowp[c];
          if (a->ccb_dist) v = v + a->ccb_ratio * cc_std(rowp[16 + c], a->ccb_lmin, a->ccb_lmax);
          if (c == 0 || v > best) best = v;
        }
        a->ccb_out[(size_t)z * a->rows + row0 + tid] = best;
        if (a->post.nl > 0) {   // the post chain's bound column (and its input save)
          T[tid * LDH + c0] = best;
          if (a->post_x) a->post_x[((size_t)z * a->rows + row0 + tid) * (c0 + 1) + c0] = best;
        }
      }
      if (a->post.nl > 0) {
        // post chain: the multiplier on [s, bound] (src/ssac.py:473-478,548-552) in this
        // workgroup; its input assembled in T (the heads' first hidden tile, consumed),
        // the bound's column written above by the thread that formed it
        const int kp = round_up(c0 + 1, 16);
        for (int e = tid; e < ROWS * kp; e += FW_NT) {
          const int r = e / kp, k = e - r * kp;
          if (k == c0) continue;
          const int64_t row = row0 + r;
          float v = 0.f;
          if (r < nrows && k < c0) {
            v = a->src[0][(size_t)z * a->sstride[0] + row * a->ld[0] + k];
            if (a->post_x) a->post_x[((size_t)z * a->rows + row) * (c0 + 1) + k] = v;
          }
          T[r * LDH + k] = v;
        }
        lds_barrier();
        run_net_g<RB>(a->post, a->rows, T, bA, bB, z, row0, nrows, red);
      }
    }
  } else {
    float* t = run_net_g<RB>(a->net[0], a->rows, xin, bA, bB, z, row0, nrows, red);
    const int w = a->net[0].L[a->net[0].nl - 1].dout;
    const int wpad = round_up(w, 16);
    for (int e = tid; e < ROWS * wpad; e += FW_NT) {
      const int r = e / wpad, k = e - r * wpad;
      T[r * LDH + k] = t[r * LDH + k];
    }
    lds_barrier();
    outp = nullptr;
    for (int h = 1; h < a->nnets; ++h) run_net_g<RB>(a->net[h], a->rows, T, bA, bB, z, row0, nrows, red);
  }
  // fused squashed-Gaussian heads on net 0's output (non-trunk jobs) and, for a pair
  // job, on net 1's (head2; its log-prob scratch after head's)
  const drpo_policy_head_t& hd = a->head;
  if (hd.mode != 0 && outp && net == 0) {
    squash_head_tile<ROWS>(outp, row0, nrows, hd, m.seed, m.ctr, red);
  }
  if (outp2 && a->head2.mode != 0) squash_head_tile<ROWS>(outp2, row0, nrows, a->head2, m.seed, m.ctr, red + ROWS * 8);
  STAMP(15);
}

DRPO_API int drpo_mlp_forward_multi(const drpo_mlp_fwd_t* jobs_host, const drpo_mlp_fwd_t* jobs_dev, int njobs,
                                    uint64_t seed, uint64_t ctr, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(jobs_host && jobs_dev && njobs >= 1 && njobs <= 8, "drpo_mlp_forward_multi: 1..8 jobs");
  MultiArgs m{};
  m.jobs = jobs_dev;
  m.seed = seed;
  m.ctr = ctr;
  int slots = 0;
  int64_t tiles = 0;
  int nbatch = 1;
  for (int j = 0; j < njobs; ++j) {
    const drpo_mlp_fwd_t* a = jobs_host + j;
    DRPO_REQUIRE(a->nnets >= 1 && a->nnets <= MAXN && a->nbatch >= 1 && !a->split_heads,
                 "drpo_mlp_forward_multi: bad job %d", j);
    const int din0 = a->cols[0] + a->cols[1] + a->cols[2];
    DRPO_REQUIRE(din0 >= 1 && din0 <= 256, "drpo_mlp_forward_multi: job %d input width %d", j, din0);
    if (a->trunk) {
      DRPO_REQUIRE(check_net(a->net[0], din0), "drpo_mlp_forward_multi: job %d bad trunk", j);
      const int tw = a->net[0].L[a->net[0].nl - 1].dout;
      for (int h = 1; h < a->nnets; ++h)
        DRPO_REQUIRE(check_net(a->net[h], tw), "drpo_mlp_forward_multi: job %d bad head %d", j, h);
      DRPO_REQUIRE(a->head.mode == 0, "drpo_mlp_forward_multi: policy head on a trunk job");
    } else {
      for (int h = 0; h < a->nnets; ++h)
        DRPO_REQUIRE(check_net(a->net[h], din0), "drpo_mlp_forward_multi: job %d bad net %d", j, h);
    }
    if (a->head.mode != 0)
      DRPO_REQUIRE(a->head.mode <= 3 && a->head.A >= 1 && a->head.A <= 8 &&
                       2 * a->head.A == a->net[0].L[a->net[0].nl - 1].dout,
                   "drpo_mlp_forward_multi: job %d policy head shape", j);
    if (a->pair) {
      DRPO_REQUIRE(pair_ok(a), "drpo_mlp_forward_multi: job %d: a pair job needs two 3-layer ReLU nets of one shape "
                               "[K <= 16 or 49..64 -> 256 -> 256 -> <= 16]", j);
      if (a->head2.mode != 0)
        DRPO_REQUIRE(a->head2.mode <= 3 && a->head2.A >= 1 && a->head2.A <= 8 &&
                         2 * a->head2.A == a->net[1].L[2].dout,
                     "drpo_mlp_forward_multi: job %d second policy head shape", j);
    } else {
      DRPO_REQUIRE(a->head2.mode == 0, "drpo_mlp_forward_multi: job %d: head2 needs a pair job", j);
    }
    if (a->pre.nl > 0) {
      const drpo_mlp_net_t& pn = a->pre;
      DRPO_REQUIRE(check_net(pn, a->cols[0]) && (a->pre_head.mode == 1 || a->pre_head.mode == 2) &&
                       a->pre_head.A == a->cols[1] && a->pre_head.A >= 1 && a->pre_head.A <= 8 &&
                       2 * a->pre_head.A == pn.L[pn.nl - 1].dout && !a->save_x && !a->nmean,
                   "drpo_mlp_forward_multi: job %d: a chain needs a policy net on the src[0] columns whose sampled "
                   "action is the src[1] block (no input save / normalizer)", j);
    }
    if (a->ccb_out) {   // the same conditions as heads_pairable (device side)
      const drpo_mlp_net_t &n1 = a->net[1], &n2 = a->net[2];
      DRPO_REQUIRE(a->trunk && a->nnets == 3 && n1.nl == 2 && n2.nl == 2 && n1.L[0].din == 256 &&
                       n2.L[0].din == 256 && n1.L[0].dout == n2.L[0].dout && n1.L[0].act == n2.L[0].act &&
                       n1.L[1].act == n2.L[1].act && n1.L[1].dout <= 16 && n2.L[1].dout <= 16,
                   "drpo_mlp_forward_multi: job %d: the constraint bound needs a trunk job with paired heads", j);
    }
    if (a->post.nl > 0) {
      const drpo_mlp_net_t& pn = a->post;
      DRPO_REQUIRE(a->ccb_out && a->cols[0] + 1 <= 64 && check_net(pn, a->cols[0] + 1) && !a->nmean,
                   "drpo_mlp_forward_multi: job %d: a post chain needs the job's constraint bound (ccb_out) and a "
                   "net on [src[0] (<= 63 columns), bound]", j);
    } else {
      DRPO_REQUIRE(!a->post_x, "drpo_mlp_forward_multi: job %d: post_x without a post net", j);
    }
    const int ns = (a->trunk || a->pair) ? 1 : a->nnets;
    DRPO_REQUIRE(slots + ns <= MJ_MAXSLOT, "drpo_mlp_forward_multi: too many nets");
    for (int h = 0; h < ns; ++h) {
      m.slot_job[slots] = (unsigned char)j;
      m.slot_net[slots] = (unsigned char)h;
      ++slots;
    }
    tiles = max(tiles, (a->rows + FW_ROWS - 1) / FW_ROWS);
    nbatch = max(nbatch, a->nbatch);
  }
  if (tiles == 0) return DRPO_OK;
  // 32-row tiles halve the weight bytes per MFMA but allow only one 8-wave workgroup
  // per CU (LDS); measured slower at B=4096 (profiles/r01, profiles/r04/bench_stats), so
  // only for launches with >= 8 workgroups per CU at 16-row tiles
  if (tiles * slots * nbatch >= 2048) {
    const size_t lds = sizeof(float) * ((size_t)4 * 2 * FW_ROWS * LDH + FW_NW * 2 * 256);
    mlp_fwd_multi_kernel<2><<<dim3((unsigned)((tiles + 1) / 2), slots, nbatch), FW_NT, lds, stream>>>(m);
  } else {
    mlp_fwd_multi_kernel<1><<<dim3((unsigned)tiles, slots, nbatch), FW_NT, fwd_lds(), stream>>>(m);
  }
  DRPO_LAUNCH_CHECK("mlp_forward_multi");
  return DRPO_OK;
}


DRPO_API int drpo_mlp_forward(const drpo_mlp_fwd_t* a, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(a && a->nnets >= 1 && a->nnets <= MAXN && a->nbatch >= 1, "drpo_mlp_forward: bad descriptor");
  const int din0 = a->cols[0] + a->cols[1] + a->cols[2];
  DRPO_REQUIRE(din0 >= 1 && din0 <= 256, "drpo_mlp_forward: input width %d", din0);
  if (a->trunk) {
    DRPO_REQUIRE(check_net(a->net[0], din0), "drpo_mlp_forward: bad trunk");
    const int tw = a->net[0].L[a->net[0].nl - 1].dout;
    for (int h = 1; h < a->nnets; ++h) DRPO_REQUIRE(check_net(a->net[h], tw), "drpo_mlp_forward: bad head %d", h);
  } else {
    for (int h = 0; h < a->nnets; ++h) DRPO_REQUIRE(check_net(a->net[h], din0), "drpo_mlp_forward: bad net %d", h);
  }
  if (a->rows == 0) return DRPO_OK;
  DRPO_REQUIRE(!a->split_heads || (a->trunk && a->nnets >= 2), "drpo_mlp_forward: split_heads needs a trunk + heads");
  dim3 grid((unsigned)((a->rows + FW_ROWS - 1) / FW_ROWS),
            a->trunk ? (a->split_heads ? a->nnets - 1 : 1) : a->nnets, a->nbatch);
  mlp_fwd_kernel<<<grid, FW_NT, fwd_lds(), stream>>>(*a);
  DRPO_LAUNCH_CHECK("mlp_forward");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// backward-data
// ---------------------------------------------------------------------------
__device__ __forceinline__ float act_grad(int act, float y, float z) {
  switch (act) {
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_TANH: return 1.f - y * y;
    case ACT_SILU: {
      const float s = fast_sigmoid(z);
      return s * (1.f + z * (1.f - s));
    }
    default: return 1.f;
  }
}

// The one saved value act_grad reads for layer L (post-activation y for relu / tanh,
// pre-activation z for swish), 8 elements per thread of the tile's [16][wpad] grid,
// loaded into registers one layer AHEAD: issued before the previous layer's
// backward GEMM, they arrive while it runs instead of stalling the elementwise phase.
constexpr int BW_PER = FW_ROWS * 256 / FW_NT;   // 8 elements per thread (widths <= 256)

__device__ __forceinline__ void bwd_fetch_act(const drpo_mlp_bwd_layer_t& __restrict__ L, int z, int64_t rows,
                                              int row0, int nrows, float (&v)[BW_PER]) {
  const int tid = threadIdx.x;
  const int dout = L.dout, act = L.act;
  const float* __restrict__ src = act == ACT_SILU ? L.sz : L.sy;
  const size_t so = ((size_t)z * rows + row0) * dout;
  const int wpad = round_up(dout, 16);
#pragma unroll
  for (int i = 0; i < BW_PER; ++i) {
    const int e = tid + i * FW_NT;
    const int r = e / wpad, k = e - r * wpad;
    v[i] = (act != ACT_NONE && src && e < FW_ROWS * wpad && r < nrows && k < dout)
               ? gload(src + so + (size_t)r * dout + k) : 0.f;
  }
}

__device__ __forceinline__ float act_grad_saved(int act, float saved) {
  return act == ACT_SILU ? act_grad(act, 0.f, saved) : act_grad(act, saved, 0.f);
}

// G (LDS, width of the net output) -> gradient w.r.t. the net input (returned LDS buffer)
__device__ __forceinline__ float* bwd_net(const drpo_mlp_bwd_net_t& __restrict__ net, float* G, float* bA, float* bB, int z, int64_t rows,
                          int row0, int nrows, bool need_dx0, bool alt = false) {
  const int tid = threadIdx.x;
  float* cur = G;
  float sv[BW_PER];
  bwd_fetch_act(net.L[net.nl - 1], z, rows, row0, nrows, sv);
  for (int l = net.nl - 1; l >= 0; --l) {
    const drpo_mlp_bwd_layer_t& L = net.L[l];
    // descriptor fields into registers once per layer (no reloads inside the loops)
    const int dout = L.dout, din = L.din, act = L.act;
    float* __restrict__ dzp = alt ? L.dz2 : L.dz;
    const float* W = L.W + (size_t)z * L.wstride;
    const size_t so = ((size_t)z * rows + row0) * dout;
    const int wpad = round_up(dout, 16);
#pragma unroll
    for (int i = 0; i < BW_PER; ++i) {
      const int e = tid + i * FW_NT;
      if (e >= FW_ROWS * wpad) break;
      const int r = e / wpad, k = e - r * wpad;
      float g = 0.f;
      if (r < nrows && k < dout) {
        g = cur[r * LDH + k];
        if (act != ACT_NONE) g *= act_grad_saved(act, sv[i]);
        if (dzp) gstore(dzp + so + (size_t)r * dout + k, g);
      }
      cur[r * LDH + k] = g;
    }
    lds_barrier();
    if (l == 0 && !need_dx0) return nullptr;   // input gradient not wanted: dZ_0 (saved) is all wgrad needs
    if (l > 0) bwd_fetch_act(net.L[l - 1], z, rows, row0, nrows, sv);   // next layer's, during this GEMM
    float* out = (cur == bA) ? bB : bA;
    // dY_prev = dZ W: transposed mirror, N = din, K = dout
    tile_dense<FW_NW, 1, FW_MAXC, ACT_NONE>(cur, LDH, dout, W, nullptr, din, out, LDH);
    lds_barrier();
    cur = out;
  }
  return cur;
}

// Two heads of the same shape on a shared trunk (the dynamics model's diff / log-var
// heads, src/dynamics.py:84-91; the constraint critic's mean / log-std heads,
// src/ssac.py:46-92), each [trunk width -> H -> out] with an identity output layer:
// backed through TOGETHER. Their output layers' products run side by side (one
// two-input pair layer), and the trunk-output gradient -- the sum of the two heads'
// hidden-layer products -- is ONE product with the concatenated K (dZ_1 | dZ_2) x
// [W_1; W_2]: three dependent GEMM phases instead of five, and no LDS accumulation.
__device__ __forceinline__ bool bwd_paired_heads(const drpo_mlp_bwd_t& a) {
  if (!a.trunk || a.split_heads || a.nnets != 3) return false;
  const drpo_mlp_bwd_net_t &h1 = a.net[1], &h2 = a.net[2];
  if (h1.nl != 2 || h2.nl != 2 || h1.dx || h2.dx) return false;
  for (int l = 0; l < 2; ++l)
    if (h1.L[l].din != h2.L[l].din || h1.L[l].dout != h2.L[l].dout || h1.L[l].act != h2.L[l].act) return false;
  const int hid = h1.L[0].dout, out = h1.L[1].dout;
  return h1.L[1].act == ACT_NONE && (hid == 200 || hid == 256) && out <= 64 && h1.L[0].din <= 256;
}

template <int NK>
__device__ __forceinline__ void bwd_heads_catk(const drpo_mlp_bwd_net_t& h1, const drpo_mlp_bwd_net_t& h2, const float* D1,
                                               const float* D2, float* out, int z) {
  tile_dense_catk<FW_NW, 1, FW_MAXC, ACT_NONE, NK>(D1, D2, LDH, h1.L[0].W + (size_t)z * h1.L[0].wstride,
                                                   h2.L[0].W + (size_t)z * h2.L[0].wstride, nullptr, h1.L[0].din, out,
                                                   LDH);
}

template <int NK>
__device__ __forceinline__ void bwd_heads_out(const drpo_mlp_bwd_net_t& h1, const drpo_mlp_bwd_net_t& h2, const float* G1,
                                              const float* G2, float* o1, float* o2, int z) {
  const int hid = h1.L[1].din;
  tile_dense_pair2<FW_NW, 1, 4, ACT_NONE, NK, 2>(G1, G2, LDH, h1.L[1].W + (size_t)z * h1.L[1].wstride, nullptr, hid, o1,
                                              h2.L[1].W + (size_t)z * h2.L[1].wstride, nullptr, hid, o2, LDH);
}

// the critic head of a drpo_mlp_backward_multi_head launch, read in place from the
// kernarg segment (scalar loads; taking a generic address of the by-value argument
// would copy it to scratch)
typedef const __attribute__((address_space(4))) drpo_critic_head_t CriticHeadK;

// a loss partial of every thread of the workgroup -> the workgroup's sum written to
// *dst (one slot per workgroup, no atomics; waves summed in order; every thread calls)
__device__ __forceinline__ void wg_loss_partial(float v, float* dst) {
  __shared__ float s_wl[FW_NW];
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) s_wl[threadIdx.x >> 6] = v;
  lds_barrier();
  if (threadIdx.x == 0) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < FW_NW; ++w) t += s_wl[w];
    *dst = t;
  }
}

// DRPO_UPSTREAM_CERT: the certificate loss gradients of rows [row0, row0+nrows)
// (cert_element, src/ssac.py:304-435) as the mean / log-std heads' output gradients:
// dmu -> Gm, dls -> Gl (LDS, width padded to 16; either may be NULL: the generic trunk
// path takes one head at a time), saved as that head's output-layer dZ; with add_loss
// the loss term is accumulated into head->loss[1]
__device__ __forceinline__ void cert_upstream(CriticHeadK& ch, const drpo_mlp_bwd_net_t* hm,
                                              const drpo_mlp_bwd_net_t* hl, float* Gm, float* Gl, int row0,
                                              int nrows, bool add_loss) {
  const int tiles = (int)((ch.B + FW_ROWS - 1) / FW_ROWS);
  const int C = ch.C, opad = round_up(C, 16);
  float lc = 0.f;
  for (int e = threadIdx.x; e < FW_ROWS * opad; e += FW_NT) {
    const int r = e / opad, k = e - r * opad;
    float dmu = 0.f, dls = 0.f;
    if (r < nrows && k < C) {
      const int64_t i = row0 + r;
      lc += cert_element(ch, i, k, dmu, dls);
      const size_t o = (size_t)i * C + k;
      if (Gm && hm->L[hm->nl - 1].dz) gstore(hm->L[hm->nl - 1].dz + o, dmu);
      if (Gl && hl->L[hl->nl - 1].dz) gstore(hl->L[hl->nl - 1].dz + o, dls);
    }
    if (Gm) Gm[r * LDH + k] = dmu;
    if (Gl) Gl[r * LDH + k] = dls;
  }
  if (add_loss) wg_loss_partial(lc, ch.loss_part + 2 * tiles + row0 / FW_ROWS);
}

// the fit's upstream, read in place from the kernarg segment (see CriticHeadK)
typedef const __attribute__((address_space(4))) drpo_ens_upstream_t EnsUpK;

// DRPO_UPSTREAM_ENS: the heteroscedastic NLL of rows [row0, row0+nrows) of member z
// (drpo_ens_loss's arithmetic, csrc/ensemble.hip; src/dynamics.py:143-153,236-253):
// d loss / d diff-head -> Gd, d loss / d raw log-var -> Gl (+ the output layers' saved
// dZ), and this tile's loss partials (mse, and per column the min / max log-var bound
// gradients) at partial block (z, bx) of the drpo_ens_loss workspace layout. Cm / Cx:
// LDS scratch (16 rows each). Thread t owns column t % 16-padded-width of row t / width,
// the element mapping and summation order of ens_loss_kernel at S+1 <= 16.
// split < 0: both heads (paired backward; the output layers' dZ saved here). split = h
// (split-heads backward, one workgroup per head): the output layers' dZ are saved by the
// head's own backward pass, and only head 0's workgroup writes the loss partials.
__device__ __forceinline__ void ens_upstream(EnsUpK& u, const drpo_mlp_bwd_net_t& hd, const drpo_mlp_bwd_net_t& hl,
                                             float* Gd, float* Gl, float* Cm, float* Cx, int z, int bx, int row0,
                                             int nrows, int split = -1) {
  const int tid = threadIdx.x;
  const int S = u.S, S1 = S + 1, opad = round_up(S1, 16);
  const int64_t b = u.b;
  const float inv_n = 1.f / (float)(b * S1);
  const float g = (u.gscale ? *u.gscale : 1.f) * inv_n;
  float acc = 0.f;
  STAMPW(5);
  for (int e = tid; e < FW_ROWS * opad; e += FW_NT) {
    const int r = e / opad, k = e - r * opad;
    float gd = 0.f, gl = 0.f, cmn = 0.f, cmx = 0.f;
    if (r < nrows && k < S1) {
      const int64_t row = row0 + r;
      const int64_t o = ((int64_t)z * b + row) * S1 + k;
      const float hi = gload(u.maxlv + k), lo = gload(u.minlv + k);
      const float raw = gload(u.LVR + o);
      const float l1 = hi - softplusf(hi - raw);
      const float l = lo + softplusf(l1 - lo);
      const float m = gload(u.D + o) + (k < S ? gload(u.s + (int64_t)z * u.s_zstride + row * S + k) : 0.f);
      const float diff = gload(u.t + (int64_t)z * u.t_zstride + row * S1 + k) - m;
      const float iv = expf(-l);
      acc += diff * diff * iv + l;
      const float dl = (1.f - diff * diff * iv) * g;
      const float s1 = sp_grad(l1 - lo), s2 = sp_grad(hi - raw);
      gd = -2.f * diff * iv * g;
      gl = dl * s1 * s2;
      cmn = dl * (1.f - s1);
      cmx = dl * s1 * (1.f - s2);
      if (split < 0 && hd.L[1].dz) gstore(hd.L[1].dz + o, gd);
      if (split < 0 && hl.L[1].dz) gstore(hl.L[1].dz + o, gl);
    }
    Gd[r * LDH + k] = gd;
    Gl[r * LDH + k] = gl;
    Cm[r * LDH + k] = cmn;
    Cx[r * LDH + k] = cmx;
  }
  STAMPW(6);
  // mse partial: per-wave sums, then the waves in order (thread 0)
  float v = acc * inv_n;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  __shared__ float s_red[FW_NW];
  if ((tid & 63) == 0) s_red[tid >> 6] = v;
  lds_barrier();
  STAMPW(7);
  const int nbx = (int)((b + FW_ROWS - 1) / FW_ROWS);
  float* part_mse = u.part;
  float* part_min = part_mse + (size_t)u.Z * nbx;
  float* part_max = part_min + (size_t)u.Z * nbx * S1;
  const size_t pb = (size_t)z * nbx + bx;
  if (split > 0) return;
  if (tid == 0) {
    float t = 0.f;
    for (int w = 0; w < FW_NW; ++w) t += s_red[w];
    part_mse[pb] = t;
  }
  if (tid < S1) {
    float a0 = 0.f, a1 = 0.f;
    for (int r = 0; r < FW_ROWS; ++r) {
      a0 += Cm[r * LDH + tid];
      a1 += Cx[r * LDH + tid];
    }
    part_min[pb * S1 + tid] = a0;
    part_max[pb * S1 + tid] = a1;
  }
}

// the actor update's head (drpo_mlp_backward_multi_actor), read in place from kernarg
typedef const __attribute__((address_space(4))) drpo_actor_head_t ActorHeadK;

// DRPO_UPSTREAM_ACTOR_CC / _SAFE_CC: the actor losses' gradient w.r.t. the constraint
// critic's mean / raw log-std heads at (s, a) or (s, a_safe) (drpo_actor_upstream's
// arithmetic, csrc/sac.hip; src/ssac.py:474-494): weight lam / B (actor) or 1 / B
// (safe actor) on the arg-max constraint of the quantile bound mu + ratio * std; the
// head outputs are the forward's saves (hm / hl last-layer sy). Gm / Gl (LDS) + the
// output layers' saved dZ.
__device__ __forceinline__ void actor_cc_upstream(ActorHeadK& h, int side, const drpo_mlp_bwd_net_t& hm,
                                                  const drpo_mlp_bwd_net_t* hl, float* Gm, float* Gl, int row0,
                                                  int nrows) {
  const int C = h.C, opad = round_up(C, 16);
  const bool dist = h.distributional;
  const float* __restrict__ mu = hm.L[hm.nl - 1].sy;
  const float* __restrict__ ls = hl ? hl->L[hl->nl - 1].sy : nullptr;
  const float invB = 1.f / (float)h.B;
  for (int e = threadIdx.x; e < FW_ROWS * opad; e += FW_NT) {
    const int r = e / opad, k = e - r * opad;
    float gm = 0.f, gs = 0.f;
    if (r < nrows && k < C) {
      const int64_t i = row0 + r;
      float best = 0.f, lbest = 0.f;
      int bi = 0;
      for (int c = 0; c < C; ++c) {
        float v = gload(mu + i * C + c);
        const float l = dist ? gload(ls + i * C + c) : 0.f;
        if (dist) v = v + h.std_ratio * cc_std(l, h.log_std_min, h.log_std_max);
        if (c == 0 || v > best) { best = v; bi = c; lbest = l; }
      }
      float g = invB;
      if (side == 0) {
        float lam = h.lams ? gload(h.lams + i) : h.fixed_lam;
        const float ub = h.lam_upper_bound;
        if (h.lams && ub > 0.f) lam = ub / 2.f * (1.f + tanhf(lam / ub * 2.f));   // MLPMultiplier.forward
        if (!h.lams && (best < h.clamp_lb || best > h.clamp_ub)) lam = 0.f;       // clamped scalar-lam term
        g = lam * invB;
      }
      float gl = 0.f;
      if (dist && g != 0.f) {
        const float sd = cc_std(lbest, h.log_std_min, h.log_std_max);
        gl = g * h.std_ratio * cc_dstd_draw(lbest, h.log_std_min, h.log_std_max, sd);
      }
      gm = k == bi ? g : 0.f;
      gs = k == bi ? gl : 0.f;
      const size_t o = (size_t)i * C + k;
      if (Gm && hm.L[hm.nl - 1].dz) gstore(hm.L[hm.nl - 1].dz + o, gm);
      if (Gl && hl->L[hl->nl - 1].dz) gstore(hl->L[hl->nl - 1].dz + o, gs);
    }
    if (Gm) Gm[r * LDH + k] = gm;
    if (Gl) Gl[r * LDH + k] = gs;
  }
}

// DRPO_UPSTREAM_SQUASH / _SQUASH_SAFE: the chain rule through rsample + tanh + log_prob
// of the squashed Gaussian (drpo_squash_backward's arithmetic, csrc/sac.hip;
// src/policy.py:89-97, src/ssac.py:458-505) to the net's raw [mu | log-std] outputs
// (the forward's save), and the alpha-loss sum for the actor
__device__ __forceinline__ void squash_upstream(ActorHeadK& h, int side, const drpo_mlp_bwd_net_t& n, float* G,
                                                int row0, int nrows) {
  const int A = h.A;
  const float* __restrict__ raw = n.L[n.nl - 1].sy;
  const float* __restrict__ u = h.u[side];
  const float* __restrict__ ep = h.e[side];
  const float* __restrict__ dA = h.dA[side];
  const float* __restrict__ dA2 = h.dA2[side];
  const float glp = (side == 0 && h.log_alpha) ? expf(*h.log_alpha) * h.lp_scale : 0.f;
  float asum = 0.f;
  for (int e = threadIdx.x; e < FW_ROWS * 16; e += FW_NT) {
    const int r = e >> 4, k = e & 15;
    float gv = 0.f;
    if (r < nrows && k < 2 * A) {
      const int64_t i = row0 + r;
      const int d = k < A ? k : k - A;
      const float mu = gload(raw + i * 2 * A + d), rr = gload(raw + i * 2 * A + A + d);
      const float uu = gload(u + i * A + d), ee = gload(ep + i * A + d);
      const float dAv = dA2 ? gload(dA + i * A + d) + gload(dA2 + i * A + d) : gload(dA + i * A + d);
      const float sg = sigmoidf(rr);
      const float sd = expf(-6.f + 10.f * sg) * 1.0f;
      const float a = tanhf(uu);
      const float diff = uu - mu;
      const float var = sd * sd;
      const float du = dAv * (1.f - a * a) + glp * (-diff / var + 2.f - 4.f * sp_grad(-2.f * uu));
      if (k < A) {
        gv = du + glp * diff / var;
      } else {
        const float dsd = du * ee + glp * (diff * diff / (var * sd) - 1.f / sd);
        gv = dsd * sd * 10.f * sg * (1.f - sg);
      }
      if (side == 0 && h.alpha_sum && k == 0) asum = gload(h.logp + i) + h.target_entropy;
    }
    G[r * LDH + k] = gv;
  }
  if (side == 0 && h.alpha_sum) wg_loss_partial(asum, h.alpha_sum + row0 / FW_ROWS);
}

// upstream families compiled into a backward kernel instantiation (each launch kind
// gets only the producer code it uses, so none of them adds register pressure -- and
// spills -- to the others' GEMM phases)
constexpr int UPF_CRITIC = 1, UPF_ENS = 2, UPF_ACTOR = 4;

// heads' output gradients -> trunk-output gradient in G (bA, bB, DT are scratch)
template <int UPF>
__device__ __forceinline__ void bwd_heads_paired(const drpo_mlp_bwd_t& __restrict__ a, float* G, float* bA, float* bB,
                                                 float* DT, int z, int row0, int nrows, CriticHeadK* ch,
                                                 EnsUpK* eu = nullptr, ActorHeadK* ah = nullptr) {
  const int tid = threadIdx.x;
  const drpo_mlp_bwd_net_t &h1 = a.net[1], &h2 = a.net[2];
  const int hid = h1.L[0].dout, out = h1.L[1].dout;
  const int opad = round_up(out, 16), hpad = round_up(hid, 16);
  float sv1[BW_PER], sv2[BW_PER];
  bwd_fetch_act(h1.L[0], z, a.rows, row0, nrows, sv1);   // head 1's hidden saved values, one phase ahead
  // output layers (identity): dZ = the given output gradient, saved for the weight gradients
  const size_t so = ((size_t)z * a.rows + row0) * out;
  bool done = false;
  if constexpr ((UPF & UPF_ENS) != 0) {
    if (eu) { ens_upstream(*eu, h1, h2, G, bA, bB, DT, z, row0 / FW_ROWS, row0, nrows); done = true; }
  }
  if constexpr ((UPF & UPF_CRITIC) != 0) {
    if (ch) { cert_upstream(*ch, &h1, &h2, G, bA, row0, nrows, true); done = true; }
  }
  if constexpr ((UPF & UPF_ACTOR) != 0) {
    if (ah) { actor_cc_upstream(*ah, a.upstream == DRPO_UPSTREAM_SAFE_CC, h1, &h2, G, bA, row0, nrows); done = true; }
  }
  if (!done)
  for (int e = tid; e < 2 * FW_ROWS * opad; e += FW_NT) {
    const int w = e / (FW_ROWS * opad), e2 = e - w * FW_ROWS * opad;
    const int r = e2 / opad, k = e2 - r * opad;
    const drpo_mlp_bwd_net_t& h = w ? h2 : h1;
    float gv = 0.f;
    if (r < nrows && k < out) {
      gv = gload(h.gout + so + (size_t)r * out + k);
      if (h.L[1].dz) gstore(h.L[1].dz + so + (size_t)r * out + k, gv);
    }
    (w ? bA : G)[r * LDH + k] = gv;
  }
  lds_barrier();
  STAMPW(1);
  // dY(hidden) of both heads: one two-input pair layer (K = out)
  switch ((out + 15) >> 4) {
    case 1: bwd_heads_out<1>(h1, h2, G, bA, bB, DT, z); break;
    case 2: bwd_heads_out<2>(h1, h2, G, bA, bB, DT, z); break;
    case 3: bwd_heads_out<3>(h1, h2, G, bA, bB, DT, z); break;
    default: bwd_heads_out<4>(h1, h2, G, bA, bB, DT, z); break;
  }
  bwd_fetch_act(h2.L[0], z, a.rows, row0, nrows, sv2);   // (after the product: 128-VGPR budget)
  lds_barrier();
  STAMPW(2);
  // hidden activations' gradient, saved dZ
  const size_t sh = ((size_t)z * a.rows + row0) * hid;
  const int act = h1.L[0].act;
#pragma unroll
  for (int i = 0; i < BW_PER; ++i) {
    const int e = tid + i * FW_NT;
    if (e >= FW_ROWS * hpad) break;
    const int r = e / hpad, k = e - r * hpad;
    float g1 = 0.f, g2 = 0.f;
    if (r < nrows && k < hid) {
      g1 = bB[r * LDH + k];
      g2 = DT[r * LDH + k];
      if (act != ACT_NONE) {
        g1 *= act_grad_saved(act, sv1[i]);
        g2 *= act_grad_saved(act, sv2[i]);
      }
      if (h1.L[0].dz) gstore(h1.L[0].dz + sh + (size_t)r * hid + k, g1);
      if (h2.L[0].dz) gstore(h2.L[0].dz + sh + (size_t)r * hid + k, g2);
    }
    bB[r * LDH + k] = g1;
    DT[r * LDH + k] = g2;
  }
  lds_barrier();
  STAMPW(3);
  // trunk-output gradient = dZ_1 W_1 + dZ_2 W_2 as one concatenated-K product
  if (hid == 200) bwd_heads_catk<13>(h1, h2, bB, DT, G, z);
  else bwd_heads_catk<16>(h1, h2, bB, DT, G, z);
  lds_barrier();
  STAMPW(4);
}

// one (job, net) slot of the fused backward-data pass; `a` may live in kernarg
// (single launch) or global memory (multi-job launch)
template <int UPF>
__device__ __forceinline__ void bwd_body(const drpo_mlp_bwd_t& __restrict__ a, int sel, int bx, int bz, float* smem,
                                         CriticHeadK* ch = nullptr, EnsUpK* eu = nullptr, ActorHeadK* ah = nullptr) {
  float* G = smem;
  float* bA = G + FW_ROWS * LDH;
  float* bB = bA + FW_ROWS * LDH;
  float* DT = bB + FW_ROWS * LDH;   // trunk output gradient accumulator
  const int tid = threadIdx.x;
  const int z = bz;
  const int row0 = bx * FW_ROWS;
  if (row0 >= a.rows) return;
  const int nrows = (int)min((int64_t)FW_ROWS, a.rows - row0);
  STAMPW(0);

  auto load_gout = [&](const drpo_mlp_bwd_net_t& n, float* dst) {
    const int w = n.L[n.nl - 1].dout;
    const int wpad = round_up(w, 16);
    for (int e = tid; e < FW_ROWS * wpad; e += FW_NT) {
      const int r = e / wpad, k = e - r * wpad;
      dst[r * LDH + k] = (r < nrows && k < w) ? gload(n.gout + ((size_t)z * a.rows + row0 + r) * w + k) : 0.f;
    }
    lds_barrier();
  };
  auto store_dx = [&](const drpo_mlp_bwd_net_t& n, const float* src) {
    if (!n.dx) return;
    for (int e = tid; e < nrows * n.dx_cols; e += FW_NT) {
      const int r = e / n.dx_cols, k = e - r * n.dx_cols;
      float* p = n.dx + ((size_t)z * a.rows + row0 + r) * n.dx_cols + k;
      const float v = src[r * LDH + n.dx_col0 + k];
      gstore(p, n.dx_accumulate ? gload(p) + v : v);
    }
  };

  // output gradients formed in-kernel from the launch's critic head (no head launch)
  if constexpr ((UPF & UPF_CRITIC) == 0) ch = nullptr;
  if constexpr ((UPF & UPF_ENS) == 0) eu = nullptr;
  if constexpr ((UPF & UPF_ACTOR) == 0) ah = nullptr;
  CriticHeadK* hq = (ch && a.upstream == DRPO_UPSTREAM_CRITIC) ? ch : nullptr;
  CriticHeadK* hc = (ch && a.upstream == DRPO_UPSTREAM_CERT) ? ch : nullptr;
  const bool acc_up = a.upstream == DRPO_UPSTREAM_ACTOR_CC || a.upstream == DRPO_UPSTREAM_SAFE_CC;
  ActorHeadK* ha = (ah && acc_up) ? ah : nullptr;
  if (!a.trunk) {
    const drpo_mlp_bwd_net_t& n = a.net[sel];
    if (hq) {
      // twin critic `sel`: dL/dq = (q - y) / B of the mean-of-twins MSE (src/ssac.py:295-302);
      // the critic loss 0.5 mean((q - y)^2) per twin is accumulated into loss[0]
      float lq = 0.f;
      for (int e = tid; e < FW_ROWS * 16; e += FW_NT) {
        const int r = e >> 4, k = e & 15;
        float g = 0.f;
        if (r < nrows && k == 0) {
          const int64_t i = row0 + r;
          const float invB = 1.f / (float)hq->B;
          const float y = critic_target(*hq, i, expf(*hq->log_alpha));
          const float err = gload((sel ? hq->q1 : hq->q0) + i) - y;
          g = err * invB;
          lq = err * err * (0.5f * invB);
        }
        G[r * LDH + k] = g;
      }
      wg_loss_partial(lq, hq->loss_part + (size_t)sel * ((hq->B + FW_ROWS - 1) / FW_ROWS) + row0 / FW_ROWS);
      lds_barrier();
    } else if (ah && a.upstream == DRPO_UPSTREAM_NEG_MEAN) {
      // the actor loss's -mean(Q_k) (src/ssac.py:472): dL/dQ = -1/B
      for (int e = tid; e < FW_ROWS * 16; e += FW_NT) {
        const int r = e >> 4, k = e & 15;
        G[r * LDH + k] = (r < nrows && k == 0) ? -1.f / (float)ah->B : 0.f;
      }
      lds_barrier();
    } else if (ah && (a.upstream == DRPO_UPSTREAM_SQUASH || a.upstream == DRPO_UPSTREAM_SQUASH_SAFE)) {
      squash_upstream(*ah, a.upstream == DRPO_UPSTREAM_SQUASH_SAFE, n, G, row0, nrows);
      lds_barrier();
    } else {
      load_gout(n, G);
    }
    const float* gx = bwd_net(n, G, bA, bB, z, a.rows, row0, nrows, n.dx != nullptr);
    if (gx) store_dx(n, gx);
    return;
  }
  if (a.split_heads) {
    // head sel + 1 alone: the trunk gradient is linear in the head gradients, so its
    // share backs through the trunk here (dz for head 1, dz2 for head 2)
    const drpo_mlp_bwd_net_t& n = a.net[sel + 1];
    bool up = false;
    if constexpr ((UPF & UPF_ENS) != 0) {
      if (eu && a.upstream == DRPO_UPSTREAM_ENS) {
        // both heads' NLL gradients are formed (they share the element's terms); this
        // workgroup keeps its own head's in G
        ens_upstream(*eu, a.net[1], a.net[2], sel == 0 ? G : bA, sel == 0 ? bA : G, bB, DT, z, row0 / FW_ROWS, row0,
                     nrows, sel);
        lds_barrier();   // Cm / Cx (bB, DT) are read by the partial sums above; bwd_net reuses bB
        up = true;
      }
    }
    if (!up) load_gout(n, G);
    STAMPW(1);
    float* gh = bwd_net(n, G, bA, bB, z, a.rows, row0, nrows, true);
    STAMPW(2);
    bwd_net(a.net[0], gh, bA, bB, z, a.rows, row0, nrows, false, sel == 1);
    STAMPW(12);
    return;
  }
  if (bwd_paired_heads(a)) {
    bwd_heads_paired<UPF>(a, G, bA, bB, DT, z, row0, nrows, hc, a.upstream == DRPO_UPSTREAM_ENS ? eu : nullptr, ha);
    const float* gx = bwd_net(a.net[0], G, bA, bB, z, a.rows, row0, nrows, a.net[0].dx != nullptr);
    STAMPW(12);
    if (gx) store_dx(a.net[0], gx);
    return;
  }
  const int tw = a.net[0].L[a.net[0].nl - 1].dout;
  const int twpad = round_up(tw, 16);
  STAMPW(5);
  for (int e = tid; e < FW_ROWS * twpad; e += FW_NT) DT[(e / twpad) * LDH + e % twpad] = 0.f;
  lds_barrier();
  for (int h = 1; h < a.nnets; ++h) {
    // generic trunk path (unpaired head shapes): one head at a time, head 1 = mean,
    // head 2 = log-std (distributional); the certificate loss is added once
    if (hc) {
      cert_upstream(*hc, &a.net[1], a.nnets > 2 ? &a.net[2] : nullptr, h == 1 ? G : nullptr, h == 2 ? G : nullptr,
                    row0, nrows, h == 1);
      lds_barrier();
    } else if (ha) {
      actor_cc_upstream(*ha, a.upstream == DRPO_UPSTREAM_SAFE_CC, a.net[1], a.nnets > 2 ? &a.net[2] : nullptr,
                        h == 1 ? G : nullptr, h == 2 ? G : nullptr, row0, nrows);
      lds_barrier();
    } else {
      load_gout(a.net[h], G);
    }
    if (h == 1) STAMPW(6); else STAMPW(9);
    const float* gh = bwd_net(a.net[h], G, bA, bB, z, a.rows, row0, nrows, true);
    if (h == 1) STAMPW(7); else STAMPW(10);
    for (int e = tid; e < FW_ROWS * twpad; e += FW_NT) {
      const int r = e / twpad, k = e - r * twpad;
      DT[r * LDH + k] += gh[r * LDH + k];
    }
    lds_barrier();
    if (h == 1) STAMPW(8); else STAMPW(11);
  }
  const float* gx = bwd_net(a.net[0], DT, bA, bB, z, a.rows, row0, nrows, a.net[0].dx != nullptr);
  STAMPW(12);
  if (gx) store_dx(a.net[0], gx);
  STAMPW(13);
}

__global__ __launch_bounds__(FW_NT) __attribute__((amdgpu_waves_per_eu(4, 4))) void mlp_bwd_kernel(drpo_mlp_bwd_t a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const LogicalBlock lb = xcd_block();   // one member's tiles per XCD (shared weights in L2)
  bwd_body<0>(a, lb.y, lb.x, lb.z, smem);
}

// the model fit's backward with the NLL loss fused in (one workgroup per (row tile,
// member); drpo_mlp_backward_ens)
struct BwdEnsArgs {
  drpo_mlp_bwd_t a;
  drpo_ens_upstream_t u;
};

__global__ __launch_bounds__(FW_NT) __attribute__((amdgpu_waves_per_eu(4, 4))) void mlp_bwd_ens_kernel(BwdEnsArgs m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  typedef const __attribute__((address_space(4))) BwdEnsArgs* ArgsK;
  ArgsK k = (ArgsK)__builtin_amdgcn_kernarg_segment_ptr();
  const LogicalBlock lb = xcd_block();   // one member's tiles per XCD (shared weights in L2)
  bwd_body<UPF_ENS>(m.a, lb.y, lb.x, lb.z, smem, nullptr, &k->u);
}

struct BwdMultiArgs {
  const drpo_mlp_bwd_t* jobs;
  unsigned char slot_job[16], slot_net[16];
  int has_head, has_actor;
  drpo_critic_head_t head;
  drpo_actor_head_t actor;
};

template <int UPF>
__global__ __launch_bounds__(FW_NT) __attribute__((amdgpu_waves_per_eu(4, 4))) void mlp_bwd_multi_kernel(
    BwdMultiArgs m) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const drpo_mlp_bwd_t* __restrict__ ap = m.jobs + m.slot_job[blockIdx.y];
  const drpo_mlp_bwd_t& a = *ap;
  if (blockIdx.z >= (unsigned)a.nbatch) return;
  typedef const __attribute__((address_space(4))) BwdMultiArgs* ArgsK;
  ArgsK k = (ArgsK)__builtin_amdgcn_kernarg_segment_ptr();
  bwd_body<UPF>(a, m.slot_net[blockIdx.y], blockIdx.x, blockIdx.z, smem, m.has_head ? &k->head : nullptr, nullptr,
                m.has_actor ? &k->actor : nullptr);
}

static size_t bwd_lds() { return sizeof(float) * (size_t)4 * FW_ROWS * LDH; }

DRPO_API int drpo_mlp_backward(const drpo_mlp_bwd_t* a, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(a && a->nnets >= 1 && a->nnets <= MAXN && a->nbatch >= 1, "drpo_mlp_backward: bad descriptor");
  for (int h = 0; h < a->nnets; ++h) {
    const drpo_mlp_bwd_net_t& n = a->net[h];
    DRPO_REQUIRE(n.nl >= 1 && n.nl <= MAXL && n.gout || (a->trunk && h == 0 && n.nl >= 1),
                 "drpo_mlp_backward: bad net %d", h);
    for (int l = 0; l < n.nl; ++l)
      DRPO_REQUIRE(n.L[l].din >= 1 && n.L[l].din <= 256 && n.L[l].dout >= 1 && n.L[l].dout <= 256 && n.L[l].W,
                   "drpo_mlp_backward: bad layer %d of net %d", l, h);
    if (n.dx) DRPO_REQUIRE(n.dx_col0 >= 0 && n.dx_col0 + n.dx_cols <= n.L[0].din, "drpo_mlp_backward: dx columns");
  }
  if (a->split_heads) {
    DRPO_REQUIRE(a->trunk && a->nnets >= 2 && a->nnets <= 3 && !a->net[0].dx,
                 "drpo_mlp_backward: split_heads needs a trunk, 1-2 heads and no trunk input gradient");
    for (int l = 0; l < a->net[0].nl; ++l)
      DRPO_REQUIRE(a->nnets < 3 || !a->net[0].L[l].dz == !a->net[0].L[l].dz2,
                   "drpo_mlp_backward: split_heads trunk layer %d needs dz2 with dz", l);
  }
  if (a->rows == 0) return DRPO_OK;
  dim3 grid((unsigned)((a->rows + FW_ROWS - 1) / FW_ROWS),
            a->trunk ? (a->split_heads ? a->nnets - 1 : 1) : a->nnets, a->nbatch);
  mlp_bwd_kernel<<<grid, FW_NT, bwd_lds(), stream>>>(*a);
  DRPO_LAUNCH_CHECK("mlp_backward");
  return DRPO_OK;
}

DRPO_API int drpo_mlp_backward_ens(const drpo_mlp_bwd_t* a, const drpo_ens_upstream_t* up,
                                   const drpo_ens_reduce_t* red_in, drpo_ens_reduce_t* reduce_out,
                                   drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(a && up && red_in && reduce_out, "drpo_mlp_backward_ens: null argument");
  DRPO_REQUIRE(a->upstream == DRPO_UPSTREAM_ENS && a->trunk && a->nnets == 3 && a->nbatch == up->Z &&
                   a->rows == up->b,
               "drpo_mlp_backward_ens: the descriptor must be the ensemble trunk + two heads with upstream ENS");
  if (a->split_heads) {   // one workgroup per (row tile, head): the trunk dZ leaves as dz + dz2
    DRPO_REQUIRE(!a->net[0].dx, "drpo_mlp_backward_ens: split heads and a trunk input gradient");
    for (int l = 0; l < a->net[0].nl; ++l)
      DRPO_REQUIRE(!a->net[0].L[l].dz == !a->net[0].L[l].dz2,
                   "drpo_mlp_backward_ens: split heads: trunk layer %d needs dz2 with dz", l);
  }
  const drpo_mlp_bwd_net_t &h1 = a->net[1], &h2 = a->net[2];
  DRPO_REQUIRE(h1.nl == 2 && h2.nl == 2 && h1.L[1].dout == up->S + 1 && h2.L[1].dout == up->S + 1 &&
                   up->S + 1 <= 64 && h1.L[1].act == ACT_NONE && h2.L[1].act == ACT_NONE &&
                   (h1.L[0].dout == 200 || h1.L[0].dout == 256) && h1.L[0].dout == h2.L[0].dout &&
                   h1.L[0].act == h2.L[0].act && !h1.dx && !h2.dx,
               "drpo_mlp_backward_ens: heads must be paired [H -> 200|256 -> S+1] (S+1 <= 64)");
  DRPO_REQUIRE(up->D && up->LVR && up->s && up->t && up->minlv && up->maxlv && up->part && up->b >= 1 &&
                   up->Z >= 1 && up->Z <= 256,
               "drpo_mlp_backward_ens: bad upstream");
  for (int l = 0; l < a->net[0].nl; ++l)
    DRPO_REQUIRE(a->net[0].L[l].din <= 256 && a->net[0].L[l].dout <= 256 && a->net[0].L[l].W,
                 "drpo_mlp_backward_ens: bad trunk layer %d", l);
  const int nbx = (int)((up->b + FW_ROWS - 1) / FW_ROWS);
  *reduce_out = *red_in;
  reduce_out->part = up->part;
  reduce_out->nbx = nbx;
  reduce_out->Z = up->Z;
  reduce_out->S1 = up->S + 1;
  reduce_out->minlv = up->minlv;
  reduce_out->maxlv = up->maxlv;
  reduce_out->gscale = up->gscale;
  BwdEnsArgs m{*a, *up};
  dim3 grid((unsigned)nbx, a->split_heads ? 2 : 1, a->nbatch);
  mlp_bwd_ens_kernel<<<grid, FW_NT, bwd_lds(), stream>>>(m);
  DRPO_LAUNCH_CHECK("mlp_backward_ens");
  return DRPO_OK;
}

static int check_bwd(const drpo_mlp_bwd_t* a) {
  if (!(a && a->nnets >= 1 && a->nnets <= MAXN && a->nbatch >= 1 && !a->split_heads)) return 0;
  for (int h = 0; h < a->nnets; ++h) {
    const drpo_mlp_bwd_net_t& n = a->net[h];
    if (!(n.nl >= 1 && n.nl <= MAXL && (n.gout || (a->trunk && h == 0)))) return 0;
    for (int l = 0; l < n.nl; ++l)
      if (!(n.L[l].din >= 1 && n.L[l].din <= 256 && n.L[l].dout >= 1 && n.L[l].dout <= 256 && n.L[l].W)) return 0;
    if (n.dx && !(n.dx_col0 >= 0 && n.dx_col0 + n.dx_cols <= n.L[0].din)) return 0;
  }
  return 1;
}

DRPO_API int drpo_mlp_backward_multi(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                                     drpo_stream_t stream_) {
  return drpo_mlp_backward_multi_head(jobs_host, jobs_dev, njobs, nullptr, stream_);
}

static int bwd_multi_launch(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                            const drpo_critic_head_t* head, const drpo_actor_head_t* actor, hipStream_t stream);

DRPO_API int drpo_mlp_backward_multi_head(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                                          const drpo_critic_head_t* head, drpo_stream_t stream_) {
  return bwd_multi_launch(jobs_host, jobs_dev, njobs, head, nullptr, (hipStream_t)stream_);
}

DRPO_API int drpo_mlp_backward_multi_actor(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                                           const drpo_actor_head_t* actor, drpo_stream_t stream_) {
  DRPO_REQUIRE(actor && actor->B >= 0 && actor->A >= 1 && actor->A <= 8 && actor->C >= 1 && actor->C <= 16,
               "drpo_mlp_backward_multi_actor: bad actor head");
  return bwd_multi_launch(jobs_host, jobs_dev, njobs, nullptr, actor, (hipStream_t)stream_);
}

static int bwd_multi_launch(const drpo_mlp_bwd_t* jobs_host, const drpo_mlp_bwd_t* jobs_dev, int njobs,
                            const drpo_critic_head_t* head, const drpo_actor_head_t* actor, hipStream_t stream) {
  DRPO_REQUIRE(jobs_host && jobs_dev && njobs >= 1 && njobs <= 8, "drpo_mlp_backward_multi: 1..8 jobs");
  BwdMultiArgs m{};
  m.jobs = jobs_dev;
  if (actor) {
    m.has_actor = 1;
    m.actor = *actor;
  }
  if (head) {
    DRPO_REQUIRE(head->C >= 1 && head->B >= 0 && head->loss_part && head->log_alpha && head->q0 && head->q1 &&
                     head->mu,
                 "drpo_mlp_backward_multi_head: bad critic head (loss_part required)");
    m.has_head = 1;
    m.head = *head;
  }
  for (int j = 0; j < njobs; ++j) {
    const drpo_mlp_bwd_t& J = jobs_host[j];
    DRPO_REQUIRE(J.upstream >= DRPO_UPSTREAM_GOUT && J.upstream <= DRPO_UPSTREAM_SQUASH_SAFE &&
                     J.upstream != DRPO_UPSTREAM_ENS,
                 "drpo_mlp_backward_multi: job %d upstream %d", j, J.upstream);
    if (J.upstream == DRPO_UPSTREAM_GOUT) continue;
    if (J.upstream >= DRPO_UPSTREAM_ACTOR_CC) {
      DRPO_REQUIRE(actor && J.nbatch == 1 && J.rows == actor->B, "drpo_mlp_backward_multi: job %d needs the actor head",
                   j);
      const drpo_mlp_bwd_net_t& n0 = J.net[0];
      if (J.upstream == DRPO_UPSTREAM_NEG_MEAN)
        DRPO_REQUIRE(!J.trunk && J.nnets == 1 && n0.L[n0.nl - 1].dout == 1,
                     "drpo_mlp_backward_multi: job %d: -1/B upstream needs one single-output net", j);
      else if (J.upstream >= DRPO_UPSTREAM_SQUASH)
        DRPO_REQUIRE(!J.trunk && J.nnets == 1 && n0.L[n0.nl - 1].dout == 2 * actor->A && n0.L[n0.nl - 1].sy &&
                         actor->u[J.upstream - DRPO_UPSTREAM_SQUASH] && actor->e[J.upstream - DRPO_UPSTREAM_SQUASH] &&
                         actor->dA[J.upstream - DRPO_UPSTREAM_SQUASH],
                     "drpo_mlp_backward_multi: job %d: squash upstream needs the policy net and its samples", j);
      else
        DRPO_REQUIRE(J.trunk && J.nnets >= 2 && J.net[1].L[J.net[1].nl - 1].dout == actor->C &&
                         J.net[1].L[J.net[1].nl - 1].sy &&
                         (!actor->distributional || (J.nnets == 3 && J.net[2].L[J.net[2].nl - 1].sy)),
                     "drpo_mlp_backward_multi: job %d: constraint-critic upstream needs its saved head outputs", j);
      continue;
    }
    DRPO_REQUIRE(head && J.nbatch == 1 && J.rows == head->B, "drpo_mlp_backward_multi: job %d needs the critic head", j);
    DRPO_REQUIRE(!head->cost || (head->v && !head->distributional),
                 "drpo_mlp_backward_multi: cost target needs v, not distributional");
    if (J.upstream == DRPO_UPSTREAM_CRITIC)
      DRPO_REQUIRE(!J.trunk && J.nnets == 2 && J.net[0].L[J.net[0].nl - 1].dout == 1 &&
                       J.net[1].L[J.net[1].nl - 1].dout == 1,
                   "drpo_mlp_backward_multi: critic-upstream job %d must be the twin critics", j);
    else
      DRPO_REQUIRE(J.trunk && J.nnets >= 2 && J.net[1].L[J.net[1].nl - 1].dout == head->C &&
                       (J.nnets == 2 || (head->distributional && J.net[2].L[J.net[2].nl - 1].dout == head->C)),
                   "drpo_mlp_backward_multi: certificate-upstream job %d must be the constraint critic", j);
  }
  int slots = 0, nbatch = 1;
  int64_t tiles = 0;
  for (int j = 0; j < njobs; ++j) {
    const drpo_mlp_bwd_t* a = jobs_host + j;
    DRPO_REQUIRE(check_bwd(a), "drpo_mlp_backward_multi: bad job %d", j);
    const int ns = a->trunk ? 1 : a->nnets;
    DRPO_REQUIRE(slots + ns <= 16, "drpo_mlp_backward_multi: too many nets");
    for (int h = 0; h < ns; ++h) {
      m.slot_job[slots] = (unsigned char)j;
      m.slot_net[slots] = (unsigned char)h;
      ++slots;
    }
    tiles = max(tiles, (a->rows + FW_ROWS - 1) / FW_ROWS);
    nbatch = max(nbatch, a->nbatch);
  }
  if (tiles == 0) return DRPO_OK;
  const dim3 grid((unsigned)tiles, slots, nbatch);
  if (m.has_head)
    mlp_bwd_multi_kernel<UPF_CRITIC><<<grid, FW_NT, bwd_lds(), stream>>>(m);
  else if (m.has_actor)
    mlp_bwd_multi_kernel<UPF_ACTOR><<<grid, FW_NT, bwd_lds(), stream>>>(m);
  else
    mlp_bwd_multi_kernel<0><<<grid, FW_NT, bwd_lds(), stream>>>(m);
  DRPO_LAUNCH_CHECK("mlp_backward_multi");
  return DRPO_OK;
}

