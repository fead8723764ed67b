// Shared device/host helpers for libdrpo_hip (gfx950 / CDNA4 only).
//
//  * C-ABI error plumbing (thread-local last-error string, DRPO_* return codes)
//  * Philox4x32-10 counter RNG + Box-Muller (production-mode noise; parity mode
//    reads caller-provided noise instead)
//  * tile_dense<>: one MLP layer for a 16/32-row tile held in LDS, computed with
//    the exact-fp32 MFMA v_mfma_f32_16x16x4_f32 by a 256-thread workgroup
//    (4 wave64s, waves split the output columns into 16-wide blocks).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "drpo_hip.h"

#define DRPO_API extern "C" __attribute__((visibility("default")))

void drpo_set_error(const char* fmt, ...);

#define DRPO_REQUIRE(cond, ...)             \
  do {                                      \
    if (!(cond)) {                          \
      drpo_set_error(__VA_ARGS__);          \
      return DRPO_EINVAL;                   \
    }                                       \
  } while (0)

#define DRPO_CHECK_HIP(expr)                                                  \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      drpo_set_error("%s failed: %s", #expr, hipGetErrorString(_e));          \
      return DRPO_EHIP;                                                       \
    }                                                                         \
  } while (0)

#define DRPO_LAUNCH_CHECK(name)                                               \
  do {                                                                        \
    hipError_t _e = hipGetLastError();                                        \
    if (_e != hipSuccess) {                                                   \
      drpo_set_error("%s launch failed: %s", name, hipGetErrorString(_e));    \
      return DRPO_EHIP;                                                       \
    }                                                                         \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

// sub-phase stamps of the layer cores: a profiling build's translation unit may define
// CORE_STAMP before including this header (rollout.hip under DRPO_STAMPS)
#ifndef CORE_STAMP
#define CORE_STAMP(i) \
  do {                \
  } while (0)
#define CORE_STAMP_W4(i) \
  do {                   \
  } while (0)
#endif

namespace drpo {

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_SILU = 2, ACT_TANH = 3 };

constexpr int WG = 256;     // threads per workgroup (4 x wave64)

__host__ __device__ inline int round_up(int x, int m) { return (x + m - 1) / m * m; }

// XCD-aware block order. The hardware deals workgroups round-robin over the 8 XCDs
// (blocks b, b+8, ... share one L2; MI355X_MICROARCH.md, workgroup dispatch). This
// returns a logical linear block index such that each XCD runs one CONTIGUOUS range
// of logical blocks (a bijection on [0, nblocks)), so blocks that read the same data
// -- one ensemble member's weights, one dZ / Y column tile -- share an L2 instead of
// every XCD fetching everything. Logical order is x fastest, then y, then z.
// Measured neutral at the fit shapes (E=7 x 200-wide members: fwd 28.8 / bwd 33.8 /
// wgrad 21.1 us with and without), kept for larger ensembles whose weights exceed
// one XCD's 4 MiB L2.
struct LogicalBlock {
  unsigned x, y, z;
};
__device__ __forceinline__ LogicalBlock xcd_block() {
  const unsigned nb = gridDim.x * gridDim.y * gridDim.z;
  const unsigned bid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  const unsigned q = nb >> 3, r = nb & 7, k = bid & 7;
  const unsigned l = k * q + (k < r ? k : r) + (bid >> 3);
  const unsigned t = l / gridDim.x;
  return {l - t * gridDim.x, t % gridDim.y, t / gridDim.y};
}

// LDS row stride (floats) for an activation tile of width K: K rounded up to a
// multiple of 64, +8. Row stride == 8 (mod 64) dwords makes the 16x16x4 A-fragment
// ds_read_b128 pattern (rows l&15, k-offset 4*(l>>4)) bank-conflict free.
__host__ __device__ inline int lds_ld(int K) { return round_up(K, 64) + 8; }

// sigmoid on the hardware transcendentals (v_exp_f32 + v_rcp_f32, ~1 ulp each): the
// libm expf + IEEE division forms cost ~40 VALU ops per element, which in the MLP
// epilogues (8-16 elements per lane per layer) made every swish layer of the
// ensemble ~2k cycles slower than the same layer with ReLU (rollout stamps).
// Saturates cleanly: x -> -inf gives rcp(inf) = 0, x -> +inf gives 1.
__device__ __forceinline__ float fast_sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}

template <int ACT>
__device__ __forceinline__ float act_fn(float x) {
  if constexpr (ACT == ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == ACT_SILU) return x * fast_sigmoid(x);
  else if constexpr (ACT == ACT_TANH) return tanhf(x);
  else return x;
}

// torch softplus(beta=1, threshold=20)
__device__ __forceinline__ float softplusf(float x) { return x > 20.f ? x : log1pf(expf(x)); }

// Hardware-transcendental forms (v_exp_f32 / v_log_f32 / v_rcp_f32, ~1 ulp each) for the
// fused rollout's per-row epilogues, where the libm forms (range reduction, IEEE
// division) cost more than the layer they follow (tracking: 4.4k cycles of 10.6k in the
// output-head phase). Relative error ~1e-6 at the magnitudes on the path, inside the
// rollout parity tolerance (2e-4).
__device__ __forceinline__ float fast_exp(float x) { return __builtin_amdgcn_exp2f(1.44269504088896341f * x); }
__device__ __forceinline__ float fast_softplus(float x) {   // max(x, 0) + log1p(exp(-|x|)), threshold 20
  if (x > 20.f) return x;
  const float y = __builtin_amdgcn_exp2f(-1.44269504088896341f * fabsf(x));
  return fmaxf(x, 0.f) + 0.69314718055994531f * __builtin_amdgcn_logf(1.f + y);
}
__device__ __forceinline__ float fast_tanh(float x) {        // 1 - 2 / (exp(2x) + 1), saturating
  return 1.f - 2.f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(2.88539008177792682f * x) + 1.f);
}
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ float torch_lerp(float s, float e, float w) {
  // at::native lerp: w < 0.5 ? s + w*(e-s) : e - (e-s)*(1-w)
  return (fabsf(w) < 0.5f) ? fmaf(w, e - s, s) : fmaf(-(e - s), 1.f - w, e);
}

// torch.optim.Adam's single-tensor step for one element (coupled L2 weight decay),
// shared by the fused optimizer launch and the weight-gradient launch's fused step so
// both round identically. Opt: any descriptor with lr_over_bc1, bc2_sqrt, beta1,
// beta2, eps, weight_decay (drpo_optim_seg_t, drpo_wgrad_adam_t).
template <typename Opt>
__device__ __forceinline__ void adam_step(const Opt& S, float coef, float g, float& p, float& m, float& v) {
  float ge = g * coef;
  if (S.weight_decay != 0.f) ge = fmaf(p, S.weight_decay, ge);
  m = torch_lerp(m, ge, 1.f - S.beta1);
  v = fmaf(v, S.beta2, (1.f - S.beta2) * ge * ge);
  const float denom = sqrtf(v) / S.bc2_sqrt + S.eps;
  p = p - S.lr_over_bc1 * (m / denom);
}

// ---------------------------------------------------------------------------
// Philox4x32-10
// ---------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = {hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float u32_to_unit(uint32_t v) {   // (0, 1]
  return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// 4 standard normals for (stream, counter words)
__device__ __forceinline__ void philox_normal4(uint64_t seed, uint32_t c0, uint32_t c1, uint32_t c2,
                                               uint32_t c3, float out[4]) {
  u32x4 r = philox({c0, c1, c2, c3}, (uint32_t)seed, (uint32_t)(seed >> 32));
  float u1 = u32_to_unit(r.x), u2 = u32_to_unit(r.y), u3 = u32_to_unit(r.z), u4 = u32_to_unit(r.w);
  // Box-Muller on the hardware transcendentals: v_log_f32 is log2, v_sin/v_cos take
  // the angle in turns (sin(2*pi*x)), so no range reduction is needed for u in (0,1]
  const float m1 = __builtin_amdgcn_sqrtf(-1.38629436112f * __builtin_amdgcn_logf(u1));
  const float m2 = __builtin_amdgcn_sqrtf(-1.38629436112f * __builtin_amdgcn_logf(u3));
  out[0] = m1 * __builtin_amdgcn_cosf(u2); out[1] = m1 * __builtin_amdgcn_sinf(u2);
  out[2] = m2 * __builtin_amdgcn_cosf(u4); out[3] = m2 * __builtin_amdgcn_sinf(u4);
}

// element idx of a recorded draw array, or the Philox normal of (seed, ctr, site)
__device__ __forceinline__ float normal_at(const float* eps, int64_t idx, uint64_t seed, uint64_t ctr, uint32_t site) {
  if (eps) return eps[idx];
  float z[4];
  philox_normal4(seed, (uint32_t)(idx >> 2), (uint32_t)(idx >> 34), site, (uint32_t)ctr, z);
  const int j = (int)(idx & 3);   // selects, not an indexed (private-memory) array
  return j == 0 ? z[0] : (j == 1 ? z[1] : (j == 2 ? z[2] : z[3]));
}

// squashed-Gaussian head of one row (src/policy.py:88-97; Independent(Tanh(Normal))
// log_prob at the cached pre-tanh u). mode 0 sample, 1 rsample, 2 mean only.
// raw = [mu | log-std pre-activation] (2A values, any stride source).
template <typename RawAt>
__device__ __forceinline__ void squashed_gaussian_row(RawAt raw_at, int64_t i, int A, int mode, const float* eps,
                                                      uint64_t seed, uint64_t ctr, uint32_t site, float* a_out,
                                                      float* logp, float* u_out, float* e_out, float* amean) {
  float lp = 0.f;
  for (int d = 0; d < A; ++d) {
    const float mu = raw_at(d);
    const float ls = -6.f + 10.f * sigmoidf(raw_at(A + d));
    const float sd = expf(ls) * 1.0f;
    if (amean) amean[i * A + d] = tanhf(mu);
    if (mode == 2) continue;
    const float e = normal_at(eps, i * A + d, seed, ctr, site);
    const float u = (mode == 0) ? e * sd + mu : mu + e * sd;
    if (a_out) a_out[i * A + d] = tanhf(u);
    if (u_out) u_out[i * A + d] = u;
    if (e_out) e_out[i * A + d] = e;
    const float ladj = 2.f * (0.69314718055994531f - u - softplusf(-2.f * u));
    const float base = -((u - mu) * (u - mu)) / (2.f * (sd * sd)) - logf(sd) - 0.91893853320467274f;
    lp += (0.f - ladj) + base;
  }
  if (logp && mode != 2) logp[i] = lp;
}

// ---------------------------------------------------------------------------
// tile_dense: out[r][c] = act(sum_k in[r][k] * W[c][k] + b[c]) for a tile of RB*16
// rows. `in` / `out` are LDS tiles with row strides ldi / ldo; columns
// [N, round_up(N,16)) of `out` are written as 0 so the next layer can read a
// zero-padded K.
//
// MFMA 16x16x4 f32 mapping (CDNA4): lane l supplies A[row=l&15][k=l>>4] and
// B[k=l>>4][col=l&15]; D[row=4*(l>>4)+r][col=l&15] in acc[r]. A k-chunk of 16 is
// fed as 4 MFMAs where lane group g=l>>4 supplies k = k0+4g+m for MFMA m, so
// both operands are loaded as one float4 per lane (A: ds_read_b128 from LDS).
//
// Weights are read from a PACKED mirror (csrc/pack.hip, drpo_pack_weights): the
// B fragment of (16-column block cb, 16-deep k-step s) is 256 contiguous floats,
// lane l's float4 at offset 4*l, zero-padded beyond N and K:
//     P[(cb*NKS + s)*256 + 4*l + i] = W[16*cb + (l&15)][16*s + 4*(l>>4) + i]
// so every weight load is one lane-linear 1 KB wave access (8 full 128-B lines)
// instead of 16 rows x 64 B (measured 2x slower per MFMA:
// profiles/probes/load_probe.hip), and needs no clamping or masks. The
// backward-data product (dY = dZ W) reads the transposed mirror of the same
// shape with the roles of N and K exchanged.
// ---------------------------------------------------------------------------
//
// Two address forms, chosen per translation unit. Default: one 64-bit per-lane
// address per load (fastest for the MLP kernels: the scalar form below measured
// 5-7% slower there). DRPO_UNIFORM_WEIGHT_LOADS=1 (rollout.hip): (cb, s) are
// wave-uniform at every call site, so the fragment base is formed in SGPRs and
// the only per-lane term is the 32-bit lane offset (saddr-form loads). Inside
// rollout_persist_kernel's horizon loop the per-lane 64-bit addresses are
// loop-invariant, get hoisted and spill (80 spill slots); the scalar form has none.
#ifndef DRPO_UNIFORM_WEIGHT_LOADS
#define DRPO_UNIFORM_WEIGHT_LOADS 0
#endif

// Load / store through a global (address space 1) pointer. Pointers that reach the
// MLP cores as generic (rebuilt from SGPRs by uniform_ptr, or read from a device
// descriptor) otherwise compile to FLAT accesses, which count against lgkmcnt as
// well as vmcnt and complete out of order: every LDS wait then becomes
// "s_waitcnt vmcnt(0) lgkmcnt(0)" and drains the whole weight prefetch ring
// (rollout actor 256x256 layer: 12.9k -> 10.7k cycles per step with global loads).
template <typename T>
static __device__ __forceinline__ T gload(const T* p) {
  return *(const __attribute__((address_space(1))) T*)(p);
}

template <typename T>
static __device__ __forceinline__ void gstore(T* p, T v) {
  *(__attribute__((address_space(1))) T*)(p) = v;
}

// An input tile [tile_rows][kpad] staged into LDS from up to three column-concatenated
// row-major sources (torch.cat([s, a, ...], -1)); the src[0] columns optionally
// normalised as (x - mean) / (std + 1e-6) (src/normalization.py:22-23), columns past
// c0 + c1 + c2 zero. s0 / s1 / s2 are the sources already offset to this member; a
// source whose columns are skipped (skip1: the action block a chain job fills from LDS)
// may be null. Each lane issues its value, mean and std loads together from valid
// addresses and selects afterwards: one memory round trip per element, where indexing
// the descriptor's source array by a per-lane block index cost a pointer load plus
// dependent value / mean / std loads (four round trips; fit staging 2.4 k cycles).
template <int NT>
__device__ __forceinline__ void stage_input_tile(float* xin, int ldx, int tile_rows, int nrows, int64_t row0, int kpad,
                                                 const float* s0, const float* s1, const float* s2, int c0, int c1,
                                                 int c2, int ld0, int ld1, int ld2, const float* nmean,
                                                 const float* nstd, bool skip1, float* save_x, int64_t save_row0) {
  const int din0 = c0 + c1 + c2;
  for (int e = threadIdx.x; e < tile_rows * kpad; e += NT) {
    const int r = e / kpad, k = e - r * kpad;
    float v = 0.f;
    if (r < nrows && k < din0) {
      const int q = k < c0 ? 0 : (k - c0 < c1 ? 1 : 2);
      const int kk = q == 0 ? k : (q == 1 ? k - c0 : k - c0 - c1);
      const bool zero = skip1 && q == 1;
      const bool use0 = q == 0 || zero;
      const float* sp = use0 ? s0 : (q == 1 ? s1 : s2);
      const int ld = use0 ? ld0 : (q == 1 ? ld1 : ld2);
      const float x = gload(sp + (row0 + r) * ld + (zero ? 0 : kk));
      if (nmean) {
        const int km = q == 0 ? kk : 0;
        const float mu = gload(nmean + km), sd = gload(nstd + km);
        v = q == 0 ? (x - mu) / (sd + 1e-6f) : x;
      } else {
        v = x;
      }
      if (zero) v = 0.f;
      if (save_x) gstore(save_x + (save_row0 + r) * din0 + k, v);
    }
    xin[r * ldx + k] = v;
  }
}

static __device__ __forceinline__ const float* uniform_ptr(const float* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
}

static __device__ __forceinline__ f32x4 load_pk(const float* __restrict__ P, int cb, int s, int NKS) {
  if constexpr (DRPO_UNIFORM_WEIGHT_LOADS) {
    const float* base = uniform_ptr(P) + ((size_t)__builtin_amdgcn_readfirstlane(cb * NKS + s) << 8);
    return gload(reinterpret_cast<const f32x4*>(base + ((threadIdx.x & 63) << 2)));
  } else {
    return gload(reinterpret_cast<const f32x4*>(P + ((size_t)(cb * NKS + s) << 8) + ((threadIdx.x & 63) << 2)));
  }
}

// Weight fragments are streamed through a static register ring of depth PF_D:
// the loads for k-step s+PF_D-1 are issued while k-step s computes. The ring is
// indexed only by compile-time constants (unrolled), so it stays in VGPRs.
// Shallow rings: one k-step ahead is enough, and deeper rings only queue behind the
// CU's L1 (round 6: rollout -1.5 %, SAC +0.3 % for 2 against 4-6 deep;
// profiles/r06/ring_ab, and profiles/r06/feed_probe for the stand-alone k-loop).
constexpr int PF_D = 2;

// Ring depth of the unrolled (compile-time K) cores: deeper for waves that own one
// column block (each k-step is then only 4 MFMAs of cover per wave)
constexpr int PF_SCALE = 4;
template <int MAXC>
__host__ __device__ constexpr int pf_depth() {
  return PF_SCALE / MAXC > PF_D ? PF_SCALE / MAXC : PF_D;
}

// Optional global saves of the tile (rows < nrows only): gy = post-activation,
// gz = pre-activation, row stride ldg (already offset to the tile's first row).
struct GSave {
  float* gy;
  float* gz;
  int ldg;
  int nrows;
};

// bias values of this lane's output columns, loaded before the k-loop so their
// latency hides behind it (loaded after the loop they cost a full L2 round trip
// per layer)
template <int NW, int MAXC>
__device__ __forceinline__ void load_bias(const float* __restrict__ bias, int N, float (&bv)[MAXC]) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int col = (wave + NW * c) * 16 + (lane & 15);
    bv[c] = (bias && col < N) ? gload(bias + col) : 0.f;
  }
}

// LDS stores of MFMA accumulators: a 16x16 accumulator's register r holds row 4g + r
// (g = lane >> 4) of column lane & 15. With a row stride == 8 (mod 32) (lds_ld) lane
// groups g = 2h and 2h + 1 of one ds_write_b32 land on the same 16 banks: a 2-way
// conflict that fits inside the store's own 4-cycle transfer (MI355X_MICROARCH.md, LDS),
// so it costs no time. (A conflict-free swizzled order measured slower: profiles/r05/swz_ab.)

// A layer's [rows][N] output tile saved to global from LDS after the layer's barrier,
// as 16-byte stores by every thread of the workgroup (at N = 256 one wave-instruction
// writes one whole 1 KB row) instead of the epilogue's row-strided 4-byte stores (four
// 64 B pieces per wave-instruction, 4x the store instructions).
// N % 4 == 0 and a 16-byte aligned destination (checked by the callers); rows < nrows.
template <int NT, int ROWS>
__device__ __forceinline__ void save_tile_lds(const float* t, int ldt, float* gy, int N, int nrows) {
  const int n4 = N >> 2;
  for (int e = threadIdx.x; e < ROWS * n4; e += NT) {
    const int r = n4 == 64 ? e >> 6 : e / n4, c = e - r * n4;
    if (r < nrows)
      gstore(reinterpret_cast<f32x4*>(gy + (size_t)r * N) + c, *reinterpret_cast<const f32x4*>(t + r * ldt + 4 * c));
  }
}

// a layer save the caller may defer to save_tile_lds: post-activation only, 4-aligned width
__device__ __forceinline__ bool save_deferrable(const float* gy, const float* gz, int N) {
  return gy && !gz && N > 16 && (N & 3) == 0 && (((uintptr_t)gy) & 15) == 0;
}

template <int NW, int RB, int MAXC, int ACT>
__device__ __forceinline__ void dense_epilogue(const f32x4 (&acc)[RB][MAXC], const float (&bvs)[MAXC], int N,
                                               float* out, int ldo, const GSave& gs, int wv = -1) {
  const int lane = threadIdx.x & 63, wave = wv >= 0 ? wv : (int)(threadIdx.x >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int NB = (N + 15) >> 4;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int cb = wave + NW * c;
    if (cb >= NB) continue;
    const int col = cb * 16 + l15;
    const float bv = bvs[c];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rb * 16 + 4 * g + r;
        const float z = acc[rb][c][r] + bv;
        const float y = act_fn<ACT>(z);
        if (out) out[row * ldo + col] = (col < N) ? y : 0.f;
        if (col < N && row < gs.nrows) {
          if (gs.gy) gstore(gs.gy + (size_t)row * gs.ldg + col, y);
          if (gs.gz) gstore(gs.gz + (size_t)row * gs.ldg + col, z);
        }
      }
  }
}

// One layer for an RB*16-row tile by NW waves (NW*64 threads); wave w owns the
// 16-column blocks w, w+NW, ... (MAXC of them; blocks past N compute discarded
// values from a clamped, valid fragment).
// NK > 0: compile-time number of 16-deep k-steps -> fully unrolled, so the weight
// ring and the one-step-ahead LDS A prefetch are indexed statically and the
// compiler's vmcnt accounting never has to cross a loop back-edge (a back-edge
// forces vmcnt(0), collapsing the prefetch distance). NK == 0: runtime K loop.
// Workgroup barrier for LDS hand-offs only. __syncthreads() is a workgroup-scope
// acq_rel fence + s_barrier, and the fence waits for every outstanding global load
// (vmcnt(0)), which drains weight fragments issued ahead of the barrier. Here each
// wave waits only for its own LDS traffic (lgkmcnt(0); LDS ops complete in order)
// before s_barrier (gfx950 backs off barriers with memory operations in flight),
// and the empty asm with a memory clobber keeps the compiler from moving memory
// accesses across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Wave-local LDS hand-off: a wave reads back, in another lane mapping, values that it
// wrote itself (a layer's own output columns as the A operand of a split-K head). A
// wave's LDS operations complete in order, so waiting for its own writes
// (lgkmcnt(0)) suffices; the memory clobbers keep the compiler from moving the reads
// above the writes (per thread the addresses differ, so nothing else orders them).
__device__ __forceinline__ void wave_lds_sync() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // vmcnt(63) expcnt(7) lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}

// Core of tile_dense_impl for a wave that owns exactly MAXC valid column blocks
// (the dispatcher below picks the instantiation per wave).
// NL > 0 (unrolled cores only): the first NL k-steps of every column block are read
// from an LDS copy Pl of the packed mirror, laid out [cb][NL][256] (weights that stay
// the same across the calls of a persistent kernel: fewer bytes per MFMA from L2).
template <int NL>
__device__ __forceinline__ f32x4 load_frag(const float* __restrict__ P, const float* Pl, int cb, int s, int NKS) {
  if (s < NL)
    return *(const __attribute__((address_space(3))) f32x4*)(Pl + ((cb * NL + s) << 8) + ((threadIdx.x & 63) << 2));
  return load_pk(P, cb, s, NKS);
}

// The MFMA part of tile_dense_core for a wave owning exactly MAXC column blocks and a
// compile-time K (NK k-steps): the accumulators and the bias values of the wave's
// columns, for callers that fuse their own epilogue (rollout: the actor's output head
// reduced straight from the hidden layer's accumulators).
template <int NW, int RB, int MAXC, int NK, int NL = 0>
__device__ __forceinline__ void tile_dense_mma(const float* in, int ldi, const float* __restrict__ P,
                                               const float* __restrict__ bias, int N, f32x4 (&acc)[RB][MAXC],
                                               float (&bvs)[MAXC], const float* Pl = nullptr) {
  static_assert(NK > 0, "compile-time K only");
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  int cbs[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) cbs[c] = wave + NW * c;
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) acc[rb][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int PF = pf_depth<MAXC>();
  f32x4 bq[PF][MAXC];
#pragma unroll
  for (int u = 0; u < PF - 1; ++u)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) bq[u][c] = load_frag<NL>(P, Pl, cbs[c], u < NK ? u : NK - 1, NK);
  load_bias<NW, MAXC>(bias, N, bvs);
  f32x4 an[RB], ac[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) an[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 4 * g);
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    if (s + PF - 1 < NK) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) bq[(s + PF - 1) % PF][c] = load_frag<NL>(P, Pl, cbs[c], s + PF - 1, NK);
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) ac[rb] = an[rb];
    if (s + 1 < NK) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
        an[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 16 * (s + 1) + 4 * g);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[rb][m], bq[s % PF][c][m], acc[rb][c], 0, 0, 0);
  }
}

// wv >= 0: the wave index within a sub-group of NW waves (a workgroup split into halves
// that run different layers, e.g. pair_nets); RING > 0: the weight ring depth
template <int NW, int RB, int MAXC, int ACT, int NK, int NL = 0, int RING = 0, int STK = -1>
__device__ __forceinline__ void tile_dense_core(const float* in, int ldi, int K, const float* __restrict__ P,
                                                const float* __restrict__ bias, int N, float* out, int ldo,
                                                const GSave& gs, const float* Pl = nullptr, int wv = -1) {
  static_assert(NL == 0 || NK > 0, "LDS-resident k-steps need the unrolled core");
  static_assert(RING == 0 || NK > 0, "a ring depth needs the unrolled core");
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = wv >= 0 ? wv : (int)(tid >> 6);
  const int l15 = lane & 15, g = lane >> 4;
  const int NKS = NK > 0 ? NK : (K + 15) >> 4;
  int cbs[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) cbs[c] = wave + NW * c;

  f32x4 acc[RB][MAXC];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) acc[rb][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int PF = RING > 0 ? RING : (NK > 0 ? pf_depth<MAXC>() : PF_D);
  f32x4 bq[PF][MAXC];
#pragma unroll
  for (int u = 0; u < PF - 1; ++u)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) bq[u][c] = load_frag<NL>(P, Pl, cbs[c], min(u, NKS - 1), NKS);
  float bvs[MAXC];
  if (wv >= 0) {
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int col = cbs[c] * 16 + l15;
      bvs[c] = (bias && col < N) ? gload(bias + col) : 0.f;
    }
  } else {
    load_bias<NW, MAXC>(bias, N, bvs);
  }

  if constexpr (NK > 0) {
    f32x4 an[RB], ac[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) an[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 4 * g);
#pragma unroll
    for (int s = 0; s < NK; ++s) {
      if (s + PF - 1 < NK) {
#pragma unroll
        for (int c = 0; c < MAXC; ++c) bq[(s + PF - 1) % PF][c] = load_frag<NL>(P, Pl, cbs[c], s + PF - 1, NKS);
      }
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) ac[rb] = an[rb];
      if (s + 1 < NK) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          an[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 16 * (s + 1) + 4 * g);
      }
      // keep the prefetches where they are: without this fence the scheduler sinks
      // them next to their consumers and the ring degenerates to distance 1
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int c = 0; c < MAXC; ++c)
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
            acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[rb][m], bq[s % PF][c][m], acc[rb][c], 0, 0, 0);
    }
    if constexpr (STK >= 0) CORE_STAMP(STK);   // k-loop issued (profiling builds)
  } else {
    for (int kb = 0; kb < NKS; kb += PF_D) {
#pragma unroll
      for (int u = 0; u < PF_D; ++u) {
        const int s = kb + u;
#pragma unroll
        for (int c = 0; c < MAXC; ++c)
          bq[(u + PF_D - 1) % PF_D][c] = load_pk(P, cbs[c], min(s + PF_D - 1, NKS - 1), NKS);
        if (s < NKS) {
          f32x4 a[RB];
#pragma unroll
          for (int rb = 0; rb < RB; ++rb)
            a[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 16 * s + 4 * g);
#pragma unroll
          for (int m = 0; m < 4; ++m)
#pragma unroll
            for (int c = 0; c < MAXC; ++c)
#pragma unroll
              for (int rb = 0; rb < RB; ++rb)
                acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb][m], bq[u][c][m], acc[rb][c], 0, 0, 0);
        }
      }
    }
  }
  dense_epilogue<NW, RB, MAXC, ACT>(acc, bvs, N, out, ldo, gs, wv);
}

// Wave w owns column blocks w, w+NW, ... < NCB: when NW does not divide NCB (13
// blocks of a 200-wide layer on 8 waves) the waves own different counts, and each
// runs the instantiation for its own count, so no wave loads or multiplies a
// padding block (the branch is wave-uniform).
template <int NW, int RB, int NC, int ACT, int NK, int NL = 0>
__device__ __forceinline__ void tile_dense_nc(int nc, const float* in, int ldi, int K, const float* __restrict__ P,
                                              const float* __restrict__ bias, int N, float* out, int ldo,
                                              const GSave& gs, const float* Pl = nullptr) {
  if (nc == NC) tile_dense_core<NW, RB, NC, ACT, NK, NL>(in, ldi, K, P, bias, N, out, ldo, gs, Pl);
  else if constexpr (NC > 1) tile_dense_nc<NW, RB, NC - 1, ACT, NK, NL>(nc, in, ldi, K, P, bias, N, out, ldo, gs, Pl);
}

template <int NW, int RB, int MAXC, int ACT, int NK, int NL = 0>
__device__ __forceinline__ void tile_dense_impl(const float* in, int ldi, int K, const float* __restrict__ P,
                                                const float* __restrict__ bias, int N, float* out, int ldo,
                                                const GSave& gs = GSave{nullptr, nullptr, 0, 0},
                                                const float* Pl = nullptr) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NCB = (N + 15) >> 4;
  const int nc = wave < NCB ? min(MAXC, (NCB - wave + NW - 1) / NW) : 0;
  tile_dense_nc<NW, RB, MAXC, ACT, NK, NL>(nc, in, ldi, K, P, bias, N, out, ldo, gs, Pl);
}

// 200-wide layer with K = 200 (13 column blocks x 13 k-steps) on 8 waves, balanced over
// the 4 SIMDs (wave w runs on SIMD w % 4): waves 0-3 own blocks w and w + 8, waves 4-7
// own block w plus a quarter of block 12's k-steps (4 / 3 / 3 / 3). Each SIMD then
// issues 3.25 blocks of MFMAs instead of 4 on SIMD 0 and 3 on the others. Block 12's
// partial tiles go to red[4][256]; after the caller's barrier tile_dense_13s_finish
// sums them (fixed order), adds the bias and applies the activation. Returns the bias
// value that thread (< 256) needs for the finish. Weight ring 2 deep: deeper rings only
// queue behind the L1 (6 / 8 deep: +3 % per rollout launch; profiles/r06/ring_ab).
template <int ACT>
__device__ __forceinline__ float tile_dense_13s(const float* in, int ldi, const float* __restrict__ P,
                                                const float* __restrict__ bias, float* out, int ldo, float* red) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  if (wave < 4) {
    const int col = 192 + (threadIdx.x & 15);
    const float b12 = col < 200 ? gload(bias + col) : 0.f;
    tile_dense_core<8, 1, 2, ACT, 13, 0, 2>(in, ldi, 200, P, bias, 200, out, ldo, GSave{nullptr, nullptr, 0, 0});
    return b12;
  }
  const int q = wave - 4;
  const int ks0 = q == 0 ? 0 : 1 + 3 * q, nks = q == 0 ? 4 : 3;
  f32x4 bq[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) bq[u] = load_pk(P, 12, ks0 + (u < nks ? u : nks - 1), 13);
  tile_dense_core<8, 1, 1, ACT, 13, 0, 2>(in, ldi, 200, P, bias, 200, out, ldo, GSave{nullptr, nullptr, 0, 0});
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (u < nks) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(in + l15 * ldi + 16 * (ks0 + u) + 4 * g);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], bq[u][m], acc, 0, 0, 0);
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[q * 256 + (4 * g + r) * 16 + l15] = acc[r];
  return 0.f;
}

template <int ACT>
__device__ __forceinline__ void tile_dense_13s_finish(const float* red, float b12, float* out, int ldo) {
  const int tid = threadIdx.x;
  if (tid < 256) {
    const int r = tid >> 4, c = tid & 15;
    const float z = ((red[tid] + red[256 + tid]) + (red[512 + tid] + red[768 + tid])) + b12;
    out[r * ldo + 192 + c] = 192 + c < 200 ? act_fn<ACT>(z) : 0.f;
  }
}

// K (input width) -> compile-time k-step count for the widths on the path
// (<= 16 inputs -> 1 step, 49..64 -> 4, 200 -> 13, 256 -> 16), else the runtime loop.
template <int NW, int RB, int MAXC, int ACT>
__device__ __forceinline__ void tile_dense(const float* in, int ldi, int K, const float* P, const float* bias, int N,
                                           float* out, int ldo, const GSave& gs = GSave{nullptr, nullptr, 0, 0}) {
  switch ((K + 15) >> 4) {
    case 1: tile_dense_impl<NW, RB, MAXC, ACT, 1>(in, ldi, K, P, bias, N, out, ldo, gs); break;
    // tracking's 51 / 53 inputs: unrolled, so all four k-steps' fragments are in flight at once
    case 4: tile_dense_impl<NW, RB, MAXC, ACT, 4>(in, ldi, K, P, bias, N, out, ldo, gs); break;
    case 13: tile_dense_impl<NW, RB, MAXC, ACT, 13>(in, ldi, K, P, bias, N, out, ldo, gs); break;
    case 16: tile_dense_impl<NW, RB, MAXC, ACT, 16>(in, ldi, K, P, bias, N, out, ldo, gs); break;
    default: tile_dense_impl<NW, RB, MAXC, ACT, 0>(in, ldi, K, P, bias, N, out, ldo, gs); break;
  }
}

// Narrow layer (N <= 16, one column block): the K reduction is split over the NW
// waves (k-steps s == wave mod NW), partial 16x16 tiles are summed through LDS
// (`red`: NW*RB*256 floats), then bias + activation. Avoids one wave doing the
// whole narrow head serially while the others idle.
//
// tile_dense_narrow_partials stops after the hand-off: the value of (row, col) is
// narrow_sum<NW, RB>(red, row, col) + bias[col], summed in the same order as
// tile_dense_narrow's epilogue (callers fuse their own elementwise work there).
template <int NW, int RB>
__device__ __forceinline__ float narrow_sum(const float* red, int row, int col) {
  const int rb = row >> 4, rr = row & 15;
  float v = 0.f;
#pragma unroll
  for (int w = 0; w < NW; ++w) v += red[(w * RB + rb) * 256 + rr * 16 + col];
  return v;
}

template <int NW, int RB, bool LDSW = false>
__device__ __forceinline__ void tile_dense_narrow_partials(const float* in, int ldi, int K,
                                                           const float* __restrict__ P, float* red,
                                                           const float* Pl = nullptr) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int NKS = (K + 15) >> 4;
  f32x4 acc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int MAXS = (16 + NW - 1) / NW;
  f32x4 b[MAXS], a[MAXS][RB];
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    const int s = wave + NW * q;
    const int sc = s < NKS ? s : 0;
    b[q] = LDSW ? load_frag<16>(P, Pl, 0, sc, 16) : load_pk(P, 0, sc, NKS);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) a[q][rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + sc * 16 + 4 * g);
  }
  for (int kb = NW * MAXS; kb < NKS; kb += NW) {
    if (kb + wave < NKS) {
      const f32x4 bb = load_pk(P, 0, kb + wave, NKS);   // K > 256 (never LDS-resident)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const f32x4 aa = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + (kb + wave) * 16 + 4 * g);
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa[m], bb[m], acc[rb], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    if (wave + NW * q < NKS) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][rb][m], b[q][m], acc[rb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * RB + rb) * 256 + (4 * g + r) * 16 + l15] = acc[rb][r];
  lds_barrier();
}

template <int NW, int RB, int ACT>
__device__ __forceinline__ void tile_dense_narrow(const float* in, int ldi, int K, const float* __restrict__ P,
                                                  const float* __restrict__ bias, int N, float* out, int ldo,
                                                  float* red, const GSave& gs = GSave{nullptr, nullptr, 0, 0}) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int NKS = (K + 15) >> 4;
  f32x4 acc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // each wave: at most ceil(16/NW) k-steps for K <= 256; issue all loads first
  constexpr int MAXS = (16 + NW - 1) / NW;
  f32x4 b[MAXS], a[MAXS][RB];
  const float bias_v = (bias && (tid & 15) < N) ? gload(bias + (tid & 15)) : 0.f;   // column (e & 15) == (tid & 15) below
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    const int s = wave + NW * q;
    const int sc = s < NKS ? s : 0;
    b[q] = load_pk(P, 0, sc, NKS);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) a[q][rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + sc * 16 + 4 * g);
  }
  for (int kb = NW * MAXS; kb < NKS; kb += NW) {   // K > 16*NW*MAXS (only for K > 256)
    if (kb + wave < NKS) {
      const f32x4 bb = load_pk(P, 0, kb + wave, NKS);
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const f32x4 aa = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + (kb + wave) * 16 + 4 * g);
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(aa[m], bb[m], acc[rb], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    if (wave + NW * q < NKS) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][rb][m], b[q][m], acc[rb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * RB + rb) * 256 + (4 * g + r) * 16 + l15] = acc[rb][r];
  lds_barrier();
  for (int e = tid; e < RB * 256; e += NW * 64) {
    const int rb = e >> 8, rr = (e >> 4) & 15, col = e & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) v += red[(w * RB + rb) * 256 + rr * 16 + col];
    const float z = v + bias_v;
    const float y = act_fn<ACT>(z);
    const int row = rb * 16 + rr;
    if (out) out[row * ldo + col] = (col < N) ? y : 0.f;
    if (col < N && row < gs.nrows) {
      if (gs.gy) gstore(gs.gy + (size_t)row * gs.ldg + col, y);
      if (gs.gz) gstore(gs.gz + (size_t)row * gs.ldg + col, z);
    }
  }
}


// Two independent layers on the SAME input tile, fused into one k-loop (e.g. the
// dynamics model's diff and log-var heads, src/dynamics.py:84-91): column blocks
// [0, NCB1) come from mirror P1 (N1 outputs -> out1), [NCB1, NCB1+NCB2) from P2
// (N2 -> out2). One pass instead of two halves the layer's serial latency and
// gives each wave more independent accumulators.
template <int NW, int RB, int MAXC, int ACT, int NK, int RING = 0>
__device__ __forceinline__ void tile_dense_pair_core(const float* in, int ldi, int K, const float* __restrict__ P1,
                                                     const float* __restrict__ b1, int N1, float* out1,
                                                     const float* __restrict__ P2, const float* __restrict__ b2,
                                                     int N2, float* out2, int ldo, const GSave& gs1,
                                                     const GSave& gs2) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int NCB1 = (N1 + 15) >> 4, NCB2 = (N2 + 15) >> 4;
  const float* Pc[MAXC];
  int cbs[MAXC];
  float bvs[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int cb = wave + NW * c;   // < NCB1 + NCB2 (the dispatcher's count)
    const bool second = cb >= NCB1;
    Pc[c] = second ? P2 : P1;
    cbs[c] = second ? cb - NCB1 : cb;
    const int col = cbs[c] * 16 + l15;
    const float* bb = second ? b2 : b1;
    const int nn = second ? N2 : N1;
    bvs[c] = (bb && col < nn) ? gload(bb + col) : 0.f;
  }
  f32x4 acc[RB][MAXC];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) acc[rb][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  // ring depth (RING = 0: PF_D); a 4-waves-per-SIMD kernel has 128 VGPRs, where 2 fits
  // 4 blocks per wave (one k-step ahead still covers 16 MFMAs per wave)
  constexpr int PFP = RING > 0 ? RING : PF_D;
  f32x4 bq[PFP][MAXC];
#pragma unroll
  for (int u = 0; u < PFP - 1; ++u)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) bq[u][c] = load_pk(Pc[c], cbs[c], min(u, NK - 1), NK);
  f32x4 an[RB], ac[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) an[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 4 * g);
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    if (s + PFP - 1 < NK) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) bq[(s + PFP - 1) % PFP][c] = load_pk(Pc[c], cbs[c], s + PFP - 1, NK);
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) ac[rb] = an[rb];
    if (s + 1 < NK) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
        an[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 16 * (s + 1) + 4 * g);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[rb][m], bq[s % PFP][c][m], acc[rb][c], 0, 0, 0);
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int cb = wave + NW * c;
    if (cb >= NCB1 + NCB2) continue;
    const bool second = cb >= NCB1;
    float* out = second ? out2 : out1;
    const int nn = second ? N2 : N1;
    const GSave& gs = second ? gs2 : gs1;
    const int col = cbs[c] * 16 + l15;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rb * 16 + 4 * g + r;
        const float z = acc[rb][c][r] + bvs[c];
        const float y = act_fn<ACT>(z);
        out[row * ldo + col] = (col < nn) ? y : 0.f;
        if (col < nn && row < gs.nrows) {
          if (gs.gy) gstore(gs.gy + (size_t)row * gs.ldg + col, y);
          if (gs.gz) gstore(gs.gz + (size_t)row * gs.ldg + col, z);
        }
      }
  }
}

template <int NW, int RB, int NC, int ACT, int NK, int RING = 0>
__device__ __forceinline__ void tile_dense_pair_nc(int nc, const float* in, int ldi, int K, const float* P1,
                                                   const float* b1, int N1, float* out1, const float* P2,
                                                   const float* b2, int N2, float* out2, int ldo, const GSave& gs1,
                                                   const GSave& gs2) {
  if (nc == NC) tile_dense_pair_core<NW, RB, NC, ACT, NK, RING>(in, ldi, K, P1, b1, N1, out1, P2, b2, N2, out2, ldo, gs1, gs2);
  else if constexpr (NC > 1)
    tile_dense_pair_nc<NW, RB, NC - 1, ACT, NK, RING>(nc, in, ldi, K, P1, b1, N1, out1, P2, b2, N2, out2, ldo, gs1, gs2);
}

// per-wave block count dispatch as in tile_dense_impl
template <int NW, int RB, int MAXC, int ACT, int NK, int RING = 0>
__device__ __forceinline__ void tile_dense_pair(const float* in, int ldi, int K, const float* P1, const float* b1,
                                                int N1, float* out1, const float* P2, const float* b2, int N2,
                                                float* out2, int ldo,
                                                const GSave& gs1 = GSave{nullptr, nullptr, 0, 0},
                                                const GSave& gs2 = GSave{nullptr, nullptr, 0, 0}) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NCB = ((N1 + 15) >> 4) + ((N2 + 15) >> 4);
  const int nc = wave < NCB ? min(MAXC, (NCB - wave + NW - 1) / NW) : 0;
  tile_dense_pair_nc<NW, RB, MAXC, ACT, NK, RING>(nc, in, ldi, K, P1, b1, N1, out1, P2, b2, N2, out2, ldo, gs1, gs2);
}

// Two independent layers on DIFFERENT input tiles in one k-loop: column blocks
// [0, NCB1) are in1 x P1 (N1 outputs -> out1), [NCB1, NCB1+NCB2) in2 x P2 (N2 -> out2);
// both K = NK k-steps. Each k-step reads both inputs' A fragments and every block
// multiplies the one of its layer (the diff and log-var output layers of the dynamics
// model side by side; the heads of a trunk network backward together).
template <int NW, int RB, int MAXC, int ACT, int NK, int RING = 0>
__device__ __forceinline__ void tile_dense_pair2_core(const float* in1, const float* in2, int ldi,
                                                      const float* __restrict__ P1, const float* __restrict__ b1,
                                                      int N1, float* out1, const float* __restrict__ P2,
                                                      const float* __restrict__ b2, int N2, float* out2, int ldo,
                                                      const GSave& gs1, const GSave& gs2) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int NCB1 = (N1 + 15) >> 4, NCB2 = (N2 + 15) >> 4;
  const float* Pc[MAXC];
  int cbs[MAXC];
  bool sec[MAXC];
  float bvs[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int cb = wave + NW * c;
    sec[c] = cb >= NCB1;
    Pc[c] = sec[c] ? P2 : P1;
    cbs[c] = sec[c] ? cb - NCB1 : cb;
    const int col = cbs[c] * 16 + l15;
    const float* bb = sec[c] ? b2 : b1;
    const int nn = sec[c] ? N2 : N1;
    bvs[c] = (bb && col < nn) ? gload(bb + col) : 0.f;
  }
  // one block per wave: even / odd k-steps into two accumulators, two independent MFMA
  // chains instead of one 4*NK-long dependent chain (summed in the epilogue)
  constexpr int NACC = MAXC == 1 && NK > 1 ? 2 : 1;
  f32x4 acc[RB][MAXC], acc2[RB][MAXC];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) acc[rb][c] = acc2[rb][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int PFP = RING > 0 ? RING : PF_D;
  f32x4 bq[PFP][MAXC];
#pragma unroll
  for (int u = 0; u < PFP - 1; ++u)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) bq[u][c] = load_pk(Pc[c], cbs[c], u < NK ? u : NK - 1, NK);
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    if (s + PFP - 1 < NK) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) bq[(s + PFP - 1) % PFP][c] = load_pk(Pc[c], cbs[c], s + PFP - 1, NK);
    }
    f32x4 a1[RB], a2[RB];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      a1[rb] = *reinterpret_cast<const f32x4*>(in1 + (rb * 16 + l15) * ldi + 16 * s + 4 * g);
      a2[rb] = *reinterpret_cast<const f32x4*>(in2 + (rb * 16 + l15) * ldi + 16 * s + 4 * g);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb) {
          f32x4& ac = (NACC == 2 && (s & 1)) ? acc2[rb][c] : acc[rb][c];
          ac = __builtin_amdgcn_mfma_f32_16x16x4f32(sec[c] ? a2[rb][m] : a1[rb][m], bq[s % PFP][c][m], ac, 0, 0, 0);
        }
  }
  if constexpr (NACC == 2) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int c = 0; c < MAXC; ++c) acc[rb][c] += acc2[rb][c];
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int cb = wave + NW * c;
    if (cb >= NCB1 + NCB2) continue;
    float* out = sec[c] ? out2 : out1;
    const int nn = sec[c] ? N2 : N1;
    const GSave& gs = sec[c] ? gs2 : gs1;
    const int col = cbs[c] * 16 + l15;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = rb * 16 + 4 * g + r;
        const float z = acc[rb][c][r] + bvs[c];
        const float y = act_fn<ACT>(z);
        if (out) out[row * ldo + col] = (col < nn) ? y : 0.f;
        if (col < nn && row < gs.nrows) {
          if (gs.gy) gstore(gs.gy + (size_t)row * gs.ldg + col, y);
          if (gs.gz) gstore(gs.gz + (size_t)row * gs.ldg + col, z);
        }
      }
  }
}

template <int NW, int RB, int NC, int ACT, int NK, int RING>
__device__ __forceinline__ void tile_dense_pair2_nc(int nc, const float* in1, const float* in2, int ldi,
                                                    const float* P1, const float* b1, int N1, float* out1,
                                                    const float* P2, const float* b2, int N2, float* out2, int ldo,
                                                    const GSave& gs1, const GSave& gs2) {
  if (nc == NC)
    tile_dense_pair2_core<NW, RB, NC, ACT, NK, RING>(in1, in2, ldi, P1, b1, N1, out1, P2, b2, N2, out2, ldo, gs1, gs2);
  else if constexpr (NC > 1)
    tile_dense_pair2_nc<NW, RB, NC - 1, ACT, NK, RING>(nc, in1, in2, ldi, P1, b1, N1, out1, P2, b2, N2, out2, ldo, gs1,
                                                       gs2);
}

template <int NW, int RB, int MAXC, int ACT, int NK, int RING = 0>
__device__ __forceinline__ void tile_dense_pair2(const float* in1, const float* in2, int ldi, const float* P1,
                                                 const float* b1, int N1, float* out1, const float* P2,
                                                 const float* b2, int N2, float* out2, int ldo,
                                                 const GSave& gs1 = GSave{nullptr, nullptr, 0, 0},
                                                 const GSave& gs2 = GSave{nullptr, nullptr, 0, 0}) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NCB = ((N1 + 15) >> 4) + ((N2 + 15) >> 4);
  const int nc = wave < NCB ? min(MAXC, (NCB - wave + NW - 1) / NW) : 0;
  tile_dense_pair2_nc<NW, RB, MAXC, ACT, NK, RING>(nc, in1, in2, ldi, P1, b1, N1, out1, P2, b2, N2, out2, ldo, gs1, gs2);
}

// out = act([in1 | in2] x [P1; P2] + bias): one layer whose K is the concatenation of
// two inputs (NK k-steps each) with their own packed mirrors -- the sum of two heads'
// contributions to a shared trunk gradient as ONE product (one pipeline fill, one
// epilogue, no intermediate LDS round trip).
template <int NW, int RB, int MAXC, int ACT, int NK>
__device__ __forceinline__ void tile_dense_catk_core(const float* in1, const float* in2, int ldi,
                                                     const float* __restrict__ P1, const float* __restrict__ P2,
                                                     const float* __restrict__ bias, int N, float* out, int ldo,
                                                     const GSave& gs) {
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  int cbs[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) cbs[c] = wave + NW * c;
  f32x4 acc[RB][MAXC];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) acc[rb][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int PF = pf_depth<MAXC>();
  constexpr int NS = 2 * NK;
  f32x4 bq[PF][MAXC];
  // k-step s of the concatenation: s < NK from (in1, P1), else (in2, P2) at s - NK
  auto frag = [&](int c, int s) { return s < NK ? load_pk(P1, cbs[c], s, NK) : load_pk(P2, cbs[c], s - NK, NK); };
  auto afrag = [&](int rb, int s) {
    const float* in = s < NK ? in1 : in2;
    const int ks = s < NK ? s : s - NK;
    return *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 16 * ks + 4 * g);
  };
#pragma unroll
  for (int u = 0; u < PF - 1; ++u)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) bq[u][c] = frag(c, u);
  float bvs[MAXC];
  load_bias<NW, MAXC>(bias, N, bvs);
  f32x4 an[RB], ac[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) an[rb] = afrag(rb, 0);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (s + PF - 1 < NS) {
#pragma unroll
      for (int c = 0; c < MAXC; ++c) bq[(s + PF - 1) % PF][c] = frag(c, s + PF - 1);
    }
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) ac[rb] = an[rb];
    if (s + 1 < NS) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) an[rb] = afrag(rb, s + 1);
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < MAXC; ++c)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[rb][m], bq[s % PF][c][m], acc[rb][c], 0, 0, 0);
  }
  dense_epilogue<NW, RB, MAXC, ACT>(acc, bvs, N, out, ldo, gs);
}

template <int NW, int RB, int NC, int ACT, int NK>
__device__ __forceinline__ void tile_dense_catk_nc(int nc, const float* in1, const float* in2, int ldi, const float* P1,
                                                   const float* P2, const float* bias, int N, float* out, int ldo,
                                                   const GSave& gs) {
  if (nc == NC) tile_dense_catk_core<NW, RB, NC, ACT, NK>(in1, in2, ldi, P1, P2, bias, N, out, ldo, gs);
  else if constexpr (NC > 1) tile_dense_catk_nc<NW, RB, NC - 1, ACT, NK>(nc, in1, in2, ldi, P1, P2, bias, N, out, ldo, gs);
}

template <int NW, int RB, int MAXC, int ACT, int NK>
__device__ __forceinline__ void tile_dense_catk(const float* in1, const float* in2, int ldi, const float* P1,
                                                const float* P2, const float* bias, int N, float* out, int ldo,
                                                const GSave& gs = GSave{nullptr, nullptr, 0, 0}) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NCB = (N + 15) >> 4;
  const int nc = wave < NCB ? min(MAXC, (NCB - wave + NW - 1) / NW) : 0;
  tile_dense_catk_nc<NW, RB, MAXC, ACT, NK>(nc, in1, in2, ldi, P1, P2, bias, N, out, ldo, gs);
}

// Which head (bit 2) and which base block (bits 0-1) a wave of an 8-wave workgroup runs in
// the paired 200-wide heads (rollout.hip pair_split_heads, fit.hip's heads phase): the diff
// head on waves 0, 1, 2, 7 (bases 0, 1, 2, 3), the log-var head on waves 3-6 (bases 0-3).
// Base 0 owns 4 of the 13 blocks, so SIMD 0 (waves 0 / 4) and SIMD 3 (waves 3 / 7) carry 7
// blocks each, the older wave the 4-block one on both. The round-5 map (head by wave half,
// base w / 7 - w) had the 4-block wave older on SIMD 0 and younger on SIMD 3, and ran the
// rollout 4.7 % and the fit 1.3 % slower at config 2 (profiles/r06/pair_map); making both
// SIMDs alike either way (4-block wave older, or younger on both) measured the same.
// The partial slot of (head, base) stays where narrow_pair_sum expects it:
// head 0 slot base, head 1 slot NW/2 + 3 - base.
__device__ __forceinline__ unsigned pair_wave_code(int wave) { return (0x37654210u >> (4 * wave)) & 7u; }

// Partials-only form of tile_dense_narrow_pair (below): the value of layer `which`
// at (row, col) is narrow_pair_sum<NW, RB>(red, which, row, col) + its bias, in the
// same summation order as tile_dense_narrow_pair's epilogue.
template <int NW, int RB>
__device__ __forceinline__ float narrow_pair_sum(const float* red, int which, int row, int col) {
  constexpr int HW = NW / 2;
  const int rb = row >> 4, rr = row & 15;
  float v = 0.f;
#pragma unroll
  for (int w = 0; w < HW; ++w) v += red[((which * HW + w) * RB + rb) * 256 + rr * 16 + col];
  return v;
}

template <int NW, int RB>
__device__ __forceinline__ void tile_dense_narrow_pair_partials(const float* in1, const float* in2, int ldi, int K,
                                                                const float* __restrict__ P1,
                                                                const float* __restrict__ P2, float* red) {
  constexpr int HW = NW / 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int NKS = (K + 15) >> 4;
  const bool second = wave >= HW;
  const int wl = second ? wave - HW : wave;
  const float* P = second ? P2 : P1;
  const float* in = second ? in2 : in1;
  f32x4 acc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int MAXS = (16 + HW - 1) / HW;      // K <= 256
  f32x4 b[MAXS], a[MAXS][RB];
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    const int s = wl + HW * q;
    const int sc = s < NKS ? s : 0;
    b[q] = load_pk(P, 0, sc, NKS);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) a[q][rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + sc * 16 + 4 * g);
  }
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    if (wl + HW * q < NKS) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][rb][m], b[q][m], acc[rb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * RB + rb) * 256 + (4 * g + r) * 16 + l15] = acc[rb][r];
  lds_barrier();
}

// Two narrow layers (N1, N2 <= 16) on two input tiles at once: waves [0, NW/2) split
// layer 1's K, waves [NW/2, NW) layer 2's; partials summed through `red`.
template <int NW, int RB, int ACT>
__device__ __forceinline__ void tile_dense_narrow_pair(const float* in1, const float* in2, int ldi, int K,
                                                       const float* __restrict__ P1, const float* __restrict__ b1,
                                                       int N1, float* out1, const float* __restrict__ P2,
                                                       const float* __restrict__ b2, int N2, float* out2, int ldo,
                                                       float* red, const GSave& gs1 = GSave{nullptr, nullptr, 0, 0},
                                                       const GSave& gs2 = GSave{nullptr, nullptr, 0, 0}) {
  constexpr int HW = NW / 2;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l15 = lane & 15, g = lane >> 4;
  const int NKS = (K + 15) >> 4;
  const bool second = wave >= HW;
  const int wl = second ? wave - HW : wave;
  const float* P = second ? P2 : P1;
  const float* in = second ? in2 : in1;
  f32x4 acc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float bias1 = (b1 && (tid & 15) < N1) ? gload(b1 + (tid & 15)) : 0.f;
  const float bias2 = (b2 && (tid & 15) < N2) ? gload(b2 + (tid & 15)) : 0.f;
  constexpr int MAXS = (16 + HW - 1) / HW;      // K <= 256
  f32x4 b[MAXS], a[MAXS][RB];
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    const int s = wl + HW * q;
    const int sc = s < NKS ? s : 0;
    b[q] = load_pk(P, 0, sc, NKS);
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) a[q][rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + sc * 16 + 4 * g);
  }
#pragma unroll
  for (int q = 0; q < MAXS; ++q) {
    if (wl + HW * q < NKS) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][rb][m], b[q][m], acc[rb], 0, 0, 0);
    }
  }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wave * RB + rb) * 256 + (4 * g + r) * 16 + l15] = acc[rb][r];
  lds_barrier();
  for (int e = tid; e < 2 * RB * 256; e += NW * 64) {
    const int which = e / (RB * 256), e2 = e - which * RB * 256;
    const int rb = e2 >> 8, rr = (e2 >> 4) & 15, col = e2 & 15;
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < HW; ++w) v += red[((which * HW + w) * RB + rb) * 256 + rr * 16 + col];
    const int nn = which ? N2 : N1;
    const float z = v + (which ? bias2 : bias1);
    float* out = which ? out2 : out1;
    const float y = act_fn<ACT>(z);
    const int row = rb * 16 + rr;
    out[row * ldo + col] = (col < nn) ? y : 0.f;
    const GSave& gs = which ? gs2 : gs1;
    if (col < nn && row < gs.nrows) {
      if (gs.gy) gstore(gs.gy + (size_t)row * gs.ldg + col, y);
      if (gs.gz) gstore(gs.gz + (size_t)row * gs.ldg + col, z);
    }
  }
}

}  // namespace drpo
