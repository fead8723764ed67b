// Fused imagined-rollout step (SMBPO.rollout, src/smbpo.py:229-249).
//
// One launch of rollout_step_kernel processes one horizon step for every alive
// row: each 512-thread workgroup (8 wave64s, 2 per SIMD) owns a 16- or 32-row tile and keeps all of its
// activations in LDS while it runs
//   actor MLP S->H->H->2A (ReLU)  +  squashed-Gaussian sample   (src/policy.py:89-97)
//   elite member MLP trunk/diff/log-var heads (SiLU) + log-var clamp + Gaussian
//   sample                                                      (src/dynamics.py:112-122,198-203)
//   env constraint functions                                    (env_constraints.hpp)
//   the 7-component row write into the circular virtual buffer  (src/sampling.py:128-145)
// and emits per-tile alive counts plus an in-tile compaction map. The next step's
// launch performs the order-preserving `next_states[~dones]` compaction
// (src/smbpo.py:243-246) itself: each workgroup scans the previous step's tile
// counts and binary-searches the source row of each of its rows, so a horizon
// step is ONE launch. Row counts and buffer offsets live on the device, so a whole
// rollout needs no host synchronisation.
#include <stdarg.h>
#include <stdio.h>

#include <hip/hip_runtime.h>

#define DRPO_UNIFORM_WEIGHT_LOADS 1   // scalar-base weight loads (see load_pk)

#ifdef DRPO_STAMPS
// profiling builds only (profiles/stamps.py): per-workgroup s_memtime stamps
__device__ unsigned long long g_stamps_roll[1 << 14][16];
#define RSTAMP(i)                                                                                 \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long _t;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (threadIdx.x == 0 && blockIdx.x < (1u << 14)) g_stamps_roll[blockIdx.x][(i)] = _t;         \
  } while (0)
#define CORE_STAMP(i) RSTAMP(i)   // sub-phase stamps inside the layer cores (profiles/stamps.py)
#define CORE_STAMP_W4(i)                                                                          \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long _t;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (threadIdx.x == 256 && blockIdx.x < (1u << 14)) g_stamps_roll[blockIdx.x][(i)] = _t;       \
  } while (0)
extern "C" __attribute__((visibility("default"))) int drpo_debug_stamps_rollout(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps_roll), sizeof(unsigned long long) * 16 * (size_t)n);
}
#else
#define RSTAMP(i) \
  do {            \
  } while (0)
#endif

#include "common.hpp"
#include "env_constraints.hpp"

using namespace drpo;

struct RolloutStepArgs {
  int S, A, C, Ha, Hm, t, Bmax;
  EnvParams env;
  // actor (row-major [out][in] weights)
  const float *aW1, *ab1, *aW2, *ab2, *aW3, *ab3;
  // elite member slices of the ensemble
  const float *mW1, *mb1, *mW2, *mb2, *dW1, *db1, *dW2, *db2, *lW1, *lb1, *lW2, *lb2;
  const float *norm_mean, *norm_std, *min_lv, *max_lv;
  // step-0 source: replay buffer states (physical layout) + chronological indices
  const float* replay_states;
  const int64_t* init_idx;        // nullptr -> device PRP sample without replacement
  int64_t replay_len, replay_ptr, replay_cap;
  uint32_t prp_key[4];
  int prp_half_bits;
  // step t>0 source: previous step's next states + compaction map
  const float* prev_nxt;
  const int* prev_cnt;
  const int* prev_inv;
  // device step bookkeeping (n[t], off[t] written by workgroup 0 of step t)
  int* n;
  int64_t* off;
  // noise: parity mode (caller-provided eps rows for this step) or Philox
  const float* eps_a;             // [Bmax][A]
  const float* eps_m;             // [Bmax][S+1]
  uint64_t seed, ctr;
  // virtual buffer
  float *vs, *va, *vs2, *vr, *vh;
  uint8_t *vd, *vv;
  const int64_t* vptr;
  int64_t vcap;
  // this step's outputs for the next step
  float* nxt;
  int* cnt;
  int* inv;
  // LDS strides
  int ldx, ldh, ldm, lds;
};

__device__ __forceinline__ uint32_t prp_round(uint32_t r, uint32_t k) {
  uint32_t h = r * 0x9E3779B1u ^ k;
  h ^= h >> 15;
  h *= 0x85EBCA77u;
  h ^= h >> 13;
  h *= 0xC2B2AE3Du;
  h ^= h >> 16;
  return h;
}

// Keyed 4-round Feistel permutation of [0, 2^(2*hb)) with cycle walking into
// [0, N): the first B outputs are B distinct indices (sampling without
// replacement, the production stand-in for np.random.choice(N, B, replace=False)).
__device__ inline int64_t prp_index(uint64_t i, uint64_t N, int hb, const uint32_t key[4]) {
  const uint32_t mask = (hb >= 32) ? 0xFFFFFFFFu : ((1u << hb) - 1u);
  uint64_t x = i;
  for (int it = 0; it < 64; ++it) {
    uint32_t L = (uint32_t)(x >> hb) & mask, R = (uint32_t)x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint32_t F = prp_round(R, key[r]) & mask;
      uint32_t nl = R;
      R = L ^ F;
      L = nl;
    }
    x = ((uint64_t)L << hb) | R;
    if (x < N) return (int64_t)x;
  }
  return (int64_t)(x % N);   // unreachable in practice (expected walk < 4)
}

template <int RB, int NW>
__global__ __launch_bounds__(NW * 64) void rollout_step_kernel(RolloutStepArgs p) {
  constexpr int ROWS = RB * 16;
  constexpr int NT = NW * 64;                   // 2 waves per SIMD at NW = 8
  constexpr int MAXC = (16 + NW - 1) / NW;      // column blocks per wave for widths <= 256
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int S = p.S, A = p.A, C = p.C, S1 = p.S + 1;

  float* xin = smem;                       // ROWS x ldx  actor in / model in / next states
  float* h1 = xin + ROWS * p.ldx;          // ROWS x ldh
  float* h2 = h1 + ROWS * p.ldh;           // ROWS x ldh
  float* h3 = h2 + ROWS * p.ldh;           // ROWS x ldh  (log-var head hidden)
  float* sraw = h3 + ROWS * p.ldh;         // ROWS x lds  raw states
  float* ao = sraw + ROWS * p.lds;         // ROWS x 20   actor head
  float* dout = ao + ROWS * 20;            // ROWS x ldm  diff head
  float* lout = dout + ROWS * p.ldm;       // ROWS x ldm  log-var head
  float* act = lout + ROWS * p.ldm;        // ROWS x 8    sampled actions
  float* rew = act + ROWS * 8;             // ROWS
  float* hval = rew + ROWS;                // ROWS x 8    constraint values
  int* flags = reinterpret_cast<int*>(hval + ROWS * 8);   // ROWS: bit0 done, bit1 violation
  int* srcrow = flags + ROWS;                              // ROWS
  float* red = reinterpret_cast<float*>(srcrow + ROWS);    // NW*RB*256 narrow-layer partials
  int* s_part = reinterpret_cast<int*>(red + NW * RB * 256);   // NT scan partials
  int* scan = s_part + NT;                                 // prev tiles + 1 (exclusive prefix)
  float* vecs = reinterpret_cast<float*>(scan + ((p.Bmax + ROWS - 1) / ROWS) + 1);   // 4 x 64: small vectors
  float* v_nm = vecs;            // normalizer mean
  float* v_ns = vecs + 64;       // normalizer std + 1e-6
  float* v_lo = vecs + 128;      // min_log_var
  float* v_hi = vecs + 192;      // max_log_var
  // issue these tiny loads first: their latency hides behind the scan / gather
  if (tid < 256) {
    const int j = tid & 63, w = tid >> 6;
    if (w == 0 && j < S) v_nm[j] = p.norm_mean[j];
    if (w == 1 && j < S) v_ns[j] = p.norm_std[j] + 1e-6f;
    if (w == 2 && j < S1) v_lo[j] = p.min_lv[j];
    if (w == 3 && j < S1) v_hi[j] = p.max_lv[j];
  }

  RSTAMP(0);
  // ---- 0. row count / buffer offset of this step + compaction map ----------
  int n;
  int64_t off;
  const int row0 = blockIdx.x * ROWS;
  if (p.t == 0) {
    n = p.Bmax;
    off = 0;
  } else {
    const int n_prev = p.n[p.t - 1];
    const int T = (n_prev + ROWS - 1) / ROWS;
    // exclusive scan of the previous step's tile counts (T <= ntiles), NT threads
    const int per = (T + NT - 1) / NT;
    const int b0 = tid * per;
    int run = 0;
    for (int i = 0; i < per; ++i) {
      const int ti = b0 + i;
      if (ti < T) {
        scan[ti] = run;
        run += p.prev_cnt[ti];
      }
    }
    s_part[tid] = run;
    __syncthreads();
    if (tid < 64) {   // exclusive scan of the NT partials in one wave
      constexpr int PPL = NT / 64;
      int v[PPL], sum = 0;
      for (int q = 0; q < PPL; ++q) { v[q] = s_part[tid * PPL + q]; sum += v[q]; }
      int incl = sum;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (tid >= o) incl += y;
      }
      int e = incl - sum;
      for (int q = 0; q < PPL; ++q) { const int x = v[q]; s_part[tid * PPL + q] = e; e += x; }
    }
    __syncthreads();
    for (int i = 0; i < per; ++i) {
      const int ti = b0 + i;
      if (ti < T) scan[ti] += s_part[tid];
    }
    if (tid == NT - 1) scan[T] = s_part[NT - 1] + run;    // total alive == n for this step
    __syncthreads();
    n = scan[T];
    off = p.off[p.t - 1] + n_prev;
    if (tid < ROWS && row0 + tid < n) {   // binary search: last tile with scan[tile] <= i
      const int i = row0 + tid;
      int lo = 0, hi = T - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (scan[mid] <= i) lo = mid; else hi = mid - 1;
      }
      srcrow[tid] = lo * ROWS + p.prev_inv[lo * ROWS + (i - scan[lo])];
    }
  }
  if (blockIdx.x == 0 && tid == 0) {
    p.n[p.t] = n;
    p.off[p.t] = off;
  }
  if (row0 >= n) return;
  const int rows = min(ROWS, n - row0);
  const int64_t vbase = *p.vptr + off + row0;
  __syncthreads();

  // ---- 1. gather the tile's states (zero-padded) ---------------------------
  const int kpad = round_up(S + A, 16);
  for (int e = tid; e < ROWS * kpad; e += NT) {
    const int r = e / kpad, k = e - r * kpad;
    float v = 0.f;
    if (r < rows && k < S) {
      if (p.t == 0) {
        int64_t c = p.init_idx ? p.init_idx[row0 + r]
                               : prp_index((uint64_t)(row0 + r), (uint64_t)p.replay_len, p.prp_half_bits, p.prp_key);
        int64_t phys = (p.replay_ptr > p.replay_cap) ? (p.replay_ptr % p.replay_cap + c) % p.replay_cap : c;
        v = p.replay_states[phys * S + k];
      } else {
        v = p.prev_nxt[(int64_t)srcrow[r] * S + k];
      }
    }
    xin[r * p.ldx + k] = v;
    if (k < S) sraw[r * p.lds + k] = v;
  }
  __syncthreads();

  RSTAMP(1);
  // ---- 2. actor MLP (src/policy.py:61-100; mlp() ReLU hidden) ---------------
  tile_dense<NW, RB, MAXC, ACT_RELU>(xin, p.ldx, S, p.aW1, p.ab1, p.Ha, h1, p.ldh);
  __syncthreads();
  RSTAMP(2);
  tile_dense<NW, RB, MAXC, ACT_RELU>(h1, p.ldh, p.Ha, p.aW2, p.ab2, p.Ha, h2, p.ldh);
  __syncthreads();
  RSTAMP(3);
  tile_dense_narrow<NW, RB, ACT_NONE>(h2, p.ldh, p.Ha, p.aW3, p.ab3, 2 * A, ao, 20, red);
  __syncthreads();
  RSTAMP(4);

  // ---- 3. squashed Gaussian sample + model input [normalize(s), a] ----------
  for (int e = tid; e < ROWS * A; e += NT) {
    const int r = e / A, d = e - r * A;
    const float mu = ao[r * 20 + d], raw = ao[r * 20 + A + d];
    const float ls = -6.f + 10.f * sigmoidf(raw);
    const float sd = expf(ls) * 1.0f;
    float eps;
    if (p.eps_a) {
      eps = (r < rows) ? p.eps_a[(int64_t)(row0 + r) * A + d] : 0.f;
    } else {
      float z[4];
      philox_normal4(p.seed, (uint32_t)(row0 + r), ((uint32_t)p.t << 8) | 0u, (uint32_t)(d >> 2), (uint32_t)p.ctr, z);
      eps = z[d & 3];
    }
    const float a = tanhf(eps * sd + mu);
    act[r * 8 + d] = a;
    xin[r * p.ldx + S + d] = a;
  }
  for (int e = tid; e < ROWS * S; e += NT) {
    const int r = e / S, k = e - r * S;
    xin[r * p.ldx + k] = (sraw[r * p.lds + k] - v_nm[k]) / v_ns[k];
  }
  __syncthreads();

  RSTAMP(5);
  // ---- 4. elite member forward (src/dynamics.py:112-122, swish) -------------
  tile_dense<NW, RB, MAXC, ACT_SILU>(xin, p.ldx, S + A, p.mW1, p.mb1, p.Hm, h1, p.ldh);
  __syncthreads();
  RSTAMP(6);
  tile_dense<NW, RB, MAXC, ACT_SILU>(h1, p.ldh, p.Hm, p.mW2, p.mb2, p.Hm, h2, p.ldh);
  __syncthreads();
  RSTAMP(7);
  if (S1 <= 16 && p.Hm == 200) {
    // diff and log-var heads side by side: one fused hidden layer (2 x 13 column
    // blocks, 4 per wave) and one fused split-K output layer
    tile_dense_pair<NW, RB, (26 + NW - 1) / NW, ACT_SILU, 13>(h2, p.ldh, p.Hm, p.dW1, p.db1, p.Hm, h1, p.lW1,
                                                               p.lb1, p.Hm, h3, p.ldh);
    __syncthreads();
    RSTAMP(8);
    RSTAMP(9);
    tile_dense_narrow_pair<NW, RB, ACT_NONE>(h1, h3, p.ldh, p.Hm, p.dW2, p.db2, S1, dout, p.lW2, p.lb2, S1, lout,
                                             p.ldm, red);
    __syncthreads();
    RSTAMP(10);
    RSTAMP(11);
  } else {
    tile_dense<NW, RB, MAXC, ACT_SILU>(h2, p.ldh, p.Hm, p.dW1, p.db1, p.Hm, h1, p.ldh);
    __syncthreads();
    RSTAMP(8);
    if (S1 <= 16) tile_dense_narrow<NW, RB, ACT_NONE>(h1, p.ldh, p.Hm, p.dW2, p.db2, S1, dout, p.ldm, red);
    else tile_dense<NW, RB, MAXC, ACT_NONE>(h1, p.ldh, p.Hm, p.dW2, p.db2, S1, dout, p.ldm);
    __syncthreads();
    RSTAMP(9);
    tile_dense<NW, RB, MAXC, ACT_SILU>(h2, p.ldh, p.Hm, p.lW1, p.lb1, p.Hm, h1, p.ldh);
    __syncthreads();
    RSTAMP(10);
    if (S1 <= 16) tile_dense_narrow<NW, RB, ACT_NONE>(h1, p.ldh, p.Hm, p.lW2, p.lb2, S1, lout, p.ldm, red);
    else tile_dense<NW, RB, MAXC, ACT_NONE>(h1, p.ldh, p.Hm, p.lW2, p.lb2, S1, lout, p.ldm);
    __syncthreads();
    RSTAMP(11);
  }

  // ---- 5. residual mean, log-var soft clamp, Gaussian sample ---------------
  for (int e = tid; e < ROWS * S1; e += NT) {
    const int r = e / S1, j = e - r * S1;
    const float mean = dout[r * p.ldm + j] + (j < S ? sraw[r * p.lds + j] : 0.f);
    float lv = lout[r * p.ldm + j];
    lv = v_hi[j] - softplusf(v_hi[j] - lv);
    lv = v_lo[j] + softplusf(lv - v_lo[j]);
    const float sd = sqrtf(expf(lv));
    float eps;
    if (p.eps_m) {
      eps = (r < rows) ? p.eps_m[(int64_t)(row0 + r) * S1 + j] : 0.f;
    } else {
      float z[4];
      philox_normal4(p.seed, (uint32_t)(row0 + r), ((uint32_t)p.t << 8) | 1u, (uint32_t)(j >> 2), (uint32_t)p.ctr, z);
      eps = z[j & 3];
    }
    const float x = mean + sd * eps;
    if (j < S) xin[r * p.ldx + j] = x;
    else rew[r] = x;
  }
  __syncthreads();

  RSTAMP(12);
  // ---- 6. constraints + in-tile compaction ranks ---------------------------
  if (tid < 64) {
    bool alive_r = false;
    if (tid < rows) {
      bool dn, vl;
      float hh[8];
      env_constraints_row(p.env, xin + tid * p.ldx, dn, vl, hh);
      for (int c = 0; c < C; ++c) hval[tid * 8 + c] = hh[c];
      flags[tid] = (dn ? 1 : 0) | (vl ? 2 : 0);
      alive_r = !dn;
    }
    const uint64_t m = __ballot(alive_r);
    if (alive_r) p.inv[row0 + __popcll(m & ((1ull << tid) - 1ull))] = tid;   // k-th alive row of the tile
    if (tid == 0) p.cnt[blockIdx.x] = __popcll(m);
  }
  __syncthreads();

  RSTAMP(13);
  // ---- 7. row writes into the circular virtual buffer + next-state scratch --
  int64_t* qrow = reinterpret_cast<int64_t*>(red);           // ROWS physical buffer rows (red is free now)
  if (tid < rows) qrow[tid] = (vbase + tid) % p.vcap;
  __syncthreads();
  for (int e = tid; e < rows * S; e += NT) {
    const int r = e / S, k = e - r * S;
    const int64_t q = qrow[r];
    p.vs[q * S + k] = sraw[r * p.lds + k];
    const float x = xin[r * p.ldx + k];
    p.vs2[q * S + k] = x;
    p.nxt[(int64_t)(row0 + r) * S + k] = x;
  }
  for (int e = tid; e < rows * A; e += NT) {
    const int r = e / A, d = e - r * A;
    p.va[qrow[r] * A + d] = act[r * 8 + d];
  }
  for (int e = tid; e < rows * C; e += NT) {
    const int r = e / C, c = e - r * C;
    p.vh[qrow[r] * C + c] = hval[r * 8 + c];
  }
  if (tid < rows) {
    const int64_t q = qrow[tid];
    p.vr[q] = rew[tid];
    p.vd[q] = flags[tid] & 1;
    p.vv[q] = (flags[tid] >> 1) & 1;
  }
  RSTAMP(14);
}

// total rows written = off[H-1] + n[H-1]; advance the buffer pointer
__global__ void rollout_finalize_kernel(int64_t* vptr, const int* n, int64_t* off, int H) {
  const int64_t total = off[H - 1] + n[H - 1];
  off[H] = total;
  *vptr += total;
}

// ---------------------------------------------------------------------------
// Fused-horizon engine (engine 2). A row's trajectory depends only on its own
// earlier steps (SMBPO.rollout, src/smbpo.py:229-249: the batch only loses rows),
// so each workgroup keeps its 16/32-row tile for ALL H steps, with the states in
// LDS, and no workgroup ever waits for another. Rows that finish (done) stay in
// the tile masked off. Each step's surviving rows go to a staging area indexed
// [t][original row] together with per-(t, tile) counts and in-tile maps;
// rollout_emit_kernel then writes them into the circular buffer in the
// reference's order (step-major, surviving rows in batch order), which is the
// order the step engine's compaction produces.
//
// Against one launch per step this removes the per-step launch and drain, the
// device-wide count scan and the binary-searched gather of the previous step's
// states (bench workload: 37.3 -> 30.9 us per step). The step's Gaussian draws
// are generated into LDS by waves 1..7 while wave 0 evaluates the previous
// step's constraints, and the LDS hand-offs use lds_barrier() (no wait on
// outstanding global loads or the staging stores).
//
// Measured and rejected: issuing each layer's first weight k-steps ahead of the
// barrier / elementwise phase in front of it (and holding the actor's
// loop-invariant input/output fragments in registers). Across all placements the
// step time did not change, and the held fragments pushed the kernel to 256 VGPRs
// with scratch reloads in front of the MFMA loops.
// ---------------------------------------------------------------------------
constexpr int PERSIST_MAX_H = 128;

// The actor's weights are the same every step: without this the compiler hoists
// all of a layer's (restrict, loop-invariant) fragment loads out of the horizon
// loop and keeps them live in registers for the whole loop (hundreds of spills).
__device__ __forceinline__ const float* step_opaque(const float* ptr) {
  asm volatile("" : "+s"(ptr));
  return ptr;
}

// Two choices of the persistent kernel, each measured (A/B, one box):
//  - the per-step pointers / sizes are read through an opaque kernarg pointer at their
//    point of use (PARG: scalar loads) instead of holding the whole argument block in
//    SGPRs across the loop (SGPR spills): config 2 248 -> 242 us per launch
//    (profiles/r03/ab_persist);
//  - the elite member's first-layer fragments and biases are issued at the top of the
//    step, so they arrive while the actor runs: +0.7-1.3 % (profiles/r05/rollout_ab).
// (Actor biases staged in LDS once per launch measured no gain: profiles/r05/rollout_ab.)

struct PersistArgs {
  int S, A, C, Ha, Hm, B, H, ntiles;
  EnvParams env;
  const float *aW1, *ab1, *aW2, *ab2, *aW3, *ab3;
  // member 0 of the ensemble mirrors / biases; member m adds m * (mstride | bstride)
  const float *mW1, *mb1, *mW2, *mb2, *dW1, *db1, *dW2, *db2, *lW1, *lb1, *lW2, *lb2;
  int64_t ms_in, ms_hid, ms_out;    // packed strides: (S+A -> Hm), (Hm -> Hm), (Hm -> S+1)
  const float *norm_mean, *norm_std, *min_lv, *max_lv;
  const float* replay_states;
  const int64_t* init_idx;
  int64_t replay_len, replay_ptr, replay_cap;
  uint32_t prp_key[4];
  int prp_half_bits;
  const float* eps_a;   // [H][B][A] original-row layout, or nullptr (Philox)
  const float* eps_m;   // [H][B][S+1]
  uint64_t seed, ctr;
  float *st_s, *st_s2, *st_a, *st_r, *st_h;
  uint8_t* st_dv;       // bit0 done, bit1 violation
  int* cnt;             // [H][ntiles] rows alive at the start of step t
  int* inv;             // [H][ntiles*ROWS] in-tile index of the k-th alive row
  int ldx, ldh, ldm, lds;
  // small rollouts: block 0 copies the buffer pointer into base_slot before any emit
  // (rollout_emit_self_kernel then reads the copy and advances *vptr itself)
  const int64_t* vptr_in;
  int64_t* base_slot;
  int members[PERSIST_MAX_H];
};

typedef const __attribute__((address_space(4))) PersistArgs* PersistArgsK;   // scalar (constant) loads
__device__ __forceinline__ PersistArgsK persist_args() {
  PersistArgsK q = (PersistArgsK)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(q));
  return q;
}
#define PARG(f) (persist_args()->f)

// First layer with K <= 16 (one k-step) whose fragments / biases were loaded ahead
// (top of the step): the wave's MAXC blocks, clamped to the last valid block (its
// duplicate results are discarded by the epilogue).
template <int NW, int MAXC>
struct Layer1Frags {
  f32x4 w[MAXC];
  float b[MAXC];
};

template <int NW, int MAXC>
__device__ __forceinline__ void layer1_prefetch(const float* P, const float* bias, int N, Layer1Frags<NW, MAXC>& f) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int NCB = (N + 15) >> 4;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) f.w[c] = load_pk(P, min(wave + NW * c, NCB - 1), 0, 1);
  load_bias<NW, MAXC>(bias, N, f.b);
}

template <int NW, int RB, int MAXC, int ACT>
__device__ __forceinline__ void layer1_run(const float* in, int ldi, const Layer1Frags<NW, MAXC>& f, int N, float* out,
                                           int ldo) {
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  f32x4 acc[RB][MAXC], a[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    a[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 4 * g);
#pragma unroll
    for (int c = 0; c < MAXC; ++c) acc[rb][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
      for (int rb = 0; rb < RB; ++rb)
        acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[rb][m], f.w[c][m], acc[rb][c], 0, 0, 0);
  dense_epilogue<NW, RB, MAXC, ACT>(acc, f.b, N, out, ldo, GSave{nullptr, nullptr, 0, 0});
}

// The dynamics model's two hidden heads and their narrow output layers
// (src/dynamics.py:84-91, 112-122) as ONE phase. Each wave runs one head's hidden layer
// (pair_wave_code: waves 0, 1, 2, 7 the diff head, 3-6 the log-var head) and owns its
// blocks base, base + NW/2, ...: 7 / 6 / 6 / 7 blocks on the four SIMDs for 13 blocks
// per head, the 4-block wave the older one on both 7-block SIMDs. Each wave then forms its split-K share of
// its head's output layer from exactly the columns it produced (read back from LDS by the
// same wave: no workgroup barrier between the two layers), the output layer's fragments
// issued before the hidden epilogue. Partials land in red slot [head][w mod NW/2], the
// layout narrow_pair_sum reduces.
template <int NW, int RB, int NC, int NK>
__device__ __forceinline__ void pair_split_core(int base, const float* in, int ldi, const float* __restrict__ P,
                                                const float* __restrict__ bias, int N, float* out, int ldo,
                                                const float* __restrict__ Pn, float* red_slot) {
  constexpr int HW = NW / 2;
  const int lane = threadIdx.x & 63, l15 = lane & 15, g = lane >> 4;
  int cbs[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) cbs[c] = base + HW * c;
  f32x4 acc[RB][NC];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[rb][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  // a 2-deep ring: deeper rings only queue behind the L1 (4: +0.6-0.9 %, 6: +3 %, 8: +5 %
  // per launch; profiles/r06/ring_ab, profiles/r06/feed_probe)
  constexpr int PF = 2;
  f32x4 bq[PF][NC];
#pragma unroll
  for (int u = 0; u < PF - 1; ++u)
#pragma unroll
    for (int c = 0; c < NC; ++c) bq[u][c] = load_pk(P, cbs[c], u < NK ? u : NK - 1, NK);
  float bvs[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = cbs[c] * 16 + l15;
    bvs[c] = col < N ? gload(bias + col) : 0.f;
  }
  f32x4 an[RB], ac[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) an[rb] = *reinterpret_cast<const f32x4*>(in + (rb * 16 + l15) * ldi + 4 * g);
#pragma unroll
  for (int s = 0; s < NK; ++s) {
    if (s + PF - 1 < NK) {
#pragma unroll
      for (int c = 0; c < NC; ++c) bq[(s + PF - 1) % PF][c] = load_pk(P, cbs[c], s + PF - 1, NK);
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
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
          acc[rb][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ac[rb][m], bq[s % PF][c][m], acc[rb][c], 0, 0, 0);
  }
  CORE_STAMP(13);
  CORE_STAMP_W4(11);
  // the output layer's k-steps == this wave's hidden column blocks (K = N = Hm)
  f32x4 nb[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) nb[c] = load_pk(Pn, 0, cbs[c], NK);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int col = cbs[c] * 16 + l15;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float y = act_fn<ACT_SILU>(acc[rb][c][r] + bvs[c]);
        out[(rb * 16 + 4 * g + r) * ldo + col] = col < N ? y : 0.f;
      }
  }
  CORE_STAMP_W4(12);
  CORE_STAMP(14);
  wave_lds_sync();
  f32x4 pacc[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) pacc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(out + (rb * 16 + l15) * ldo + 16 * cbs[c] + 4 * g);
#pragma unroll
      for (int m = 0; m < 4; ++m) pacc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], nb[c][m], pacc[rb], 0, 0, 0);
    }
#pragma unroll
  for (int rb = 0; rb < RB; ++rb)
#pragma unroll
    for (int r = 0; r < 4; ++r) red_slot[rb * 256 + (4 * g + r) * 16 + l15] = pacc[rb][r];
  CORE_STAMP(15);
}

template <int NW, int RB, int NC, int NK>
__device__ __forceinline__ void pair_split_nc(int nc, int base, const float* in, int ldi, const float* P,
                                              const float* bias, int N, float* out, int ldo, const float* Pn,
                                              float* red_slot) {
  if (nc == NC) pair_split_core<NW, RB, NC, NK>(base, in, ldi, P, bias, N, out, ldo, Pn, red_slot);
  else if constexpr (NC > 1) pair_split_nc<NW, RB, NC - 1, NK>(nc, base, in, ldi, P, bias, N, out, ldo, Pn, red_slot);
}

// in: the trunk output (K = N = Hm, NK k-steps); out1 / out2: the heads' hidden
// activations; Pn1 / Pn2: the output layers (Hm -> S+1 <= 16). Ends with the barrier
// that publishes the partials.
template <int NW, int RB, int MAXC, int NK>
__device__ __forceinline__ void pair_split_heads(const float* in, int ldi, int N, const float* P1, const float* b1,
                                                 float* out1, const float* Pn1, const float* P2, const float* b2,
                                                 float* out2, const float* Pn2, float* red) {
  constexpr int HW = NW / 2;
  static_assert(NW == 8, "pair_wave_code maps 8 waves");
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const unsigned code = pair_wave_code(wave);
  const bool second = code >> 2;
  const int base = code & 3;
  const int NCB = (N + 15) >> 4;
  const int nc = base < NCB ? min(MAXC, (NCB - base + HW - 1) / HW) : 0;
  // head 0's slot q holds base q, head 1's slot q holds base HW - 1 - q (narrow_pair_sum's order)
  float* slot = red + (size_t)(second ? HW + (HW - 1 - base) : base) * RB * 256;
  if (nc > 0)
    pair_split_nc<NW, RB, MAXC, NK>(nc, base, in, ldi, second ? P2 : P1, second ? b2 : b1, N, second ? out2 : out1,
                                    ldi, second ? Pn2 : Pn1, slot);

  else {   // a wave without blocks contributes zero partials
    const int lane = threadIdx.x & 63;
    for (int e = lane; e < RB * 256; e += 64) slot[e] = 0.f;
  }
  lds_barrier();
}

// This step's Gaussian draws into LDS: recorded (original-row layout) or the step
// engine's Philox keys with the original row. Threads [first, first + count) work.
template <int ROWS>
__device__ __forceinline__ void persist_noise(const float* eps_a, const float* eps_m, uint64_t seed, uint64_t ctr,
                                              int A, int S1, int B, int t, int row0, int nrows, float* nz_a,
                                              float* nz_m, int first, int count) {
  const int NA4 = (A + 3) >> 2, NM4 = (S1 + 3) >> 2;
  const int total = ROWS * (NA4 + NM4);
  for (int base = 0; base < total; base += count) {   // uniform trip count, divergent body
    const int i = base + (int)threadIdx.x - first;
    if (i < base || i >= base + count || i >= total) continue;
    const int r = i / (NA4 + NM4), q = i - r * (NA4 + NM4);
    const uint32_t row = (uint32_t)(row0 + r);
    if (eps_a) {
      if (q < NA4) {
        for (int d = 4 * q; d < min(A, 4 * q + 4); ++d)
          nz_a[r * 8 + d] = r < nrows ? eps_a[((size_t)t * B + row) * A + d] : 0.f;
      } else {
        const int q2 = q - NA4;
        for (int j = 4 * q2; j < min(S1, 4 * q2 + 4); ++j)
          nz_m[r * 64 + j] = r < nrows ? eps_m[((size_t)t * B + row) * S1 + j] : 0.f;
      }
    } else {
      float z[4];
      if (q < NA4) {
        philox_normal4(seed, row, ((uint32_t)t << 8) | 0u, (uint32_t)q, (uint32_t)ctr, z);
        for (int u = 0; u < 4; ++u) nz_a[r * 8 + 4 * q + u] = z[u];
      } else {
        const int q2 = q - NA4;
        philox_normal4(seed, row, ((uint32_t)t << 8) | 1u, (uint32_t)q2, (uint32_t)ctr, z);
        for (int u = 0; u < 4; ++u) nz_m[r * 64 + 4 * q2 + u] = z[u];
      }
    }
  }
}

// LW: the actor's first layer, its output head and the first PERSIST_L2_LDS k-steps of
// its hidden layer stay in LDS for the whole launch (the actor is the same every
// step; with one 16-row tile per CU every weight byte is otherwise re-read from L2
// each step, and the layers run at the CU's L2 read rate). Needs S <= 16,
// Ha == 256, 2A <= 16 and the LDS to spare (host check).
constexpr int PERSIST_L2_LDS = 3;

// PM: the dynamics heads' path fixed at compile time (1: paired heads, S+1 <= 16 and
// Hm = 200; 0: the general path), so each kernel holds registers for one path only
// (spilled VGPRs 53 -> 33 / 1 -> 0 against one kernel with a run-time path choice,
// profiles/r03/pm_ab)
template <int RB, int NW, bool LW, int PM>
__global__ __launch_bounds__(NW * 64) void rollout_persist_kernel(PersistArgs p) {
  constexpr int ROWS = RB * 16;
  constexpr int NT = NW * 64;
  constexpr int MAXC = (16 + NW - 1) / NW;      // column blocks per wave for widths <= 256
  constexpr int PMAXC = (32 + NW - 1) / NW;     // paired 200-wide heads: 26 blocks
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x;
  const int S = p.S, A = p.A, C = p.C, S1 = p.S + 1, B = p.B;
  if (p.base_slot && blockIdx.x == 0 && tid == 0) *p.base_slot = *p.vptr_in;

  // LDS carve-up. Re-derived at the top of every horizon step from an opaque zero
  // and opaque leading dimensions: otherwise LICM hoists every (loop-invariant)
  // per-lane LDS address of the unrolled layers out of the loop and spills them.
#define PERSIST_LDS_LAYOUT(ZO, LDX, LDH, LDM, LDSS)                                         \
  float* xin = smem + (ZO);                  /* ROWS x ldx  actor in / model in / next states */ \
  float* h1 = xin + ROWS * (LDX);                                                             \
  float* h2 = h1 + ROWS * (LDH);                                                              \
  float* h3 = h2 + ROWS * (LDH);                                                              \
  float* sraw = h3 + ROWS * (LDH);           /* ROWS x lds  states at the start of the step */  \
  float* dout = sraw + ROWS * (LDSS);       /* ROWS x ldm  (tracking's output layers) */        \
  float* lout = dout + ROWS * (LDM);                                                          \
  float* act = lout + ROWS * (LDM);          /* ROWS x 8 */                                     \
  float* rew = act + ROWS * 8;                                                                \
  float* nz_a = rew + ROWS;                  /* ROWS x 8    this step's action draws */         \
  float* nz_m = nz_a + ROWS * 8;             /* ROWS x 64   this step's model draws */          \
  int* flags = reinterpret_cast<int*>(nz_m + ROWS * 64);                                      \
  int* alive = flags + ROWS;                                                                  \
  int* s_nalive = alive + ROWS;                                                               \
  float* red = reinterpret_cast<float*>(s_nalive + 4);  /* NW*RB*256 narrow partials */       \
  float* vecs = red + NW * RB * 256;                    /* 4 x 64 */                          \
  float* v_nm = vecs;                                                                         \
  float* v_ns = vecs + 64;                                                                    \
  float* v_lo = vecs + 128;                                                                   \
  float* v_hi = vecs + 192;                                                                   \
  float* wl1 = vecs + 256;                  /* LW: actor L1 mirror [16 cb][256] */               \
  float* wl3 = wl1 + 16 * 256;              /* LW: actor head mirror [16 k-steps][256] */        \
  float* wl2 = wl3 + 16 * 256;              /* LW: actor L2 [16 cb][PERSIST_L2_LDS][256] */      \
  (void)wl1; (void)wl2; (void)wl3;                                                            \
  (void)h3; (void)dout; (void)lout; (void)act; (void)rew; (void)nz_a; (void)nz_m;    \
  (void)flags; (void)alive; (void)s_nalive; (void)red; (void)v_nm; (void)v_ns; (void)v_lo; (void)v_hi;
  const int tile = blockIdx.x;
  const int row0 = tile * ROWS;
  const int nrows = min(ROWS, B - row0);
  const int Ha = p.Ha, Hm = p.Hm;
  constexpr bool paired = PM == 1;
  {
  PERSIST_LDS_LAYOUT(0, p.ldx, p.ldh, p.ldm, p.lds)
  if (tid < 256) {
    const int j = tid & 63, w = tid >> 6;
    if (w == 0 && j < S) v_nm[j] = p.norm_mean[j];
    if (w == 1 && j < S) v_ns[j] = p.norm_std[j] + 1e-6f;
    if (w == 2 && j < S1) v_lo[j] = p.min_lv[j];
    if (w == 3 && j < S1) v_hi[j] = p.max_lv[j];
  }
  if constexpr (LW) {
    // packed mirrors: aW1 is [16 cb][1 k-step][256], aW3 [1 cb][16 k-steps][256];
    // aW2 keeps k-steps [0, PERSIST_L2_LDS) of each of its 16 column blocks
    const f32x4* a1 = reinterpret_cast<const f32x4*>(p.aW1);
    const f32x4* a3 = reinterpret_cast<const f32x4*>(p.aW3);
    const f32x4* a2 = reinterpret_cast<const f32x4*>(p.aW2);
    for (int e = tid; e < 16 * 64; e += NT) {
      reinterpret_cast<f32x4*>(wl1)[e] = gload(a1 + e);
      reinterpret_cast<f32x4*>(wl3)[e] = gload(a3 + e);
    }
    for (int e = tid; e < 16 * PERSIST_L2_LDS * 64; e += NT) {
      const int cb = e / (PERSIST_L2_LDS * 64), r = e - cb * PERSIST_L2_LDS * 64;
      reinterpret_cast<f32x4*>(wl2)[e] = gload(a2 + cb * 16 * 64 + r);
    }
  }

  // ---- initial states (t = 0): chronological replay index -> physical row -----
  const int kpad = round_up(S + A, 16);
  for (int e = tid; e < ROWS * kpad; e += NT) {
    const int r = e / kpad, k = e - r * kpad;
    float v = 0.f;
    if (r < nrows && k < S) {
      const int64_t c = p.init_idx ? p.init_idx[row0 + r]
                                   : prp_index((uint64_t)(row0 + r), (uint64_t)p.replay_len, p.prp_half_bits, p.prp_key);
      const int64_t phys = (p.replay_ptr > p.replay_cap) ? (p.replay_ptr % p.replay_cap + c) % p.replay_cap : c;
      v = p.replay_states[phys * S + k];
    }
    xin[r * p.ldx + k] = v;
    if (k < S) sraw[r * p.lds + k] = v;
  }
  if (tid < ROWS) alive[tid] = tid < nrows;
  persist_noise<ROWS>(p.eps_a, p.eps_m, p.seed, p.ctr, A, S1, B, 0, row0, nrows, nz_a, nz_m, 0, NT);   // step 0's draws
  lds_barrier();
  }
  for (int t = 0; t < p.H; ++t) {
    int zo = 0, ldx = p.ldx, ldh = p.ldh, ldm = p.ldm, ldss = p.lds;
    asm volatile("" : "+s"(zo), "+s"(ldx), "+s"(ldh), "+s"(ldm), "+s"(ldss));
    PERSIST_LDS_LAYOUT(zo, ldx, ldh, ldm, ldss)
    const int m = PARG(members[t]);
    const float* aW2 = step_opaque(PARG(aW2));
    const float* ab2 = step_opaque(PARG(ab2));
    // the elite member's slices, formed where they are used (PARG: re-read per use)
#define MW(f, st) (PARG(f) + (size_t)m * PARG(st))
#define MB(f, n) (PARG(f) + (size_t)m * (n))
    Layer1Frags<NW, MAXC> m1;
    const bool m1_pre = S + A <= 16;
    if (m1_pre) layer1_prefetch<NW, MAXC>(MW(mW1, ms_in), MB(mb1, Hm), Hm, m1);

    if (t == 2) RSTAMP(0);
    if (t == 2) RSTAMP(1);
    // alive flags of this step's rows / of the next step's (double-buffered: the
    // constraint wave writes the next step's while the staging waves read these)
    int* alive_cur = (t & 1) ? flags : alive;
    int* alive_nxt = (t & 1) ? alive : flags;
    // ---- actor MLP (src/policy.py:61-100) ------------------------------------
    if constexpr (LW) {
      tile_dense_impl<NW, RB, MAXC, ACT_RELU, 1, 1>(xin, ldx, S, step_opaque(PARG(aW1)),
                                                   step_opaque(PARG(ab1)), Ha, h1, ldh,
                                                   GSave{nullptr, nullptr, 0, 0}, wl1);
      lds_barrier();
      if (t == 2) RSTAMP(2);
      tile_dense_impl<NW, RB, MAXC, ACT_RELU, 16, PERSIST_L2_LDS>(h1, ldh, Ha, aW2, ab2,
                                                                 Ha, h2, ldh, GSave{nullptr, nullptr, 0, 0}, wl2);
    } else {
      tile_dense<NW, RB, MAXC, ACT_RELU>(xin, ldx, S, step_opaque(PARG(aW1)), step_opaque(PARG(ab1)), Ha, h1, ldh);
      lds_barrier();
      if (t == 2) RSTAMP(2);
      tile_dense<NW, RB, MAXC, ACT_RELU>(h1, ldh, Ha, aW2, ab2, Ha, h2, ldh);
    }
    // the head's split-K share of wave w is k-steps w, w + NW, ...: exactly the hidden
    // column blocks wave w just wrote (Ha <= 256), so no workgroup barrier here. That
    // holds while tile_dense's column-block map (block wave + NW*c) and
    // tile_dense_narrow_partials' k-step map (step wave + NW*q) are the same map and
    // NW divides the 16 blocks of a 256-wide layer.
    static_assert(16 % NW == 0, "wave-local head hand-off needs NW | 16");
    wave_lds_sync();
    if (t == 2) RSTAMP(3);
    // ---- actor head + squashed Gaussian sample + model input [normalize(s), a]:
    //      the head's split-K partials are reduced by the threads that sample
    //      (one thread per (row, action dim) sums the mu and log-std columns) ----
    {
      float bmu = 0.f, braw = 0.f;
      if (tid < ROWS * A) {   // ROWS * A <= NT (A <= 8)
        const int d = tid % A;
        const float* ab3 = step_opaque(PARG(ab3));
        bmu = gload(ab3 + d);
        braw = gload(ab3 + A + d);
      }
      tile_dense_narrow_partials<NW, RB, LW>(h2, ldh, Ha, step_opaque(PARG(aW3)), red, wl3);
      if (tid < ROWS * A) {
        const int r = tid / A, d = tid - r * A;
        const float mu = narrow_sum<NW, RB>(red, r, d) + bmu;
        const float raw = narrow_sum<NW, RB>(red, r, A + d) + braw;
        const float ls = -6.f + 10.f * fast_sigmoid(raw);
        const float a = fast_tanh(nz_a[r * 8 + d] * fast_exp(ls) + mu);
        act[r * 8 + d] = a;
        xin[r * ldx + S + d] = a;
      }
      for (int e = tid; e < ROWS * S; e += NT) {
        const int r = e / S, k = e - r * S;
        xin[r * ldx + k] = (sraw[r * ldss + k] - v_nm[k]) / v_ns[k];
      }
    }
    lds_barrier();
    if (t == 2) RSTAMP(4);

    // ---- elite member forward (src/dynamics.py:112-122) -----------------------
    if (m1_pre) layer1_run<NW, RB, MAXC, ACT_SILU>(xin, ldx, m1, Hm, h1, ldh);
    else
    tile_dense<NW, RB, MAXC, ACT_SILU>(xin, ldx, S + A, MW(mW1, ms_in), MB(mb1, Hm), Hm, h1, ldh);
    lds_barrier();
    if (t == 2) RSTAMP(5);
    if (RB == 1 && NW == 8 && Hm == 200) {
      // member hidden layer balanced over the SIMDs (13th block split over K;
      // profiles/r04/m2_split)
      const float b12 = tile_dense_13s<ACT_SILU>(h1, ldh, MW(mW2, ms_hid), MB(mb2, Hm), h2, ldh, red);
      lds_barrier();
      tile_dense_13s_finish<ACT_SILU>(red, b12, h2, ldh);
    } else
    tile_dense<NW, RB, MAXC, ACT_SILU>(h1, ldh, Hm, MW(mW2, ms_hid), MB(mb2, Hm), Hm, h2, ldh);
    lds_barrier();
    if (t == 2) RSTAMP(6);
    const float* dW1 = MW(dW1, ms_hid);
    const float* lW1 = MW(lW1, ms_hid);
    const float* db1 = MB(db1, Hm);
    const float* lb1 = MB(lb1, Hm);
    if (paired) {
      // output-layer biases first (their latency hides behind the hidden layers)
      float bd = 0.f, bl = 0.f;
      if (tid < ROWS * S1) {   // ROWS * S1 <= NT (S1 <= 16)
        const int j = tid % S1;
        bd = gload(MB(db2, S1) + j);
        bl = gload(MB(lb2, S1) + j);
      }
      // both hidden heads + their output layers' split-K partials, one barrier
      pair_split_heads<NW, RB, (13 + NW / 2 - 1) / (NW / 2), 13>(h2, ldh, Hm, dW1, db1, h1, MW(dW2, ms_out), lW1,
                                                                 lb1, h3, MW(lW2, ms_out), red);
      if (t == 2) RSTAMP(7);
      // the partials reduced by the threads that form the residual mean, soft-clamp the
      // log-variance and sample the next state
      if (tid < ROWS * S1) {
        const int r = tid / S1, j = tid - r * S1;
        const float mean = (narrow_pair_sum<NW, RB>(red, 0, r, j) + bd) + (j < S ? sraw[r * ldss + j] : 0.f);
        float lv = narrow_pair_sum<NW, RB>(red, 1, r, j) + bl;
        lv = v_hi[j] - fast_softplus(v_hi[j] - lv);
        lv = v_lo[j] + fast_softplus(lv - v_lo[j]);
        const float x = mean + fast_exp(0.5f * lv) * nz_m[r * 64 + j];
        if (j < S) xin[r * ldx + j] = x;
        else rew[r] = x;
      }
    } else {
      if (Hm == 200 && 2 * ((S1 + 15) >> 4) <= NW) {
        // wide state (tracking, S + 1 = 52): the two hidden layers as one 400-wide layer,
        // then both output layers side by side (two inputs, one block per wave): two
        // phases instead of four
        tile_dense_pair<NW, RB, PMAXC, ACT_SILU, 13>(h2, ldh, Hm, dW1, db1, Hm, h1, lW1, lb1, Hm, h3, ldh);
        lds_barrier();
        if (t == 2) RSTAMP(7);
        // one block per wave: a ring as deep as K (every fragment in flight at once), else
        // this latency-bound layer waits one L2 round trip per few k-steps
        tile_dense_pair2<NW, RB, 1, ACT_NONE, 13, 13>(h1, h3, ldh, MW(dW2, ms_out), MB(db2, S1), S1, dout,
                                                       MW(lW2, ms_out), MB(lb2, S1), S1, lout, ldm);
      } else {
        const float* dW2 = MW(dW2, ms_out);
        const float* lW2 = MW(lW2, ms_out);
        const float* db2 = MB(db2, S1);
        const float* lb2 = MB(lb2, S1);
        tile_dense<NW, RB, MAXC, ACT_SILU>(h2, ldh, Hm, dW1, db1, Hm, h1, ldh);
        lds_barrier();
        if (S1 <= 16) tile_dense_narrow<NW, RB, ACT_NONE>(h1, ldh, Hm, dW2, db2, S1, dout, ldm, red);
        else tile_dense<NW, RB, MAXC, ACT_NONE>(h1, ldh, Hm, dW2, db2, S1, dout, ldm);
        lds_barrier();
        tile_dense<NW, RB, MAXC, ACT_SILU>(h2, ldh, Hm, lW1, lb1, Hm, h1, ldh);
        lds_barrier();
        if (t == 2) RSTAMP(7);
        if (S1 <= 16) tile_dense_narrow<NW, RB, ACT_NONE>(h1, ldh, Hm, lW2, lb2, S1, lout, ldm, red);
        else tile_dense<NW, RB, MAXC, ACT_NONE>(h1, ldh, Hm, lW2, lb2, S1, lout, ldm);
      }
      lds_barrier();
      if (t == 2) RSTAMP(10);
      // residual mean, log-var soft clamp, Gaussian sample
      for (int e = tid; e < ROWS * S1; e += NT) {
        const int r = e / S1, j = e - r * S1;
        const float mean = dout[r * ldm + j] + (j < S ? sraw[r * ldss + j] : 0.f);
        float lv = lout[r * ldm + j];
        lv = v_hi[j] - fast_softplus(v_hi[j] - lv);
        lv = v_lo[j] + fast_softplus(lv - v_lo[j]);
        const float x = mean + fast_exp(0.5f * lv) * nz_m[r * 64 + j];
        if (j < S) xin[r * ldx + j] = x;
        else rew[r] = x;
      }
    }
    lds_barrier();
    if (t == 2) RSTAMP(8);

    // ---- one phase: constraints + alive map + their staging writes (wave 0, one
    //      lane per row), the states / actions staging writes and the state
    //      hand-off (waves 1 .. NW/2-1), the next step's draws (waves NW/2 ..) ----
    const size_t sb = (size_t)t * B + row0;
    if (tid < 64) {
      bool in_r = false, dn = false, vl = false;
      if (tid < ROWS && alive_cur[tid]) {
        float hh[8];
        env_constraints_row(p.env, xin + tid * ldx, dn, vl, hh);
        for (int c = 0; c < C; ++c) PARG(st_h)[(sb + tid) * C + c] = hh[c];
        PARG(st_r)[sb + tid] = rew[tid];
        PARG(st_dv)[sb + tid] = (uint8_t)((dn ? 1 : 0) | (vl ? 2 : 0));
        in_r = true;
      }
      const uint64_t mk = __ballot(in_r);
      if (in_r) PARG(inv)[((size_t)t * PARG(ntiles) + tile) * ROWS + __popcll(mk & ((1ull << tid) - 1ull))] = tid;
      if (tid == 0) PARG(cnt)[(size_t)t * PARG(ntiles) + tile] = __popcll(mk);
      const uint64_t still = __ballot(in_r && !dn);
      if (tid < ROWS) alive_nxt[tid] = in_r && !dn;
      if (tid == 0) *s_nalive = __popcll(still);
    } else if (tid < NT / 2) {
      constexpr int NS = NT / 2 - 64;
      const int ts = tid - 64;
      for (int e = ts; e < ROWS * S; e += NS) {
        const int r = e / S, k = e - r * S;
        const float x = xin[r * ldx + k];
        if (alive_cur[r]) {
          PARG(st_s)[(sb + r) * S + k] = sraw[r * ldss + k];
          PARG(st_s2)[(sb + r) * S + k] = x;
        }
        sraw[r * ldss + k] = x;   // same element, same thread
      }
      for (int e = ts; e < nrows * A; e += NS) {
        const int r = e / A, d = e - r * A;
        if (alive_cur[r]) PARG(st_a)[(sb + r) * A + d] = act[r * 8 + d];
      }
    } else if (t + 1 < PARG(H)) {
      persist_noise<ROWS>(PARG(eps_a), PARG(eps_m), PARG(seed), PARG(ctr), A, S1, B, t + 1, row0, nrows, nz_a, nz_m, NT / 2, NT / 2);
    }
    lds_barrier();
    if (t == 2) RSTAMP(9);
    const int n_alive = __builtin_amdgcn_readfirstlane(*s_nalive);   // uniform exit
    if (n_alive == 0) {   // the whole tile finished: later steps see no rows from it
      for (int t2 = t + 1 + tid; t2 < PARG(H); t2 += NT) PARG(cnt)[(size_t)t2 * PARG(ntiles) + tile] = 0;
      break;
    }
  }
}

#undef MW
#undef MB
#undef PERSIST_LDS_LAYOUT

// per step t: exclusive prefix of the tile counts -> pos[t][tile], n[t]
__global__ __launch_bounds__(256) void rollout_scan_kernel(const int* __restrict__ cnt, int* __restrict__ pos,
                                                           int* __restrict__ n, int ntiles) {
  __shared__ int part[256];
  const int t = blockIdx.x, tid = threadIdx.x;
  const int* c = cnt + (size_t)t * ntiles;
  int* ps = pos + (size_t)t * ntiles;
  const int per = (ntiles + 255) / 256, b0 = tid * per;
  int run = 0;
  for (int i = 0; i < per; ++i)
    if (b0 + i < ntiles) run += c[b0 + i];
  part[tid] = run;
  __syncthreads();
  if (tid < 64) {   // exclusive scan of the 256 partials in one wave
    int v[4], sum = 0;
    for (int q = 0; q < 4; ++q) { v[q] = part[tid * 4 + q]; sum += v[q]; }
    int incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      if (tid >= o) incl += y;
    }
    int e = incl - sum;
    for (int q = 0; q < 4; ++q) { const int x = v[q]; part[tid * 4 + q] = e; e += x; }
    if (tid == 63) n[t] = incl;
  }
  __syncthreads();
  int e = part[tid];
  for (int i = 0; i < per; ++i)
    if (b0 + i < ntiles) { ps[b0 + i] = e; e += c[b0 + i]; }
}

// staged rows -> circular virtual buffer, in the reference's order
template <int ROWS>
__global__ __launch_bounds__(256) void rollout_emit_kernel(PersistArgs p, const int* __restrict__ pos,
                                                           const int* __restrict__ n, const int64_t* __restrict__ vptr,
                                                           int advanced, const int64_t* __restrict__ offs,
                                                           int64_t vcap, float* __restrict__ vs, float* __restrict__ va,
                                                           float* __restrict__ vs2, float* __restrict__ vr,
                                                           float* __restrict__ vh, uint8_t* __restrict__ vd,
                                                           uint8_t* __restrict__ vv) {
  __shared__ int64_t s_off;
  const int t = blockIdx.y, tid = threadIdx.x;
  if (tid == 0) {
    int64_t o = 0;
    for (int u = 0; u < t; ++u) o += n[u];
    // rollout_scanfin_kernel already advanced the pointer by the total (offs[H])
    s_off = o + *vptr - (advanced ? offs[p.H] : 0);
  }
  __syncthreads();
  const int slot = blockIdx.x * 256 + tid;
  const int tile = slot / ROWS, k = slot - tile * ROWS;
  if (tile >= p.ntiles) return;
  const size_t ti = (size_t)t * p.ntiles + tile;
  if (k >= p.cnt[ti]) return;
  const int S = p.S, A = p.A, C = p.C;
  const size_t src = (size_t)t * p.B + (size_t)tile * ROWS + p.inv[ti * ROWS + k];
  const int64_t q = (s_off + pos[ti] + k) % vcap;
  for (int j = 0; j < S; ++j) {
    vs[q * S + j] = p.st_s[src * S + j];
    vs2[q * S + j] = p.st_s2[src * S + j];
  }
  for (int d = 0; d < A; ++d) va[q * A + d] = p.st_a[src * A + d];
  for (int c = 0; c < C; ++c) vh[q * C + c] = p.st_h[src * C + c];
  vr[q] = p.st_r[src];
  const uint8_t dv = p.st_dv[src];
  vd[q] = dv & 1;
  vv[q] = (dv >> 1) & 1;
}

// Small rollouts (H x tiles <= EMIT_SELF_MAX counts): count scan, ordered emit and
// pointer advance in ONE launch. Every workgroup reads the whole [H][ntiles] count
// array (<= 32 KB, L2-resident: the persist kernel just wrote it) and reduces it to
// its own flat prefix (all rows of steps < t, and of tiles before its first tile at
// step t) and the total, so no workgroup waits on another. The buffer pointer was
// copied into base_slot by rollout_persist_kernel, so the one workgroup that advances
// *vptr races with no reader.
constexpr int EMIT_SELF_MAX = 8192;
template <int ROWS>
__global__ __launch_bounds__(256) void rollout_emit_self_kernel(PersistArgs p, const int64_t* __restrict__ base_slot,
                                                                int64_t* __restrict__ vptr, int64_t* __restrict__ off,
                                                                int64_t vcap, float* __restrict__ vs,
                                                                float* __restrict__ va, float* __restrict__ vs2,
                                                                float* __restrict__ vr, float* __restrict__ vh,
                                                                uint8_t* __restrict__ vd, uint8_t* __restrict__ vv) {
  constexpr int TPB = 256 / ROWS;   // tiles per workgroup
  __shared__ int s_pre[4], s_tot[4], s_loc[TPB];
  const int t = blockIdx.y, tid = threadIdx.x;
  const int tile0 = blockIdx.x * TPB;
  const int nflat = p.H * p.ntiles, P = t * p.ntiles + tile0;
  const int* __restrict__ cnt = p.cnt;
  int pre = 0, tot = 0;
  for (int i = tid; i < nflat; i += 256) {
    const int c = cnt[i];
    tot += c;
    pre += i < P ? c : 0;
  }
  for (int o = 32; o > 0; o >>= 1) {
    pre += __shfl_xor(pre, o, 64);
    tot += __shfl_xor(tot, o, 64);
  }
  if ((tid & 63) == 0) { s_pre[tid >> 6] = pre; s_tot[tid >> 6] = tot; }
  if (tid < TPB) s_loc[tid] = tile0 + tid < p.ntiles ? cnt[(size_t)t * p.ntiles + tile0 + tid] : 0;
  __syncthreads();
  pre = s_pre[0] + s_pre[1] + s_pre[2] + s_pre[3];
  tot = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
  const int64_t base = *base_slot;
  if (t == p.H - 1 && blockIdx.x == gridDim.x - 1 && tid == 0) {
    off[p.H] = tot;
    *vptr = base + tot;
  }
  const int j = tid / ROWS, k = tid - j * ROWS, tile = tile0 + j;
  if (tile >= p.ntiles || k >= s_loc[j]) return;
  int loc = 0;
  for (int u = 0; u < j; ++u) loc += s_loc[u];
  const int S = p.S, A = p.A, C = p.C;
  const size_t ti = (size_t)t * p.ntiles + tile;
  const size_t src = (size_t)t * p.B + (size_t)tile * ROWS + p.inv[ti * ROWS + k];
  const int64_t q = (base + pre + loc + k) % vcap;
  for (int jj = 0; jj < S; ++jj) {
    vs[q * S + jj] = p.st_s[src * S + jj];
    vs2[q * S + jj] = p.st_s2[src * S + jj];
  }
  for (int d = 0; d < A; ++d) va[q * A + d] = p.st_a[src * A + d];
  for (int c = 0; c < C; ++c) vh[q * C + c] = p.st_h[src * C + c];
  vr[q] = p.st_r[src];
  const uint8_t dv = p.st_dv[src];
  vd[q] = dv & 1;
  vv[q] = (dv >> 1) & 1;
}

// Mid-size rollouts (H x tiles <= 16384 counts): the per-step scans, the step offsets and
// the pointer advance of rollout_scan_kernel + rollout_persist_finalize_kernel in ONE
// single-workgroup launch (the emit then reads the advanced pointer minus the total).
__global__ __launch_bounds__(256) void rollout_scanfin_kernel(const int* __restrict__ cnt, int* __restrict__ pos,
                                                              int* __restrict__ n, int64_t* __restrict__ off,
                                                              int64_t* __restrict__ vptr, int ntiles, int H) {
  __shared__ int part[256];
  __shared__ int s_tot;
  const int tid = threadIdx.x;
  int64_t total = 0;
  for (int t = 0; t < H; ++t) {
    const int* c = cnt + (size_t)t * ntiles;
    int* ps = pos + (size_t)t * ntiles;
    const int per = (ntiles + 255) / 256, b0 = tid * per;
    int run = 0;
    for (int i = 0; i < per; ++i)
      if (b0 + i < ntiles) run += c[b0 + i];
    part[tid] = run;
    __syncthreads();
    if (tid < 64) {
      int v[4], sum = 0;
      for (int q = 0; q < 4; ++q) { v[q] = part[tid * 4 + q]; sum += v[q]; }
      int incl = sum;
      for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(incl, o, 64);
        if (tid >= o) incl += y;
      }
      int e = incl - sum;
      for (int q = 0; q < 4; ++q) { const int x = v[q]; part[tid * 4 + q] = e; e += x; }
      if (tid == 63) { n[t] = incl; s_tot = incl; }
    }
    __syncthreads();
    int e = part[tid];
    for (int i = 0; i < per; ++i)
      if (b0 + i < ntiles) { ps[b0 + i] = e; e += c[b0 + i]; }
    if (tid == 0) off[t] = total;
    total += s_tot;
    __syncthreads();
  }
  if (tid == 0) {
    off[H] = total;
    *vptr += total;
  }
}

// off[t] = sum n[<t], off[H] = total; advance the buffer pointer
__global__ void rollout_persist_finalize_kernel(int64_t* vptr, const int* n, int64_t* off, int H) {
  int64_t o = 0;
  for (int t = 0; t < H; ++t) {
    off[t] = o;
    o += n[t];
  }
  off[H] = o;
  *vptr += o;
}

// ---------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------

static size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

struct RolloutWs {
  float* nxt[2];
  int* cnt[2];
  int* inv[2];
  int* n;
  int64_t* off;
};

// Byte offsets of the workspace pieces (in order); returns total bytes.
// pieces 0-7: step-engine scratch + n/off; 8-16: fused-engine staging, indexed
// [t][original row] (A, C <= 8 slots), per-(t, tile) counts / in-tile maps / positions
constexpr int WS_PIECES = 17;
static size_t rollout_ws_offsets(int B, int S, int H, size_t off[WS_PIECES]) {
  const size_t HB = (size_t)H * B, T16 = (size_t)B / 16 + 1;
  const size_t bytes[WS_PIECES] = {sizeof(float) * (size_t)B * S, sizeof(float) * (size_t)B * S,
                                   sizeof(int) * T16, sizeof(int) * T16,
                                   sizeof(int) * (size_t)B, sizeof(int) * (size_t)B,
                                   sizeof(int) * (size_t)(H + 1), sizeof(int64_t) * (size_t)(H + 2),
                                   sizeof(float) * HB * S, sizeof(float) * HB * S, sizeof(float) * HB * 8,
                                   sizeof(float) * HB, sizeof(float) * HB * 8, HB,
                                   sizeof(int) * (size_t)H * T16, sizeof(int) * (size_t)H * (B + 32),
                                   sizeof(int) * (size_t)H * T16};
  size_t o = 0;
  for (int i = 0; i < WS_PIECES; ++i) {
    off[i] = o;
    o += align256(bytes[i]);
  }
  return o;
}

static RolloutWs rollout_ws(int B, int S, int H, char* base) {
  size_t o[WS_PIECES];
  rollout_ws_offsets(B, S, H, o);
  RolloutWs w;
  w.nxt[0] = (float*)(base + o[0]);
  w.nxt[1] = (float*)(base + o[1]);
  w.cnt[0] = (int*)(base + o[2]);
  w.cnt[1] = (int*)(base + o[3]);
  w.inv[0] = (int*)(base + o[4]);
  w.inv[1] = (int*)(base + o[5]);
  w.n = (int*)(base + o[6]);
  w.off = (int64_t*)(base + o[7]);
  return w;
}

DRPO_API size_t drpo_rollout_workspace_size(int B, int S, int H) {
  size_t o[WS_PIECES];
  return rollout_ws_offsets(B, S, H, o);
}

// Byte offset (inside the workspace) of the device int64 that holds the number of
// transitions written by the last drpo_rollout call (off[H]).
DRPO_API size_t drpo_rollout_count_offset(int B, int S, int H) {
  size_t o[WS_PIECES];
  rollout_ws_offsets(B, S, H, o);
  return o[7] + sizeof(int64_t) * (size_t)H;
}

static int hb_for(int64_t n) {
  int b = 1;
  while ((1ull << (2 * b)) < (uint64_t)n) ++b;
  return b;
}

// LDS bytes of rollout_persist_kernel for `rpt`-row tiles (without the LDS-resident
// actor weights): per row xin, h1-h3, sraw, dout, lout, act, rew, nz_a, nz_m, flags,
// alive; then s_nalive, the split-K partials and the normalizer / log-var vectors.
// (Tracking, S = 51: 162.7 KB at 32-row tiles, inside the 160 KiB, so B >= 8192 runs
// 32-row tiles there too.)
static size_t persist_lds_bytes(int S, int A, int Ha, int Hm, int rpt, int nw) {
  const int S1 = S + 1;
  const int ldx = lds_ld(S + A), ldh = lds_ld(Ha > Hm ? Ha : Hm), ldm = round_up(S1, 16) + 4, ldss = round_up(S, 4);
  return sizeof(float) * ((size_t)rpt * (ldx + 3 * ldh + ldss + 2 * ldm + 8 + 1 + 8 + 64 + 2) + 4 +
                          (size_t)nw * (rpt / 16) * 256 + 256);
}

// engine 2: fused-horizon kernel + count scan + ordered emit + pointer advance
static int rollout_fused(const drpo_rollout_desc_t* d, int rpt, int64_t rlen, hipStream_t stream) {
  DRPO_REQUIRE(d->H <= PERSIST_MAX_H, "drpo_rollout: engine 2 supports horizon <= %d", PERSIST_MAX_H);
  const int S = d->S, A = d->A, S1 = d->S + 1, B = d->B, H = d->H;
  size_t o[WS_PIECES];
  rollout_ws_offsets(B, S, H, o);
  char* base = (char*)d->workspace;
  PersistArgs a{};
  a.S = S; a.A = A; a.C = d->C; a.Ha = d->Ha; a.Hm = d->Hm; a.B = B; a.H = H;
  a.ntiles = (B + rpt - 1) / rpt;
  a.env.id = d->env_id; a.env.surr_start = d->tracking_surr_start; a.env.n_surr = d->tracking_n_surr;
  a.env.thr0 = d->env_thr0; a.env.thr1 = d->env_thr1;
  a.aW1 = d->aW1; a.ab1 = d->ab1; a.aW2 = d->aW2; a.ab2 = d->ab2; a.aW3 = d->aW3; a.ab3 = d->ab3;
  a.mW1 = d->mW1; a.mb1 = d->mb1; a.mW2 = d->mW2; a.mb2 = d->mb2; a.dW1 = d->dW1; a.db1 = d->db1;
  a.dW2 = d->dW2; a.db2 = d->db2; a.lW1 = d->lW1; a.lb1 = d->lb1; a.lW2 = d->lW2; a.lb2 = d->lb2;
  a.ms_in = drpo_packed_size(S + A, d->Hm);
  a.ms_hid = drpo_packed_size(d->Hm, d->Hm);
  a.ms_out = drpo_packed_size(d->Hm, S1);
  a.norm_mean = d->norm_mean; a.norm_std = d->norm_std; a.min_lv = d->min_lv; a.max_lv = d->max_lv;
  a.replay_states = d->replay_states; a.init_idx = d->init_idx;
  a.replay_len = rlen; a.replay_ptr = d->replay_ptr; a.replay_cap = d->replay_cap;
  a.prp_half_bits = hb_for(rlen);
  for (int i = 0; i < 4; ++i) a.prp_key[i] = (uint32_t)(d->seed >> (8 * i)) * 0x9E3779B9u + (uint32_t)d->ctr * (2 * i + 1) + i;
  a.eps_a = d->eps_a; a.eps_m = d->eps_m;
  a.seed = d->seed; a.ctr = d->ctr;
  a.st_s = (float*)(base + o[8]); a.st_s2 = (float*)(base + o[9]); a.st_a = (float*)(base + o[10]);
  a.st_r = (float*)(base + o[11]); a.st_h = (float*)(base + o[12]); a.st_dv = (uint8_t*)(base + o[13]);
  a.cnt = (int*)(base + o[14]); a.inv = (int*)(base + o[15]);
  int* pos = (int*)(base + o[16]);
  int* n = (int*)(base + o[6]);
  int64_t* off = (int64_t*)(base + o[7]);
  a.ldx = lds_ld(S + A);
  a.ldh = lds_ld(d->Ha > d->Hm ? d->Ha : d->Hm);
  a.ldm = round_up(S1, 16) + 4;
  a.lds = round_up(S, 4);
  for (int t = 0; t < H; ++t) a.members[t] = d->members[t];

  // 8-wave workgroups (16 waves measured 3.5 % slower at config 2, profiles/r02/rollout_ab)
  const size_t lds_bytes = persist_lds_bytes(S, A, d->Ha, d->Hm, rpt, 8);
  DRPO_REQUIRE(lds_bytes <= 160 * 1024, "drpo_rollout: LDS %zu too large", lds_bytes);
  // LDS-resident actor weights (see rollout_persist_kernel) when they fit
  const size_t lw_bytes = sizeof(float) * (size_t)(32 + 16 * PERSIST_L2_LDS) * 256;
  const bool lw = rpt == 16 && S <= 16 && d->Ha == 256 && 2 * A <= 16 && lds_bytes + lw_bytes <= 160 * 1024;
  const bool paired = S1 <= 16 && d->Hm == 200;   // the kernel's PM specialisation
  const bool self_emit = (int64_t)H * a.ntiles <= EMIT_SELF_MAX;
  if (self_emit) {
    a.vptr_in = d->vptr;
    a.base_slot = off + H + 1;
  }
  if (d->step_events) hipEventRecord((hipEvent_t)d->step_events[0], stream);
  if (rpt == 32) {
    if (paired) rollout_persist_kernel<2, 8, false, 1><<<a.ntiles, 8 * 64, lds_bytes, stream>>>(a);
    else rollout_persist_kernel<2, 8, false, 0><<<a.ntiles, 8 * 64, lds_bytes, stream>>>(a);
  } else if (lw) {
    if (paired) rollout_persist_kernel<1, 8, true, 1><<<a.ntiles, 8 * 64, lds_bytes + lw_bytes, stream>>>(a);
    else rollout_persist_kernel<1, 8, true, 0><<<a.ntiles, 8 * 64, lds_bytes + lw_bytes, stream>>>(a);
  } else {
    if (paired) rollout_persist_kernel<1, 8, false, 1><<<a.ntiles, 8 * 64, lds_bytes, stream>>>(a);
    else rollout_persist_kernel<1, 8, false, 0><<<a.ntiles, 8 * 64, lds_bytes, stream>>>(a);
  }
  DRPO_LAUNCH_CHECK("rollout_persist");
  if (d->step_events) hipEventRecord((hipEvent_t)d->step_events[1], stream);
  const dim3 eg((unsigned)((a.ntiles * rpt + 255) / 256), (unsigned)H);
  if (self_emit) {
    if (rpt == 32)
      rollout_emit_self_kernel<32><<<eg, 256, 0, stream>>>(a, off + H + 1, d->vptr, off, d->vcap, d->vs, d->va,
                                                           d->vs2, d->vr, d->vh, d->vd, d->vv);
    else
      rollout_emit_self_kernel<16><<<eg, 256, 0, stream>>>(a, off + H + 1, d->vptr, off, d->vcap, d->vs, d->va,
                                                           d->vs2, d->vr, d->vh, d->vd, d->vv);
    DRPO_LAUNCH_CHECK("rollout_emit_self");
    return DRPO_OK;
  }
  // mid-size rollouts: scan + offsets + pointer advance in one single-workgroup launch
  const int fin1 = (int64_t)H * a.ntiles <= 16384;
  if (fin1) {
    rollout_scanfin_kernel<<<1, 256, 0, stream>>>(a.cnt, pos, n, off, d->vptr, a.ntiles, H);
    DRPO_LAUNCH_CHECK("rollout_scanfin");
  } else {
    rollout_scan_kernel<<<H, 256, 0, stream>>>(a.cnt, pos, n, a.ntiles);
    DRPO_LAUNCH_CHECK("rollout_scan");
  }
  if (rpt == 32)
    rollout_emit_kernel<32><<<eg, 256, 0, stream>>>(a, pos, n, d->vptr, fin1, off, d->vcap, d->vs, d->va,
                                                    d->vs2, d->vr, d->vh, d->vd, d->vv);
  else
    rollout_emit_kernel<16><<<eg, 256, 0, stream>>>(a, pos, n, d->vptr, fin1, off, d->vcap, d->vs, d->va,
                                                    d->vs2, d->vr, d->vh, d->vd, d->vv);
  DRPO_LAUNCH_CHECK("rollout_emit");
  if (fin1) return DRPO_OK;
  rollout_persist_finalize_kernel<<<1, 1, 0, stream>>>(d->vptr, n, off, H);
  DRPO_LAUNCH_CHECK("rollout_finalize");
  return DRPO_OK;
}

DRPO_API int drpo_rollout(const drpo_rollout_desc_t* d, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(d, "drpo_rollout: null descriptor");
  DRPO_REQUIRE(d->S >= 1 && d->S <= 64 && d->A >= 1 && d->A <= 8, "drpo_rollout: S=%d A=%d out of range", d->S, d->A);
  DRPO_REQUIRE(d->Ha >= 1 && d->Ha <= 256 && d->Hm >= 1 && d->Hm <= 256, "drpo_rollout: hidden dims must be <= 256");
  DRPO_REQUIRE(d->S + 1 <= 64, "drpo_rollout: state_dim+1 must be <= 64");
  DRPO_REQUIRE(d->C >= 1 && d->C <= 8 && d->C == env_con_dim(d->env_id, d->tracking_n_surr),
               "drpo_rollout: con_dim %d does not match env %d", d->C, d->env_id);
  DRPO_REQUIRE(d->B >= 1 && d->H >= 1 && (int64_t)d->B * d->H <= d->vcap,
               "drpo_rollout: B*H=%lld exceeds buffer capacity %lld", (long long)d->B * d->H, (long long)d->vcap);
  DRPO_REQUIRE(d->workspace && d->vptr && d->replay_states, "drpo_rollout: null pointer");
  DRPO_REQUIRE(d->B <= 16 * 8192, "drpo_rollout: batch %d too large (max 131072)", d->B);
  const int64_t rlen = d->replay_ptr < d->replay_cap ? d->replay_ptr : d->replay_cap;
  DRPO_REQUIRE(rlen >= d->B, "drpo_rollout: replay has %lld rows < batch %d (sampling without replacement)",
               (long long)rlen, d->B);
  if (d->env_id == ENV_TRACKING)
    DRPO_REQUIRE(d->tracking_surr_start + 4 * d->tracking_n_surr <= d->S, "drpo_rollout: tracking layout");

  RolloutWs w = rollout_ws(d->B, d->S, d->H, (char*)d->workspace);
  // 32-row tiles halve the weight bytes per MFMA once the batch fills the chip with
  // them (B >= 8192), when the wider tile still fits the LDS (not for tracking's S=51)
  const int rpt = d->rows_per_tile ? d->rows_per_tile
                                   : (d->B >= 256 * 32 &&
                                              persist_lds_bytes(d->S, d->A, d->Ha, d->Hm, 32, 8) <= 160 * 1024
                                          ? 32 : 16);
  DRPO_REQUIRE(rpt == 16 || rpt == 32, "drpo_rollout: rows_per_tile must be 16 or 32");
  const int S = d->S, A = d->A, S1 = d->S + 1;
  DRPO_REQUIRE(d->engine >= 0 && d->engine <= 2 && (d->eps_layout == 0 || d->eps_layout == 1),
               "drpo_rollout: engine %d / eps_layout %d", d->engine, d->eps_layout);
  DRPO_REQUIRE((d->eps_a == nullptr) == (d->eps_m == nullptr), "drpo_rollout: eps_a and eps_m go together");
  int engine = d->engine;
  if (engine == 0) engine = (d->eps_a && d->eps_layout == 0) || d->H > PERSIST_MAX_H ? 1 : 2;
  if (d->eps_a)
    DRPO_REQUIRE(d->eps_layout == engine - 1, "drpo_rollout: eps_layout %d cannot drive engine %d (compacted draws "
                 "need engine 1, original-row draws engine 2)", d->eps_layout, engine);
  if (engine == 2) return rollout_fused(d, rpt, rlen, stream);

  RolloutStepArgs a{};
  a.S = S; a.A = A; a.C = d->C; a.Ha = d->Ha; a.Hm = d->Hm; a.Bmax = d->B;
  a.env.id = d->env_id; a.env.surr_start = d->tracking_surr_start; a.env.n_surr = d->tracking_n_surr;
  a.env.thr0 = d->env_thr0; a.env.thr1 = d->env_thr1;
  a.aW1 = d->aW1; a.ab1 = d->ab1; a.aW2 = d->aW2; a.ab2 = d->ab2; a.aW3 = d->aW3; a.ab3 = d->ab3;
  a.norm_mean = d->norm_mean; a.norm_std = d->norm_std; a.min_lv = d->min_lv; a.max_lv = d->max_lv;
  a.replay_states = d->replay_states; a.init_idx = d->init_idx;
  a.replay_len = rlen; a.replay_ptr = d->replay_ptr; a.replay_cap = d->replay_cap;
  a.prp_half_bits = hb_for(rlen);
  for (int i = 0; i < 4; ++i) a.prp_key[i] = (uint32_t)(d->seed >> (8 * i)) * 0x9E3779B9u + (uint32_t)d->ctr * (2 * i + 1) + i;
  a.seed = d->seed; a.ctr = d->ctr;
  a.vs = d->vs; a.va = d->va; a.vs2 = d->vs2; a.vr = d->vr; a.vh = d->vh; a.vd = d->vd; a.vv = d->vv;
  a.vptr = d->vptr; a.vcap = d->vcap;
  a.n = w.n; a.off = w.off;
  a.ldx = lds_ld(S + A);
  a.ldh = lds_ld(d->Ha > d->Hm ? d->Ha : d->Hm);
  a.ldm = round_up(S1, 16) + 4;
  a.lds = round_up(S, 4);

  const int tiles = (d->B + rpt - 1) / rpt;
  constexpr int NW = 8;
  const size_t lds_bytes = sizeof(float) * ((size_t)rpt * (a.ldx + 3 * a.ldh + a.lds + 20 + 2 * a.ldm + 8 + 1 + 8 + 2) +
                                            (size_t)NW * (rpt / 16) * 256 + NW * 64 + (size_t)tiles + 1 + 256);
  DRPO_REQUIRE(lds_bytes <= 160 * 1024, "drpo_rollout: LDS %zu too large", lds_bytes);

  const int E_out_in[6][2] = {{d->Hm, S + A}, {d->Hm, d->Hm}, {d->Hm, d->Hm}, {S1, d->Hm}, {d->Hm, d->Hm}, {S1, d->Hm}};
  const float* Wb[6] = {d->mW1, d->mW2, d->dW1, d->dW2, d->lW1, d->lW2};
  const float* Bb[6] = {d->mb1, d->mb2, d->db1, d->db2, d->lb1, d->lb2};

  for (int t = 0; t < d->H; ++t) {
    const int m = d->members[t];
    const float* Wm[6];
    const float* Bm[6];
    for (int i = 0; i < 6; ++i) {
      // packed mirrors: member stride = drpo_packed_size(in, out)
      Wm[i] = Wb[i] + (size_t)m * drpo_packed_size(E_out_in[i][1], E_out_in[i][0]);
      Bm[i] = Bb[i] + (size_t)m * E_out_in[i][0];
    }
    a.mW1 = Wm[0]; a.mW2 = Wm[1]; a.dW1 = Wm[2]; a.dW2 = Wm[3]; a.lW1 = Wm[4]; a.lW2 = Wm[5];
    a.mb1 = Bm[0]; a.mb2 = Bm[1]; a.db1 = Bm[2]; a.db2 = Bm[3]; a.lb1 = Bm[4]; a.lb2 = Bm[5];
    a.t = t;
    const int cur = t & 1, prv = cur ^ 1;
    a.prev_nxt = w.nxt[prv]; a.prev_cnt = w.cnt[prv]; a.prev_inv = w.inv[prv];
    a.nxt = w.nxt[cur]; a.cnt = w.cnt[cur]; a.inv = w.inv[cur];
    a.eps_a = d->eps_a ? d->eps_a + (size_t)t * d->B * A : nullptr;
    a.eps_m = d->eps_m ? d->eps_m + (size_t)t * d->B * S1 : nullptr;
    if (d->step_events) hipEventRecord((hipEvent_t)d->step_events[2 * t], stream);
    if (rpt == 32)
      rollout_step_kernel<2, NW><<<tiles, NW * 64, lds_bytes, stream>>>(a);
    else
      rollout_step_kernel<1, NW><<<tiles, NW * 64, lds_bytes, stream>>>(a);
    DRPO_LAUNCH_CHECK("rollout_step");
    if (d->step_events) hipEventRecord((hipEvent_t)d->step_events[2 * t + 1], stream);
  }
  rollout_finalize_kernel<<<1, 1, 0, stream>>>(d->vptr, w.n, w.off, d->H);
  DRPO_LAUNCH_CHECK("rollout_finalize");
  return DRPO_OK;
}

// Standalone batched constraint evaluation (tests, evaluation, robust target).
__global__ void env_constraints_kernel(EnvParams ep, const float* s, int64_t n, int S, int C, uint8_t* done,
                                       uint8_t* viol, float* h) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  bool dn, vl;
  float hh[8];
  env_constraints_row(ep, s + i * S, dn, vl, hh);
  if (done) done[i] = dn;
  if (viol) viol[i] = vl;
  if (h)
    for (int c = 0; c < C; ++c) h[i * C + c] = hh[c];
}

DRPO_API int drpo_env_constraints(int env_id, int tracking_surr_start, int tracking_n_surr, double env_thr0,
                                  double env_thr1, const float* states, int64_t n, int S, uint8_t* done,
                                  uint8_t* violation, float* h, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(env_id >= 0 && env_id <= 3, "drpo_env_constraints: unknown env id %d", env_id);
  if (n == 0) return DRPO_OK;
  EnvParams ep{env_id, tracking_surr_start, tracking_n_surr, env_thr0, env_thr1};
  const int C = env_con_dim(env_id, tracking_n_surr);
  env_constraints_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(ep, states, n, S, C, done, violation, h);
  DRPO_LAUNCH_CHECK("env_constraints");
  return DRPO_OK;
}

__global__ void prp_kernel(int64_t* out, int64_t B, int64_t N, int hb, uint32_t k0, uint32_t k1, uint32_t k2,
                           uint32_t k3) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const uint32_t key[4] = {k0, k1, k2, k3};
  out[i] = prp_index((uint64_t)i, (uint64_t)N, hb, key);
}

DRPO_API int drpo_sample_without_replacement(int64_t* out, int64_t B, int64_t N, uint64_t seed, uint64_t ctr,
                                             drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(B >= 0 && B <= N && N < (1ll << 62), "drpo_sample_without_replacement: need 0 <= B <= N");
  if (B == 0) return DRPO_OK;
  uint32_t k[4];
  for (int i = 0; i < 4; ++i) k[i] = (uint32_t)(seed >> (8 * i)) * 0x9E3779B9u + (uint32_t)ctr * (2 * i + 1) + i;
  prp_kernel<<<(unsigned)((B + 255) / 256), 256, 0, stream>>>(out, B, N, hb_for(N), k[0], k[1], k[2], k[3]);
  DRPO_LAUNCH_CHECK("prp");
  return DRPO_OK;
}
