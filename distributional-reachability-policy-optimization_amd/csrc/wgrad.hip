// Grouped weight gradients dW = dZ^T Y, db = colsum(dZ) for every layer of a
// parameter group in ONE launch (the reference's autograd of BatchedLinear /
// nn.Linear, src/dynamics.py:26-52, src/torch_util.py:190-211), plus the per-tile
// sums of squares of the finished gradient that clip_grad_norm_ needs
// (src/ssac.py:454,494-527, torch.nn.utils.clip_grad_norm_).
//
// Work split. An item (one layer x nbatch members) is cut into output tiles of
// TO x TI (TO, TI = 64, or 16 for a layer with <= 16 outputs / inputs, so the
// narrow output heads and the S+A-wide input layers do not pay for 64-wide
// padding) times row chunks. One 256-thread workgroup owns a (tile, chunk) unit:
// its 4 waves split the chunk's rows (4-row k-groups, interleaved), and every wave
// streams its own dZ / Y fragments straight from global memory into a register ring
// (no LDS staging, no barriers in the main loop): per k-group one 16-byte load of 4
// consecutive outputs and one of 4 consecutive inputs feed 4 x 4 MFMAs
// (v_mfma_f32_16x16x4_f32, exact f32), MFMA m covering o = o0 + 4*(lane&15) + m and
// MFMA n covering i = i0 + 4*(lane&15) + n, k = the 4 rows. The chunk sizes are
// chosen on the host so that every unit costs about the same and all units are
// resident at once (<= 2 workgroups per CU): no partial second round.
//
// Hand-off. The 4 waves' partial tiles are summed through LDS. A tile with one row
// chunk adds its sum to the gradient directly. Otherwise each unit writes its partial
// (and bias partial) to a slab with write-through (sc1) stores, waits for them
// (vmcnt(0)), and one lane adds 1 to the tile's arrival counter (agent-scope atomic).
// The workgroup whose add returns nch-1 is the last: it resets the counter, loads
// every slab of the tile with sc1 loads, sums them in chunk order (deterministic, no
// float atomics), adds the sum to the gradient and writes the tile's sum of squares.
// That is MI355X_MICROARCH.md's validated hand-off (sc1 payload, drained, one
// ticket add per workgroup, last arriver by the returned value, sc1 loads); nothing
// ever waits, so no schedule can hang it.
//
// Memory-model note. Every operation of the hand-off is RELAXED (agent scope): the
// slab stores, the ticket add and the slab loads. Under the C++ / HIP memory model
// nothing orders the slab stores before the ticket or the ticket before the loads;
// the hand-off is correct because of gfx950's ordering, not because of
// release/acquire semantics:
//   - an agent-scope relaxed store is a write-through `global_store ... sc1` (the bytes
//     leave the XCD's L2 for the agent-coherent memory side);
//   - `s_waitcnt vmcnt(0)` after the stores, then a workgroup barrier, then the one
//     ticket add: the add issues only after every wave's stores have completed;
//   - the last arriver learns it from the add's returned value and reads the slabs with
//     `global_load ... sc1` (bypassing the per-CU L1, which is never refreshed by
//     other CUs' stores), issued only after the add returned.
// This is the first row of MI355X_MICROARCH.md's table of hand-offs measured with sc1
// loads in place of the acquire (one lane per storing workgroup adds to one counter after
// every wave's vmcnt(0) wait; the last adder, told by the returned value, loads with sc1).
// An __ATOMIC_ACQ_REL ticket would lower to `buffer_wbl2 sc1` + `buffer_inv sc1` around
// the add: a write-back of the XCD's whole L2 and an L1 invalidate, each ~1.7 us per
// workgroup (the guide's price list) -- measured and rejected (profiles/r05/wgrad_setup).
#include "common.hpp"
#include "ens_reduce.hpp"

using namespace drpo;

namespace {
constexpr int WG_NW = 4;                 // waves per workgroup
constexpr int WG_NT = WG_NW * 64;
constexpr int WG_D = 3;                  // register ring slots (k-groups of 4 rows each; 3 measured best, profiles/r04/wgrad)
constexpr int WG_ROWQ = 64;              // chunk granularity (rows)
constexpr int WG_MAXITEMS = 16;
constexpr int WG_SLD = 264;              // LDS slab stride per accumulator block (== 8 mod 32)
}  // namespace

#ifdef DRPO_STAMPS
// profiling builds only (profiles/wgrad_probe.py): per-workgroup s_memtime stamps
__device__ unsigned long long g_stamps_wg[1 << 14][8];
#define STAMPG(i)                                                                                 \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    unsigned long long _t;                                                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(_t)::"memory");                    \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (threadIdx.x == 0 && blockIdx.x < (1u << 14)) g_stamps_wg[blockIdx.x][(i)] = _t;           \
  } while (0)
DRPO_API int drpo_debug_stamps_wgrad(unsigned long long* dst, int n) {
  return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_stamps_wg), sizeof(unsigned long long) * 8 * (size_t)n);
}
DRPO_API int drpo_debug_stamps_wgrad_clear() {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_stamps_wg)) != hipSuccess) return 1;
  return (int)hipMemset(p, 0, sizeof(g_stamps_wg));
}
#else
#define STAMPG(i) \
  do {            \
  } while (0)
#endif

struct WgradPlan {
  int to, ti;              // tile shape (64 or 16)
  int nto, nti, nch;       // tiles along outputs / inputs, row chunks
  int chunk;               // rows per chunk (multiple of WG_ROWQ)
  int va, vb;              // 16-byte loads of dZ / Y rows (widths % 4 == 0, aligned)
  int z2;                  // a second dZ term (item dz2)
  int pk_layer;            // fused Adam: the item's matrix in the pack map (-1: none)
  int pk_z0;               // its first member within that matrix (a member shard's slice)
  int vf;                  // 64x64 tiles, 16-byte aligned rows: the finish in float4s
  int64_t first_unit;      // first logical workgroup of the item
  int64_t first_tile;      // first arrival counter of the item
  int64_t slab_off;        // first slab float of the item (tiles with nch > 1)
};

constexpr int WG_MAXSUMS = 4;

struct WgradArgs {   // (kernarg: <= 4 KB, static_assert below)
  int64_t first[WG_MAXITEMS];        // first logical workgroup per item (unused: INT64_MAX)
  drpo_wgrad_item_t it[WG_MAXITEMS];
  WgradPlan pl[WG_MAXITEMS];
  int64_t units;
  int n;
  int has_red;
  drpo_ens_reduce_t red;
  int nsums;                         // > 0: one extra (logically last) block adds partial sums
  drpo_sum_t sums[WG_MAXSUMS];
  int has_adam;                      // fused Adam step (drpo_mlp_wgrad_adam)
  drpo_wgrad_adam_t adam;
  float* slab;
  unsigned* ctr;
};

// The launch arguments are read in place from the kernarg segment (address space 4,
// scalar loads): with the by-value parameter the compiler copies the 3 KB struct to
// scratch once the kernel's code grows (dynamic item index + many instantiations).
typedef const __attribute__((address_space(4))) WgradArgs WgradArgsK;

// *out = part[0] + ... + part[n-1] for every entry, in a fixed order (256 strided
// lanes, then a fixed tree): deterministic, no float atomics
__device__ __forceinline__ void sums_block(WgradArgsK& a, float* red) {
  for (int q = 0; q < a.nsums; ++q) {
    const auto& S = a.sums[q];
    float v = 0.f;
    for (int j = threadIdx.x; j < S.n; j += WG_NT) v += S.part[j];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int w = WG_NT / 2; w > 0; w >>= 1) {
      if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) *S.out = red[0];
    __syncthreads();
  }
}

// write-through (sc1) float store / load: the slab hand-off between workgroups
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// 4 consecutive columns c..c+3 (W == 4) or column c (W == 1, in .x) of row `row` of a
// row-major [.][ld] matrix. No value is masked here: the caller clamps row / c to
// valid addresses, a column past the matrix only feeds output elements that are never
// stored, and rows past the chunk are zeroed where the fragment is consumed (a
// select right after the load would make the wave wait for it, collapsing the ring).
template <int W, bool VEC>
__device__ __forceinline__ f32x4 frag_load(const float* __restrict__ M, int64_t row, int64_t ld, int c, int ncols) {
  const float* p = M + row * ld + c;
  f32x4 v;
  if constexpr (W == 4 && VEC) {
    v = gload(reinterpret_cast<const f32x4*>(p));
  } else if constexpr (W == 4) {
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = gload(c + u < ncols ? p + u : p);
  } else {
    v = f32x4{gload(p), 0.f, 0.f, 0.f};
  }
  return v;
}

template <int TO, int TI>
__device__ __forceinline__ void frag_mma(const f32x4& a, const f32x4& b, f32x4 (&acc)[TO / 16][TI / 16]) {
  constexpr int MA = TO / 16, MB = TI / 16;
  if constexpr (MA == 4 && MB == 4) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], b[n], acc[m][n], 0, 0, 0);
  } else if constexpr (MA == 4) {
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], b[0], acc[m][0], 0, 0, 0);
  } else if constexpr (MB == 4) {
#pragma unroll
    for (int n = 0; n < 4; ++n) acc[0][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[n], acc[0][n], 0, 0, 0);
  } else {
    acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], acc[0][0], 0, 0, 0);
  }
}

// LDS float index, inside wave w's slab, of tile element (ol, il) (accumulator
// layout: acc[m][n][rr] of lane (G, L) holds o = 4*(4G + rr) + m (TO 64) or
// 4G + rr (TO 16), i = 4L + n (TI 64) or L (TI 16))
template <int TO, int TI>
__device__ __forceinline__ int slab_index(int w, int ol, int il) {
  constexpr int NA = (TO / 16) * (TI / 16), NB = TI / 16;
  int m, rr, G, n, L;
  if constexpr (TO == 64) {
    m = ol & 3; rr = (ol >> 2) & 3; G = ol >> 4;
  } else {
    m = 0; rr = ol & 3; G = ol >> 2;
  }
  if constexpr (TI == 64) {
    n = il & 3; L = il >> 2;
  } else {
    n = 0; L = il;
  }
  return (w * NA + m * NB + n) * WG_SLD + rr * 64 + 16 * G + L;
}

__device__ __forceinline__ float wg_block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < WG_NW; ++i) s += red[i];
  return s;   // valid in thread 0
}

template <int TO, int TI, bool VA, bool VB, bool Z2>
__device__ __forceinline__ void wgrad_unit(WgradArgsK& a, int q, int64_t u, float* lds) {
  constexpr int MA = TO / 16, MB = TI / 16, NA = MA * MB;
  constexpr int WA = TO == 64 ? 4 : 1, WB = TI == 64 ? 4 : 1;
  constexpr int E = TO * TI / WG_NT;          // tile elements per thread (16, 4 or 1)
  const auto& I = a.it[q];
  const auto& P = a.pl[q];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, l15 = lane & 15;
  // 32-bit decode (an item has < 2^31 units): a 64-bit division expands to a long
  // stretch of scalar code, fetched cold by every workgroup at every dispatch
  const unsigned uu = (unsigned)u;
  const int it_i = (int)(uu % (unsigned)P.nti);
  unsigned rest = uu / (unsigned)P.nti;
  const int it_o = (int)(rest % (unsigned)P.nto);
  rest /= (unsigned)P.nto;
  const int ch = (int)(rest % (unsigned)P.nch);
  const int zb = (int)(rest / (unsigned)P.nch);
  const int64_t tile_local = ((int64_t)zb * P.nto + it_o) * P.nti + it_i;
  const int dout = I.dout, din = I.din;
  const float* __restrict__ dz = I.dz + (size_t)zb * I.zstride;
  const float* __restrict__ dz2 = Z2 ? I.dz2 + (size_t)zb * I.zstride : nullptr;
  const float* __restrict__ y = I.y + (size_t)zb * I.ystride;
  const int o0 = it_o * TO, i0 = it_i * TI;
  const int64_t r0 = (int64_t)ch * P.chunk;
  const int64_t r1 = min(I.rows, r0 + P.chunk);
  const bool do_bias = it_i == 0;

  // this lane's columns, clamped to valid addresses (masked to zero when out of range)
  const int ca_raw = o0 + (WA == 4 ? 4 * l15 : l15);
  const int cb_raw = i0 + (WB == 4 ? 4 * l15 : l15);
  const int ca = ca_raw < dout ? ca_raw : 0, cb = cb_raw < din ? cb_raw : 0;

  f32x4 acc[MA][MB];
#pragma unroll
  for (int m = 0; m < MA; ++m)
#pragma unroll
    for (int n = 0; n < MB; ++n) acc[m][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 bsum = {0.f, 0.f, 0.f, 0.f};

  // wave k-group j covers rows r0 + 16 j + 4 wave + (0..3); lane group g takes row 4.. + g
  const int nj = P.chunk / (4 * WG_NW);      // k-groups per wave
  const int64_t rlane = r0 + 4 * wave + g;
  auto ld = [&](int j, f32x4& fa, f32x4& fb, f32x4& fa2) {
    const int64_t r = rlane + 16 * (int64_t)j;
    const int64_t rc = r < r1 ? r : r1 - 1;
    fa = frag_load<WA, VA>(dz, rc, dout, ca, dout);
    fb = frag_load<WB, VB>(y, rc, din, cb, din);
    if constexpr (Z2) fa2 = frag_load<WA, VA>(dz2, rc, dout, ca, dout);
  };
  auto use = [&](int j, f32x4 fa, const f32x4& fb, const f32x4& fa2) {
    if constexpr (Z2) fa += fa2;   // the two dZ terms, added at use (see frag_load)
    if (rlane + 16 * (int64_t)j >= r1) fa = f32x4{0.f, 0.f, 0.f, 0.f};   // row past the chunk
    frag_mma<TO, TI>(fa, fb, acc);
    if (do_bias) bsum += fa;
  };
  // Register ring of WG_D slots: step s loads k-group s into slot s % D and consumes
  // k-group s - (D - 1) (D - 1 k-groups of cover). Every load is inside the loop: with
  // a prologue of loads outside it the compiler drains vmcnt at every loop entry. Steps
  // past the chunk load clamped rows that are never consumed or are zeroed at use.
  f32x4 ra[WG_D], rb[WG_D], ra2[Z2 ? WG_D : 1];
#pragma unroll
  for (int v = 0; v < WG_D; ++v) ra[v] = rb[v] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int v = 0; v < (Z2 ? WG_D : 1); ++v) ra2[v] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int steps = (nj + WG_D - 1 + WG_D - 1) / WG_D * WG_D;
  STAMPG(6);
  for (int s0 = 0; s0 < steps; s0 += WG_D) {
#pragma unroll
    for (int v = 0; v < WG_D; ++v) {
      ld(s0 + v, ra[v], rb[v], ra2[Z2 ? v : 0]);
      // keep the prefetch here: the scheduler would otherwise sink the loads past the
      // MFMAs, next to their first use
      __builtin_amdgcn_sched_barrier(0);
      if (s0 + v >= WG_D - 1)
        use(s0 + v - (WG_D - 1), ra[(v + 1) % WG_D], rb[(v + 1) % WG_D], ra2[Z2 ? (v + 1) % WG_D : 0]);
    }
#ifdef DRPO_STAMPS
    if (s0 == 0) STAMPG(7);      // the first k-group consumed: the ring's fill latency
    if (s0 == WG_D) STAMPG(5);
#endif
  }

  STAMPG(1);
  // Thread t owns tile elements t + 256 e: il = t % TI, ol = t / TI + (256 / TI) e; with
  // P.vf (64x64 tiles) it owns 4 runs of 4 consecutive inputs instead: run f = t + 256 j
  // is row ol = f / 16, inputs 4 (f % 16) .. + 3 -- the gradient / Adam reads and writes
  // then go as float4s (a quarter of the memory instructions; the forward mirror's 4
  // components are one float4 too). A slab (nch > 1) stores element e at t + 256 e in
  // either mapping: the writer and the last arriver of a tile use the same one.
  const bool vf = TO == 64 && TI == 64 && P.vf;
  auto elem = [&](int e, int& ol, int& il) {
    if (vf) {
      const int f = tid + WG_NT * (e >> 2);
      ol = f >> 4;
      il = ((f & 15) << 2) + (e & 3);
    } else {
      const int idx = tid + WG_NT * e;
      ol = idx / TI;
      il = idx % TI;
    }
  };
  constexpr int SL = TO * TI + TO;            // slab floats per unit (tile + bias)
  float* gW = I.gW + (size_t)zb * I.gwstride;
  float* gb = I.gb + (size_t)zb * I.gbstride;
  float* red = lds + WG_NW * NA * WG_SLD + WG_NW * TO;   // 4 floats
  // the gradient's current values: loaded by the workgroup that finishes the tile,
  // before (and in flight with) the slab loads; every load precedes the first store.
  // A single-chunk tile (nch == 1) is finished by its only workgroup: its loads are
  // issued here, ahead of the partial tiles' LDS reduction, which covers their latency
  float gv[E];
  const bool bias_mine = do_bias && tid < TO && o0 + tid < dout;
  float gbv = 0.f;
  // fused Adam (drpo_mlp_wgrad_adam): the parameters and moments of the tile, loaded with
  // the gradient's current values
  const bool adam = a.has_adam;
  const int64_t eW = adam ? gW - a.adam.g : 0, eb = adam ? gb - a.adam.g : 0;   // flat element offsets
  float ap[E], am[E], av[E], bp = 0.f, bm = 0.f, bvv = 0.f;
  auto ld4 = [&](const float* base, int64_t k, bool in, float* dst) {
    const f32x4 v = in ? *reinterpret_cast<const f32x4*>(base + k) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) dst[c] = v[c];
  };
  auto load_grad = [&]() {
    if (vf) {   // din % 4 == 0: a run of 4 is wholly inside or outside the matrix
#pragma unroll
      for (int j = 0; j < E / 4; ++j) {
        int ol, il;
        elem(4 * j, ol, il);
        const int o = o0 + ol, i = i0 + il;
        const bool in = o < dout && i < din;
        const int64_t k = (int64_t)o * din + i;
        ld4(gW, k, in, gv + 4 * j);
        if (adam) {
          ld4(a.adam.p + eW, k, in, ap + 4 * j);
          ld4(a.adam.m + eW, k, in, am + 4 * j);
          ld4(a.adam.v + eW, k, in, av + 4 * j);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        int ol, il;
        elem(e, ol, il);
        const int o = o0 + ol, i = i0 + il;
        const bool in = o < dout && i < din;
        const int64_t k = (int64_t)o * din + i;
        gv[e] = in ? gW[k] : 0.f;
        if (adam) {
          ap[e] = in ? a.adam.p[eW + k] : 0.f;
          am[e] = in ? a.adam.m[eW + k] : 0.f;
          av[e] = in ? a.adam.v[eW + k] : 0.f;
        }
      }
    }
    gbv = bias_mine ? gb[o0 + tid] : 0.f;
    if (adam && bias_mine) {
      bp = a.adam.p[eb + o0 + tid];
      bm = a.adam.m[eb + o0 + tid];
      bvv = a.adam.v[eb + o0 + tid];
    }
  };
  if (P.nch == 1) load_grad();
  // the 4 waves' partial tiles -> LDS slabs (conflict-free: lanes write consecutive words)
  float* R = lds;
#pragma unroll
  for (int m = 0; m < MA; ++m)
#pragma unroll
    for (int n = 0; n < MB; ++n)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) R[(wave * NA + m * MB + n) * WG_SLD + rr * 64 + lane] = acc[m][n][rr];
  // bias partials: sum over the 4 row lanes g of each column, then over waves (LDS)
  float* Rb = lds + WG_NW * NA * WG_SLD;      // [WG_NW][TO]
  if (do_bias) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float s = bsum[c];
      s += __shfl_xor(s, 16, 64);
      s += __shfl_xor(s, 32, 64);
      bsum[c] = s;
    }
    if (g == 0) {
      if constexpr (WA == 4) {
#pragma unroll
        for (int c = 0; c < 4; ++c) Rb[wave * TO + 4 * l15 + c] = bsum[c];
      } else {
        Rb[wave * TO + l15] = bsum[0];
      }
    }
  }
  __syncthreads();
  float pv[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    int ol, il;
    elem(e, ol, il);
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < WG_NW; ++w) s += R[slab_index<TO, TI>(w, ol, il)];
    pv[e] = s;
  }
  float pb = 0.f;
  if (do_bias && tid < TO) {
#pragma unroll
    for (int w = 0; w < WG_NW; ++w) pb += Rb[w * TO + tid];
  }
  STAMPG(2);
  if (P.nch > 1) {
    float* my = a.slab + P.slab_off + (tile_local * P.nch + ch) * SL;
#pragma unroll
    for (int e = 0; e < E; ++e) st_sc1(my + tid + WG_NT * e, pv[e]);
    if (do_bias && tid < TO) st_sc1(my + TO * TI + tid, pb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int& s_last = *reinterpret_cast<int*>(red + 4);
    if (tid == 0) {
      unsigned* c = a.ctr + P.first_tile + tile_local;
      // relaxed: see the memory-model note at the top (gfx950 ordering, not C++ acq_rel)
      const unsigned old = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = old == (unsigned)(P.nch - 1);
      if (last) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_last = last;
    }
    __syncthreads();
    STAMPG(3);
    if (!s_last) return;
    load_grad();
    // last arriver: the tile's partials in chunk order, CG chunks' loads in flight at a
    // time (one memory round trip per group of chunks, not per chunk)
    const float* base = a.slab + P.slab_off + tile_local * P.nch * SL;
    const bool bias_lane = do_bias && tid < TO;
#pragma unroll
    for (int e = 0; e < E; ++e) pv[e] = 0.f;
    pb = 0.f;
    constexpr int CG = E >= 16 ? 4 : 8;
    for (int c0 = 0; c0 < P.nch; c0 += CG) {
      float t[CG][E], tb[CG];
#pragma unroll
      for (int u = 0; u < CG; ++u) {
        const int c = min(c0 + u, P.nch - 1);     // clamped: a duplicate load, not added
#pragma unroll
        for (int e = 0; e < E; ++e) t[u][e] = ld_sc1(base + c * SL + tid + WG_NT * e);
        tb[u] = bias_lane ? ld_sc1(base + c * SL + TO * TI + tid) : 0.f;
      }
#pragma unroll
      for (int u = 0; u < CG; ++u) {
        if (c0 + u < P.nch) {
#pragma unroll
          for (int e = 0; e < E; ++e) pv[e] += t[u][e];
          pb += tb[u];
        }
      }
    }
  }
  if (adam) {
    // the finished gradient g = current terms + this launch's sum -> Adam (the
    // drpo_optim_step arithmetic), the tile's forward / transposed mirrors refreshed; the
    // gradient itself is never written (nonzero input terms are cleared)
    const drpo_pack_map_t* md = P.pk_layer >= 0 ? (const drpo_pack_map_t*)a.adam.map : nullptr;
    const int ncb = (dout + 15) >> 4, nks = (din + 15) >> 4;
    const int64_t mb = md ? md->poff[P.pk_layer] + (int64_t)(P.pk_z0 + zb) * ncb * nks * 256 : 0;
    float* PM = md ? md->P : nullptr;
    float* PTM = md ? md->PT : nullptr;
    if (vf) {
#pragma unroll
      for (int j = 0; j < E / 4; ++j) {
        int ol, il;
        elem(4 * j, ol, il);
        const int o = o0 + ol, i = i0 + il;
        if (o >= dout || i >= din) continue;
        const int64_t k = (int64_t)o * din + i;
        f32x4 p4, m4, v4;
        bool nz = false;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float pe = ap[4 * j + c], me = am[4 * j + c], ve = av[4 * j + c];
          adam_step(a.adam, 1.f, gv[4 * j + c] + pv[4 * j + c], pe, me, ve);
          p4[c] = pe;
          m4[c] = me;
          v4[c] = ve;
          nz = nz || gv[4 * j + c] != 0.f;
        }
        *reinterpret_cast<f32x4*>(a.adam.p + eW + k) = p4;
        *reinterpret_cast<f32x4*>(a.adam.m + eW + k) = m4;
        *reinterpret_cast<f32x4*>(a.adam.v + eW + k) = v4;
        if (nz) *reinterpret_cast<f32x4*>(gW + k) = f32x4{0.f, 0.f, 0.f, 0.f};
        if (PM)   // i .. i+3 are the 4 components of one lane of fragment (o>>4, i>>4)
          *reinterpret_cast<f32x4*>(PM + mb + ((int64_t)((o >> 4) * nks + (i >> 4)) << 8) +
                                    ((((i >> 2) & 3) * 16 + (o & 15)) << 2)) = p4;
#pragma unroll
        for (int c = 0; c < 4; ++c) ap[4 * j + c] = p4[c];   // the new parameters (the transposed refresh)
      }
      if (PTM) {
        // transposed mirror: a float4 there is 4 consecutive outputs of one input, so the
        // tile goes through LDS ([64][65] floats over the partial-tile slabs) and each
        // thread stores 4 such float4s instead of 16 scattered floats
        float* T = lds;
        __syncthreads();   // every thread's reads of the partial-tile slabs are done
#pragma unroll
        for (int j = 0; j < E / 4; ++j) {
          int ol, il;
          elem(4 * j, ol, il);
          const bool in = o0 + ol < dout && i0 + il < din;
#pragma unroll
          for (int c = 0; c < 4; ++c) T[ol * 65 + il + c] = in ? ap[4 * j + c] : 0.f;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < E / 4; ++j) {
          const int f = tid + WG_NT * j;
          const int il = f >> 4, ol = (f & 15) << 2;   // input il, outputs ol .. ol + 3
          const int o = o0 + ol, i = i0 + il;
          if (o >= dout || i >= din) continue;
          f32x4 v;
#pragma unroll
          for (int c = 0; c < 4; ++c) v[c] = T[(ol + c) * 65 + il];   // zero past dout: the padding
          *reinterpret_cast<f32x4*>(PTM + mb + ((int64_t)((i >> 4) * ncb + (o >> 4)) << 8) +
                                    ((((o >> 2) & 3) * 16 + (i & 15)) << 2)) = v;
        }
      }
    } else
#pragma unroll
    for (int e = 0; e < E; ++e) {
      int ol, il;
      elem(e, ol, il);
      const int o = o0 + ol, i = i0 + il;
      if (o < dout && i < din) {
        const int64_t k = (int64_t)o * din + i;
        float pe = ap[e], me = am[e], ve = av[e];
        adam_step(a.adam, 1.f, gv[e] + pv[e], pe, me, ve);
        a.adam.p[eW + k] = pe;
        a.adam.m[eW + k] = me;
        a.adam.v[eW + k] = ve;
        if (gv[e] != 0.f) gW[k] = 0.f;
        if (PM)   // forward mirror: fragment (o>>4, i>>4), lane ((i>>2)&3)*16 + (o&15), component i&3
          PM[mb + ((int64_t)((o >> 4) * nks + (i >> 4)) << 8) + ((((i >> 2) & 3) * 16 + (o & 15)) << 2) + (i & 3)] = pe;
        if (PTM)  // transposed: fragment (i>>4, o>>4), lane ((o>>2)&3)*16 + (i&15), component o&3
          PTM[mb + ((int64_t)((i >> 4) * ncb + (o >> 4)) << 8) + ((((o >> 2) & 3) * 16 + (i & 15)) << 2) + (o & 3)] = pe;
      }
    }
    if (bias_mine) {
      adam_step(a.adam, 1.f, gbv + pb, bp, bm, bvv);
      a.adam.p[eb + o0 + tid] = bp;
      a.adam.m[eb + o0 + tid] = bm;
      a.adam.v[eb + o0 + tid] = bvv;
      if (gbv != 0.f) gb[o0 + tid] = 0.f;
    }
    STAMPG(4);
    return;
  }
  // gradient += sum (the caller's gradient is zeroed or holds terms to accumulate)
  float sq = 0.f;
  if (vf) {
#pragma unroll
    for (int j = 0; j < E / 4; ++j) {
      int ol, il;
      elem(4 * j, ol, il);
      const int o = o0 + ol, i = i0 + il;
      if (o >= dout || i >= din) continue;
      f32x4 v4;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        v4[c] = gv[4 * j + c] + pv[4 * j + c];
        sq = fmaf(v4[c], v4[c], sq);
      }
      *reinterpret_cast<f32x4*>(gW + (size_t)o * din + i) = v4;
    }
  } else
#pragma unroll
  for (int e = 0; e < E; ++e) {
    int ol, il;
    elem(e, ol, il);
    const int o = o0 + ol, i = i0 + il;
    if (o < dout && i < din) {
      const float v = gv[e] + pv[e];
      gW[(size_t)o * din + i] = v;
      sq = fmaf(v, v, sq);
    }
  }
  if (bias_mine) {
    const float v = gbv + pb;
    gb[o0 + tid] = v;
    sq = fmaf(v, v, sq);
  }
  if (I.sq) {
    const float s = wg_block_sum(sq, red);
    if (tid == 0) I.sq[I.sq_off + tile_local] = s;
  }
  STAMPG(4);
}

template <int TO, int TI, bool Z2>
__device__ __forceinline__ void wgrad_unit_z(WgradArgsK& a, int q, int64_t u, float* lds) {
  const auto& P = a.pl[q];
  if (P.va && P.vb) wgrad_unit<TO, TI, true, true, Z2>(a, q, u, lds);
  else if (P.va) wgrad_unit<TO, TI, true, false, Z2>(a, q, u, lds);
  else if (P.vb) wgrad_unit<TO, TI, false, true, Z2>(a, q, u, lds);
  else wgrad_unit<TO, TI, false, false, Z2>(a, q, u, lds);
}

template <int TO, int TI>
__device__ __forceinline__ void wgrad_unit_v(WgradArgsK& a, int q, int64_t u, float* lds) {
  if (a.pl[q].z2) wgrad_unit_z<TO, TI, true>(a, q, u, lds);
  else wgrad_unit_z<TO, TI, false>(a, q, u, lds);
}

__global__ __launch_bounds__(WG_NT, 2) void mlp_wgrad_kernel(WgradArgs args) {
  extern __shared__ __attribute__((aligned(16))) float wsm[];
  WgradArgsK& a = *(const __attribute__((address_space(4))) WgradArgs*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)args;
  // logical order: item, then (member, chunk, o-tile, i-tile) with i fastest, spread so
  // that each XCD runs one contiguous range: the units of one row chunk (which read the
  // same dZ / Y rows) share an L2
  STAMPG(0);
  const int64_t bid = xcd_block().x;
  if (bid >= a.units) {        // the extra blocks: deferred reductions
    if (a.has_red && bid == a.units) {
      typedef const __attribute__((address_space(4))) drpo_wgrad_adam_t AdamK;
      ens_loss_reduce_block(a.red, a.has_adam ? &a.adam : (AdamK*)nullptr);
    }
    else if (a.nsums) sums_block(a, wsm);
    return;
  }
  // the item: the number of item starts <= bid, all read at once (independent scalar
  // loads, one kernarg round trip; a dependent search costs one per item passed)
  int q = 0;
#pragma unroll
  for (int i = 1; i < WG_MAXITEMS; ++i) q += bid >= a.first[i] ? 1 : 0;
  const auto& P = a.pl[q];
  const int64_t u = bid - P.first_unit;
  if (P.to == 64 && P.ti == 64) wgrad_unit_v<64, 64>(a, q, u, wsm);
  else if (P.to == 64) wgrad_unit_v<64, 16>(a, q, u, wsm);
  else if (P.ti == 64) wgrad_unit_v<16, 64>(a, q, u, wsm);
  else wgrad_unit_v<16, 16>(a, q, u, wsm);
}

static_assert(sizeof(WgradArgs) <= 4096, "weight-gradient kernarg");

// LDS: 4 wave slabs of the largest tile + bias partials + the block-sum scratch
static size_t wgrad_lds() { return sizeof(float) * ((size_t)WG_NW * 16 * WG_SLD + WG_NW * 64 + 8); }

namespace {

struct Plan {
  WgradArgs a;
  int64_t tiles;     // arrival counters
  int64_t slab;      // slab floats
};

int wg_cus() {
  static int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  return cus;
}

// per-k-group cost of a tile shape in MFMA-issue units (a 16-MFMA k-group is MFMA
// bound; the narrow shapes are bound by their 1.25 / 0.5 KB of loads)
int kg_cost(int to, int ti) { return to == 64 && ti == 64 ? 16 : (to == 64 || ti == 64 ? 6 : 3); }

int plan(const drpo_wgrad_item_t* items, int n, const drpo_ens_reduce_t* red, Plan& p) {
  WgradArgs& a = p.a;
  a = WgradArgs{};
  int m = 0;
  struct Shape { int to, ti, nto, nti; int64_t rows, nb; };
  Shape sh[WG_MAXITEMS];
  for (int k = 0; k < n; ++k) {
    const drpo_wgrad_item_t& I = items[k];
    DRPO_REQUIRE(I.dz && I.y && I.gW && I.gb && I.dout >= 1 && I.din >= 1 && I.rows >= 0 && I.nbatch >= 1,
                 "drpo_mlp_wgrad: bad item %d", k);
    DRPO_REQUIRE(!I.sq || I.sq_off >= 0, "drpo_mlp_wgrad: item %d sq_off", k);
    for (int j = 0; j < k; ++j)
      DRPO_REQUIRE(items[j].gW != I.gW, "drpo_mlp_wgrad: items %d and %d write the same gradient", j, k);
    if (I.rows == 0) continue;
    a.it[m] = I;
    Shape& s = sh[m];
    s.to = I.dout <= 16 ? 16 : 64;
    s.ti = I.din <= 16 ? 16 : 64;
    s.nto = (I.dout + s.to - 1) / s.to;
    s.nti = (I.din + s.ti - 1) / s.ti;
    s.rows = I.rows;
    s.nb = I.nbatch;
    ++m;
  }
  a.n = m;
  // chunk sizes: every unit about the same cost, all units resident at once (2 per CU;
  // 1, 3 or 4 per CU and minimum row counts per unit measured slower, profiles/r04)
  const int64_t slots = 2 * (int64_t)wg_cus();
  auto units_for = [&](double per, int* nch, int* chunk) {
    int64_t tot = 0;
    for (int k = 0; k < m; ++k) {
      const Shape& s = sh[k];
      const double rows_per = per * 16.0 / kg_cost(s.to, s.ti);   // rows whose cost per wave is `per`
      int64_t c = (int64_t)((double)s.rows / (rows_per > 1 ? rows_per : 1) + 0.5);
      c = c < 1 ? 1 : c;
      int64_t ck = (s.rows + c - 1) / c;
      ck = (ck + WG_ROWQ - 1) / WG_ROWQ * WG_ROWQ;
      c = (s.rows + ck - 1) / ck;
      nch[k] = (int)c;
      chunk[k] = (int)ck;
      tot += c * s.nto * s.nti * s.nb;
    }
    return tot;
  };
  double total = 0;
  for (int k = 0; k < m; ++k)
    total += (double)sh[k].nb * sh[k].nto * sh[k].nti * ((sh[k].rows + 15) / 16) * kg_cost(sh[k].to, sh[k].ti);
  int nch[WG_MAXITEMS], chunk[WG_MAXITEMS];
  double per = total / (double)slots;
  if (per < 1) per = 1;
  // grow the per-unit cost until the units fit the resident slots (one round)
  for (int it = 0; it < 64 && units_for(per, nch, chunk) > slots; ++it) per *= 1.08;
  int64_t unit = 0, tile = 0, slab = 0;
  for (int k = 0; k < m; ++k) {
    const Shape& s = sh[k];
    WgradPlan& P = a.pl[k];
    const drpo_wgrad_item_t& I = a.it[k];
    P.to = s.to; P.ti = s.ti; P.nto = s.nto; P.nti = s.nti; P.nch = nch[k]; P.chunk = chunk[k];
    P.va = (I.dout & 3) == 0 && ((uintptr_t)I.dz & 15) == 0 && ((uintptr_t)I.dz2 & 15) == 0 && (I.zstride & 3) == 0;
    P.z2 = I.dz2 != nullptr;
    P.vb = (I.din & 3) == 0 && ((uintptr_t)I.y & 15) == 0 && (I.ystride & 3) == 0;
    P.vf = s.to == 64 && s.ti == 64 && (I.din & 3) == 0 && ((uintptr_t)I.gW & 15) == 0 && (I.gwstride & 3) == 0;
    P.first_unit = unit;
    P.first_tile = tile;
    P.slab_off = slab;
    const int64_t ntile = (int64_t)s.nto * s.nti * s.nb;
    unit += ntile * P.nch;
    tile += ntile;
    if (P.nch > 1) slab += ntile * P.nch * ((int64_t)s.to * s.ti + s.to);
  }
  for (int k = 0; k < WG_MAXITEMS; ++k) a.first[k] = k < m ? a.pl[k].first_unit : INT64_MAX;
  a.units = unit;
  p.tiles = tile;
  p.slab = slab;
  if (red) {
    DRPO_REQUIRE(red->part && red->mse && red->Z >= 1 && red->Z <= 256 && red->S1 >= 1 && red->S1 <= LOSS_MAXS1 &&
                     red->nbx >= 1,
                 "drpo_mlp_wgrad_reduce: bad reduction");
    a.has_red = 1;
    a.red = *red;
  }
  return DRPO_OK;
}

size_t ws_bytes(const Plan& p) { return (size_t)((p.tiles * 4 + 255) / 256 * 256) + sizeof(float) * (size_t)p.slab; }

}  // namespace

DRPO_API int drpo_mlp_wgrad_tiles(const drpo_wgrad_item_t* I) {
  if (!I || I->dout < 1 || I->din < 1 || I->nbatch < 1) return 0;
  const int to = I->dout <= 16 ? 16 : 64, ti = I->din <= 16 ? 16 : 64;
  return ((I->dout + to - 1) / to) * ((I->din + ti - 1) / ti) * I->nbatch;
}

DRPO_API size_t drpo_mlp_wgrad_workspace_size(const drpo_wgrad_item_t* items, int n) {
  if (n < 0 || n > WG_MAXITEMS || (n > 0 && !items)) return 0;
  Plan p;
  if (plan(items, n, nullptr, p) != DRPO_OK) return 0;
  return ws_bytes(p);
}

DRPO_API int drpo_mlp_wgrad(const drpo_wgrad_item_t* items, int n, void* workspace, size_t workspace_bytes,
                            drpo_stream_t stream) {
  return drpo_mlp_wgrad_reduce(items, n, nullptr, workspace, workspace_bytes, stream);
}

static int wgrad_launch(const drpo_wgrad_item_t* items, int n, const drpo_ens_reduce_t* red, const drpo_sum_t* sums,
                        int nsums, void* workspace, size_t workspace_bytes, hipStream_t stream,
                        const drpo_wgrad_adam_t* adam = nullptr);

DRPO_API int drpo_mlp_wgrad_adam(const drpo_wgrad_item_t* items, int n, const drpo_ens_reduce_t* red,
                                 const drpo_wgrad_adam_t* adam, void* workspace, size_t workspace_bytes,
                                 drpo_stream_t stream_) {
  DRPO_REQUIRE(adam && adam->g && adam->p && adam->m && adam->v && adam->bc2_sqrt > 0.f &&
                   (!adam->map == !adam->map_host),
               "drpo_mlp_wgrad_adam: bad Adam descriptor (g, p, m, v; map with its host copy)");
  for (int k = 0; k < n; ++k)
    DRPO_REQUIRE(!items[k].sq, "drpo_mlp_wgrad_adam: item %d asks for clip partials (no clip in the fused step)", k);
  return wgrad_launch(items, n, red, nullptr, 0, workspace, workspace_bytes, (hipStream_t)stream_, adam);
}

DRPO_API int drpo_mlp_wgrad_reduce(const drpo_wgrad_item_t* items, int n, const drpo_ens_reduce_t* red,
                                   void* workspace, size_t workspace_bytes, drpo_stream_t stream_) {
  return wgrad_launch(items, n, red, nullptr, 0, workspace, workspace_bytes, (hipStream_t)stream_);
}

DRPO_API int drpo_mlp_wgrad_sums(const drpo_wgrad_item_t* items, int n, const drpo_sum_t* sums, int nsums,
                                 void* workspace, size_t workspace_bytes, drpo_stream_t stream_) {
  DRPO_REQUIRE(nsums >= 0 && nsums <= WG_MAXSUMS && (nsums == 0 || sums), "drpo_mlp_wgrad_sums: 0..%d sums",
               WG_MAXSUMS);
  for (int q = 0; q < nsums; ++q)
    DRPO_REQUIRE(sums[q].n >= 0 && sums[q].out && (sums[q].n == 0 || sums[q].part), "drpo_mlp_wgrad_sums: sum %d", q);
  return wgrad_launch(items, n, nullptr, sums, nsums, workspace, workspace_bytes, (hipStream_t)stream_);
}

static int wgrad_launch(const drpo_wgrad_item_t* items, int n, const drpo_ens_reduce_t* red, const drpo_sum_t* sums,
                        int nsums, void* workspace, size_t workspace_bytes, hipStream_t stream,
                        const drpo_wgrad_adam_t* adam) {
  DRPO_REQUIRE(n >= 0 && n <= WG_MAXITEMS && (n == 0 || items), "drpo_mlp_wgrad: at most %d items", WG_MAXITEMS);
  static Plan p;   // host scratch (the library is driven by one host thread per process)
  const int rc = plan(items, n, red, p);
  if (rc != DRPO_OK) return rc;
  const size_t need = ws_bytes(p);
  DRPO_REQUIRE(workspace_bytes >= need && (need == 0 || workspace),
               "drpo_mlp_wgrad: workspace %zu bytes < %zu (drpo_mlp_wgrad_workspace_size)", workspace_bytes, need);
  p.a.ctr = (unsigned*)workspace;
  p.a.slab = (float*)((char*)workspace + (size_t)((p.tiles * 4 + 255) / 256 * 256));
  p.a.nsums = nsums;
  for (int q = 0; q < nsums; ++q) p.a.sums[q] = sums[q];
  p.a.has_adam = adam != nullptr;
  if (adam) {
    p.a.adam = *adam;
    // each item's matrix in the group's pack map (by its flat offset), for the mirrors
    const drpo_pack_map_t* mh = (const drpo_pack_map_t*)adam->map_host;
    for (int k = 0; k < p.a.n; ++k) {
      const drpo_wgrad_item_t& I = p.a.it[k];
      p.a.pl[k].pk_layer = -1;
      p.a.pl[k].pk_z0 = 0;
      if (!mh) continue;
      const int64_t off = I.gW - adam->g;
      // the item is members [z0, z0 + nbatch) of one [nbatch][dout][din] matrix of the map
      // (the whole matrix, or a member shard's contiguous slice of it)
      for (int l = 0; l < mh->nlayers && l < 16; ++l) {
        const int64_t per = (int64_t)mh->din[l] * mh->dout[l], rel = off - mh->off[l];
        if (mh->din[l] != I.din || mh->dout[l] != I.dout || rel < 0 || rel % per != 0) continue;
        const int64_t z0 = rel / per;
        if (z0 + I.nbatch > mh->nbatch[l] || (I.nbatch > 1 && I.gwstride != per)) continue;
        DRPO_REQUIRE(p.a.pl[k].pk_layer < 0, "drpo_mlp_wgrad_adam: item %d matches layers %d and %d of the pack map", k,
                     p.a.pl[k].pk_layer, l);
        p.a.pl[k].pk_layer = l;
        p.a.pl[k].pk_z0 = (int)z0;
      }
      DRPO_REQUIRE(p.a.pl[k].pk_layer >= 0, "drpo_mlp_wgrad_adam: item %d is not a matrix of the pack map", k);
    }
    // the float4 finish also reads / writes p, m, v at the gradient's flat offsets
    const bool al = ((uintptr_t)adam->p & 15) == 0 && ((uintptr_t)adam->m & 15) == 0 &&
                    ((uintptr_t)adam->v & 15) == 0 && ((uintptr_t)adam->g & 15) == 0 &&
                    (!mh || (((uintptr_t)mh->P & 15) == 0 && ((uintptr_t)mh->PT & 15) == 0));
    for (int k = 0; k < p.a.n; ++k) p.a.pl[k].vf = p.a.pl[k].vf && al && ((p.a.it[k].gW - adam->g) & 3) == 0;
  }
  const int64_t blocks = p.a.units + (red ? 1 : 0) + (nsums ? 1 : 0);
  if (blocks == 0) return DRPO_OK;
  mlp_wgrad_kernel<<<(unsigned)blocks, WG_NT, wgrad_lds(), stream>>>(p.a);
  DRPO_LAUNCH_CHECK("mlp_wgrad");
  return DRPO_OK;
}
