// Optimizer-side kernels over flat parameter groups (one launch covers a whole
// group or clip segment, HBM-bound):
//   drpo_grad_sumsq  : per-block partial sums of g^2 (first pass of clip_grad_norm_)
//   drpo_adam        : torch.optim.Adam (coupled L2 weight decay, single-tensor
//                      formulas) with the clip coefficient min(1, max/(||g||+1e-6))
//                      applied on the fly from the partial sums (deterministic:
//                      every block reduces the same partials in the same order)
//   drpo_ema         : target <- rate*p + (1-rate)*target (src/torch_util.py:223-226)
//   drpo_normalizer_fit : column mean / unbiased std over the replay states
//                      (src/normalization.py:14-19)
#include <algorithm>

#include "common.hpp"

using namespace drpo;

static constexpr int SUMSQ_BLOCK_ELEMS = 2048;

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, int64_t n, float* partial) {
  __shared__ float red[256];
  const int64_t base = (int64_t)blockIdx.x * SUMSQ_BLOCK_ELEMS;
  float s = 0.f;
  for (int64_t i = base + threadIdx.x; i < min(n, base + (int64_t)SUMSQ_BLOCK_ELEMS); i += 256) {
    const float v = g[i];
    s = fmaf(v, v, s);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

DRPO_API int drpo_grad_sumsq_blocks(int64_t n) { return (int)((n + SUMSQ_BLOCK_ELEMS - 1) / SUMSQ_BLOCK_ELEMS); }

DRPO_API int drpo_grad_sumsq(const float* g, int64_t n, float* partial, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(n >= 0, "drpo_grad_sumsq: n < 0");
  if (n == 0) return DRPO_OK;
  sumsq_kernel<<<drpo_grad_sumsq_blocks(n), 256, 0, stream>>>(g, n, partial);
  DRPO_LAUNCH_CHECK("grad_sumsq");
  return DRPO_OK;
}

struct AdamArgs {
  float* p;
  const float* g;
  float *m, *v;
  int64_t n;
  float lr_over_bc1;      // lr / (1 - beta1^t)
  float bc2_sqrt;         // sqrt(1 - beta2^t)
  float beta1, beta2, one_minus_beta1, one_minus_beta2, eps, wd;
  const float* partial;   // clip: partial sums of squares (nullptr = no clipping)
  int n_partial;
  float max_norm;
  const float* lr_scale;  // optional device scalar multiplying the step (nullptr = 1)
};

__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a) {
  __shared__ float s_coef;
  if (a.partial) {
    if (threadIdx.x < 64) {
      float s = 0.f;
      for (int i = threadIdx.x; i < a.n_partial; i += 64) s += a.partial[i];
      for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
      if (threadIdx.x == 0) {
        const float norm = sqrtf(s);
        const float c = a.max_norm / (norm + 1e-6f);
        s_coef = c < 1.f ? c : 1.f;
      }
    }
    __syncthreads();
  }
  const float coef = a.partial ? s_coef : 1.f;
  const float step = a.lr_over_bc1 * (a.lr_scale ? *a.lr_scale : 1.f);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (int64_t)gridDim.x * blockDim.x) {
    const float p = a.p[i];
    float g = a.g[i] * coef;
    if (a.wd != 0.f) g = fmaf(p, a.wd, g);
    const float m = torch_lerp(a.m[i], g, a.one_minus_beta1);
    const float v = fmaf(a.v[i], a.beta2, a.one_minus_beta2 * g * g);
    a.m[i] = m;
    a.v[i] = v;
    const float denom = sqrtf(v) / a.bc2_sqrt + a.eps;
    a.p[i] = p - step * (m / denom);
  }
}

DRPO_API int drpo_adam(float* p, const float* g, float* m, float* v, int64_t n, float lr_over_bc1, float bc2_sqrt,
                       float beta1, float beta2, float eps, float weight_decay, const float* clip_partial,
                       int n_partial, float max_norm, const float* lr_scale, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(n >= 0 && p && g && m && v, "drpo_adam: bad arguments");
  if (n == 0) return DRPO_OK;
  AdamArgs a{p, g, m, v, n, lr_over_bc1, bc2_sqrt, beta1, beta2, 1.f - beta1, 1.f - beta2, eps, weight_decay,
             clip_partial, n_partial, max_norm, lr_scale};
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  adam_kernel<<<blocks, 256, 0, stream>>>(a);
  DRPO_LAUNCH_CHECK("adam");
  return DRPO_OK;
}

__global__ void ema_kernel(float* t, const float* p, int64_t n, float rate, float keep) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    t[i] = rate * p[i] + keep * t[i];
}

DRPO_API int drpo_ema(float* target, const float* source, int64_t n, float rate, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(rate >= 0.f && rate <= 1.f, "drpo_ema: rate must be in [0,1]");
  if (n == 0) return DRPO_OK;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  // (1 - rate) is formed in double like the Python reference, then rounded once
  ema_kernel<<<blocks, 256, 0, stream>>>(target, source, n, rate, (float)(1.0 - (double)rate));
  DRPO_LAUNCH_CHECK("ema");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// Normalizer.fit: column mean and unbiased std over X [N][S] (double accumulation)
// ---------------------------------------------------------------------------
static constexpr int NORM_ROWS = 2048;

__global__ __launch_bounds__(256) void colstats_partial_kernel(const float* X, int64_t N, int S, double* part) {
  // block b: rows [b*NORM_ROWS, ...); thread t: column t % S, row lane t / S
  extern __shared__ double sh[];
  const int lanes = 256 / S;
  const int c = threadIdx.x % S, rl = threadIdx.x / S;
  double s = 0.0, q = 0.0;
  if (rl < lanes) {
    const int64_t r0 = (int64_t)blockIdx.x * NORM_ROWS;
    const int64_t r1 = min(N, r0 + NORM_ROWS);
    for (int64_t r = r0 + rl; r < r1; r += lanes) {
      const double x = X[r * S + c];
      s += x;
      q += x * x;
    }
  }
  sh[threadIdx.x] = (rl < lanes) ? s : 0.0;
  sh[256 + threadIdx.x] = (rl < lanes) ? q : 0.0;
  __syncthreads();
  if (threadIdx.x < S) {
    double ts = 0.0, tq = 0.0;
    for (int l = 0; l < lanes; ++l) {
      ts += sh[l * S + threadIdx.x];
      tq += sh[256 + l * S + threadIdx.x];
    }
    part[(int64_t)blockIdx.x * 2 * S + threadIdx.x] = ts;
    part[(int64_t)blockIdx.x * 2 * S + S + threadIdx.x] = tq;
  }
}

__global__ void colstats_final_kernel(const double* part, int nb, int64_t N, int S, float* mean, float* std) {
  const int c = threadIdx.x;
  if (c >= S) return;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < nb; ++b) {
    s += part[(int64_t)b * 2 * S + c];
    q += part[(int64_t)b * 2 * S + S + c];
  }
  const double mu = s / (double)N;
  double var = N > 1 ? (q - s * mu) / (double)(N - 1) : __longlong_as_double(0x7ff8000000000000LL);
  if (var < 0) var = 0;
  float sd = (float)sqrt(var);
  if (!(sd >= 1e-6f)) sd = (sd < 1e-6f) ? 1.0f : sd;   // std[std < 1e-6] = 1.0 (NaN stays NaN)
  mean[c] = (float)mu;
  std[c] = sd;
}

DRPO_API size_t drpo_normalizer_workspace_size(int64_t N, int S) {
  return sizeof(double) * 2 * (size_t)S * (size_t)((N + NORM_ROWS - 1) / NORM_ROWS);
}

DRPO_API int drpo_normalizer_fit(const float* X, int64_t N, int S, float* mean, float* std, void* workspace,
                                 drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(N >= 1 && S >= 1 && S <= 256, "drpo_normalizer_fit: N=%lld S=%d", (long long)N, S);
  const int nb = (int)((N + NORM_ROWS - 1) / NORM_ROWS);
  colstats_partial_kernel<<<nb, 256, 2 * 256 * sizeof(double), stream>>>(X, N, S, (double*)workspace);
  DRPO_LAUNCH_CHECK("normalizer_partial");
  colstats_final_kernel<<<1, 256, 0, stream>>>((const double*)workspace, nb, N, S, mean, std);
  DRPO_LAUNCH_CHECK("normalizer_final");
  return DRPO_OK;
}

__global__ void normalize_kernel(const float* x, const float* mean, const float* std, float eps, float* y,
                                 int64_t n, int S) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n * S; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % S);
    y[i] = (x[i] - mean[c]) / (std[c] + eps);
  }
}

DRPO_API int drpo_normalize(const float* x, const float* mean, const float* std, float eps, float* y, int64_t n,
                            int S, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (n == 0) return DRPO_OK;
  int64_t blocks = (n * S + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  normalize_kernel<<<(unsigned)blocks, 256, 0, stream>>>(x, mean, std, eps, y, n, S);
  DRPO_LAUNCH_CHECK("normalize");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// Fused optimizer step over segments of flat groups (one launch per SAC update
// phase): clip coefficient from precomputed partial sums, Adam, gradient zeroing
// for the next backward, EMA of a target group, and the refresh of the packed
// weight mirrors the MLP kernels stream (so no separate zero / EMA / pack
// launches). Elements are processed independently; segments never overlap.
// ---------------------------------------------------------------------------
namespace {
constexpr int OPT_MAXSEG = 8;
constexpr int OPT_MAXTASK = 32;
constexpr int OPT_BLOCK_ELEMS = 1024;   // flat task: elements per workgroup (256 threads x 4)
constexpr int OPT_BLOCKS4 = 64;         // matrix task: 4x4 blocks per workgroup (one per lane quad)
}

// A launch is a list of tasks, each a run of workgroups over one segment:
//  * flat: elements [a, b), 4 consecutive per thread (biases, scalars, anything
//    outside a weight matrix, and matrices of segments without a host map);
//  * matrix: whole members [z0, z0 + nz) of one [nbatch][dout][din] weight matrix,
//    one 4x4 block (4 rows x 4 columns) per lane quad. Every access is then a 16-byte
//    row segment: the flat group's p / g / m / v / EMA target rows, the forward
//    mirror (a fragment lane holds 4 consecutive columns of one row) and the
//    transposed mirror (a fragment lane holds 4 consecutive rows of one column) --
//    where the flat form issued 4 scattered 4-byte transposed-mirror stores per
//    thread (round 3 probe: 13.8 us -> 7.6 us per fit step without the mirror stores).
struct OptTask {
  int64_t a, b;                         // flat: element range; matrix: flat offset of member 0, blocks
  int seg, kind;                        // kind 0 flat, 1 matrix (din % 4 == 0), 2 matrix (scalar rows)
  int layer, din, dout, z0;             // matrix: its entry in the segment's (device) pack map
  int map_needed;                       // flat: the range overlaps a weight matrix
};

struct OptimArgs {
  int64_t first[OPT_MAXTASK];           // first workgroup of each task (unused slots: INT64_MAX)
  OptTask task[OPT_MAXTASK];
  drpo_optim_seg_t seg[OPT_MAXSEG];
  int ntask;
};
static_assert(sizeof(OptimArgs) <= 4096, "optimizer kernarg");

// Packed-mirror refresh for the n (<= 4) consecutive flat elements i0.. of one thread.
// The weight matrix holding i0 is found once; the (member, row, column) coordinates
// are divided out once and then stepped (consecutive elements are consecutive
// columns), so the per-element cost is a few integer adds instead of two 32-bit
// divisions and a layer search. (Flat tasks only: segments without a host map, or
// partial members of a matrix.)
__device__ __forceinline__ void pack_write4(const drpo_pack_map_t* mp, int64_t i0, int n, const float (&pv)[4],
                                            const float (&tv)[4], bool has_t) {
  const int nl = mp->nlayers;
  int l = 0;
  int64_t rel64 = 0;
  for (; l < nl; ++l) {
    rel64 = i0 - mp->off[l];
    if (rel64 >= 0 && rel64 < (int64_t)mp->din[l] * mp->dout[l] * mp->nbatch[l]) break;
  }
  if (l == nl) return;
  const int din = mp->din[l], dout = mp->dout[l], nb = mp->nbatch[l];
  const int msz = din * dout;                         // group tensors are < 2^31 floats
  const int rel = (int)rel64;
  int z = rel / msz;
  const int w = rel - z * msz;
  int o = w / din, k = w - o * din;
  const int ncb = (dout + 15) >> 4, nks = (din + 15) >> 4;
  float* P = mp->P;
  float* Pt = has_t ? mp->Pt : nullptr;
  float* PT = mp->PT;
  for (int e = 0; e < n; ++e) {
    const int64_t base = mp->poff[l] + (int64_t)z * ncb * nks * 256;
    // forward mirror: fragment (o>>4, k>>4), lane ((k>>2)&3)*16 + (o&15), component k&3
    const int64_t pi = base + ((int64_t)((o >> 4) * nks + (k >> 4)) << 8) + ((((k >> 2) & 3) * 16 + (o & 15)) << 2) + (k & 3);
    if (P) P[pi] = pv[e];
    if (Pt) Pt[pi] = tv[e];
    if (PT) {   // transposed mirror: fragment (k>>4, o>>4), lane ((o>>2)&3)*16 + (k&15), component o&3
      const int64_t ti = base + ((int64_t)((k >> 4) * ncb + (o >> 4)) << 8) + ((((o >> 2) & 3) * 16 + (k & 15)) << 2) + (o & 3);
      PT[ti] = pv[e];
    }
    if (++k == din) {
      k = 0;
      if (++o == dout) {
        o = 0;
        if (++z == nb) return;
      }
    }
  }
}

// per-element update shared by both task kinds: g (already scaled) -> Adam on p, m, v
__device__ __forceinline__ void adam_elem(const drpo_optim_seg_t& S, float coef, float g, float& p, float& m,
                                          float& v) {
  adam_step(S, coef, g, p, m, v);
}

// EMA of one target element (one explicit fma: both task kinds round alike)
__device__ __forceinline__ float ema_elem(const drpo_optim_seg_t& S, float p, float t) {
  return fmaf(S.ema_rate, p, S.ema_keep * t);
}

// x[i] for a per-lane i, by bit masks (a select chain is turned back into an indexed
// private array, i.e. scratch memory)
__device__ __forceinline__ float pick4(const float (&x)[4], int i) {
  unsigned r = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) r |= __float_as_uint(x[k]) & (0u - (unsigned)(i == k));
  return __uint_as_float(r);
}

// One 4x4 block of a weight matrix per 4 adjacent lanes: lane rr = tid & 3 owns row
// o0 + rr, columns k0..k0+3 (masked past dout / din; VEC: din % 4 == 0, so the row
// segment is one 16-byte access). After the update a 4x4 transpose inside the lane
// quad (3 xor shuffles) hands lane rr column k0 + rr of rows o0..o0+3: the transposed
// mirror's 16-byte fragment component group.
template <bool VEC>
__device__ __forceinline__ void opt_matrix_block(const drpo_optim_seg_t& S, const OptTask& T, int64_t blk, int rr,
                                                 bool live, float coef, float gscale) {
  const int din = T.din, dout = T.dout;
  const int nkb = (din + 3) >> 2, nob = (dout + 3) >> 2;
  const int per = nkb * nob;
  const int64_t zb = blk / per;
  const int z = T.z0 + (int)zb;
  const int r = (int)(blk - zb * per);
  const int ob = r / nkb, kb = r - ob * nkb;
  const int o0 = 4 * ob, k0 = 4 * kb;
  const int o = o0 + rr;
  const bool row = live && o < dout;
  const int64_t i = T.a + (int64_t)z * din * dout + (int64_t)o * din + k0;
  float p[4] = {0.f, 0.f, 0.f, 0.f}, g[4] = {0.f, 0.f, 0.f, 0.f}, m[4] = {0.f, 0.f, 0.f, 0.f};
  float v[4] = {0.f, 0.f, 0.f, 0.f}, t[4] = {0.f, 0.f, 0.f, 0.f};
  const bool has_t = S.ema_target != nullptr;
  auto ld = [&](const float* src, float (&dst)[4]) {
    if (!row) return;
    if constexpr (VEC) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(src + i);
      dst[0] = x[0]; dst[1] = x[1]; dst[2] = x[2]; dst[3] = x[3];
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) dst[c] = k0 + c < din ? src[i + c] : 0.f;
    }
  };
  auto st = [&](float* dst, const float (&src)[4]) {
    if (!row) return;
    if constexpr (VEC) {
      *reinterpret_cast<f32x4*>(dst + i) = f32x4{src[0], src[1], src[2], src[3]};
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (k0 + c < din) dst[i + c] = src[c];
    }
  };
  ld(S.p, p);
  if (S.adam) {
    ld(S.g, g);
    ld(S.m, m);
    ld(S.v, v);
  }
  if (has_t) ld(S.ema_target, t);
  if (S.adam) {
#pragma unroll
    for (int c = 0; c < 4; ++c) adam_elem(S, coef, g[c] * gscale, p[c], m[c], v[c]);
    st(S.m, m);
    st(S.v, v);
    st(S.p, p);
  }
  if (S.zero_grad) {
    const float zz[4] = {0.f, 0.f, 0.f, 0.f};
    st(S.g, zz);
  }
  if (has_t) {
#pragma unroll
    for (int c = 0; c < 4; ++c) t[c] = ema_elem(S, p[c], t[c]);
    st(S.ema_target, t);
  }
  // mirrors (device map, scalar loads). Masked elements are 0, the mirrors' padding value.
  const drpo_pack_map_t* md = S.map;
  const int ncb = (dout + 15) >> 4, nks = (din + 15) >> 4;
  const int64_t mb = md->poff[T.layer] + (int64_t)z * ncb * nks * 256;
  float* P = md->P;
  float* PT = md->PT;
  float* Pt = has_t ? md->Pt : nullptr;
  // forward mirror: row o's columns k0..k0+3 are the 4 components of fragment
  // (o>>4, k0>>4), lane ((k0>>2)&3)*16 + (o&15)
  if (row) {
    const int64_t pi = mb + ((int64_t)((o >> 4) * nks + (k0 >> 4)) << 8) + ((((k0 >> 2) & 3) * 16 + (o & 15)) << 2);
    if (P) *reinterpret_cast<f32x4*>(P + pi) = f32x4{p[0], p[1], p[2], p[3]};
    if (Pt) *reinterpret_cast<f32x4*>(Pt + pi) = f32x4{t[0], t[1], t[2], t[3]};
  }
  if (PT) {
    // quad transpose: q[j] = row o0 + j, column k0 + rr
    float q[4];
    q[0] = q[1] = q[2] = q[3] = 0.f;
#pragma unroll
    for (int x = 0; x < 4; ++x) {
      const float sent = pick4(p, rr ^ x);
      const float got = x == 0 ? sent : __shfl_xor(sent, x, 64);
      const unsigned gb = __float_as_uint(got), j = (unsigned)(rr ^ x);
#pragma unroll
      for (int c = 0; c < 4; ++c)   // q[j] = got (masks: see pick4)
        q[c] = __uint_as_float(__float_as_uint(q[c]) | (gb & (0u - (unsigned)(j == (unsigned)c))));
    }
    // transposed mirror: column k's rows o0..o0+3 are the 4 components of fragment
    // (k>>4, o0>>4), lane ((o0>>2)&3)*16 + (k&15)
    const int k = k0 + rr;
    if (live && k < din) {
      const int64_t ti = mb + ((int64_t)((k >> 4) * ncb + (o0 >> 4)) << 8) + ((((o0 >> 2) & 3) * 16 + (k & 15)) << 2);
      *reinterpret_cast<f32x4*>(PT + ti) = f32x4{q[0], q[1], q[2], q[3]};
    }
  }
}

__global__ __launch_bounds__(256) void optim_step_kernel(OptimArgs a) {
  __shared__ float s_coef, s_gsum;
  // the segment's pack map (flat tasks overlapping a matrix), staged once per workgroup:
  // the per-thread layer search of pack_write4 then reads LDS instead of a chain of
  // dependent global loads
  __shared__ __attribute__((aligned(16))) int s_map[(sizeof(drpo_pack_map_t) + 3) / 4];
  const int64_t bid = blockIdx.x;
  // the task: the number of prefixes <= bid. All prefixes are read at once (independent
  // scalar loads, one kernarg round trip) instead of a chain of dependent ones.
  int lo = -1;
#pragma unroll
  for (int i = 0; i < OPT_MAXTASK; ++i) lo += bid >= a.first[i] ? 1 : 0;
  const OptTask& T = a.task[lo];
  const drpo_optim_seg_t& S = a.seg[T.seg];
  const int64_t lb = bid - a.first[lo];
  const bool matrix = T.kind != 0;
  // Flat: each thread owns 4 consecutive elements, whose loads are issued FIRST, so
  // they are in flight together with the pack-map staging and the clip partial sums
  // (one memory latency per workgroup instead of three in a row).
  const int64_t e0 = T.a + lb * OPT_BLOCK_ELEMS;
  const int64_t e1 = min(T.b, e0 + OPT_BLOCK_ELEMS);
  const int64_t i0 = e0 + 4 * (int64_t)threadIdx.x;
  const bool live = !matrix && i0 < e1;
  const int n = live ? (int)min((int64_t)4, e1 - i0) : 0;
  const bool vec = n == 4 && (i0 & 3) == 0;
  float p[4] = {0.f, 0.f, 0.f, 0.f}, g[4] = {0.f, 0.f, 0.f, 0.f}, m[4] = {0.f, 0.f, 0.f, 0.f};
  float v[4] = {0.f, 0.f, 0.f, 0.f}, t[4] = {0.f, 0.f, 0.f, 0.f};
  auto ld4 = [&](const float* src, float (&dst)[4]) {
    if (vec) {
      const f32x4 x = *reinterpret_cast<const f32x4*>(src + i0);
      dst[0] = x[0]; dst[1] = x[1]; dst[2] = x[2]; dst[3] = x[3];
    } else {
      for (int e = 0; e < n; ++e) dst[e] = src[i0 + e];
    }
  };
  auto st4 = [&](float* dst, const float (&src)[4]) {
    if (vec) {
      *reinterpret_cast<f32x4*>(dst + i0) = f32x4{src[0], src[1], src[2], src[3]};
    } else {
      for (int e = 0; e < n; ++e) dst[i0 + e] = src[e];
    }
  };
  if (live) {
    ld4(S.p, p);
    if (S.adam) {
      ld4(S.g, g);
      ld4(S.m, m);
      ld4(S.v, v);
    }
    if (S.ema_target) ld4(S.ema_target, t);
  }
  const bool stage_map = !matrix && S.map && T.map_needed;
  if (stage_map) {
    const int* src = reinterpret_cast<const int*>(S.map);
    for (int i = threadIdx.x; i < (int)(sizeof(drpo_pack_map_t) / 4); i += 256) s_map[i] = src[i];
  }
  // data-parallel mean folded into the step: the partial sums are of the SUMMED
  // gradient, so the clip norm is sqrt(sum) * scale (exact for power-of-2 ranks)
  const float gscale = S.grad_scale != 0.f ? S.grad_scale : 1.f;
  if (S.partial && threadIdx.x < 64) {
    float s = 0.f;
    for (int i = threadIdx.x; i < S.n_partial; i += 64) s += S.partial[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (threadIdx.x == 0) {
      const float c = S.max_norm / (sqrtf(s) * gscale + 1e-6f);
      s_coef = c < 1.f ? c : 1.f;
    }
  }
  // a scalar's gradient from device loss partials: the first wave adds them (lane-strided,
  // then a fixed shuffle tree: deterministic), instead of one thread walking the list
  if (S.grad_from_sum && threadIdx.x < 64) {
    const int ns = S.grad_sum_n > 1 ? S.grad_sum_n : 1;
    float s = 0.f;
    for (int i = threadIdx.x; i < ns; i += 64) s += S.grad_from_sum[i];
    for (int o = 32; o > 0; o >>= 1) s += __shfl_down(s, o, 64);
    if (threadIdx.x == 0) s_gsum = s;
  }
  if (stage_map || S.partial || S.grad_from_sum) __syncthreads();
  const float coef = S.partial ? s_coef : 1.f;
  if (matrix) {
    // every lane of a quad takes part in the transpose: out-of-range quads run masked
    const int64_t blk = lb * OPT_BLOCKS4 + (threadIdx.x >> 2);
    const bool in = blk < T.b;
    const int64_t b = in ? blk : T.b - 1;
    if (T.kind == 1) opt_matrix_block<true>(S, T, b, threadIdx.x & 3, in, coef, gscale);
    else opt_matrix_block<false>(S, T, b, threadIdx.x & 3, in, coef, gscale);
    return;
  }
  if (!live) return;
  if (S.grad_from_sum) {   // a scalar's gradient from a device loss sum (see drpo_optim_seg_t)
    const float gs = s_gsum * (1.f / (float)S.grad_sum_rows);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float c = S.grad_from_sum_kind == 1 ? 1.f / (1.f + expf(-p[e])) : (S.grad_from_sum_kind == 2 ? 1.f : expf(p[e]));
      g[e] = -c * gs;
    }
  } else if (gscale != 1.f) {
#pragma unroll
    for (int e = 0; e < 4; ++e) g[e] *= gscale;
  }
  if (S.adam) {
#pragma unroll
    for (int e = 0; e < 4; ++e) adam_elem(S, coef, g[e], p[e], m[e], v[e]);
    st4(S.m, m);
    st4(S.v, v);
    st4(S.p, p);
  }
  if (S.zero_grad) {
    const float zz[4] = {0.f, 0.f, 0.f, 0.f};
    st4(S.g, zz);
  }
  if (S.ema_target) {
#pragma unroll
    for (int e = 0; e < 4; ++e) t[e] = ema_elem(S, p[e], t[e]);
    st4(S.ema_target, t);
  }
  if (stage_map) {
    const drpo_pack_map_t* map = reinterpret_cast<const drpo_pack_map_t*>(s_map);
    pack_write4(map, i0, n, p, t, S.ema_target != nullptr);
  }
}

namespace {
// task list of one segment: each whole-member run of a weight matrix (from the host
// map) as a matrix task, the ranges between them as flat tasks
int plan_segment(const drpo_optim_seg_t& S, int k, OptimArgs& a, int64_t& tot) {
  auto flat = [&](int64_t x, int64_t y, int needed) {
    if (y <= x) return DRPO_OK;
    DRPO_REQUIRE(a.ntask < OPT_MAXTASK, "drpo_optim_step: more than %d tasks", OPT_MAXTASK);
    OptTask& T = a.task[a.ntask++];
    T = OptTask{};
    a.first[a.ntask - 1] = tot;
    T.a = x; T.b = y; T.seg = k; T.kind = 0; T.map_needed = needed;
    tot += (y - x + OPT_BLOCK_ELEMS - 1) / OPT_BLOCK_ELEMS;
    return DRPO_OK;
  };
  const drpo_pack_map_t* mh = S.map ? S.map_host : nullptr;
  if (!mh) return flat(S.start, S.end, S.map != nullptr);
  // matrices in flat order
  int order[16], nl = mh->nlayers < 16 ? mh->nlayers : 16;
  for (int l = 0; l < nl; ++l) order[l] = l;
  for (int i = 1; i < nl; ++i)
    for (int j = i; j > 0 && mh->off[order[j]] < mh->off[order[j - 1]]; --j) std::swap(order[j], order[j - 1]);
  int64_t cur = S.start;
  for (int q = 0; q < nl; ++q) {
    const int l = order[q];
    const int64_t msz = (int64_t)mh->din[l] * mh->dout[l];
    const int64_t off = mh->off[l], endm = off + msz * mh->nbatch[l];
    const int64_t x = std::max(off, S.start), y = std::min(endm, S.end);
    if (y <= x || msz == 0) continue;
    const int64_t za = (x - off + msz - 1) / msz, zb = (y - off) / msz;   // whole members inside
    if (za >= zb || a.ntask + 2 > OPT_MAXTASK - 1) continue;   // partial only / list full: flat
    int rc = flat(cur, off + za * msz, 1);
    if (rc != DRPO_OK) return rc;
    OptTask& T = a.task[a.ntask++];
    T = OptTask{};
    a.first[a.ntask - 1] = tot;
    T.seg = k; T.kind = (mh->din[l] & 3) == 0 ? 1 : 2;
    T.a = off; T.layer = l; T.din = mh->din[l]; T.dout = mh->dout[l]; T.z0 = (int)za;
    T.b = (zb - za) * (int64_t)((mh->din[l] + 3) / 4) * ((mh->dout[l] + 3) / 4);   // 4x4 blocks
    tot += (T.b + OPT_BLOCKS4 - 1) / OPT_BLOCKS4;
    cur = off + zb * msz;
  }
  return flat(cur, S.end, 1);
}
}  // namespace

DRPO_API int drpo_optim_step(const drpo_optim_seg_t* segs, int n, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(n >= 0 && n <= OPT_MAXSEG, "drpo_optim_step: at most %d segments", OPT_MAXSEG);
  static OptimArgs a;   // host scratch (the library is driven by one host thread per process)
  a = OptimArgs{};
  for (int i = 0; i < OPT_MAXTASK; ++i) a.first[i] = INT64_MAX;
  int64_t tot = 0;
  for (int k = 0; k < n; ++k) {
    const drpo_optim_seg_t& S = segs[k];
    DRPO_REQUIRE(S.p && S.end >= S.start && (!S.adam || (S.g && S.m && S.v)), "drpo_optim_step: bad segment %d", k);
    DRPO_REQUIRE(!S.grad_from_sum || S.grad_sum_rows >= 1, "drpo_optim_step: segment %d: grad_sum_rows", k);
    a.seg[k] = S;
    if (S.end == S.start) continue;
    const int rc = plan_segment(S, k, a, tot);
    if (rc != DRPO_OK) return rc;
  }
  if (tot == 0) return DRPO_OK;
  optim_step_kernel<<<(unsigned)tot, 256, 0, stream>>>(a);
  DRPO_LAUNCH_CHECK("optim_step");
  return DRPO_OK;
}

// partial sums of squares for several clip segments in one launch:
// segment k writes drpo_grad_sumsq_blocks(end-start) partials at out[k]
namespace {
constexpr int SQ_MAXSEG = 8;
}
struct SumsqArgs {
  const float* g[SQ_MAXSEG];
  int64_t n[SQ_MAXSEG];
  float* out[SQ_MAXSEG];
  int64_t first[SQ_MAXSEG + 1];
  int cnt;
};

__global__ __launch_bounds__(256) void sumsq_multi_kernel(SumsqArgs a) {
  __shared__ float red[256];
  const int64_t bid = blockIdx.x;
  int q = 0;
  while (q + 1 < a.cnt && bid >= a.first[q + 1]) ++q;
  const int64_t lb = bid - a.first[q];
  const int64_t base = lb * SUMSQ_BLOCK_ELEMS;
  const float* g = a.g[q];
  float s = 0.f;
  for (int64_t i = base + threadIdx.x; i < min(a.n[q], base + (int64_t)SUMSQ_BLOCK_ELEMS); i += 256) {
    const float v = g[i];
    s = fmaf(v, v, s);
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) a.out[q][lb] = red[0];
}

DRPO_API int drpo_grad_sumsq_multi(const float* const* g, const int64_t* n, float* const* out, int cnt,
                                   drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(cnt >= 0 && cnt <= SQ_MAXSEG, "drpo_grad_sumsq_multi: at most %d segments", SQ_MAXSEG);
  SumsqArgs a{};
  int64_t tot = 0;
  for (int k = 0; k < cnt; ++k) {
    a.g[k] = g[k];
    a.n[k] = n[k];
    a.out[k] = out[k];
    a.first[k] = tot;
    tot += drpo_grad_sumsq_blocks(n[k]);
  }
  a.first[cnt] = tot;
  a.cnt = cnt;
  if (tot == 0) return DRPO_OK;
  sumsq_multi_kernel<<<(unsigned)tot, 256, 0, stream>>>(a);
  DRPO_LAUNCH_CHECK("grad_sumsq_multi");
  return DRPO_OK;
}
