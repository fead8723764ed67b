// Row-wise kernels around the fused ensemble MLP (mlp.hip) for the dynamics
// ensemble API and its fit (src/dynamics.py:112-253):
//
//  drpo_ens_gather  fit / holdout minibatch: chronological replay indices (recorded
//                   or Philox) -> raw states, actions and targets [s', r]
//                   (src/dynamics.py:156-166,175-177; SampleBuffer.get order,
//                   src/sampling.py:87-92)
//  drpo_ens_head    Gaussian head: mu = diff + [s, 0], the soft log-var clamp, and
//                   optionally a sample mu + sqrt(exp(lv)) * eps split into (s', r)
//                   (src/dynamics.py:112-134,198-234)
//  drpo_ens_loss    heteroscedastic NLL per member + log-var bound term, and its
//                   gradients w.r.t. the head outputs and min/max_log_var
//                   (src/dynamics.py:143-153,236-253)
// All are HBM/latency-bound epilogues; the GEMM work is in mlp.hip.
#include "common.hpp"
#include "ens_reduce.hpp"

using namespace drpo;

namespace {

// torch softplus backward: x > 20 ? 1 : e^x / (e^x + 1)
__device__ __forceinline__ float sp_grad(float x) {
  if (x > 20.f) return 1.f;
  const float z = expf(x);
  return z / (z + 1.f);
}

__device__ __forceinline__ float lv_clamp(float raw, float lo, float hi) {
  const float l1 = hi - softplusf(hi - raw);
  return lo + softplusf(l1 - lo);
}

__device__ __forceinline__ int64_t chrono_to_phys(int64_t j, int64_t ptr, int64_t cap) {
  // SampleBuffer._get1: when wrapped, chronological order starts at ptr % cap
  return ptr > cap ? (ptr % cap + j) % cap : j;
}

}  // namespace

// ---------------------------------------------------------------------------
// gather
// ---------------------------------------------------------------------------
// One thread per gathered ELEMENT (row x [s | a | s' | r] column): the replay rows
// are random, so the copy is latency-bound; spreading it over rows * (2S+A+1)
// threads (instead of one thread per row walking its 2S+A+1 columns) keeps the whole
// chip's memory pipes busy. Each thread derives its row's index itself (recorded,
// or the row's Philox draw -- the same value for every column of the row).
// steps > 1: the minibatches of `steps` consecutive fit steps in ONE launch (step k:
// rows [k*rows, (k+1)*rows) of every output, indices idx[k*rows ..] or Philox counter
// ctr + k), so the fit loop pays one latency-bound gather per chunk of steps instead
// of one per step (the replay is not written during a fit).
__global__ void ens_gather_kernel(const float* __restrict__ bs, const float* __restrict__ ba,
                                  const float* __restrict__ bs2, const float* __restrict__ br, int64_t ptr,
                                  const int64_t* ptr_dev, int64_t cap, int64_t rows, int64_t steps,
                                  const int64_t* idx, uint64_t seed, uint64_t ctr, int S, int A,
                                  float* __restrict__ xs, float* __restrict__ xa, float* __restrict__ xt) {
  const int W = 2 * S + A + 1;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= steps * rows * W) return;
  const int64_t gi = e / W;                  // row over all steps
  const int c = (int)(e - gi * W);
  const int64_t st = gi / rows, i = gi - st * rows;
  const int64_t p = ptr_dev ? *ptr_dev : ptr;
  const int64_t n = p < cap ? p : cap;
  int64_t j;
  if (idx) {
    j = idx[gi];
  } else {
    const uint64_t cs = ctr + (uint64_t)st;
    const u32x4 r = philox({(uint32_t)i, (uint32_t)(i >> 32), 0xe5e3b1u, (uint32_t)cs}, (uint32_t)seed,
                           (uint32_t)(seed >> 32));
    j = (int64_t)((((uint64_t)r.y << 32) | r.x) % (uint64_t)n);
  }
  const int64_t q = chrono_to_phys(j, p, cap);
  if (c < S) {
    xs[gi * S + c] = bs[q * S + c];
  } else if (c < S + A) {
    xa[gi * A + (c - S)] = ba[q * A + (c - S)];
  } else if (c < 2 * S + A) {
    xt[gi * (S + 1) + (c - S - A)] = bs2[q * S + (c - S - A)];
  } else {
    xt[gi * (S + 1) + S] = br[q];
  }
}

DRPO_API int drpo_ens_gather_steps(const float* states, const float* actions, const float* next_states,
                                   const float* rewards, int64_t ptr, const int64_t* ptr_dev, int64_t cap,
                                   int64_t rows, int64_t steps, const int64_t* idx, uint64_t seed, uint64_t ctr,
                                   int S, int A, float* xs, float* xa, float* xt, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(states && actions && next_states && rewards && cap >= 1 && rows >= 0 && steps >= 0 && S >= 1 &&
                   A >= 1,
               "drpo_ens_gather: bad arguments");
  DRPO_REQUIRE(ptr_dev || ptr >= 1, "drpo_ens_gather: empty buffer");
  const int64_t elems = steps * rows * (2 * S + A + 1);
  if (elems == 0) return DRPO_OK;
  DRPO_REQUIRE((elems + 255) / 256 <= 0x7fffffff, "drpo_ens_gather: %lld elements", (long long)elems);
  ens_gather_kernel<<<(unsigned)((elems + 255) / 256), 256, 0, stream>>>(states, actions, next_states, rewards, ptr,
                                                                         ptr_dev, cap, rows, steps, idx, seed, ctr,
                                                                         S, A, xs, xa, xt);
  DRPO_LAUNCH_CHECK("ens_gather");
  return DRPO_OK;
}

DRPO_API int drpo_ens_gather(const float* states, const float* actions, const float* next_states,
                             const float* rewards, int64_t ptr, const int64_t* ptr_dev, int64_t cap, int64_t rows,
                             const int64_t* idx, uint64_t seed, uint64_t ctr, int S, int A, float* xs, float* xa,
                             float* xt, drpo_stream_t stream) {
  return drpo_ens_gather_steps(states, actions, next_states, rewards, ptr, ptr_dev, cap, rows, 1, idx, seed, ctr, S,
                               A, xs, xa, xt, stream);
}

// ---------------------------------------------------------------------------
// Gaussian head (forward)
// ---------------------------------------------------------------------------
// D, LV: [Z][n][S1] head outputs (member-major); s: raw states [*][n][S] with
// member stride s_zstride (0 when every member sees the same rows). zsel: optional
// output-member -> input-member map (elite_samples). Outputs [Zo][n][*].
__global__ void ens_head_kernel(const float* D, const float* LVR, const float* s, int64_t s_zstride, int64_t n,
                                int S, const float* minlv, const float* maxlv, const int* zsel, const float* eps,
                                uint64_t seed, uint64_t ctr, float* mu, float* lv, float* s2, float* r) {
  const int S1 = S + 1;
  const int zo = blockIdx.y;
  const int zi = zsel ? zsel[zo] : zo;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n * S1) return;
  const int64_t row = e / S1;
  const int k = (int)(e - row * S1);
  const int64_t src = (int64_t)zi * n * S1 + e;
  const float m = D[src] + (k < S ? s[(int64_t)zi * s_zstride + row * S + k] : 0.f);
  const float l = lv_clamp(LVR[src], minlv[k], maxlv[k]);
  const int64_t dst = (int64_t)zo * n * S1 + e;
  if (mu) mu[dst] = m;
  if (lv) lv[dst] = l;
  if (s2 || r) {
    float z;
    if (eps) {
      z = eps[dst];
    } else {
      float zz[4];
      philox_normal4(seed, (uint32_t)(dst >> 2), (uint32_t)(dst >> 34), 0xe5a1u, (uint32_t)ctr, zz);
      z = zz[dst & 3];
    }
    const float x = m + sqrtf(expf(l)) * z;
    if (k < S) {
      if (s2) s2[((int64_t)zo * n + row) * S + k] = x;
    } else if (r) {
      r[(int64_t)zo * n + row] = x;
    }
  }
}

DRPO_API int drpo_ens_head(const float* D, const float* LVR, const float* s, int64_t s_zstride, int64_t n, int S,
                           int nz_out, const float* minlv, const float* maxlv, const int* zsel, const float* eps,
                           uint64_t seed, uint64_t ctr, float* mu, float* lv, float* s2, float* r,
                           drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(D && LVR && s && minlv && maxlv && n >= 0 && S >= 1 && nz_out >= 1, "drpo_ens_head: bad arguments");
  if (n == 0) return DRPO_OK;
  dim3 grid((unsigned)((n * (S + 1) + 255) / 256), nz_out);
  ens_head_kernel<<<grid, 256, 0, stream>>>(D, LVR, s, s_zstride, n, S, minlv, maxlv, zsel, eps, seed, ctr, mu, lv, s2,
                                            r);
  DRPO_LAUNCH_CHECK("ens_head");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// NLL loss + gradients
// ---------------------------------------------------------------------------
// grid (row blocks of 256 / KP rows, member). Thread t owns column k = t % KP of row
// r0 + t / KP (KP = S1 rounded up to a power of two >= 16): one row per thread, so a
// block waits one memory latency (64-row blocks looped 4 times: 9.2 us per launch at
// E=7, b=256; the per-column log-var-bound partials are reduced through LDS). Each
// block leaves its partial sums in the workspace and ens_loss_reduce_kernel (one
// block) sums them in a fixed order into the per-member NLL, the total loss and the
// bound gradients: deterministic, no memset, and no in-kernel cross-workgroup hand-
// off (a device-scope fence writes back the whole XCD L2 on gfx950: measured 22 us
// for a last-block variant of this kernel).

__global__ __launch_bounds__(256) void ens_loss_kernel(const float* __restrict__ D, const float* __restrict__ LVR,
                                                       const float* __restrict__ s, int64_t s_zstride,
                                                       const float* __restrict__ t, int64_t t_zstride, int64_t b,
                                                       int S, int Z, int KP, const float* __restrict__ minlv,
                                                       const float* __restrict__ maxlv, const float* gscale,
                                                       float* gD, float* gLVR, float* __restrict__ part) {
  __shared__ float red[4];
  __shared__ float rmin[256], rmax[256];
  const int S1 = S + 1;
  const int nbx = gridDim.x;
  const int z = blockIdx.y, bx = blockIdx.x;
  const int tid = threadIdx.x;
  const bool grads = gD != nullptr;
  const int k = tid % KP, rl = tid / KP, RP = 256 / KP;
  const float inv_n = 1.f / (float)(b * S1);
  const float g = grads ? (gscale ? *gscale : 1.f) * inv_n : 0.f;
  const int64_t r0 = (int64_t)bx * RP;     // one row per thread (launcher: 256 / KP rows)
  const int64_t r1 = min(b, r0 + RP);
  float acc = 0.f, cmin = 0.f, cmax = 0.f;
  if (k < S1) {
    const float hi = maxlv[k], lo = minlv[k];
    for (int64_t row = r0 + rl; row < r1; row += RP) {
      const int64_t o = ((int64_t)z * b + row) * S1 + k;
      const float raw = LVR[o];
      const float l1 = hi - softplusf(hi - raw);
      const float l = lo + softplusf(l1 - lo);
      const float m = D[o] + (k < S ? s[(int64_t)z * s_zstride + row * S + k] : 0.f);
      const float diff = t[(int64_t)z * t_zstride + row * S1 + k] - m;
      const float iv = expf(-l);
      acc += diff * diff * iv + l;
      if (grads) {
        const float dl = (1.f - diff * diff * iv) * g;
        const float s1 = sp_grad(l1 - lo), s2 = sp_grad(hi - raw);
        gD[o] = -2.f * diff * iv * g;
        gLVR[o] = dl * s1 * s2;
        cmin += dl * (1.f - s1);
        cmax += dl * s1 * (1.f - s2);
      }
    }
  }
  float* part_mse = part;
  float* part_min = part_mse + (size_t)Z * nbx;
  float* part_max = part_min + (size_t)Z * nbx * S1;
  float v = acc * inv_n;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  rmin[tid] = cmin;
  rmax[tid] = cmax;
  __syncthreads();
  const size_t pb = (size_t)z * nbx + bx;
  if (tid == 0) part_mse[pb] = red[0] + red[1] + red[2] + red[3];
  if (grads && tid < S1) {
    float a0 = 0.f, a1 = 0.f;
    for (int q = 0; q < RP; ++q) {
      a0 += rmin[q * KP + tid];
      a1 += rmax[q * KP + tid];
    }
    part_min[pb * S1 + tid] = a0;
    part_max[pb * S1 + tid] = a1;
  }
}

// per-member NLL, total loss, bound gradients from the block partials
// (ens_reduce.hpp; also run as the last block of a drpo_mlp_wgrad_reduce launch)
__global__ __launch_bounds__(256) void ens_loss_reduce_kernel(drpo_ens_reduce_t r) {
  ens_loss_reduce_block(r, (const drpo_wgrad_adam_t*)nullptr);
}

// rows per loss workgroup: one row per thread (256 / KP rows of KP column lanes)
static int loss_rows(int S1);

static int loss_kp(int S1) {
  int kp = 16;
  while (kp < S1) kp <<= 1;
  return kp;
}

static int loss_rows(int S1) { return 256 / loss_kp(S1); }

DRPO_API size_t drpo_ens_loss_workspace_size(int64_t b, int S, int Z) {
  const int rows = loss_rows(S + 1);
  const size_t nbx = (size_t)((b + rows - 1) / rows);
  return sizeof(float) * (size_t)Z * nbx * (1 + 2 * (size_t)(S + 1));
}

static int ens_loss_launch(const float* D, const float* LVR, const float* s, int64_t s_zstride, const float* t,
                           int64_t t_zstride, int64_t b, int S, int Z, const float* minlv, const float* maxlv,
                           float weight, const float* gscale, float* mse, float* loss, float* gD, float* gLVR,
                           float* gmin, float* gmax, void* workspace, drpo_ens_reduce_t* reduce_out,
                           drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(D && LVR && s && t && minlv && maxlv && mse && workspace && b >= 1 && S >= 1 &&
                   S + 1 <= LOSS_MAXS1 && Z >= 1,
               "drpo_ens_loss: bad arguments");
  DRPO_REQUIRE(!gD == !gLVR && !gD == !gmin && !gD == !gmax, "drpo_ens_loss: gradient outputs all or none");
  DRPO_REQUIRE(Z <= 256, "drpo_ens_loss: at most 256 members");
  const int rows = loss_rows(S + 1);
  const int64_t nbx64 = (b + rows - 1) / rows;
  DRPO_REQUIRE(nbx64 <= (1 << 30), "drpo_ens_loss: too many rows");
  const int nbx = (int)nbx64;
  ens_loss_kernel<<<dim3((unsigned)nbx, Z), 256, 0, stream>>>(D, LVR, s, s_zstride, t, t_zstride, b, S, Z,
                                                             loss_kp(S + 1), minlv, maxlv, gscale, gD, gLVR,
                                                             (float*)workspace);
  DRPO_LAUNCH_CHECK("ens_loss");
  const drpo_ens_reduce_t r{(const float*)workspace, nbx, Z, S + 1, minlv, maxlv, weight, gscale, mse, loss, gmin, gmax};
  if (reduce_out) {
    *reduce_out = r;   // deferred: the caller runs it (drpo_mlp_wgrad_reduce)
    return DRPO_OK;
  }
  ens_loss_reduce_kernel<<<1, 256, 0, stream>>>(r);
  DRPO_LAUNCH_CHECK("ens_loss_reduce");
  return DRPO_OK;
}

DRPO_API int drpo_ens_loss(const float* D, const float* LVR, const float* s, int64_t s_zstride, const float* t,
                           int64_t t_zstride, int64_t b, int S, int Z, const float* minlv, const float* maxlv,
                           float weight, const float* gscale, float* mse, float* loss, float* gD, float* gLVR,
                           float* gmin, float* gmax, void* workspace, drpo_stream_t stream) {
  return ens_loss_launch(D, LVR, s, s_zstride, t, t_zstride, b, S, Z, minlv, maxlv, weight, gscale, mse, loss, gD,
                         gLVR, gmin, gmax, workspace, nullptr, stream);
}

DRPO_API int drpo_ens_loss_partials(const float* D, const float* LVR, const float* s, int64_t s_zstride,
                                    const float* t, int64_t t_zstride, int64_t b, int S, int Z, const float* minlv,
                                    const float* maxlv, float weight, const float* gscale, float* mse, float* loss,
                                    float* gD, float* gLVR, float* gmin, float* gmax, void* workspace,
                                    drpo_ens_reduce_t* reduce_out, drpo_stream_t stream) {
  DRPO_REQUIRE(reduce_out, "drpo_ens_loss_partials: reduce_out is required");
  return ens_loss_launch(D, LVR, s, s_zstride, t, t_zstride, b, S, Z, minlv, maxlv, weight, gscale, mse, loss, gD,
                         gLVR, gmin, gmax, workspace, reduce_out, stream);
}

DRPO_API int drpo_ens_loss_reduce(const drpo_ens_reduce_t* red, drpo_stream_t stream) {
  DRPO_REQUIRE(red && red->part && red->mse && red->Z >= 1 && red->Z <= 256 && red->S1 >= 1 &&
                   red->S1 <= LOSS_MAXS1 && red->nbx >= 1 && red->minlv && red->maxlv,
               "drpo_ens_loss_reduce: bad reduction");
  ens_loss_reduce_kernel<<<1, 256, 0, (hipStream_t)stream>>>(*red);
  DRPO_LAUNCH_CHECK("ens_loss_reduce");
  return DRPO_OK;
}
