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
__global__ void ens_gather_kernel(const float* __restrict__ bs, const float* __restrict__ ba,
                                  const float* __restrict__ bs2, const float* __restrict__ br, int64_t ptr,
                                  const int64_t* ptr_dev, int64_t cap, int64_t rows, const int64_t* idx,
                                  uint64_t seed, uint64_t ctr, int S, int A, float* xs, float* xa, float* xt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  const int64_t p = ptr_dev ? *ptr_dev : ptr;
  const int64_t n = p < cap ? p : cap;
  int64_t j;
  if (idx) {
    j = idx[i];
  } else {
    const u32x4 r = philox({(uint32_t)i, (uint32_t)(i >> 32), 0xe5e3b1u, (uint32_t)ctr}, (uint32_t)seed,
                           (uint32_t)(seed >> 32));
    j = (int64_t)((((uint64_t)r.y << 32) | r.x) % (uint64_t)n);
  }
  const int64_t q = chrono_to_phys(j, p, cap);
  for (int k = 0; k < S; ++k) {
    xs[i * S + k] = bs[q * S + k];
    xt[i * (S + 1) + k] = bs2[q * S + k];
  }
  for (int k = 0; k < A; ++k) xa[i * A + k] = ba[q * A + k];
  xt[i * (S + 1) + S] = br[q];
}

DRPO_API int drpo_ens_gather(const float* states, const float* actions, const float* next_states,
                             const float* rewards, int64_t ptr, const int64_t* ptr_dev, int64_t cap, int64_t rows,
                             const int64_t* idx, uint64_t seed, uint64_t ctr, int S, int A, float* xs, float* xa,
                             float* xt, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(states && actions && next_states && rewards && cap >= 1 && rows >= 0 && S >= 1 && A >= 1,
               "drpo_ens_gather: bad arguments");
  DRPO_REQUIRE(ptr_dev || ptr >= 1, "drpo_ens_gather: empty buffer");
  if (rows == 0) return DRPO_OK;
  ens_gather_kernel<<<(unsigned)((rows + 255) / 256), 256, 0, stream>>>(states, actions, next_states, rewards, ptr,
                                                                        ptr_dev, cap, rows, idx, seed, ctr, S, A,
                                                                        xs, xa, xt);
  DRPO_LAUNCH_CHECK("ens_gather");
  return DRPO_OK;
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
constexpr int LOSS_ROWS = 256;   // rows per block (split over blocks beyond that)
constexpr int LOSS_MAXS1 = 256;

__global__ __launch_bounds__(256) void ens_loss_kernel(const float* D, const float* LVR, const float* s,
                                                       int64_t s_zstride, const float* t, int64_t t_zstride, int64_t b,
                                                       int S, const float* minlv, const float* maxlv,
                                                       const float* gscale, float* mse, float* gD, float* gLVR,
                                                       float* gmin, float* gmax) {
  __shared__ float red[4];
  __shared__ float cmin[LOSS_MAXS1], cmax[LOSS_MAXS1];
  const int S1 = S + 1;
  const int z = blockIdx.y;
  const int tid = threadIdx.x;
  const bool grads = gD != nullptr;
  if (grads)
    for (int k = tid; k < S1; k += 256) cmin[k] = cmax[k] = 0.f;
  __syncthreads();
  const float inv_n = 1.f / (float)(b * S1);
  const float g = grads ? (gscale ? *gscale : 1.f) * inv_n : 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * LOSS_ROWS;
  const int64_t r1 = min(b, r0 + LOSS_ROWS);
  float sq = 0.f, ld = 0.f;
  for (int64_t e = r0 * S1 + tid; e < r1 * S1; e += 256) {
    const int64_t row = e / S1;
    const int k = (int)(e - row * S1);
    const int64_t o = (int64_t)z * b * S1 + e;
    const float raw = LVR[o];
    const float hi = maxlv[k], lo = minlv[k];
    const float l1 = hi - softplusf(hi - raw);
    const float l = lo + softplusf(l1 - lo);
    const float m = D[o] + (k < S ? s[(int64_t)z * s_zstride + row * S + k] : 0.f);
    const float diff = t[(int64_t)z * t_zstride + e] - m;
    const float iv = expf(-l);
    sq += diff * diff * iv;
    ld += l;
    if (grads) {
      const float dl = (1.f - diff * diff * iv) * g;
      const float s1 = sp_grad(l1 - lo), s2 = sp_grad(hi - raw);
      gD[o] = -2.f * diff * iv * g;
      gLVR[o] = dl * s1 * s2;
      atomicAdd(&cmin[k], dl * (1.f - s1));
      atomicAdd(&cmax[k], dl * s1 * (1.f - s2));
    }
  }
  // mean(sq) + mean(lv) for this member, accumulated over row blocks
  float v = (sq + ld) * inv_n;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((tid & 63) == 0) red[tid >> 6] = v;
  __syncthreads();
  if (tid == 0) atomicAdd(&mse[z], red[0] + red[1] + red[2] + red[3]);
  if (grads)
    for (int k = tid; k < S1; k += 256) {
      atomicAdd(&gmin[k], cmin[k]);
      atomicAdd(&gmax[k], cmax[k]);
    }
}

// loss = sum_z mse[z] + w * (sum(max) - sum(min)); d/dmax += w*g, d/dmin -= w*g
__global__ void ens_loss_total_kernel(const float* mse, int Z, const float* minlv, const float* maxlv, int S1,
                                      float weight, const float* gscale, float* loss, float* gmin, float* gmax) {
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int z = 0; z < Z; ++z) tot += mse[z];
    float smax = 0.f, smin = 0.f;
    for (int k = 0; k < S1; ++k) {
      smax += maxlv[k];
      smin += minlv[k];
    }
    if (loss) *loss = tot + weight * (smax - smin);
  }
  if (gmin && (int)threadIdx.x < S1) {
    const float g = (gscale ? *gscale : 1.f) * weight;
    gmax[threadIdx.x] += g;
    gmin[threadIdx.x] -= g;
  }
}

DRPO_API int drpo_ens_loss(const float* D, const float* LVR, const float* s, int64_t s_zstride, const float* t,
                           int64_t t_zstride, int64_t b, int S, int Z, const float* minlv, const float* maxlv,
                           float weight, const float* gscale, float* mse, float* loss, float* gD, float* gLVR,
                           float* gmin, float* gmax, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(D && LVR && s && t && minlv && maxlv && mse && b >= 1 && S >= 1 && S + 1 <= LOSS_MAXS1 && Z >= 1,
               "drpo_ens_loss: bad arguments");
  DRPO_REQUIRE(!gD == !gLVR && !gD == !gmin && !gD == !gmax, "drpo_ens_loss: gradient outputs all or none");
  DRPO_CHECK_HIP(hipMemsetAsync(mse, 0, sizeof(float) * Z, stream));
  dim3 grid((unsigned)((b + LOSS_ROWS - 1) / LOSS_ROWS), Z);
  ens_loss_kernel<<<grid, 256, 0, stream>>>(D, LVR, s, s_zstride, t, t_zstride, b, S, minlv, maxlv, gscale, mse, gD,
                                            gLVR, gmin, gmax);
  DRPO_LAUNCH_CHECK("ens_loss");
  if (loss || gmin) {
    ens_loss_total_kernel<<<1, 256, 0, stream>>>(mse, Z, minlv, maxlv, S + 1, weight, gscale, loss, gmin, gmax);
    DRPO_LAUNCH_CHECK("ens_loss_total");
  }
  return DRPO_OK;
}
