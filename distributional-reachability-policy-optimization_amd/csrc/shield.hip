// Safety shields around the real-environment step and the evaluation rollouts.
//
//  drpo_shield_mix     the linear shield's candidate actions (src/sampling.py:430-434):
//                      mix_i = a_safe * r_i + a_perf * (1 - r_i), r_i = (K-1-i)/(K-1),
//                      i = 0..K-1 (K = 11 in the reference), as [K][n][A]; the K
//                      candidates are then scored by ONE constraint-critic forward over
//                      K*n rows instead of K separate calls.
//  drpo_shield_select  the per-row decision on the device (no host round trip):
//                      mode 0 none (a_perf); mode 1 threshold shield
//                      (src/smbpo.py:127-136, src/sampling.py:427-429): a_safe where
//                      max_C q > thr; mode 2 linear shield (src/sampling.py:430-437):
//                      start from a_safe, take mix_i wherever max_C q_i <= thr, later i
//                      overriding earlier ones.
// Arithmetic matches PyTorch CPU fp32: the scalar ratios are rounded to float once
// (tensor * python float), products and the sum are separately rounded (no FMA).
#include "common.hpp"

namespace {

__global__ void shield_mix_kernel(const float* ap, const float* as, int64_t n, int A, int K, float* mixes) {
  const int64_t per = n * A;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= per * K) return;
  const int k = (int)(i / per);
  const int64_t j = i - (int64_t)k * per;
  const double r = (double)(K - 1 - k) / (double)(K - 1);
  const float rs = (float)r, rp = (float)(1.0 - r);
  mixes[i] = __fadd_rn(__fmul_rn(as[j], rs), __fmul_rn(ap[j], rp));
}

__device__ __forceinline__ float row_max(const float* q, int C) {
  float m = q[0];
  for (int c = 1; c < C; ++c) m = q[c] > m ? q[c] : m;
  return m;
}

__global__ void shield_select_kernel(const float* q, int K, int64_t n, int C, int A, int mode, float thr,
                                     const float* ap, const float* as, const float* mixes, float* out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  const float* src = ap + r * A;
  if (mode == 1) {
    if (row_max(q + r * C, C) > thr) src = as + r * A;
  } else if (mode == 2) {
    src = as + r * A;
    for (int k = 0; k < K; ++k)
      if (row_max(q + ((int64_t)k * n + r) * C, C) <= thr) src = mixes + ((int64_t)k * n + r) * A;
  }
  for (int c = 0; c < A; ++c) out[r * A + c] = src[c];
}

}  // namespace

DRPO_API int drpo_shield_mix(const float* a_perf, const float* a_safe, int64_t n, int A, int K, float* mixes,
                             drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(K >= 2 && A >= 1 && n >= 0, "drpo_shield_mix: need K >= 2, A >= 1 (K=%d A=%d)", K, A);
  const int64_t tot = n * A * K;
  if (tot == 0) return DRPO_OK;
  shield_mix_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, stream>>>(a_perf, a_safe, n, A, K, mixes);
  DRPO_LAUNCH_CHECK("shield_mix");
  return DRPO_OK;
}

DRPO_API int drpo_shield_select(const float* q, int K, int64_t n, int C, int A, int mode, float threshold,
                                const float* a_perf, const float* a_safe, const float* mixes, float* out,
                                drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(mode >= 0 && mode <= 2, "drpo_shield_select: unknown mode %d", mode);
  DRPO_REQUIRE(mode != 2 || (K >= 1 && mixes), "drpo_shield_select: the linear shield needs K >= 1 mixes");
  DRPO_REQUIRE(C >= 1 && A >= 1, "drpo_shield_select: need C >= 1, A >= 1");
  if (n == 0) return DRPO_OK;
  shield_select_kernel<<<(unsigned)((n + 63) / 64), 64, 0, stream>>>(q, K, n, C, A, mode, threshold, a_perf, a_safe,
                                                                      mixes, out);
  DRPO_LAUNCH_CHECK("shield_select");
  return DRPO_OK;
}
