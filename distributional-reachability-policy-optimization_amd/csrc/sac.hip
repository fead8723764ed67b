// Fused elementwise kernels of the safe-SAC update (src/ssac.py, src/smbpo.py:251-279).
// All are HBM/latency bound row-wise epilogues around the MLP kernels (mlp.hip):
//
//  drpo_sample_batch      mixed real/virtual minibatch gather + reward / constraint
//                         preprocessing (src/smbpo.py:253-270, src/sampling.py:147-151)
//  drpo_policy_head       squashed-Gaussian sample / rsample / mean + log_prob
//                         (src/policy.py:89-97, torch TanhTransform / Normal)
//  drpo_cc_head           constraint-critic log-std soft clamp, quantile upper bound
//                         mu + std_ratio*std and its max over C (src/ssac.py:64-92,588-600)
//  drpo_critic_head       soft Bellman target, reachability-certificate backup
//                         (distributional or vanilla), both critic losses and their
//                         gradients w.r.t. the critic outputs (src/ssac.py:284-435)
//  drpo_actor_upstream    dL/d(critic / constraint-critic outputs) of the actor and
//                         safe-actor losses (src/ssac.py:458-505)
//  drpo_squash_backward   chain rule through rsample + tanh + log_prob to the actor
//                         head (mu, raw log-std), plus the alpha-loss sum
//  drpo_multiplier_head   Lagrangian multiplier loss gradient (src/ssac.py:529-568)
//  drpo_alpha_grad        d alpha_loss / d log_alpha (src/ssac.py:498-501)
// Losses are accumulated (already scaled) with float atomics into caller-zeroed
// device scalars, so no host synchronisation is needed.
#include "common.hpp"
#include "critic_rows.hpp"

using namespace drpo;

namespace {

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  __syncthreads();
  return s;   // valid in thread 0
}


}  // namespace

// ---------------------------------------------------------------------------
// minibatch sampling
// ---------------------------------------------------------------------------

__global__ void sample_batch_kernel(drpo_buffer_view_t real, drpo_buffer_view_t virt, int n_real, int B, int S, int A,
                                    int C, const int64_t* idx_real, const int64_t* idx_virt, uint64_t seed,
                                    uint64_t ctr, float reward_scale, float alive_bonus, float cscale, float coffset,
                                    float* os, float* oa, float* os2, float* orw, uint8_t* od, uint8_t* ov, float* oh) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const bool isr = i < n_real;
  const drpo_buffer_view_t& bv = isr ? real : virt;
  const int j = isr ? i : i - n_real;
  int64_t len = bv.len;
  if (len < 0) {
    const int64_t p = *bv.ptr_dev;
    len = p < bv.cap ? p : bv.cap;
  }
  int64_t q;
  const int64_t* ix = isr ? idx_real : idx_virt;
  if (ix) {
    q = ix[j];
  } else {
    const u32x4 rr = philox({(uint32_t)j, isr ? 0u : 1u, 0x5a4d11u, (uint32_t)ctr}, (uint32_t)seed,
                            (uint32_t)(seed >> 32));
    q = (int64_t)(((uint64_t)rr.x * (uint64_t)len) >> 32);
  }
  // grid.y splits the row's components over 4 threads (more loads in flight)
  const int part = blockIdx.y;
  if (part == 0) {
    for (int k = 0; k < S; ++k) os[(int64_t)i * S + k] = bv.s[q * S + k];
  } else if (part == 1) {
    for (int k = 0; k < S; ++k) os2[(int64_t)i * S + k] = bv.s2[q * S + k];
  } else if (part == 2) {
    for (int k = 0; k < A; ++k) oa[(int64_t)i * A + k] = bv.a[q * A + k];
    float r = bv.r[q];
    if (reward_scale != 0.f) r = r * reward_scale;
    if (alive_bonus != 0.f) r = r + alive_bonus;
    orw[i] = r;
    od[i] = bv.d[q];
    ov[i] = bv.v[q];
  } else {
    for (int c = 0; c < C; ++c) {
      float hv = bv.h[q * C + c] * cscale;
      hv = hv + (hv > 0.f ? 1.f : 0.f) * coffset;
      oh[(int64_t)i * C + c] = hv;
    }
  }
}

DRPO_API int drpo_sample_batch(const drpo_buffer_view_t* real, const drpo_buffer_view_t* virt, int n_real, int B,
                               int S, int A, int C, const int64_t* idx_real, const int64_t* idx_virt, uint64_t seed,
                               uint64_t ctr, float reward_scale, float alive_bonus, float constraint_scale,
                               float constraint_offset, float* s, float* a, float* s2, float* r, uint8_t* d,
                               uint8_t* v, float* h, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(real && virt && B >= 0 && n_real >= 0 && n_real <= B, "drpo_sample_batch: bad sizes");
  if (B == 0) return DRPO_OK;
  sample_batch_kernel<<<dim3((B + 63) / 64, 4), 64, 0, stream>>>(*real, *virt, n_real, B, S, A, C, idx_real, idx_virt, seed,
                                                          ctr, reward_scale, alive_bonus, constraint_scale,
                                                          constraint_offset, s, a, s2, r, d, v, h);
  DRPO_LAUNCH_CHECK("sample_batch");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// policy head
// ---------------------------------------------------------------------------
// raw [B][2A] = (mu, log-std pre-activation). mode 0: sample (Normal.sample: eps*std+mu),
// 1: rsample (mu + eps*std), 2: mean only. Outputs are optional.
__global__ void policy_head_kernel(const float* raw, int64_t B, int A, int mode, const float* eps, uint64_t seed,
                                   uint64_t ctr, uint32_t site, float* a_out, float* logp, float* u_out, float* e_out,
                                   float* amean) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const float* r = raw + i * 2 * A;
  if (mode == 3) {   // distribution parameters (loc, scale) for distr()
    for (int d = 0; d < A; ++d) {
      const float mu = r[d];
      const float sd = expf(-6.f + 10.f * sigmoidf(r[A + d])) * 1.0f;
      if (amean) amean[i * A + d] = tanhf(mu);
      if (u_out) u_out[i * A + d] = mu;
      if (e_out) e_out[i * A + d] = sd;
    }
    return;
  }
  squashed_gaussian_row([&](int c) { return r[c]; }, i, A, mode, eps, seed, ctr, site, a_out, logp, u_out, e_out,
                        amean);
}

DRPO_API int drpo_policy_head(const float* raw, int64_t B, int A, int mode, const float* eps, uint64_t seed,
                              uint64_t ctr, uint32_t site, float* a, float* logp, float* u, float* e, float* amean,
                              drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(mode >= 0 && mode <= 3 && A >= 1, "drpo_policy_head: bad mode/A");
  if (B == 0) return DRPO_OK;
  policy_head_kernel<<<(unsigned)((B + 63) / 64), 64, 0, stream>>>(raw, B, A, mode, eps, seed, ctr, site, a, logp,
                                                                      u, e, amean);
  DRPO_LAUNCH_CHECK("policy_head");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// constraint-critic head: ub = mu + ratio*std (distributional) or mu; max over C
// ---------------------------------------------------------------------------
__global__ void cc_head_kernel(const float* mu, const float* lsraw, int64_t B, int C, int dist, float ratio, float lmin,
                               float lmax, float* ubmax, int* argmax) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  float best = 0.f;
  int bi = 0;
  for (int c = 0; c < C; ++c) {
    float v = mu[i * C + c];
    if (dist) v = v + ratio * cc_std(lsraw[i * C + c], lmin, lmax);
    if (c == 0 || v > best) { best = v; bi = c; }
  }
  if (ubmax) ubmax[i] = best;
  if (argmax) argmax[i] = bi;
}

DRPO_API int drpo_cc_head(const float* mu, const float* lsraw, int64_t B, int C, int distributional, float std_ratio,
                          float log_std_min, float log_std_max, float* ubmax, int* argmax, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (B == 0) return DRPO_OK;
  cc_head_kernel<<<(unsigned)((B + 63) / 64), 64, 0, stream>>>(mu, lsraw, B, C, distributional, std_ratio,
                                                                  log_std_min, log_std_max, ubmax, argmax);
  DRPO_LAUNCH_CHECK("cc_head");
  return DRPO_OK;
}

// ConstraintCritic.forward outputs per constraint (src/ssac.py:75-92): mode 0
// (uncertainty) q = mu + std_ratio*std; mode 1 (sample) std and
// q = mu + clamp(eps, -2, 2)*std. n = rows*C elements.
__global__ void cc_dist_kernel(const float* mu, const float* lsraw, int64_t n, int mode, float std_ratio, float lmin,
                               float lmax, const float* eps, uint64_t seed, uint64_t ctr, float* std_out, float* q) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float sd = cc_std(lsraw[i], lmin, lmax);
  if (mode == 0) {
    q[i] = mu[i] + std_ratio * sd;
  } else {
    float e = normal_at(eps, i, seed, ctr, 0xcc01u);
    e = fminf(fmaxf(e, -2.f), 2.f);
    if (std_out) std_out[i] = sd;
    q[i] = mu[i] + e * sd;
  }
}

DRPO_API int drpo_cc_dist(const float* mu, const float* lsraw, int64_t n, int mode, float std_ratio,
                          float log_std_min, float log_std_max, const float* eps, uint64_t seed, uint64_t ctr,
                          float* std_out, float* q, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(mu && lsraw && q && n >= 0 && (mode == 0 || mode == 1), "drpo_cc_dist: bad arguments");
  if (n == 0) return DRPO_OK;
  cc_dist_kernel<<<(unsigned)((n + 255) / 256), 256, 0, stream>>>(mu, lsraw, n, mode, std_ratio, log_std_min,
                                                                  log_std_max, eps, seed, ctr, std_out, q);
  DRPO_LAUNCH_CHECK("cc_dist");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// critic + certificate targets, losses, gradients (update_critic)
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void critic_head_kernel(drpo_critic_head_t p) {
  __shared__ float red[8];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float lq = 0.f, lc = 0.f;
  if (i < p.B) {
    const float y = critic_target(p, i, expf(*p.log_alpha));
    const float e0 = p.q0[i] - y, e1 = p.q1[i] - y;
    const float invB = 1.f / (float)p.B;
    lq = (e0 * e0 + e1 * e1) * (0.5f * invB);
    for (int c = 0; c < p.C; ++c) {
      float dmu, dls;
      lc += cert_element(p, i, c, dmu, dls);
      p.dmu[i * p.C + c] = dmu;
      if (p.dls) p.dls[i * p.C + c] = dls;
    }
    // the critic gradients are stored after the certificate loop: a store ahead of
    // the loop's loads would cost the row a second memory latency
    p.dq0[i] = e0 * invB;
    p.dq1[i] = e1 * invB;
  }
  const float s0 = block_sum(lq, red);
  const float s1 = block_sum(lc, red);
  if (threadIdx.x == 0) {
    atomicAdd(&p.loss[0], s0);
    atomicAdd(&p.loss[1], s1);
  }
}

DRPO_API int drpo_critic_head(const drpo_critic_head_t* p, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(p && p->C >= 1 && p->B >= 0, "drpo_critic_head: bad descriptor");
  DRPO_REQUIRE(!p->cost || (p->v && !p->distributional), "drpo_critic_head: cost target needs v, not distributional");
  if (p->B == 0) return DRPO_OK;
  critic_head_kernel<<<(unsigned)((p->B + 63) / 64), 64, 0, stream>>>(*p);
  DRPO_LAUNCH_CHECK("critic_head");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// actor / safe-actor upstream gradients (update_actor_and_alpha)
// ---------------------------------------------------------------------------
// For the actor loss mean(alpha*logp - Q_k) + mean(lam * max_C ub(s,a)) and the safe
// actor loss mean(max_C ub(s, a_safe)): gradients w.r.t. Q_k (-1/B), and w.r.t. the
// mean / raw-log-std heads of the constraint critic at (s,a) and (s,a_safe).
__global__ void actor_upstream_kernel(int64_t B, int C, int dist, float ratio, float lmin, float lmax,
                                      const float* lams, const float* mu_a, const float* ls_a, const float* mu_s,
                                      const float* ls_s, float* gq, float* gmu_a, float* gls_a, float* gmu_s,
                                      float* gls_s, float ub, float fixed_lam, float clb, float cub) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B) return;
  const float invB = 1.f / (float)B;
  // pass 1, loads only: the arg-max constraint of each side and its raw log-std (both
  // sides' loads are in flight together; no store sits between them)
  int bis[2] = {0, 0};
  float lsb[2] = {0.f, 0.f}, best_a = 0.f;
  float lam = gmu_a ? (lams ? lams[i] : fixed_lam) : 0.f;
  if (lams && ub > 0.f) lam = ub / 2.f * (1.f + tanhf(lam / ub * 2.f));   // MLPMultiplier.forward transform
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const float* mu = side ? mu_s : mu_a;
    const float* ls = side ? ls_s : ls_a;
    if (!(side ? gmu_s : gmu_a)) continue;
    float best = 0.f, lbest = 0.f;
    int bi = 0;
    for (int c = 0; c < C; ++c) {
      float v = mu[i * C + c];
      const float l = dist ? ls[i * C + c] : 0.f;
      if (dist) v = v + ratio * cc_std(l, lmin, lmax);
      if (c == 0 || v > best) { best = v; bi = c; lbest = l; }
    }
    bis[side] = bi;
    lsb[side] = lbest;
    if (!side) best_a = best;
  }
  // scalar multiplier: the certificate term is clamp(Qc, lb, ub) -- no gradient outside
  if (!lams && (best_a < clb || best_a > cub)) lam = 0.f;
  // pass 2, stores
  if (gq) gq[i] = -invB;
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    float* gmu = side ? gmu_s : gmu_a;
    float* gls = side ? gls_s : gls_a;
    if (!gmu) continue;
    const float g = side ? invB : lam * invB;
    float gl = 0.f;
    if (dist && g != 0.f) {
      const float sd = cc_std(lsb[side], lmin, lmax);
      gl = g * ratio * cc_dstd_draw(lsb[side], lmin, lmax, sd);
    }
    for (int c = 0; c < C; ++c) {
      const int64_t k = i * C + c;
      const bool hit = c == bis[side];
      gmu[k] = hit ? g : 0.f;
      if (gls) gls[k] = hit ? gl : 0.f;
    }
  }
}

DRPO_API int drpo_actor_upstream(int64_t B, int C, int distributional, float std_ratio, float log_std_min,
                                 float log_std_max, const float* lams, const float* mu_a, const float* ls_a,
                                 const float* mu_s, const float* ls_s, float* gq, float* gmu_a, float* gls_a,
                                 float* gmu_s, float* gls_s, float lam_upper_bound, float fixed_lam,
                                 float clamp_lb, float clamp_ub, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (B == 0) return DRPO_OK;
  actor_upstream_kernel<<<(unsigned)((B + 63) / 64), 64, 0, stream>>>(
      B, C, distributional, std_ratio, log_std_min, log_std_max, lams, mu_a, ls_a, mu_s, ls_s, gq, gmu_a, gls_a,
      gmu_s, gls_s, lam_upper_bound, fixed_lam, clamp_lb, clamp_ub);
  DRPO_LAUNCH_CHECK("actor_upstream");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// squashed-Gaussian backward
// ---------------------------------------------------------------------------
// dA [B][A]: dL/d action; g_lp = dL/d log_prob (alpha/B for the actor, 0 for the safe
// actor, read as alpha = exp(*log_alpha) * lp_scale when log_alpha != NULL).
// Writes draw [B][2A] = dL/d(mu, raw log-std). Optionally accumulates
// sum_i (logp_i + target_entropy) into *alpha_sum (alpha loss).
constexpr int SQ_MAXA = 8;   // action width bound of the row-wise heads
__global__ __launch_bounds__(256) void squash_bwd_kernel(int64_t B, int A, const float* raw, const float* u,
                                                         const float* e, const float* dA, const float* dA2, const float* log_alpha,
                                                         float lp_scale, const float* logp, float target_entropy,
                                                         float* alpha_sum, float* draw) {
  __shared__ float red[8];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float acc = 0.f;
  if (i < B) {
    // every load of the row is issued before the first store (a store between two
    // dependent load groups costs a second memory latency per row)
    float mu[SQ_MAXA], rr[SQ_MAXA], uu[SQ_MAXA], ee[SQ_MAXA], dAv[SQ_MAXA];
#pragma unroll
    for (int d = 0; d < SQ_MAXA; ++d) {
      if (d >= A) break;
      mu[d] = raw[i * 2 * A + d];
      rr[d] = raw[i * 2 * A + A + d];
      uu[d] = u[i * A + d];
      ee[d] = e[i * A + d];
      dAv[d] = dA2 ? dA[i * A + d] + dA2[i * A + d] : dA[i * A + d];
    }
    const float lpi = alpha_sum ? logp[i] : 0.f;
    const float glp = log_alpha ? expf(*log_alpha) * lp_scale : 0.f;
#pragma unroll
    for (int d = 0; d < SQ_MAXA; ++d) {
      if (d >= A) break;
      const float sg = sigmoidf(rr[d]);
      const float sd = expf(-6.f + 10.f * sg) * 1.0f;
      const float a = tanhf(uu[d]);
      const float diff = uu[d] - mu[d];
      const float var = sd * sd;
      const float du = dAv[d] * (1.f - a * a) + glp * (-diff / var + 2.f - 4.f * sp_grad(-2.f * uu[d]));
      const float dmu = du + glp * diff / var;
      const float dsd = du * ee[d] + glp * (diff * diff / (var * sd) - 1.f / sd);
      draw[i * 2 * A + d] = dmu;
      draw[i * 2 * A + A + d] = dsd * sd * 10.f * sg * (1.f - sg);
    }
    if (alpha_sum) acc = lpi + target_entropy;
  }
  if (alpha_sum) {
    const float s = block_sum(acc, red);
    if (threadIdx.x == 0) atomicAdd(alpha_sum, s);
  }
}

DRPO_API int drpo_squash_backward(int64_t B, int A, const float* raw, const float* u, const float* e, const float* dA, const float* dA2,
                                  const float* log_alpha, float lp_scale, const float* logp, float target_entropy,
                                  float* alpha_sum, float* draw, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(A >= 1 && A <= SQ_MAXA, "drpo_squash_backward: action width %d", A);
  if (B == 0) return DRPO_OK;
  squash_bwd_kernel<<<(unsigned)((B + 63) / 64), 64, 0, stream>>>(B, A, raw, u, e, dA, dA2, log_alpha, lp_scale, logp,
                                                                     target_entropy, alpha_sum, draw);
  DRPO_LAUNCH_CHECK("squash_backward");
  return DRPO_OK;
}

__global__ void alpha_grad_kernel(const float* log_alpha, const float* alpha_sum, float invB, float* grad) {
  *grad = -expf(*log_alpha) * (*alpha_sum * invB);
}

DRPO_API int drpo_alpha_grad(const float* log_alpha, const float* alpha_sum, int64_t B, float* grad,
                             drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  alpha_grad_kernel<<<1, 1, 0, stream>>>(log_alpha, alpha_sum, 1.f / (float)B, grad);
  DRPO_LAUNCH_CHECK("alpha_grad");
  return DRPO_OK;
}

// ---------------------------------------------------------------------------
// multiplier head (mlp multiplier)
// ---------------------------------------------------------------------------
// x: multiplier MLP output [B]; sqc: max_C safe constraint value; aqc: max_C actor Qc.
// lam = ub/2 (1 + tanh(2x/ub)); loss = -0.5 mean([sqc<=0] lam pen) + mean(([sqc>0](lam - (ub-eps)))^2)
__global__ __launch_bounds__(256) void multiplier_head_kernel(int64_t B, const float* x, const float* sqc,
                                                              const float* aqc, float thr, float plb, float pub,
                                                              float ub, float lam_eps, float* gx, float* loss) {
  __shared__ float red[8];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float l = 0.f;
  if (i < B && !x) {
    // scalar multiplier: the penalty sum of -mean(softplus(m) * penalty)
    l = fminf(fmaxf(aqc[i] - thr, plb), pub);
  } else if (i < B) {
    const float t = tanhf(x[i] / ub * 2.f);
    const float lam = ub / 2.f * (1.f + t);
    const float pen = fminf(fmaxf(aqc[i] - thr, plb), pub);
    const float safe = sqc[i] <= 0.f ? 1.f : 0.f, unsafe = 1.f - safe;
    const float invB = 1.f / (float)B;
    const float lu = unsafe * lam, tu = unsafe * (ub - lam_eps);
    l = (-0.5f * safe * lam * pen + (lu - tu) * (lu - tu)) * invB;
    const float glam = (-0.5f * safe * pen + 2.f * (lu - tu) * unsafe) * invB;
    gx[i] = glam * (ub / 2.f) * (1.f - t * t) * (2.f / ub);
  }
  if (loss) {
    const float s = block_sum(l, red);
    if (threadIdx.x == 0) atomicAdd(loss, s);
  }
}

DRPO_API int drpo_multiplier_head(int64_t B, const float* x, const float* safe_qc, const float* actor_qc,
                                  float threshold, float penalty_lb, float penalty_ub, float upper_bound,
                                  float lam_epsilon, float* gx, float* loss, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (B == 0) return DRPO_OK;
  multiplier_head_kernel<<<(unsigned)((B + 63) / 64), 64, 0, stream>>>(
      B, x, safe_qc, actor_qc, threshold, penalty_lb, penalty_ub, upper_bound, lam_epsilon, gx, loss);
  DRPO_LAUNCH_CHECK("multiplier_head");
  return DRPO_OK;
}

// lam = ub/2 (1 + tanh(2x/ub)) (MLPMultiplier.forward output transform)
__global__ void multiplier_out_kernel(int64_t B, const float* x, float ub, float* lam) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < B) lam[i] = ub / 2.f * (1.f + tanhf(x[i] / ub * 2.f));
}

DRPO_API int drpo_multiplier_out(int64_t B, const float* x, float upper_bound, float* lam, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  if (B == 0) return DRPO_OK;
  multiplier_out_kernel<<<(unsigned)((B + 63) / 64), 64, 0, stream>>>(B, x, upper_bound, lam);
  DRPO_LAUNCH_CHECK("multiplier_out");
  return DRPO_OK;
}
