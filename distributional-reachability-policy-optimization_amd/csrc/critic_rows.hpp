// Per-row math of the safe-SAC critic losses (src/ssac.py:284-435), shared by the
// stand-alone drpo_critic_head kernel (csrc/sac.hip) and the critic backward launch,
// which forms its own output gradients from the forward outputs (no separate head
// launch on the production path, csrc/mlp.hip).
#pragma once
#include "common.hpp"

namespace drpo {

// Transcendentals of the per-row critic math. The libm forms (range reduction, IEEE
// division) made the certificate upstream of the critic backward a 15.5 k-cycle serial
// chain per workgroup (profiles/sac_stamps.py); the hardware forms (v_exp_f32 /
// v_log_f32 / v_rcp_f32, ~1 ulp) cut it, at ~1e-6 relative error -- far inside the SAC
// parity tolerances. log1p of a small argument uses its series (log(1 + y) alone loses
// the low bits of y).
__device__ __forceinline__ float cr_exp(float x) { return fast_exp(x); }
__device__ __forceinline__ float cr_log(float x) { return 0.69314718055994531f * __builtin_amdgcn_logf(x); }
__device__ __forceinline__ float cr_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ float cr_softplus(float x) {   // torch softplus (beta 1, threshold 20)
  if (x > 20.f) return x;
  const float y = fast_exp(-fabsf(x));
  const float l1p = y < 1e-3f ? y * (1.f - 0.5f * y) : 0.69314718055994531f * __builtin_amdgcn_logf(1.f + y);
  return fmaxf(x, 0.f) + l1p;
}

__device__ __forceinline__ float sp_grad(float x) { return x > 20.f ? 1.f : cr_rcp(1.f + cr_exp(-x)); }

__device__ __forceinline__ float cc_std(float l, float lmin, float lmax) {
  float ls = lmax - cr_softplus(lmax - l);
  ls = lmin + cr_softplus(ls - lmin);
  return cr_exp(ls);
}

// d std / d raw for std = exp(lmin + sp(lmax - sp(lmax - l) - lmin))
__device__ __forceinline__ float cc_dstd_draw(float l, float lmin, float lmax, float std) {
  const float ls1 = lmax - cr_softplus(lmax - l);
  return std * sp_grad(ls1 - lmin) * sp_grad(lmax - l);
}

// The head descriptor may be referenced from the kernarg segment (address space 4:
// scalar loads) or from generic memory, hence the template parameter.
// soft Bellman target of row i with the twin-min target critics (src/ssac.py:284-294)
template <typename Head>
__device__ __forceinline__ float critic_target(const Head& p, int64_t i, float alpha) {
  // global-address-space loads (gload): the descriptor's pointers are generic, and FLAT
  // loads would also count against lgkmcnt and drain with every LDS wait
  float nv = fminf(gload(p.q0t + i), gload(p.q1t + i));
  if (!p.deterministic_backup) nv = nv - alpha * gload(p.logp2 + i);
  const float dn = gload(p.d + i) ? 1.f : 0.f;
  return gload(p.r + i) + p.discount * (1.f - dn) * nv;
}

// certificate element k = (i, c): reachability backup (src/ssac.py:304-413), the
// distributional (3-term) or MSE loss term (src/ssac.py:415-435) and its gradients
// w.r.t. the mean / raw log-std head outputs. Returns the loss term (already / (B C)).
template <typename Head>
__device__ __forceinline__ float cert_element(const Head& p, int64_t i, int c, float& dmu, float& dls) {
  const int64_t k = i * p.C + c;
  const float invN = 1.f / (float)(p.B * p.C);
  const float dn = gload(p.d + i) ? 1.f : 0.f;
  // certificate-target done flags: the batch's, or the model-predicted ones of the
  // robust branch (src/ssac.py:387-400)
  const float dnc = p.dc ? (gload(p.dc + i) ? 1.f : 0.f) : dn;
  const float mu = gload(p.mu + k);
  const float mut = gload(p.mu_t + k);
  if (p.cost) {
    // cost certificate (src/ssac.py:306-310): one-step discounted violation cost, MSE
    const float yc = (gload(p.v + i) ? 1.f : 0.f) + p.discount * (1.f - dn) * mut;
    dmu = 2.f * (mu - yc) * invN;
    dls = 0.f;
    return (mu - yc) * (mu - yc) * invN;
  }
  const float hv = gload(p.h + k);
  const float lst = p.distributional ? gload(p.ls_t + k) : 0.f;
  const float lsk = p.distributional ? gload(p.ls + k) : 0.f;
  float q2;
  if (p.distributional) {
    const float e = fminf(fmaxf(normal_at(p.eps3, k, p.seed, p.ctr, 7u), -2.f), 2.f);
    q2 = mut + e * cc_std(lst, p.lmin, p.lmax);
  } else {
    q2 = mut;
  }
  const float nonterm = (1.f - p.discount) * hv + p.discount * fmaxf(hv, q2);
  const float yc = nonterm * (1.f - dnc) + hv * dnc;
  if (p.distributional) {
    const float diff = fminf(fmaxf(yc - mu, -p.qc_td_bound), p.qc_td_bound);
    const float yb = diff + mu;
    const float sd = cc_std(lsk, p.lmin, p.lmax);
    const float var = sd * sd;
    const float ivar = cr_rcp(var), isd = cr_rcp(sd);
    const float t1 = (mu - yc) * (mu - yc) * (0.5f * ivar);
    const float t2 = (mu - yb) * (mu - yb) * (0.5f * ivar);
    dmu = (mu - yc) * ivar * invN;
    const float dsd = (-(mu - yb) * (mu - yb) * ivar * isd + isd) * invN;
    dls = dsd * cc_dstd_draw(lsk, p.lmin, p.lmax, sd);
    return (t1 + t2 + cr_log(sd)) * invN;
  }
  dmu = 2.f * (mu - yc) * invN;
  dls = 0.f;
  return (mu - yc) * (mu - yc) * invN;
}

}  // namespace drpo
