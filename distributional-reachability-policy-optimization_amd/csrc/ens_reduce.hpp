// Fixed-order reduction of the ensemble NLL block partials (csrc/ensemble.hip) for
// one 256-thread block: run by ens_loss_reduce_kernel, or as the extra last block
// of a drpo_mlp_wgrad_reduce launch (one launch fewer per fit step).
#pragma once
#include "common.hpp"

namespace drpo {
constexpr int LOSS_MAXS1 = 256;

// per-member NLL, total loss, bound gradients from the block partials. Every sum is
// spread over 16 lanes (strided partials, then a fixed xor tree), so the kernel waits
// a couple of memory latencies instead of one per partial; the order is fixed, so the
// result is deterministic.
// Reduce: drpo_ens_reduce_t, in generic memory or read in place from a kernarg segment.
// adam (drpo_wgrad_adam_t, may be NULL): the log-var bounds take their Adam step here
// (the weight-gradient launch's fused step) instead of accumulating into gmin / gmax.
template <typename Reduce, typename AdamT>
__device__ __forceinline__ void ens_loss_reduce_block(Reduce& rd, AdamT* adam) {
  const float* __restrict__ part = rd.part;
  const int nbx = rd.nbx, Z = rd.Z, S1 = rd.S1;
  const float* __restrict__ minlv = rd.minlv;
  const float* __restrict__ maxlv = rd.maxlv;
  const float weight = rd.weight;
  const float* gscale = rd.gscale;
  float *mse = rd.mse, *loss = rd.loss, *gmin = rd.gmin, *gmax = rd.gmax;
  __shared__ float red[256], smx[LOSS_MAXS1], smn[LOSS_MAXS1];
  const int tid = threadIdx.x;
  const int grp = tid >> 4, l16 = tid & 15;
  const float* part_mse = part;
  const float* part_min = part_mse + (size_t)Z * nbx;
  const float* part_max = part_min + (size_t)Z * nbx * S1;
  for (int z = grp; z < Z; z += 16) {
    float m = 0.f;
    for (int q = l16; q < nbx; q += 16) m += part_mse[(size_t)z * nbx + q];
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) m += __shfl_xor(m, o, 16);
    if (l16 == 0) {
      mse[z] = m;
      red[z] = m;
    }
  }
  const size_t Q = (size_t)Z * nbx;
  const float gw = gmin ? (gscale ? *gscale : 1.f) * weight : 0.f;
  for (int c = grp; c < S1; c += 16) {
    // the bounds' values for the loss term below, read before any fused step moves them
    if (l16 == 0) {
      smx[c] = maxlv[c];
      smn[c] = minlv[c];
    }
    if (gmin) {
      float a0 = 0.f, a1 = 0.f;
      for (size_t q = l16; q < Q; q += 16) {
        a0 += part_min[q * S1 + c];
        a1 += part_max[q * S1 + c];
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) {
        a0 += __shfl_xor(a0, o, 16);
        a1 += __shfl_xor(a1, o, 16);
      }
      if (l16 == 0) {
        if (adam) {
          // the bound's finished gradient -> Adam on the bound itself (fused step)
          const float g0 = gmin[c], g1 = gmax[c];
          const int64_t e0 = (gmin + c) - adam->g, e1 = (gmax + c) - adam->g;
          float p0 = adam->p[e0], m0 = adam->m[e0], v0 = adam->v[e0];
          float p1 = adam->p[e1], m1 = adam->m[e1], v1 = adam->v[e1];
          adam_step(*adam, 1.f, g0 + (a0 - gw), p0, m0, v0);
          adam_step(*adam, 1.f, g1 + (a1 + gw), p1, m1, v1);
          adam->p[e0] = p0;
          adam->m[e0] = m0;
          adam->v[e0] = v0;
          adam->p[e1] = p1;
          adam->m[e1] = m1;
          adam->v[e1] = v1;
          if (g0 != 0.f) gmin[c] = 0.f;
          if (g1 != 0.f) gmax[c] = 0.f;
        } else {
          gmin[c] += a0 - gw;
          gmax[c] += a1 + gw;
        }
      }
    }
  }
  __syncthreads();
  if (tid == 0 && loss) {
    float tot = 0.f;
    for (int zz = 0; zz < Z; ++zz) tot += red[zz];
    float smax = 0.f, smin = 0.f;
    for (int kk = 0; kk < S1; ++kk) {
      smax += smx[kk];
      smin += smn[kk];
    }
    *loss = tot + weight * (smax - smin);
  }
}

}  // namespace drpo
