// Packed weight mirrors for the MFMA tile (see tile_dense in common.hpp).
//
// drpo_pack_weights rewrites PyTorch-layout weights W [nbatch][dout][din]
// (nn.Linear / BatchedLinear, src/torch_util.py:190-211, src/dynamics.py:26-52)
// into the fragment-linear layouts the kernels stream:
//   P  (forward,  y = x W^T):  P [(cb*NKS + s)*256 + 4*l + i] = W[16cb + (l&15)][16s + 4(l>>4) + i]
//   PT (backward, dx = dz W):  PT[(cb*NKS'+ s)*256 + 4*l + i] = W[16s + 4(l>>4) + i][16cb + (l&15)]
// with zero padding outside [dout) x [din). One launch packs every layer of a
// parameter group (all ensemble members); it runs after each optimizer / EMA
// step of the group (HBM-bound: reads + writes ~2x the group bytes).
#include "common.hpp"

using namespace drpo;

namespace {
constexpr int PACK_MAX = 16;
}

struct PackArgs {
  drpo_pack_item_t it[PACK_MAX];
  int64_t first[PACK_MAX + 1];
  int n;
};

__global__ __launch_bounds__(256) void pack_kernel(PackArgs a) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= a.first[a.n]) return;
  int q = 0;
  while (q + 1 < a.n && t >= a.first[q + 1]) ++q;
  const drpo_pack_item_t& I = a.it[q];
  const int ncb = (I.dout + 15) >> 4, nks = (I.din + 15) >> 4;
  const int64_t per = (int64_t)ncb * nks * 64;
  int64_t loc = t - a.first[q];
  const int z = (int)(loc / per);
  loc -= (int64_t)z * per;
  const int lane = (int)(loc & 63), l15 = lane & 15, g = lane >> 4;
  const int64_t frag = loc >> 6;
  const float* W = I.W + (size_t)z * I.wstride;
  if (I.P) {   // forward fragment (cb over dout, s over din)
    const int cb = (int)(frag / nks), s = (int)(frag % nks);
    const int o = 16 * cb + l15;
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = 16 * s + 4 * g + i;
      v[i] = (o < I.dout && k < I.din) ? W[(size_t)o * I.din + k] : 0.f;
    }
    *reinterpret_cast<f32x4*>(I.P + (size_t)z * I.pstride + (frag << 8) + 4 * lane) = v;
  }
  if (I.PT) {  // transposed fragment (cb over din, s over dout): same count
    const int cb = (int)(frag / ncb), s = (int)(frag % ncb);
    const int k = 16 * cb + l15;
    f32x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int o = 16 * s + 4 * g + i;
      v[i] = (o < I.dout && k < I.din) ? W[(size_t)o * I.din + k] : 0.f;
    }
    *reinterpret_cast<f32x4*>(I.PT + (size_t)z * I.ptstride + (frag << 8) + 4 * lane) = v;
  }
}

DRPO_API int64_t drpo_packed_size(int din, int dout) {
  return (int64_t)((dout + 15) >> 4) * ((din + 15) >> 4) * 256;
}

DRPO_API int drpo_pack_weights(const drpo_pack_item_t* items, int n, drpo_stream_t stream_) {
  hipStream_t stream = (hipStream_t)stream_;
  DRPO_REQUIRE(n >= 0 && n <= PACK_MAX, "drpo_pack_weights: at most %d items", PACK_MAX);
  PackArgs a{};
  int64_t tot = 0;
  for (int k = 0; k < n; ++k) {
    const drpo_pack_item_t& I = items[k];
    DRPO_REQUIRE(I.W && (I.P || I.PT) && I.din >= 1 && I.dout >= 1 && I.nbatch >= 1, "drpo_pack_weights: bad item %d",
                 k);
    const int64_t sz = drpo_packed_size(I.din, I.dout);
    DRPO_REQUIRE(I.nbatch == 1 || ((!I.P || I.pstride >= sz) && (!I.PT || I.ptstride >= sz)),
                 "drpo_pack_weights: item %d stride too small", k);
    a.it[k] = I;
    a.first[k] = tot;
    tot += sz / 4 * I.nbatch;
  }
  a.first[n] = tot;
  a.n = n;
  if (tot == 0) return DRPO_OK;
  pack_kernel<<<(unsigned)((tot + 255) / 256), 256, 0, stream>>>(a);
  DRPO_LAUNCH_CHECK("pack_weights");
  return DRPO_OK;
}
