// Micro-probe: the MLP tile's k-loop (8 waves, 16 rows x 256 cols x K=256) with
// its operand streams, to find what bounds it (MFMA alone runs at 32 cyc/MFMA).
//   P0 tile_dense_impl on the packed mirror (before packing it read W rows: 16 lines x
//      64 B per dwordx4 instruction and measured 68 cycles per MFMA)
//   P1 same k-loop, B from 1 KB lane-linear chunks (4 lines per instruction)
//   P2 same k-loop, B from registers (no global loads), A from LDS
// Build: hipcc -O3 --offload-arch=gfx950 -I ../../include -I ../../distributional-reachability-policy-optimization_amd/csrc -o load_probe load_probe.hip
#include "common.hpp"
#include <stdio.h>
using namespace drpo;

template <int MODE>
__global__ __launch_bounds__(512) void probe(const float* __restrict__ W, float* outg, unsigned long long* cyc, int reps) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* in = smem;
  float* out = smem + 16 * 264;
  for (int e = threadIdx.x; e < 16 * 264; e += 512) in[e] = 0.001f * (e & 255);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, l15 = lane & 15, g = lane >> 4;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float sink = 0.f;
  for (int r = 0; r < reps; ++r) {
    if (MODE == 0) {
      tile_dense_impl<8, 1, 2, ACT_NONE, 16>(in, 264, 256, W + r * 64, nullptr, 256, out, 264);
    } else {
      f32x4 acc[2] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
      f32x4 bq[4][2];
      const float* base = W + r * 64 + wave * 8192 + lane * 4;
#pragma unroll
      for (int u = 0; u < 3; ++u)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          bq[u][c] = MODE == 1 ? *reinterpret_cast<const f32x4*>(base + (u * 2 + c) * 256)
                               : f32x4{0.1f * u, 0.2f * c, 0.3f, 0.4f};
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        if (s + 3 < 16) {
#pragma unroll
          for (int c = 0; c < 2; ++c)
            bq[(s + 3) % 4][c] = MODE == 1 ? *reinterpret_cast<const f32x4*>(base + ((s + 3) * 2 + c) * 256)
                                           : f32x4{0.1f * s, 0.2f * c, 0.3f, 0.4f};
        }
        f32x4 a = *reinterpret_cast<const f32x4*>(in + l15 * 264 + 16 * s + 4 * g);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int c = 0; c < 2; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], bq[s % 4][c][m], acc[c], 0, 0, 0);
      }
      sink += acc[0][0] + acc[1][1];
    }
    __syncthreads();
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  outg[blockIdx.x * 512 + threadIdx.x] = out[threadIdx.x] + sink;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *W, *out;
  unsigned long long* cyc;
  (void)hipMalloc(&W, 1 << 24);
  (void)hipMemset(W, 0, 1 << 24);
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 256 * 8);
  unsigned long long h[256];
  const int reps = 16;
  const size_t lds = 2 * 16 * 264 * 4;
  const char* names[3] = {"P0 tile_dense (packed, lane-linear)", "P1 lane-linear B (4 lines/instr)", "P2 B in registers"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 3; ++rep) {
      if (mode == 0) probe<0><<<256, 512, lds>>>(W, out, cyc, reps);
      if (mode == 1) probe<1><<<256, 512, lds>>>(W, out, cyc, reps);
      if (mode == 2) probe<2><<<256, 512, lds>>>(W, out, cyc, reps);
      (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < 256; ++i) avg += h[i];
    avg /= 256;
    printf("%-36s %8.1f cycles per MFMA per SIMD (ideal 32)\n", names[mode], avg / reps / (2 * 128.0));
  }
  return 0;
}
