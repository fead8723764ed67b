// Layer probe: what bounds tile_dense (csrc/common.hpp), the MLP layer core of every
// SAC / fit / rollout kernel? Each workgroup (8 waves) runs NL back-to-back 256x256
// layers (ReLU) on an RB*16-row tile held in LDS, weights streamed from L2 (NW_L
// distinct packed layers, 256 KB each, shared by every workgroup). Variants differ in
// rows per tile (RB), workgroups per CU (LDS padding + waves-per-EU register budget)
// and grid size; each prints TFLOP/s over back-to-back launches (HIP events).
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -I include \
//     -I distributional-reachability-policy-optimization_amd/csrc profiles/layer_probe.hip -o profiles/layer_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "common.hpp"

using namespace drpo;

void drpo_set_error(const char*, ...) {}

constexpr int LD = 264;
constexpr int NW_L = 4;   // distinct weight layers (1 MB: L2-resident)

template <int RB, int WPE, int NL, int SV = 0>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void layers_kernel(
    const float* __restrict__ P, const float* __restrict__ bias, float* out, float* save) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int ROWS = 16 * RB;
  float* a = smem;
  float* b = smem + ROWS * LD;
  for (int e = threadIdx.x; e < ROWS * LD; e += 512) a[e] = 0.001f * (float)((e * 7 + blockIdx.x) & 63);
  lds_barrier();
#pragma unroll 1
  for (int l = 0; l < NL; ++l) {
    const float* W = P + (size_t)(l % NW_L) * 65536;
    // SV: the epilogue's global saves of the post- (1) and pre-activation (2) for the
    // backward pass, one [ROWS][256] slab per workgroup and layer (as GSave in the SAC)
    float* sl = save + ((size_t)blockIdx.x * NL + l) * 2 * ROWS * 256;
    const GSave gs{SV >= 1 ? sl : nullptr, SV >= 2 ? sl + ROWS * 256 : nullptr, 256, ROWS};
    tile_dense_impl<8, RB, 2, ACT_RELU, 16>(a, LD, 256, W, bias, 256, b, LD, gs);
    lds_barrier();
    float* t = a; a = b; b = t;
  }
  if (threadIdx.x == 0) out[blockIdx.x] = a[5];
}

float* g_save = nullptr;

template <int RB, int WPE, int SV = 0>
void run(const char* name, int grid, size_t lds_extra, const float* P, const float* bias, float* out) {
  constexpr int NL = 16;
  const size_t lds = sizeof(float) * 2 * 16 * RB * LD + lds_extra;
  auto launch = [&] { layers_kernel<RB, WPE, NL, SV><<<grid, 512, lds>>>(P, bias, out, g_save); };
  for (int i = 0; i < 20; ++i) launch();
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int n = 200;
  hipEventRecord(e0, 0);
  for (int i = 0; i < n; ++i) launch();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1000.0 / n;
  const double flop = 2.0 * grid * 16 * RB * NL * 256.0 * 256.0;
  printf("%-44s grid %5d lds %6zu B  %8.2f us/launch  %6.1f TFLOP/s  %6.2f us/layer\n", name, grid, lds, us,
         flop / (us * 1e-6) / 1e12, us / NL);
  hipError_t err = hipGetLastError();
  if (err != hipSuccess) printf("  error: %s\n", hipGetErrorString(err));
}

int main() {
  float *P, *bias, *out;
  hipMalloc(&P, sizeof(float) * 65536 * NW_L);
  hipMalloc(&bias, sizeof(float) * 256);
  hipMalloc(&out, sizeof(float) * 8192);
  std::vector<float> h(65536 * NW_L);
  for (size_t i = 0; i < h.size(); ++i) h[i] = 0.01f * (float)((int)(i * 2654435761u >> 24) - 128) / 128.f;
  hipMemcpy(P, h.data(), sizeof(float) * h.size(), hipMemcpyHostToDevice);
  hipMemset(bias, 0, sizeof(float) * 256);
  hipMalloc(&g_save, sizeof(float) * (size_t)1024 * 16 * 2 * 32 * 256);   // 1 GB: every variant's slabs
  // global saves of every layer's output (the SAC forward's GSave), 16-row tiles
  run<1, 2, 1>("RB1 1 WG/CU, save y", 256, 100000 - 2 * 16 * LD * 4, P, bias, out);
  run<1, 2, 2>("RB1 1 WG/CU, save y + z", 256, 100000 - 2 * 16 * LD * 4, P, bias, out);
  run<1, 4, 1>("RB1 2 WG/CU, save y", 512, 76000 - 2 * 16 * LD * 4, P, bias, out);
  run<1, 4, 2>("RB1 2 WG/CU, save y + z", 512, 76000 - 2 * 16 * LD * 4, P, bias, out);
  run<2, 4, 1>("RB2 2 WG/CU, save y", 512, 0, P, bias, out);
  // 16-row tiles
  run<1, 2>("RB1 1 WG/CU (pad to 100 KB)", 256, 100000 - 2 * 16 * LD * 4, P, bias, out);
  run<1, 4>("RB1 2 WG/CU (76 KB, the SAC forward)", 512, 76000 - 2 * 16 * LD * 4, P, bias, out);
  run<1, 4>("RB1 2 WG/CU, 2x grid", 1024, 76000 - 2 * 16 * LD * 4, P, bias, out);
  run<1, 6>("RB1 3 WG/CU (80 VGPR)", 768, 0, P, bias, out);
  run<1, 8>("RB1 4 WG/CU (64 VGPR)", 1024, 0, P, bias, out);
  // 32-row tiles
  run<2, 2>("RB2 1 WG/CU (pad to 100 KB)", 256, 100000 - 2 * 32 * LD * 4, P, bias, out);
  run<2, 4>("RB2 2 WG/CU (68 KB)", 512, 0, P, bias, out);
  run<2, 4>("RB2 2 WG/CU, 2x grid", 1024, 0, P, bias, out);
  run<2, 6>("RB2 3 WG/CU? (80 VGPR, LDS 2 fit)", 768, 0, P, bias, out);
  return 0;
}
