// Micro-probe: cycles per v_mfma_f32_16x16x4_f32 for the dependency shapes the
// MLP tile uses (8 waves / workgroup, one workgroup per CU, operands in VGPRs).
//   chains=2 grouped : acc0 x4, acc1 x4 (what hipcc emits for tile_dense)
//   chains=2 interl. : acc0, acc1, acc0, acc1, ...
//   chains=4 interl.
// Build: hipcc -O3 --offload-arch=gfx950 -o mfma_probe mfma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void probe(float* out, unsigned long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  float a = 0.001f * lane, b = 0.002f * lane;
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    if (MODE == 0) {
#pragma unroll
      for (int m = 0; m < 4; ++m) c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
#pragma unroll
      for (int m = 0; m < 4; ++m) c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
    } else if (MODE == 1) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  f32x4 s = c0 + c1 + c2 + c3;
  out[blockIdx.x * 512 + threadIdx.x] = s[0] + s[1] + s[2] + s[3];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, 256 * 512 * 4);
  hipMalloc(&cyc, 256 * 8);
  unsigned long long h[256];
  const int iters = 1000;
  const char* names[3] = {"2 chains grouped x4", "2 chains interleaved", "4 chains interleaved"};
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      if (mode == 0) probe<0><<<256, 512>>>(out, cyc, iters);
      if (mode == 1) probe<1><<<256, 512>>>(out, cyc, iters);
      if (mode == 2) probe<2><<<256, 512>>>(out, cyc, iters);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < 256; ++i) avg += h[i];
    avg /= 256;
    // per SIMD: 2 waves x 8 MFMAs per iteration
    printf("%-24s %8.1f cycles per MFMA per SIMD (ideal 32)\n", names[mode], avg / iters / 16.0);
  }
  return 0;
}
