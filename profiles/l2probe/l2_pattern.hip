// L2 -> CU weight-stream probe: every CU (one 512-thread workgroup) streams the same
// 256 KB packed weight matrix (16 column blocks x 16 k-steps x 1 KB fragments) the
// way tile_dense does (wave w owns column blocks w and w+8, 4-deep register ring),
// in three address orders:
//   0: [cb][s] fragments (the current packed mirror: a k-step's 16 fragments 16 KB apart)
//   1: [s][cb] fragments (a k-step's 16 fragments contiguous)
//   2: [cb][s] with the k-loop of wave w rotated by w
// Prints bytes per clock per CU (2.4 GHz) for each order.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(512) void stream_kernel(const float* __restrict__ P, float* out, int reps, int rmask) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < reps; ++r) {
#pragma unroll
    for (int s0 = 0; s0 < 16; ++s0) {
      const int s = MODE == 2 ? ((s0 + w) & 15) : s0;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int cb = w + 8 * c;
        const int frag = MODE == 1 ? (s * 16 + cb) : (cb * 16 + s);
        // rmask == 0 at run time: the loads cannot be hoisted out of the rep loop
        const f32x4 v = *(const __attribute__((address_space(1))) f32x4*)(P + (frag + (r & rmask)) * 256 + lane * 4);
        acc += v;
      }
    }
  }
  if (acc[0] == 1234.5f) out[blockIdx.x * 512 + threadIdx.x] = acc[1] + acc[2] + acc[3];
}

template <int MODE>
float run(const float* P, float* out, int reps, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  stream_kernel<MODE><<<blocks, 512>>>(P, out, reps, 0);
  hipEventRecord(a);
  for (int i = 0; i < 10; ++i) stream_kernel<MODE><<<blocks, 512>>>(P, out, reps, 0);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0.f;
  hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}

int main() {
  const int n = 16 * 16 * 256;
  float *P, *out;
  hipMalloc(&P, n * sizeof(float));
  hipMalloc(&out, 256 * 512 * sizeof(float));
  std::vector<float> h(n, 0.001f);
  hipMemcpy(P, h.data(), n * sizeof(float), hipMemcpyHostToDevice);
  const int reps = 64, blocks = 256;
  const double bytes_per_cu = (double)reps * 256 * 1024;
  const char* names[3] = {"[cb][s] (current)", "[s][cb] contiguous k-step", "[cb][s] k-loop rotated by wave"};
  float t[3] = {run<0>(P, out, reps, blocks), run<1>(P, out, reps, blocks), run<2>(P, out, reps, blocks)};
  float t2[3] = {run<0>(P, out, reps, blocks), run<1>(P, out, reps, blocks), run<2>(P, out, reps, blocks)};
  for (int m = 0; m < 3; ++m) {
    const float ms = t[m] < t2[m] ? t[m] : t2[m];
    printf("%-34s %8.3f ms  %6.1f B/clk/CU\n", names[m], ms, bytes_per_cu / (ms * 1e-3 * 2.4e9));
  }
  hipFree(P);
  hipFree(out);
  return 0;
}
