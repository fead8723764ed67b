// Dependent scalar-load chains through the kernarg segment vs through a device buffer:
// per-workgroup s_memtime cycles from kernel entry until a 3-level chain (unit ->
// item index -> item fields -> a field they select) is resolved, at the weight-gradient
// launch's shape (a ~3.3 KB argument block, 420-448 workgroups of 256 threads).
//   hipcc -O3 --offload-arch=gfx950 kchain_probe.hip -o kchain_probe && ./kchain_probe
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

struct Args {
  long first[16];
  long pad[390];
  unsigned long long* out;
};
typedef const __attribute__((address_space(4))) Args ArgsK;

__device__ __forceinline__ unsigned long long memtime() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// MODE 0: fields read in place from the kernarg segment; 1: from the device copy `g`
template <int MODE>
__global__ __launch_bounds__(256) void chain(Args a, const Args* __restrict__ g) {
  (void)a;
  ArgsK& ka = *(ArgsK*)__builtin_amdgcn_kernarg_segment_ptr();
  const unsigned long long t0 = memtime();
  // an opaque zero defined after the first stamp: every load's address depends on it, so
  // none can be hoisted above the stamp (kernarg loads are invariant otherwise)
  int zr = 0;
  asm volatile("s_mov_b32 %0, 0" : "=s"(zr)::"memory");
  const long b = blockIdx.x;
  int q = 0;
#pragma unroll
  for (int i = 1; i < 16; ++i) q += b >= (MODE == 0 ? ka.first[i + zr] : g->first[i + zr]) ? 1 : 0;
  const long v = MODE == 0 ? ka.pad[q * 20 + 7] : g->pad[q * 20 + 7];
  const long w = MODE == 0 ? ka.pad[330 + (v & 31)] : g->pad[330 + (v & 31)];
  const unsigned long long t1 = memtime();
  unsigned long long* out = MODE == 0 ? ka.out : g->out;
  if (threadIdx.x == 0) {
    out[2 * b] = t1 - t0;
    out[2 * b + 1] = (unsigned long long)w;
  }
}

template <typename F>
float time_us(F f, int n = 500) {
  for (int i = 0; i < 20; ++i) f();
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, 0);
  for (int i = 0; i < n; ++i) f();
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms = 0.f;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / n;
}

int main() {
  const int nb = 448;
  Args a{};
  for (int i = 0; i < 16; ++i) a.first[i] = i * 28;
  for (int i = 0; i < 390; ++i) a.pad[i] = i * 7 + 3;
  unsigned long long* out = nullptr;
  hipMalloc(&out, sizeof(unsigned long long) * 2 * nb);
  a.out = out;
  Args* g = nullptr;
  hipMalloc(&g, sizeof(Args));
  hipMemcpy(g, &a, sizeof(Args), hipMemcpyHostToDevice);
  std::vector<unsigned long long> h(2 * nb);
  for (int mode = 0; mode < 2; ++mode) {
    for (int grid : {1, 64, nb}) {
      auto launch = [&] {
        if (mode == 0) chain<0><<<grid, 256>>>(a, g);
        else chain<1><<<grid, 256>>>(a, g);
      };
      const float us = time_us(launch);
      launch();
      hipDeviceSynchronize();
      hipMemcpy(h.data(), out, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost);
      std::vector<unsigned long long> d(grid);
      double sum = 0;
      for (int b = 0; b < grid; ++b) { d[b] = h[2 * b]; sum += (double)d[b]; }
      std::sort(d.begin(), d.end());
      printf("%-14s grid %4d: chain cycles mean %8.0f min %8llu p50 %8llu max %8llu | %.2f us/launch\n",
             mode == 0 ? "kernarg" : "device buffer", grid, sum / grid, d[0], d[grid / 2], d[grid - 1], us);
    }
  }
  hipFree(out);
  hipFree(g);
  return 0;
}
