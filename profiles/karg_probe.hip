// Kernel floor probe: per-launch time (HIP events over back-to-back launches) and
// per-kernel execution time (rocprofv3 --kernel-trace) of tiny kernels that differ
// only in kernarg size, how the kernarg is read, and their memory chain.
//   hipcc -O3 --offload-arch=gfx950 karg_probe.hip -o karg_probe && ./karg_probe
#include <hip/hip_runtime.h>
#include <cstdio>

struct Small { float* p; int n; };
struct Big { float* p; int n; long pad[400]; };   // ~3.2 KB, like the optimizer / wgrad kernargs

__global__ void k_empty(Small a) {
  if (a.n < 0) a.p[0] = 0.f;
}
__global__ void k_big_first(Big a) {   // reads a field at the start of the struct
  if (a.n < 0) a.p[0] = 0.f;
}
__global__ void k_big_dyn(Big a) {     // reads a field at a block-dependent offset
  if (a.pad[blockIdx.x % 400] == 12345) a.p[0] = 0.f;
}
__global__ void k_rmw(Small a) {       // one load -> one store per thread
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < a.n) a.p[i] = a.p[i] * 0.5f + 1.f;
}
__global__ void k_rmw_chain(Small a) { // load -> barrier -> store -> load -> store
  __shared__ float s[256];
  const int i = blockIdx.x * 256 + threadIdx.x;
  float v = i < a.n ? a.p[i] : 0.f;
  s[threadIdx.x] = v;
  __syncthreads();
  v += s[255 - threadIdx.x];
  if (i < a.n) a.p[i] = v;
  __syncthreads();
  if (i < a.n) a.p[i] = a.p[(i + 1) % a.n] + v;
}

template <typename F>
float time_us(F f, int n = 2000) {
  for (int i = 0; i < 50; ++i) f();
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
  float* p = nullptr;
  hipMalloc(&p, sizeof(float) * (1 << 22));
  hipMemset(p, 0, sizeof(float) * (1 << 22));
  Small s{p, 1 << 20};
  Big b{};
  b.p = p;
  b.n = 1 << 20;
  printf("empty 1 WG small kernarg      %.2f us/launch\n", time_us([&] { k_empty<<<1, 64>>>(s); }));
  printf("empty 256 WG small kernarg    %.2f us/launch\n", time_us([&] { k_empty<<<256, 256>>>(s); }));
  printf("big kernarg 1 WG              %.2f us/launch\n", time_us([&] { k_big_first<<<1, 64>>>(b); }));
  printf("big kernarg 256 WG            %.2f us/launch\n", time_us([&] { k_big_first<<<256, 256>>>(b); }));
  printf("big kernarg dyn read 256 WG   %.2f us/launch\n", time_us([&] { k_big_dyn<<<256, 256>>>(b); }));
  printf("rmw 1 WG                      %.2f us/launch\n", time_us([&] { k_rmw<<<1, 256>>>(s); }));
  printf("rmw 4096 WG (4 MB)            %.2f us/launch\n", time_us([&] { k_rmw<<<4096, 256>>>(s); }));
  printf("rmw chain 1 WG                %.2f us/launch\n", time_us([&] { k_rmw_chain<<<1, 256>>>(s); }));
  printf("rmw chain 4096 WG             %.2f us/launch\n", time_us([&] { k_rmw_chain<<<4096, 256>>>(s); }));
  hipFree(p);
  return 0;
}
