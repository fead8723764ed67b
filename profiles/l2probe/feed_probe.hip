// Weight-feed probe for the rollout's 200-wide phases: 8 waves (2 per SIMD), 16 rows,
// K = 208 (13 k-steps of 16), every workgroup streaming the same L2-resident packed
// fragments (1 KB per column block and k-step). Waves 0-3 own NH column blocks, waves 4-7
// NL (the paired heads: 4 / 3, i.e. 7 blocks per SIMD).
//   M0  register ring, MFMA        (production form)
//   M1  MFMA only, B from registers (matrix-pipe floor)
//   M2  register ring, no MFMA      (feed alone)
//   M3  global_load_lds ring (per-wave LDS slots, counted vmcnt), ds_read + MFMA
// Each pass ends at a workgroup barrier, as a layer phase does (a raw s_barrier). Prints cycles per pass
// (s_memtime), the SIMD's MFMA floor over that and B/clk per CU.
// Build (in profiles/l2probe): hipcc -O3 --offload-arch=gfx950 -o feed_probe feed_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int KS = 13, LDA = 264, NBMAX = 4, UNR = 8;   // passes per launch (unrolled)
constexpr int RING_OFF = 16 * LDA;   // floats: activation tile, then the LDS rings

__device__ __forceinline__ f32x4 ldg(const float* p) {
  return *(const __attribute__((address_space(1))) f32x4*)p;
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  // gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt[5:4] at [15:14]
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// One wave's passes. The ring persists across passes: the next pass's first PF - 1
// k-steps are issued before the barrier that ends a pass (the kernels' cross-phase
// prefetch), and sched_barrier pins each k-step's load issue ahead of its MFMAs.
template <int MODE, int PF, int NB>
__device__ __forceinline__ void body(const float* W, float* smem, int wave, int lane, f32x4* acc, int reps,
                                     int rmask) {
  const int l15 = lane & 15, g = lane >> 4;
  auto frag = [&](int r, int c, int s) { return W + (r & rmask) * 64 + lane * 4 + ((wave + 8 * c) * KS + s) * 256; };
  float* ring = smem + RING_OFF + wave * PF * NBMAX * 256;
  auto issue = [&](int r, int s) {
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      if constexpr (MODE == 3)
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)frag(r, c, s),
                                         (__attribute__((address_space(3))) void*)(ring + ((s % PF) * NBMAX + c) * 256), 16, 0, 0);
    }
  };
  f32x4 bq[PF][NB];
  if constexpr (MODE == 0 || MODE == 2) {
#pragma unroll
    for (int u = 0; u < PF - 1; ++u)
#pragma unroll
      for (int c = 0; c < NB; ++c) bq[u][c] = ldg(frag(0, c, u));
  } else if constexpr (MODE == 3) {
#pragma unroll
    for (int u = 0; u < PF - 1; ++u) issue(0, u);
  }
  // passes unrolled (a loop back-edge would make the compiler drain the ring at its head)
#pragma unroll
  for (int r = 0; r < UNR; ++r) {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int sn = s + PF - 1;   // the k-step issued now: this pass's, or the next pass's prologue
      if constexpr (MODE == 0 || MODE == 2) {
        if (sn < KS) {
#pragma unroll
          for (int c = 0; c < NB; ++c) bq[sn % PF][c] = ldg(frag(r, c, sn));
        }
      } else if constexpr (MODE == 3) {
        if (sn < KS) issue(r, sn);
      }
      __builtin_amdgcn_sched_barrier(0);
      f32x4 b[NB];
      if constexpr (MODE == 3) {
        if (sn < KS) wait_vm<(PF - 1) * NB>();
        else if (KS - 1 - s == 2) wait_vm<2 * NB>();
        else if (KS - 1 - s == 1) wait_vm<NB>();
        else wait_vm<0>();
#pragma unroll
        for (int c = 0; c < NB; ++c) b[c] = *reinterpret_cast<const f32x4*>(ring + ((s % PF) * NBMAX + c) * 256 + lane * 4);
      } else if constexpr (MODE == 1) {
#pragma unroll
        for (int c = 0; c < NB; ++c) b[c] = f32x4{0.5f + 0.1f * c, 0.25f, 0.125f, 0.0625f};
      } else {
#pragma unroll
        for (int c = 0; c < NB; ++c) b[c] = bq[s % PF][c];
      }
      if constexpr (MODE == 2) {
#pragma unroll
        for (int c = 0; c < NB; ++c) acc[c] += b[c];
      } else {
        const f32x4 a = *reinterpret_cast<const f32x4*>(smem + l15 * LDA + 16 * s + 4 * g);
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int c = 0; c < NB; ++c)
            acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[m], b[c][m], acc[c], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // the next pass's first k-steps, then the barrier that ends this pass
    if (r + 1 < UNR) {
      if constexpr (MODE == 0 || MODE == 2) {
#pragma unroll
        for (int u = 0; u < PF - 1; ++u)
#pragma unroll
          for (int c = 0; c < NB; ++c) bq[u][c] = ldg(frag(r + 1, c, u));
      } else if constexpr (MODE == 3) {
        // an LDS-DMA in flight across __syncthreads() would be drained by it: raw barrier
#pragma unroll
        for (int u = 0; u < PF - 1; ++u) issue(r + 1, u);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int MODE, int PF, int NH, int NL>
__global__ __launch_bounds__(512) void feed(const float* __restrict__ W, float* outg, unsigned long long* cyc,
                                            int reps, int rmask) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  for (int e = threadIdx.x; e < 16 * LDA; e += 512) smem[e] = 0.001f * (e & 255);
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  f32x4 acc[NBMAX];
#pragma unroll
  for (int c = 0; c < NBMAX; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (wave < 4) body<MODE, PF, NH>(W, smem, wave, lane, acc, reps, rmask);
  else body<MODE, PF, NL>(W, smem, wave, lane, acc, reps, rmask);
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float sink = 0.f;
#pragma unroll
  for (int c = 0; c < NBMAX; ++c) sink += acc[c][0] + acc[c][3];
  outg[blockIdx.x * 512 + threadIdx.x] = sink;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int PF, int NH, int NL>
void run(const char* name, const float* W, float* out, unsigned long long* cyc, int reps) {
  const size_t lds = (16 * LDA + (MODE == 3 ? 8 * PF * NBMAX * 256 : 0)) * sizeof(float);
  unsigned long long h[256];
  double best = 1e30;
  for (int it = 0; it < 3; ++it) {
    feed<MODE, PF, NH, NL><<<256, 512, lds>>>(W, out, cyc, reps, 0);
    (void)hipDeviceSynchronize();
    (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    double avg = 0;
    for (int i = 0; i < 256; ++i) avg += (double)h[i];
    avg /= 256.0 * UNR;
    if (avg < best) best = avg;
  }
  const double bytes = 4.0 * (NH + NL) * KS * 1024, floor_cyc = (NH + NL) * KS * 4 * 32.0;
  printf("%-40s %8.0f cycles per pass  floor/pass %.2f  %5.1f B/clk/CU\n", name, best, floor_cyc / best, bytes / best);
}

int main() {
  float *W, *out;
  unsigned long long* cyc;
  (void)hipMalloc(&W, 1 << 20);
  (void)hipMemset(W, 0, 1 << 20);
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 256 * 8);
  const int reps = UNR;
  run<1, 4, 4, 4>("M1 4/4 MFMA only", W, out, cyc, reps);
  run<2, 4, 4, 4>("M2 4/4 register ring 4, no MFMA", W, out, cyc, reps);
  run<0, 4, 4, 4>("M0 4/4 register ring 4 + MFMA", W, out, cyc, reps);
  run<0, 2, 4, 4>("M0 4/4 register ring 2 + MFMA", W, out, cyc, reps);
  run<3, 4, 4, 4>("M3 4/4 LDS-DMA ring 4 + MFMA", W, out, cyc, reps);
  run<3, 2, 4, 4>("M3 4/4 LDS-DMA ring 2 + MFMA", W, out, cyc, reps);
  run<1, 4, 4, 3>("M1 4/3 MFMA only", W, out, cyc, reps);
  run<0, 4, 4, 3>("M0 4/3 register ring 4 + MFMA", W, out, cyc, reps);
  run<3, 4, 4, 3>("M3 4/3 LDS-DMA ring 4 + MFMA", W, out, cyc, reps);
  run<0, 4, 2, 2>("M0 2/2 register ring 4 + MFMA", W, out, cyc, reps);
  run<1, 4, 2, 2>("M1 2/2 MFMA only", W, out, cyc, reps);
  return 0;
}
