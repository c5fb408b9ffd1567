// Microbenchmark: VALU issue rate of v_pk_fma_f32 vs v_fma_f32 on gfx950 at
// 1..4 waves per SIMD (grid = 256 CUs x 4 SIMDs x w waves). 8 independent
// accumulator chains per lane, 64 instructions per loop iteration.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <bool PK>
__global__ __launch_bounds__(256) void k(float* out, int iters, float s) {
  f2 a[8];
  for (int i = 0; i < 8; ++i) a[i] = f2{s * (threadIdx.x + i), s * i};
  const f2 b = f2{1.0001f, 0.9999f}, c = f2{1e-7f, 2e-7f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (PK) {
          asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        } else {
          asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i].x) : "v"(b.x), "v"(c.x));
        }
      }
    }
  }
  float acc = 0;
  for (int i = 0; i < 8; ++i) acc += a[i].x + a[i].y;
  if (acc == 12345.f) out[0] = acc;
}

int main() {
  float* out;
  hipMalloc(&out, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  for (int pk = 0; pk < 2; ++pk)
    for (int w = 1; w <= 4; w *= 2) {
      // one 64-thread block per (CU, SIMD, wave): 1024*w blocks of 64 threads
      dim3 grid(1024 * w), blk(64);
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(e0);
        if (pk) hipLaunchKernelGGL(k<true>, grid, blk, 0, 0, out, iters, 1.0f);
        else hipLaunchKernelGGL(k<false>, grid, blk, 0, 0, out, iters, 1.0f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double inst = 64.0 * iters * 1024 * w;  // wave-instructions
        const double per_simd = inst / 1024;
        if (rep) printf("%s waves/SIMD=%d: %.3f ms, %.2f ns per wave-instr per SIMD, %.1f TFLOP/s\n",
                        pk ? "v_pk_fma_f32" : "v_fma_f32   ", w, ms, ms * 1e6 / per_simd,
                        inst * 64 * (pk ? 4 : 2) / (ms * 1e-3) / 1e12);
      }
    }
  return 0;
}
