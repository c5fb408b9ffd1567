// Microbenchmark: dependent-chain cost of v_pk_fma_f32 on gfx950 — C independent
// accumulator chains per lane, W waves per SIMD (1024*W one-wave blocks).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int C>
__global__ __launch_bounds__(64) void k(float* out, int iters, float s) {
  f2 a[C];
  for (int i = 0; i < C; ++i) a[i] = f2{s * (threadIdx.x + i), s * i};
  const f2 b = f2{1.0001f, 0.9999f}, c = f2{1e-7f, 2e-7f};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 64 / C; ++r)
#pragma unroll
      for (int i = 0; i < C; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
  }
  float acc = 0;
  for (int i = 0; i < C; ++i) acc += a[i].x + a[i].y;
  if (acc == 12345.f) out[0] = acc;
}

template <int C>
void run(float* out, int w) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  float best = 1e9;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k<C>, dim3(1024 * w), dim3(64), 0, 0, out, iters, 1.0f);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  const double per_simd = 64.0 * iters * w;  // wave-instructions per SIMD
  printf("chains=%d waves/SIMD=%d: %.2f ns per wave-instr per SIMD\n", C, w, best * 1e6 / per_simd);
}

int main() {
  float* out;
  hipMalloc(&out, 4);
  for (int w = 1; w <= 2; ++w) {
    run<1>(out, w);
    run<2>(out, w);
    run<4>(out, w);
    run<8>(out, w);
  }
  return 0;
}
