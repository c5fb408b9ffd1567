// membench.hip — read-path micro-benchmark for the WBFM front's access pattern
// (not part of the product). Each variant streams the same 512 MiB cf32 buffer
// once and reports GB/s; the reduction result is written so nothing is elided.
//   hipcc -O3 --offload-arch=gfx950 scripts/membench.hip -o /tmp/membench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);      \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

// Grid-stride f4 read, 256-thread blocks.
__global__ __launch_bounds__(256) void k_stride(const f4* __restrict__ x, long long n4, float* out) {
  f4 acc = {0, 0, 0, 0};
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256)
    acc += x[i];
  if (acc.x + acc.y + acc.z + acc.w == 12345.0f) out[0] = acc.x;
}

// One wave per block, contiguous range per wave, KL f4 loads per lane per tile
// (a tile = 64*KL f4), loads for tile n+1 issued before tile n is consumed.
// STAGE: also scatter every sample into LDS like the polyphase staging.
// WR: 0 no output, 1 two floats per lane per tile (lane-contiguous float2),
// 2 the same with nontemporal stores, 3 one float4 per lane every other tile,
// 4 outputs kept in LDS and written after the wave's last load.
// NTL: nontemporal input loads.
template <int KL, bool STAGE, int WR = 0, bool NTL = false>
__global__ __launch_bounds__(64) void k_range(const f4* __restrict__ x, long long tiles_per_wave,
                                              float* out, f2* __restrict__ y = nullptr) {
  __shared__ f2 U[STAGE ? 8 * (KL * 16 + 18) + 64 : 1];
  __shared__ f2 Yl[WR == 4 ? 64 * 16 : 1];
  const int l = threadIdx.x;
  const f4* p = x + blockIdx.x * tiles_per_wave * 64 * KL;
  f4 v[KL];
#pragma unroll
  for (int k = 0; k < KL; ++k) v[k] = NTL ? __builtin_nontemporal_load(p + l + 64 * k) : p[l + 64 * k];
  f4 acc = {0, 0, 0, 0};
  for (long long n = 0; n < tiles_per_wave; ++n) {
    f4 cur[KL];
#pragma unroll
    for (int k = 0; k < KL; ++k) cur[k] = v[k];
    asm volatile("" ::: "memory");
    if (n + 1 < tiles_per_wave) {
      const f4* q = p + (n + 1) * 64 * KL;
#pragma unroll
      for (int k = 0; k < KL; ++k) v[k] = NTL ? __builtin_nontemporal_load(q + l + 64 * k) : q[l + 64 * k];
    }
    if constexpr (WR == 4) {
      Yl[(n & 15) * 64 + l] = f2{cur[0].x, cur[1].y};
    } else if constexpr (WR == 1) {
      y[(blockIdx.x * tiles_per_wave + n) * 64 + l] = f2{cur[0].x, cur[1].y};
    } else if constexpr (WR == 2) {
      __builtin_nontemporal_store(f2{cur[0].x, cur[1].y}, y + (blockIdx.x * tiles_per_wave + n) * 64 + l);
    } else if constexpr (WR == 3) {
      if (n & 1)
        reinterpret_cast<f4*>(y)[(blockIdx.x * tiles_per_wave + n) / 2 * 64 + l] =
            f4{cur[0].x, cur[1].y, cur[2].x, cur[3].y};
    }
    if constexpr (STAGE) {
      const int c0 = (-2 * l) & 7, c1 = (-2 * l - 1) & 7;
      const int LR = KL * 16 + 18;
      const int s0 = c0 * LR + (128 + 2 * l + c0) / 8, s1 = c1 * LR + (128 + 2 * l + 1 + c1) / 8;
#pragma unroll
      for (int k = 0; k < KL; ++k) {
        U[s0 + 16 * k] = f2{cur[k].x, cur[k].y};
        U[s1 + 16 * k] = f2{cur[k].z, cur[k].w};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const f4 w = *reinterpret_cast<const f4*>(U + 2 * l);
      acc += w;
    } else {
#pragma unroll
      for (int k = 0; k < KL; ++k) acc += cur[k];
    }
  }
  if constexpr (WR == 4) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int n = 0; n < tiles_per_wave && n < 16; ++n)
      y[(blockIdx.x * tiles_per_wave + n) * 64 + l] = Yl[n * 64 + l];
  }
  if (acc.x + acc.y + acc.z + acc.w == 12345.0f) out[0] = acc.x;
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

template <int KL, bool STAGE, int WR = 0, bool NTL = false>
void run_range(const f4* x, long long n4, float* out, int waves_per_cu, int ncu, f2* y = nullptr) {
  const long long tile = 64LL * KL;
  long long waves = (long long)waves_per_cu * ncu;
  long long tpw = (n4 / tile + waves - 1) / waves;
  waves = n4 / (tile * tpw);  // full tiles only
  const double bytes = (double)waves * tpw * tile * 16;
  const float ms = timeit([&] { k_range<KL, STAGE, WR, NTL><<<waves, 64>>>(x, tpw, out, y); }, 20);
  printf("range NTL=%d KL=%2d stage=%d wr=%d waves/CU=%2d tiles/wave=%4lld : %7.1f us  %6.2f TB/s (reads)\n", NTL, KL,
         STAGE, WR, waves_per_cu, tpw, ms * 1e3, bytes / ms / 1e9);
}

int main() {
  const long long n = 1LL << 26;  // cf32 samples
  const long long n4 = n / 2;
  f4* x;
  float* out;
  CK(hipMalloc(&x, n * 8));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(x, 0, n * 8));
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  f2* y;
  CK(hipMalloc(&y, n));  // n/8 f2 = one float2 per 8 samples... sized generously
  for (int w : {16}) {
    run_range<8, true, 0>(x, n4, out, w, ncu, y);
    run_range<8, true, 1>(x, n4, out, w, ncu, y);
    run_range<8, true, 2>(x, n4, out, w, ncu, y);
    run_range<8, true, 3>(x, n4, out, w, ncu, y);
    run_range<8, false, 1>(x, n4, out, w, ncu, y);
    run_range<8, true, 0, true>(x, n4, out, w, ncu, y);
    run_range<8, true, 1, true>(x, n4, out, w, ncu, y);
    run_range<8, true, 2, true>(x, n4, out, w, ncu, y);
    run_range<8, true, 4, false>(x, n4, out, w, ncu, y);
    run_range<8, true, 4, true>(x, n4, out, w, ncu, y);
    run_range<8, true, 0>(x, n4, out, w, ncu, y);
  }
  return 0;
  for (int g : {1024, 2048, 4096}) {
    const float ms = timeit([&] { k_stride<<<g, 256>>>(x, n4, out); }, 20);
    printf("stride grid=%d : %7.1f us  %6.2f TB/s\n", g, ms * 1e3, n * 8.0 / ms / 1e9);
  }
  for (int w : {4, 8, 16}) run_range<8, false>(x, n4, out, w, ncu);
  for (int w : {4, 6, 8}) run_range<24, false>(x, n4, out, w, ncu);
  for (int w : {8, 16}) run_range<8, true>(x, n4, out, w, ncu);
  for (int w : {4, 6}) run_range<24, true>(x, n4, out, w, ncu);
  for (int w : {8}) run_range<16, false>(x, n4, out, w, ncu);
  for (int w : {8}) run_range<16, true>(x, n4, out, w, ncu);
  return 0;
}
