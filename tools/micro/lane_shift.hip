// Check of the DPP / permlane lane shifts (iir.hpp wave_up<D>) against
// __shfl_up on gfx950: prints one line per D with the number of mismatching lanes.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../orion-sdr_amd/csrc/iir.hpp"

__global__ void k(const double* x, double* y) {
  const int l = threadIdx.x;
  const double v = x[l];
  y[0 * 64 + l] = orion::wave_up<1>(v);
  y[1 * 64 + l] = orion::wave_up<2>(v);
  y[2 * 64 + l] = orion::wave_up<4>(v);
  y[3 * 64 + l] = orion::wave_up<8>(v);
  y[4 * 64 + l] = orion::wave_up<16>(v);
  y[5 * 64 + l] = orion::wave_up<32>(v);
}

int main() {
  double h[64], o[384];
  for (int i = 0; i < 64; ++i) h[i] = 1000.0 + i + 1e-9 * i;
  double *dx, *dy;
  if (hipMalloc(&dx, sizeof h) || hipMalloc(&dy, sizeof o)) return 2;
  if (hipMemcpy(dx, h, sizeof h, hipMemcpyHostToDevice)) return 2;
  k<<<1, 64>>>(dx, dy);
  if (hipMemcpy(o, dy, sizeof o, hipMemcpyDeviceToHost)) return 2;
  int bad_total = 0;
  for (int s = 0; s < 6; ++s) {
    const int d = 1 << s;
    int bad = 0;
    for (int l = d; l < 64; ++l) bad += o[s * 64 + l] != h[l - d];
    printf("wave_up<%d>: %d mismatching lanes of %d\n", d, bad, 64 - d);
    bad_total += bad;
  }
  return bad_total ? 1 : 0;
}
