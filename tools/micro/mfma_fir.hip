// Micro check: (1) the operand/result lane maps of v_mfma_f32_16x16x32_f16 with exact
// integer data; (2) a 125-tap real FIR over 1024 outputs as a Toeplitz product on it,
// with the data and taps split into f16 hi + lo parts (three products), against an
// f64 reference: max relative error per output. hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

// (1) D = A B, A 16x32, B 32x16 (row-major in memory), the assumed maps:
// lane l: A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]; D[4(l>>4)+r][l&15].
__global__ void k_map(const float* A, const float* B, float* D) {
  const int l = threadIdx.x;
  h8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = (_Float16)A[(l & 15) * 32 + 8 * (l >> 4) + j];
    b[j] = (_Float16)B[(8 * (l >> 4) + j) * 16 + (l & 15)];
  }
  f4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

// (2) y[o] = sum_k a[k] f[o - k], o in [0, 1024), f[-128..1024+16) in fimg (index + 128).
// Group g (256 outputs o = 256 g + 16 J + I): window w0 = 256 g + 16 J - 128, K = 160:
// A[I][kap] = a[I + 128 - kap] (0 outside [0, 124]), B[kap][J] = f[w0 + kap].
// ah/al: per step s, lane l, the 8 A elements (host-built). fh/fl: f16 planes of f*2^sf.
__global__ void k_fir(const h8* __restrict__ ah, const h8* __restrict__ al, const _Float16* __restrict__ fh,
                      const _Float16* __restrict__ fl, float* __restrict__ y, float unscale) {
  const int l = threadIdx.x;
  const int J = l & 15, kg = l >> 4;
  f4 acc[4];
  for (int g = 0; g < 4; ++g) acc[g] = f4{0, 0, 0, 0};
  for (int s = 0; s < 5; ++s) {
    const h8 a_h = ah[s * 64 + l], a_l = al[s * 64 + l];
    for (int g = 0; g < 4; ++g) {
      const int base = 256 * g + 16 * J - 128 + 32 * s + 8 * kg + 128;  // image index
      h8 bh, bl;
      for (int j = 0; j < 8; ++j) {
        bh[j] = fh[base + j];
        bl[j] = fl[base + j];
      }
      acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_h, bh, acc[g], 0, 0, 0);
      acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_h, bl, acc[g], 0, 0, 0);
      acc[g] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_l, bh, acc[g], 0, 0, 0);
    }
  }
  for (int g = 0; g < 4; ++g)
    for (int r = 0; r < 4; ++r) y[256 * g + 16 * J + 4 * kg + r] = acc[g][r] * unscale;
}

int main() {
  // (1)
  std::vector<float> A(16 * 32), B(32 * 16), D(256), R(256, 0.0f);
  for (int i = 0; i < 16; ++i)
    for (int k = 0; k < 32; ++k) A[i * 32 + k] = static_cast<float>((i * 7 + k * 3) % 13 - 6);
  for (int k = 0; k < 32; ++k)
    for (int j = 0; j < 16; ++j) B[k * 16 + j] = static_cast<float>((k * 5 + j * 11) % 9 - 4);
  for (int i = 0; i < 16; ++i)
    for (int j = 0; j < 16; ++j)
      for (int k = 0; k < 32; ++k) R[i * 16 + j] += A[i * 32 + k] * B[k * 16 + j];
  float *dA, *dB, *dD;
  hipMalloc(&dA, A.size() * 4);
  hipMalloc(&dB, B.size() * 4);
  hipMalloc(&dD, D.size() * 4);
  hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice);
  hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice);
  k_map<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256; ++i) bad += D[i] != R[i];
  printf("map: %d of 256 wrong\n", bad);

  // (2)
  srand(7);
  std::vector<double> a(125);
  double amax = 0;
  for (int k = 0; k < 125; ++k) {
    const double x = (k - 62) / 62.0;
    a[k] = (0.5 + 0.5 * cos(M_PI * x)) * (k == 62 ? 1.0 : sin(0.1 * M_PI * (k - 62)) / (0.1 * M_PI * (k - 62))) * 0.1;
    amax = fmax(amax, fabs(a[k]));
  }
  const int st = static_cast<int>(floor(log2(30000.0 / amax)));
  const int sf = 12;
  std::vector<float> af(125);
  for (int k = 0; k < 125; ++k) af[k] = static_cast<float>(a[k]);
  std::vector<h8> AH(5 * 64), AL(5 * 64);
  for (int s = 0; s < 5; ++s)
    for (int l = 0; l < 64; ++l)
      for (int j = 0; j < 8; ++j) {
        const int I = l & 15, kap = 32 * s + 8 * (l >> 4) + j, k = I + 128 - kap;
        const float v = (k >= 0 && k <= 124) ? ldexpf(af[k], st) : 0.0f;
        const _Float16 h = (_Float16)v;
        AH[s * 64 + l][j] = h;
        AL[s * 64 + l][j] = (_Float16)(v - (float)h);
      }
  const int NI = 128 + 1024 + 32;
  std::vector<float> f(NI, 0.0f);
  std::vector<_Float16> FH(NI), FL(NI);
  for (int i = 0; i < 128 + 1024; ++i) f[i] = static_cast<float>(((rand() / (double)RAND_MAX) - 0.5) * 4.0 * pow(10.0, -3.0 * (i % 7) / 6.0));
  for (int i = 0; i < NI; ++i) {
    const float v = ldexpf(f[i], sf);
    const _Float16 h = (_Float16)v;
    FH[i] = h;
    FL[i] = (_Float16)(v - (float)h);
  }
  h8 *dah, *dal;
  _Float16 *dfh, *dfl;
  float* dy;
  hipMalloc(&dah, AH.size() * sizeof(h8));
  hipMalloc(&dal, AL.size() * sizeof(h8));
  hipMalloc(&dfh, NI * 2);
  hipMalloc(&dfl, NI * 2);
  hipMalloc(&dy, 1024 * 4);
  hipMemcpy(dah, AH.data(), AH.size() * sizeof(h8), hipMemcpyHostToDevice);
  hipMemcpy(dal, AL.data(), AL.size() * sizeof(h8), hipMemcpyHostToDevice);
  hipMemcpy(dfh, FH.data(), NI * 2, hipMemcpyHostToDevice);
  hipMemcpy(dfl, FL.data(), NI * 2, hipMemcpyHostToDevice);
  k_fir<<<1, 64>>>(dah, dal, dfh, dfl, dy, ldexpf(1.0f, -(st + sf)));
  std::vector<float> y(1024);
  hipMemcpy(y.data(), dy, 1024 * 4, hipMemcpyDeviceToHost);
  double emax = 0, e32 = 0, num = 0, den = 0;
  for (int o = 0; o < 1024; ++o) {
    double r = 0, mag = 0;
    float r32 = 0;
    for (int k = 0; k < 125; ++k) {
      r += static_cast<double>(af[k]) * f[o - k + 128];
      mag += fabs(static_cast<double>(af[k]) * f[o - k + 128]);
      r32 = fmaf(af[k], f[o - k + 128], r32);
    }
    emax = fmax(emax, fabs(y[o] - r) / mag);
    e32 = fmax(e32, fabs(r32 - r) / mag);
    num += (y[o] - r) * (y[o] - r);
    den += r * r;
  }
  printf("fir: max |err| / sum|terms| = %.3g (f32 fma chain: %.3g), nrmse %.3g, st %d\n", emax, e32, sqrt(num / den), st);
  return bad != 0;
}
