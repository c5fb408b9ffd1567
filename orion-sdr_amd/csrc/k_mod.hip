// k_mod.hip — on-device analog modulators for gfx950.
//   AmDsbMod::process          modulate/am.rs:44-120
//   PmDirectPhaseMod::process  modulate/pm.rs:36-47
//   FmPhaseAccumMod::process   modulate/fm.rs:45-74 (+ mix_with_nco, dsp/nco.rs:62-66)
//   SsbPhasingMod::process     modulate/ssb.rs:43-114 (front and back of the two
//                              LpCascade scans, which run on the k_scan kernels)
// Every oscillator is the closed form of the reference's phasor recurrence:
// sample i of a call uses w^(k0 + i + 1) (Rotator::next / Nco::next_cs advance
// before returning), evaluated by phasor_q64 from the stream index, so a call
// never depends on its predecessor's rounding. Streaming, memory-bound kernels:
// grid-stride over the samples, at most 8 workgroups per CU.
#include <algorithm>

#include "kernels.hpp"

namespace orion {
namespace {

constexpr int NT = 256;
constexpr int kMaxGrid = 2048;
constexpr int kFmC = 16;             // FM phase scan: samples per thread
constexpr int kFmCH = kFmC * NT;     // samples per workgroup chunk (4096)

int grid_for(long long n) { return static_cast<int>(std::min<long long>(kMaxGrid, std::max(1LL, (n + NT - 1) / NT))); }

// am.rs:87-89 (clamp: :56): m = (cl + mi x) [clamped to +-1] * g; out = m * r.
__global__ __launch_bounds__(NT) void k_am_mod(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                               uint64_t k0, uint64_t step, float cl, float mi, float g, int clamp) {
  for (long long i = blockIdx.x * static_cast<long long>(NT) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * NT) {
    float v = cl + mi * x[i];
    if (clamp) v = fminf(fmaxf(v, -1.0f), 1.0f);
    const float m = v * g;
    const f2 r = phasor_q64(k0 + static_cast<uint64_t>(i) + 1, step);
    y[i] = f2{m * r.x, m * r.y};
  }
}

// modulate/pm.rs:36-47 PmDirectPhaseMod: phi = kp x; base = (cos phi, sin phi) * gain
// (num-complex Complex * f32); out = mix_with_nco(base, rf) (the non-FMA product,
// nco.rs:63-66) with the RF phasor after k0 + i + 1 steps.
__global__ __launch_bounds__(NT) void k_pm_mod(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                               uint64_t k0, uint64_t step, float kp, float g) {
  for (long long i = blockIdx.x * static_cast<long long>(NT) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * NT) {
    const float phi = kp * x[i];
    const float br = cosf(phi) * g, bi = sinf(phi) * g;
    const f2 r = phasor_q64(k0 + static_cast<uint64_t>(i) + 1, step);
    y[i] = f2{br * r.x - bi * r.y, br * r.y + bi * r.x};
  }
}

// ssb.rs:52-54: the two LpCascade inputs x p.re, x p.im (p = audio NCO), planar.
__global__ __launch_bounds__(NT) void k_ssb_mod_front(const float* __restrict__ x, float* __restrict__ u,
                                                      long long n, uint64_t k0, uint64_t step) {
  for (long long i = blockIdx.x * static_cast<long long>(NT) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * NT) {
    const f2 p = phasor_q64(k0 + static_cast<uint64_t>(i) + 1, step);
    const float xi = x[i];
    u[i] = xi * p.x;
    u[n + i] = xi * p.y;
  }
}

// ssb.rs:55-60: z = (I, side Q); out = z * r (rf NCO), FMA form of rotate_block.
__global__ __launch_bounds__(NT) void k_ssb_mod_back(const float* __restrict__ v, f2* __restrict__ y, long long n,
                                                     uint64_t k0, uint64_t step, float side) {
  for (long long i = blockIdx.x * static_cast<long long>(NT) + threadIdx.x; i < n;
       i += static_cast<long long>(gridDim.x) * NT) {
    const f2 r = phasor_q64(k0 + static_cast<uint64_t>(i) + 1, step);
    const f2 z = f2{v[i], side * v[n + i]};
    y[i] = cmul_rot(z, r);
  }
}

// ---- FmPhaseAccumMod: phi_i = phi_carry + sum_{j <= i} inc_j (f64), z = e^{j phi} ----
// fm.rs:48-56 multiplies the running phasor by (cos dphi, sin dphi) rounded to
// f32, dphi = kf x_i, renormalising every 1024 samples. The angle of that f32
// pair, not dphi itself, is what the recurrence adds per sample, and its bias
// is systematic (it drifted 1.2e-2 rad from the exact sum over 2^20 samples of
// the C2 input): so the increment is atan2 of the same f32 pair, summed in f64.
// What remains is the recurrence's own multiply rounding (a random walk) and
// sincosf/sin_cos last-bit differences.
// For |dphi| < 1/8 (every WBFM-rate deviation): dphi plus the angle between the
// f32 pair and the exact (C, S) = (cos, sin) dphi, the latter from f64 Taylor
// series (truncation < 1e-21), the former to first order (it is < 1e-7 rad).
__device__ __forceinline__ double fm_inc(float kf, float x) {
  const float dphi = kf * x;  // fm.rs:50
  float s, c;
  sincosf(dphi, &s, &c);  // fm.rs:51
  const double d = dphi;
  if (fabs(d) < 0.125) {
    const double q = d * d;
    const double S = d * (1.0 - q * (1.0 / 6) * (1.0 - q * (1.0 / 20) * (1.0 - q * (1.0 / 42) *
                     (1.0 - q * (1.0 / 72) * (1.0 - q * (1.0 / 110))))));
    const double C = 1.0 - q * 0.5 * (1.0 - q * (1.0 / 12) * (1.0 - q * (1.0 / 30) * (1.0 - q * (1.0 / 56) *
                     (1.0 - q * (1.0 / 90) * (1.0 - q * (1.0 / 132))))));
    // sin of the angle between them; |(c, s)| = 1 +- 1e-7, so dividing by their
    // cosine (1 +- 1e-7) would change the ~1e-8 result by ~1e-15
    return d + (static_cast<double>(s) * C - static_cast<double>(c) * S);
  }
  return atan2(static_cast<double>(s), static_cast<double>(c));
}

// Pass 1: the f64 sum of each chunk's phase increments.
__global__ __launch_bounds__(NT) void k_fm_mod_sum(const float* __restrict__ x, long long n, float kf,
                                                   double* __restrict__ sums) {
  __shared__ double part[NT / 64];
  const long long base = static_cast<long long>(blockIdx.x) * kFmCH;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    const long long i = base + threadIdx.x + static_cast<long long>(k) * NT;
    if (i < n) s += fm_inc(kf, x[i]);
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < NT / 64; ++w) t += part[w];
    sums[blockIdx.x] = t;
  }
}

// Pass 2 (one workgroup): exclusive prefix of the chunk sums from the carried
// phase (each thread a run of consecutive chunks, one workgroup scan of the run
// totals); the carried phase of the next call (reduced mod 2 pi).
__global__ __launch_bounds__(NT) void k_fm_mod_carry(double* __restrict__ sums, int nchunk,
                                                     const double* __restrict__ carry_in,
                                                     double* __restrict__ carry_out) {
  __shared__ double tot[NT / 64];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int per = (nchunk + NT - 1) / NT;
  const int c0 = min(nchunk, t * per), c1 = min(nchunk, c0 + per);
  double run = 0.0;
  for (int c = c0; c < c1; ++c) run += sums[c];
  double inc = run;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double o = __shfl_up(inc, d, 64);
    if (lane >= d) inc += o;
  }
  if (lane == 63) tot[w] = inc;
  __syncthreads();
  double before = carry_in[0] + inc - run;
  for (int k = 0; k < w; ++k) before += tot[k];
  for (int c = c0; c < c1; ++c) {
    const double v = sums[c];
    sums[c] = before;
    before += v;
  }
  if (t == NT - 1) carry_out[0] = before - 6.283185307179586 * rint(before * 0.15915494309189535);
}

// Pass 3: per chunk, the inclusive prefix of the increments (thread-local runs,
// then a workgroup scan of the run totals), z = e^{j phi} * gain, and
// mix_with_nco's non-FMA complex product with the RF phasor (nco.rs:62-66).
__global__ __launch_bounds__(NT) void k_fm_mod_apply(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                                     float kf, float gain, const double* __restrict__ offs,
                                                     uint64_t k0, uint64_t step, const f2* __restrict__ rtab) {
  __shared__ double tot[NT / 64];
  __shared__ float xs[kFmCH + kFmCH / 16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const long long base = static_cast<long long>(blockIdx.x) * kFmCH;
  // coalesced load, then each thread owns kFmC consecutive samples
  for (int k = 0; k < kFmC; ++k) {
    const int e = t + k * NT;
    const long long i = base + e;
    xs[e + (e >> 4)] = i < n ? x[i] : 0.0f;
  }
  __syncthreads();
  double d[kFmC];
  double run = 0.0;
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    const int e = t * kFmC + k;
    d[k] = fm_inc(kf, xs[e + (e >> 4)]);
    run += d[k];
  }
  double inc = run;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const double o = __shfl_up(inc, dd, 64);
    if (lane >= dd) inc += o;
  }
  if (lane == 63) tot[w] = inc;
  __syncthreads();
  double phi = offs[blockIdx.x] + inc - run;
  for (int k = 0; k < w; ++k) phi += tot[k];
  // RF phasor of sample i0 + k = (phasor of i0) x e^{j theta k} (rtab: k < kFmC)
  const long long i0 = base + t * kFmC;
  const f2 R0 = phasor_q64(k0 + static_cast<uint64_t>(i0) + 1, step);
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    const long long i = i0 + k;
    phi += d[k];
    if (i < n) {
      const double red = phi - 6.283185307179586 * rint(phi * 0.15915494309189535);
      float s, c;
      sincosf(static_cast<float>(red), &s, &c);
      const f2 b = f2{c * gain, s * gain};  // fm.rs:66 base = z * gain
      const f2 r = cmul(R0, rtab[k]);
      y[i] = f2{b.x * r.x - b.y * r.y, b.x * r.y + b.y * r.x};  // nco.rs:65 (no FMA)
    }
  }
}

// Single pass (default; the three passes above stay behind ORION_FM_MOD_3P=1): each
// chunk computes its increments once, publishes its f64 aggregate, and takes the
// phase entering it by decoupled look-back over its predecessors (wave 0: lane i
// looks at chunk c-1-i; the nearest chunk with a published inclusive prefix, or the
// carried phase before chunk 0, closes the sum), then publishes its own inclusive
// prefix. Chunk-major grid: every predecessor was dispatched earlier and publishes
// its aggregate before it waits, so the walk always ends. Records: 8 u32 per chunk,
// [0, 2) aggregate, [2, 4) inclusive prefix (f64), 6 / 7 their flags (launch epoch).
__device__ __forceinline__ void fm_st(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t fm_ld(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void fm_st64(uint32_t* p, double v) {
  const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
  fm_st(p, static_cast<uint32_t>(b));
  fm_st(p + 1, static_cast<uint32_t>(b >> 32));
}
__device__ __forceinline__ double fm_ld64(const uint32_t* p) {
  const unsigned long long lo = fm_ld(p), hi = fm_ld(p + 1);
  return __longlong_as_double(static_cast<long long>((hi << 32) | lo));
}

__global__ __launch_bounds__(NT) void k_fm_mod_sp(const float* __restrict__ x, f2* __restrict__ y, long long n,
                                                  float kf, float gain, uint32_t* __restrict__ rec, uint32_t epoch,
                                                  const double* __restrict__ carry_in, double* __restrict__ carry_out,
                                                  uint64_t k0, uint64_t step, const f2* __restrict__ rtab,
                                                  int* __restrict__ err, uint32_t spin) {
  __shared__ double tot[NT / 64];
  __shared__ double excl_sh;
  __shared__ float xs[kFmCH + kFmCH / 16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c = static_cast<int>(blockIdx.x);
  const int nchunk = static_cast<int>((n + kFmCH - 1) / kFmCH);
  const bool last = c == nchunk - 1;
  const long long base = static_cast<long long>(c) * kFmCH;
  for (int k = 0; k < kFmC; ++k) {
    const int e = t + k * NT;
    const long long i = base + e;
    xs[e + (e >> 4)] = i < n ? x[i] : 0.0f;
  }
  __syncthreads();
  double d[kFmC];
  double run = 0.0;
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    const int e = t * kFmC + k;
    d[k] = base + e < n ? fm_inc(kf, xs[e + (e >> 4)]) : 0.0;
    run += d[k];
  }
  double inc = run;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const double o = __shfl_up(inc, dd, 64);
    if (lane >= dd) inc += o;
  }
  if (lane == 63) tot[w] = inc;
  __syncthreads();
  if (w == 0) {
    double agg = 0.0;
    for (int v = 0; v < NT / 64; ++v) agg += tot[v];
    uint32_t* my = rec + static_cast<long long>(c) * 8;
    if (!last) {
      if (lane == 0) fm_st64(my, agg);
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the aggregate is visible before its flag
      if (lane == 0) fm_st(my + 6, epoch);
    }
    double excl = 0.0;
    for (int b = c - 1;; b -= 64) {
      const int k = b - lane;
      double v = 0.0;
      bool closes = true;
      if (k >= 0) {
        const uint32_t* pr = rec + static_cast<long long>(k) * 8;
        bool seen = false;  // bounded wait (spin 0: time out at once, test-only)
        for (uint32_t it = 0; it < spin && !seen; ++it) {
          seen = fm_ld(pr + 6) == epoch || fm_ld(pr + 7) == epoch;
          if (!seen) __builtin_amdgcn_s_sleep(2);
        }
        if (!seen) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        closes = fm_ld(pr + 7) == epoch;
        v = closes ? fm_ld64(pr + 2) : fm_ld64(pr);
      } else {
        v = k == -1 ? carry_in[0] : 0.0;  // the carried phase before chunk 0
      }
      const unsigned long long bal = __ballot(closes);
      const int first = bal ? __builtin_ctzll(bal) : 64;
      double term = lane <= first ? v : 0.0;
#pragma unroll
      for (int off = 32; off >= 1; off >>= 1) term += __shfl_xor(term, off, 64);
      excl += term;
      if (first < 64) break;
    }
    if (lane == 0) {
      if (!last) {
        fm_st64(my + 2, excl + agg);
        __builtin_amdgcn_s_waitcnt(0x0F70);
        fm_st(my + 7, epoch);
      } else {
        const double end = excl + agg;  // the carried phase of the next call (reduced mod 2 pi)
        carry_out[0] = end - 6.283185307179586 * rint(end * 0.15915494309189535);
      }
      excl_sh = excl;
    }
  }
  __syncthreads();
  double phi = excl_sh + inc - run;
  for (int k = 0; k < w; ++k) phi += tot[k];
  const long long i0 = base + t * kFmC;
  const f2 R0 = phasor_q64(k0 + static_cast<uint64_t>(i0) + 1, step);
#pragma unroll
  for (int k = 0; k < kFmC; ++k) {
    const long long i = i0 + k;
    phi += d[k];
    if (i < n) {
      const double red = phi - 6.283185307179586 * rint(phi * 0.15915494309189535);
      float sn, cs;
      sincosf(static_cast<float>(red), &sn, &cs);
      const f2 bz = f2{cs * gain, sn * gain};  // fm.rs:66 base = z * gain
      const f2 r = cmul(R0, rtab[k]);
      y[i] = f2{bz.x * r.x - bz.y * r.y, bz.x * r.y + bz.y * r.x};  // nco.rs:65 (no FMA)
    }
  }
}

}  // namespace

void launch_am_mod(const float* x, f2* y, long long n, uint64_t k0, uint64_t step, float cl, float mi, float g,
                   bool clamp, hipStream_t s) {
  if (n <= 0) return;
  k_am_mod<<<grid_for(n), NT, 0, s>>>(x, y, n, k0, step, cl, mi, g, clamp ? 1 : 0);
  ORION_LAUNCH_CHECK();
}

void launch_ssb_mod_front(const float* x, float* u, long long n, uint64_t k0, uint64_t step, hipStream_t s) {
  if (n <= 0) return;
  k_ssb_mod_front<<<grid_for(n), NT, 0, s>>>(x, u, n, k0, step);
  ORION_LAUNCH_CHECK();
}

void launch_pm_mod(const float* x, f2* y, long long n, uint64_t k0, uint64_t step, float kp, float g, hipStream_t s) {
  if (n <= 0) return;
  k_pm_mod<<<grid_for(n), NT, 0, s>>>(x, y, n, k0, step, kp, g);
  ORION_LAUNCH_CHECK();
}

void launch_ssb_mod_back(const float* v, f2* y, long long n, uint64_t k0, uint64_t step, float side, hipStream_t s) {
  if (n <= 0) return;
  k_ssb_mod_back<<<grid_for(n), NT, 0, s>>>(v, y, n, k0, step, side);
  ORION_LAUNCH_CHECK();
}

long long fm_mod_chunks(long long n) { return (n + kFmCH - 1) / kFmCH; }

void launch_fm_mod_sp(const float* x, f2* y, long long n, float kf, float gain, uint32_t* rec, uint32_t epoch,
                      const double* carry_in, double* carry_out, uint64_t k0, uint64_t step, const f2* rtab,
                      int* err, hipStream_t s) {
  if (n <= 0) return;
  const long long nchunk = fm_mod_chunks(n);
  if (nchunk > (1LL << 30)) throw HipError("FM modulator: input too long");
  k_fm_mod_sp<<<static_cast<int>(nchunk), NT, 0, s>>>(x, y, n, kf, gain, rec, epoch, carry_in, carry_out, k0, step,
                                                     rtab, err, spin_limit());
  ORION_LAUNCH_CHECK();
}
int fm_mod_rtab_len() { return kFmC; }

void launch_fm_mod(const float* x, f2* y, long long n, float kf, float gain, double* sums,
                   const double* carry_in, double* carry_out, uint64_t k0, uint64_t step, const f2* rtab,
                   hipStream_t s) {
  if (n <= 0) return;
  const long long nchunk = fm_mod_chunks(n);
  if (nchunk > (1LL << 30)) throw HipError("FM modulator: input too long");
  const int g = static_cast<int>(nchunk);
  k_fm_mod_sum<<<g, NT, 0, s>>>(x, n, kf, sums);
  k_fm_mod_carry<<<1, NT, 0, s>>>(sums, g, carry_in, carry_out);
  k_fm_mod_apply<<<g, NT, 0, s>>>(x, y, n, kf, gain, sums, k0, step, rtab);
  ORION_LAUNCH_CHECK();
}

}  // namespace orion
