// hip_common.hpp — shared device/host helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>

namespace orion {

// cf32 as a packed pair: lane-level complex math maps onto v_pk_fma_f32 / v_pk_mul_f32.
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

struct HipError : std::runtime_error {
  explicit HipError(const std::string& s) : std::runtime_error(s) {}
};

#define ORION_HIP(expr)                                                                    \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      throw ::orion::HipError(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" +   \
                              __FILE__ + ":" + std::to_string(__LINE__));                  \
  } while (0)

#define ORION_LAUNCH_CHECK() ORION_HIP(hipGetLastError())

// Workgroup barrier for LDS hand-offs only. __syncthreads() on gfx950 also waits
// vmcnt(0), which drains every outstanding global load — including a prefetch
// meant to stay in flight across the barrier. This waits for this wave's LDS
// operations (lgkmcnt) and then barriers; global loads keep flying and the
// compiler still inserts its own vmcnt wait before their first use.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// A wave's own LDS operations are complete (DS operations of one wave complete
// in order); also a compiler fence. For hand-offs inside one wave: no barrier.
__device__ __forceinline__ void wave_lds_fence() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// A read-only table the host wrote before the launch, read at wave-uniform indices: in
// the constant address space the compiler reads it with scalar loads (one s_load per
// 4-16 dwords for the wave) instead of a vector load per use whose 64 lanes each
// return the same bytes through the CU's load-return path.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(4))) T* uniform_table(const T* p) {
  return (const __attribute__((address_space(4))) T*)(p);
}

__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 splat2(float x) { return f2{x, x}; }

// Complex multiply as the reference's Rotator::rotate_block writes it
// (dsp/rotator.rs:80-83): re = fma(a, p.re, -(b*p.im)), im = fma(b, p.re, a*p.im).
__device__ __forceinline__ f2 cmul_rot(f2 x, f2 p) {
  return f2{__builtin_fmaf(x.x, p.x, -(x.y * p.y)), __builtin_fmaf(x.y, p.x, x.x * p.y)};
}
// cmul_rot with the same roundings, written as packed-f32 ops (v_pk_mul_f32 +
// v_pk_fma_f32, the negation folded into a source modifier): t = (b*d, a*d)
// rounded, then (fma(a, c, -t.x), fma(b, c, t.y)) for x = (a, b), p = (c, d).
// Written in VOP3P asm: the compiler does not fold the half-negation into the
// FMA's neg_lo modifier and emits a v_pk_add + v_mov instead (4 VALU, not 2).
__device__ __forceinline__ f2 cmul_rot_pk(f2 x, f2 p) {
  f2 t, r;
  // t.lo = x.hi * p.hi, t.hi = x.lo * p.hi
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1]" : "=v"(t) : "v"(x), "v"(p));
  // r.lo = fma(x.lo, p.lo, -t.lo), r.hi = fma(x.hi, p.lo, t.hi)
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1] neg_lo:[0,0,1]" : "=v"(r) : "v"(x), "v"(p), "v"(t));
  return r;
}
// Plain complex multiply (ours, not a reference op order).
__device__ __forceinline__ f2 cmul(f2 a, f2 b) {
  return f2{__builtin_fmaf(a.x, b.x, -(a.y * b.y)), __builtin_fmaf(a.x, b.y, a.y * b.x)};
}

// Exact oscillator phase: phasor for absolute step count k is e^{j*theta*k}
// with theta/2pi = step_q64 / 2^64. (k*step) mod 2^64 is exact integer math;
// the top 24 bits give an exactly representable f32 turn count for
// sincospif, the remaining 40 bits a first-order correction (< 3.8e-7 rad, so
// the neglected second-order term is < 1e-13).
__device__ __forceinline__ f2 phasor_at(uint64_t ph);
__device__ __forceinline__ f2 phasor_q64(uint64_t k, uint64_t step_q64) { return phasor_at(k * step_q64); }
// The phasor of a Q0.64 phase (a fraction of a turn): e^{j 2 pi ph / 2^64}.
__device__ __forceinline__ f2 phasor_at(uint64_t ph) {
  const uint32_t hi24 = static_cast<uint32_t>(ph >> 40);
  const uint64_t lo40 = ph & ((1ull << 40) - 1);
  const float t2 = static_cast<float>(hi24) * (1.0f / 8388608.0f);  // 2*turns in [0,2)
  float s, c;
  sincospif(t2, &s, &c);
  const float d = static_cast<float>(lo40) * (6.28318530717958647692f / 1099511627776.0f) *
                  (1.0f / 16777216.0f);  // 2*pi * lo40 / 2^64
  return f2{__builtin_fmaf(-s, d, c), __builtin_fmaf(c, d, s)};
}

// ---- the reference's oscillator on the device (osc.hpp RefOsc, design.hpp RecTable) ----
// Output k of an oscillator (k steps after its table's start state; the phasor after
// k + 1 steps, rotator.rs:44-62 / nco.rs:42-58):
//   tab[k]                                            k < n_tab (the reference's own)
//   tab[cyc_start + (k - cyc_start) mod cyc_len]      cyc_len > 0 (its cycle, forever)
//   (mag0 + mag1 ((ctr0 + k + 1) & 1023)) e^{j 2 pi ph / 2^64}, ph = mbase + (k + 1 - n_tab) mstep
//                                                     otherwise (the drift model; the
//                                                     closed form: mag0 = 1, mag1 = 0)
// mtab: e^{j 2 pi p mstep / 2^64}, p < kOscSpan (the model within a run).
// cyc_len is 0 or >= kOscSpan (rec_table unrolls shorter cycles).
constexpr int kOscSpan = 16384;  // longest run of consecutive outputs one cursor serves
struct OscDev {
  const f2* tab;
  const f2* mtab;
  uint64_t n_tab, cyc_start, cyc_len, mbase, mstep;
  uint32_t ctr0;
  float mag0, mag1;  // the model's magnitude, linear in the renorm-counter position
};
__device__ __forceinline__ float osc_mag(const OscDev& o, uint32_t pos) {
  return __builtin_fmaf(o.mag1, static_cast<float>(pos & 1023u), o.mag0);
}
// A cursor over outputs k .. k + len - 1 (len <= kOscSpan), all fields wave-uniform:
// kind 0 every output from the table, 1 every output modelled, 2 mixed (the first
// `rem` from the table); j = the table index of k, wrapped into the cycle (with
// cyc_len >= kOscSpan a run wraps at most once; tables hold < 2^31 outputs, so table
// indices are 32-bit); S = the model phasor of k; klo = k mod 2^32 (magnitude position).
struct OscRun {
  uint32_t j, rem, klo;
  int kind;
  f2 S;
};
__device__ __forceinline__ OscRun osc_run(const OscDev& o, uint64_t k, int len) {
  OscRun r;
  const bool cyc = o.cyc_len != 0;
  r.kind = (cyc || k + static_cast<uint64_t>(len) <= o.n_tab) ? 0 : (k >= o.n_tab ? 1 : 2);
  r.j = static_cast<uint32_t>((cyc && k >= o.n_tab) ? o.cyc_start + (k - o.cyc_start) % o.cyc_len : k);
  r.rem = r.kind == 2 ? static_cast<uint32_t>(o.n_tab - k) : 0u;
  r.klo = static_cast<uint32_t>(k);
  r.S = r.kind != 0 ? phasor_at(o.mbase + (k + 1 - o.n_tab) * o.mstep) : f2{1.0f, 0.0f};
  return r;
}
// Table output r.k + off (kind 0, or kind 2 with off < rem). The device table holds
// kOscSpan entries past n_tab (the cycle's continuation, or the last entry repeated:
// osc.cpp), so a run reads tab[j + off] without a wrap; the padding lanes of a run's
// last tile read valid memory whose values are never used.
__device__ __forceinline__ f2 osc_tab(const OscDev& o, const OscRun& r, int off) {
  return o.tab[r.j + static_cast<uint32_t>(off)];
}
// Model output r.k + off from tm = mtab[off] (or any equal product of step phasors).
__device__ __forceinline__ f2 osc_model(const OscDev& o, const OscRun& r, int off, f2 tm) {
  return cmul(r.S, tm) * splat2(osc_mag(o, o.ctr0 + r.klo + static_cast<uint32_t>(off) + 1u));
}
__device__ __forceinline__ bool osc_in_tab(const OscRun& r, int off) {
  return r.kind == 0 || (r.kind == 2 && static_cast<uint32_t>(off) < r.rem);
}
// Output r.k + off in two steps, so that a kernel can issue every load first: osc_ld
// reads the table entry or mtab[off], osc_fin turns a model read into the output.
__device__ __forceinline__ f2 osc_ld(const OscDev& o, const OscRun& r, int off) {
  const f2* b = osc_in_tab(r, off) ? o.tab + r.j : o.mtab;
  return b[off];
}
__device__ __forceinline__ f2 osc_fin(const OscDev& o, const OscRun& r, int off, f2 v) {
  return osc_in_tab(r, off) ? v : osc_model(o, r, off, v);
}
// Output r.k + off (off < the run's len), from the table or the model (tm: mtab[off]).
__device__ __forceinline__ f2 osc_get_tm(const OscDev& o, const OscRun& r, int off, f2 tm) {
  if (osc_in_tab(r, off)) return osc_tab(o, r, off);
  return osc_model(o, r, off, tm);
}
__device__ __forceinline__ f2 osc_get(const OscDev& o, const OscRun& r, int off) {
  return osc_fin(o, r, off, osc_ld(o, r, off));
}

// Output k alone (no cursor: kernels that visit samples in no run order).
__device__ __forceinline__ f2 osc_at(const OscDev& o, uint64_t k) {
  if (k < o.n_tab) return o.tab[k];
  if (o.cyc_len) {
    const uint64_t d = k - o.cyc_start;
    const uint64_t j = ((d | o.cyc_len) >> 32) == 0 ? static_cast<uint32_t>(d) % static_cast<uint32_t>(o.cyc_len)
                                                    : d % o.cyc_len;
    return o.tab[o.cyc_start + j];
  }
  return phasor_at(o.mbase + (k + 1 - o.n_tab) * o.mstep) *
         splat2(osc_mag(o, o.ctr0 + static_cast<uint32_t>(k) + 1u));
}

// f32 sin and cos, correctly rounded but for rare near-ties: the argument reduced by
// pi/2 in f64 (two-part pi/2: exact enough for |x| < 2^20), then Taylor polynomials on
// |r| <= pi/4 through r^15 / r^16 (truncation < 2^-45 relative), one rounding to f32.
// The reference's f32 sin / cos / sin_cos (glibc's sinf / cosf, < 0.56 ulp) give the same
// values but for rare near-ties, with no systematic difference (a phase that sums the
// pairs' angles, FmPhaseAccumMod, must not drift). No Payne-Hanek path: the library
// sincosf's is if-converted into every call (~180 VALU); this is ~30. |x| >= 2^20: the
// library.
__device__ __forceinline__ void sincos_cr(float x, float* s, float* c) {
  if (!(fabsf(x) < 1048576.0f)) {
    sincosf(x, s, c);
    return;
  }
  const double d = x;
  const double nq = rint(d * 0.63661977236758134);
  const double r = __builtin_fma(-nq, 6.123233995736766e-17, __builtin_fma(-nq, 1.5707963267948966, d));
  const double r2 = r * r;
  double ps = -1.0 / 1307674368000.0;
  ps = __builtin_fma(ps, r2, 1.0 / 6227020800.0);
  ps = __builtin_fma(ps, r2, -1.0 / 39916800.0);
  ps = __builtin_fma(ps, r2, 1.0 / 362880.0);
  ps = __builtin_fma(ps, r2, -1.0 / 5040.0);
  ps = __builtin_fma(ps, r2, 1.0 / 120.0);
  ps = __builtin_fma(ps, r2, -1.0 / 6.0);
  double pc = 1.0 / 20922789888000.0;
  pc = __builtin_fma(pc, r2, -1.0 / 87178291200.0);
  pc = __builtin_fma(pc, r2, 1.0 / 479001600.0);
  pc = __builtin_fma(pc, r2, -1.0 / 3628800.0);
  pc = __builtin_fma(pc, r2, 1.0 / 40320.0);
  pc = __builtin_fma(pc, r2, -1.0 / 720.0);
  pc = __builtin_fma(pc, r2, 1.0 / 24.0);
  pc = __builtin_fma(pc, r2, -0.5);
  const float sr = static_cast<float>(__builtin_fma(ps * r2, r, r));
  const float cr = static_cast<float>(__builtin_fma(pc, r2, 1.0));
  const int q = static_cast<int>(static_cast<long long>(nq) & 3);
  const float s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
  *s = (q & 2) ? -s0 : s0;
  *c = ((q + 1) & 2) ? -c0 : c0;
}

// util.rs:305-322 atan2_approx, restated op for op (no contraction: this TU is
// built with -ffp-contract=off, and the division is IEEE).
__device__ __forceinline__ float atan2_approx(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const bool swap = ax < ay;
  const float mn = swap ? ax : ay;
  const float mx = swap ? ay : ax;
  const float r = mn / (mx + 1.1920929e-7f);
  const float r2 = r * r;
  float phi = r * (0.7853981633974483f + r2 * (-0.2447f + r2 * 0.0663f));
  if (swap) phi = 1.5707963267948966f - phi;
  const float sgn = (y < 0.0f) ? -1.0f : 1.0f;
  return (x < 0.0f) ? (3.14159265358979323846f - phi) * sgn : phi * sgn;
}

// FmQuadratureDemod discriminator input, demodulate/fm.rs:62-65 (non-FMA):
// prod = (z.re*p.re + z.im*p.im, z.im*p.re - z.re*p.im).
__device__ __forceinline__ float fm_disc(f2 z, f2 p, float k) {
  const float pr = z.x * p.x + z.y * p.y;
  const float pi = z.y * p.x - z.x * p.y;
  return atan2_approx(pi, pr) * k;
}

// fm_disc with the same roundings as packed ops: (z.x p.x, z.y p.x) and
// (z.y p.y, z.x p.y) rounded, then (sum, difference).
__device__ __forceinline__ float fm_disc_pk(f2 z, f2 p, float k) {
  const f2 a = z * f2{p.x, p.x};
  const f2 b = f2{z.y, z.x} * f2{p.y, p.y};
  const f2 s = a + f2{b.x, -b.y};
  return atan2_approx(s.y, s.x) * k;
}

// atan2_approx with the ratio from the hardware reciprocal (v_rcp_f32, 1 ulp)
// instead of the IEEE division sequence (~11 VALU): used where the chain is held
// to a tolerance rather than bit-exactness (the fused WBFM front).
__device__ __forceinline__ float atan2_approx_rcp(float y, float x) {
  const float ax = fabsf(x), ay = fabsf(y);
  const bool swap = ax < ay;
  const float mn = swap ? ax : ay;
  const float mx = swap ? ay : ax;
  const float r = mn * __builtin_amdgcn_rcpf(mx + 1.1920929e-7f);
  const float r2 = r * r;
  float phi = r * (0.7853981633974483f + r2 * (-0.2447f + r2 * 0.0663f));
  if (swap) phi = 1.5707963267948966f - phi;
  const float sgn = (y < 0.0f) ? -1.0f : 1.0f;
  return (x < 0.0f) ? (3.14159265358979323846f - phi) * sgn : phi * sgn;
}
__device__ __forceinline__ f2 fm_prod_pk(f2 z, f2 p) {
  f2 a, b, q;
  // a = (z.lo p.lo, z.hi p.lo)
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(a) : "v"(z), "v"(p));
  // b = (z.hi p.hi, z.lo p.hi)
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,1] op_sel_hi:[0,1]" : "=v"(b) : "v"(z), "v"(p));
  // q = (a.lo + b.lo, a.hi - b.hi)
  asm("v_pk_add_f32 %0, %1, %2 neg_hi:[0,1]" : "=v"(q) : "v"(a), "v"(b));
  return q;
}
__device__ __forceinline__ float fm_disc_pk_rcp(f2 z, f2 p, float k) {
  const f2 s = fm_prod_pk(z, p);
  return atan2_approx_rcp(s.y, s.x) * k;
}

// PmQuadratureDemod, demodulate/pm.rs:56-57: num-complex z * conj(prev),
// re = a*c - b*d, im = a*d + b*c with (c, d) = (p.re, -p.im); then k*atan2.
__device__ __forceinline__ float pm_disc(f2 z, f2 p, float k) {
  const float c = p.x, d = -p.y;
  const float wr = z.x * c - z.y * d;
  const float wi = z.x * d + z.y * c;
  return k * atan2_approx(wi, wr);
}

inline int div_up(long long a, long long b) { return static_cast<int>((a + b - 1) / b); }

// Resident workgroups per CU of `kernel` at `threads` per workgroup, and the CU
// count, of the CURRENT device; cached per (kernel, device) under a lock: segment and
// one-round geometries are sized from them, so they must not leak across devices
// with different CU counts or be torn by two first launches racing.
int resident_per_cu(const void* kernel, int threads);
int device_cus();

// Cross-workgroup waits (WBFM segment hand-offs, decoupled look-backs) poll a flag
// at most spin_limit() times before they give up and set the handle's device error
// word (blocks.hpp Block::dev_err). Process-wide; orion_debug_set_spin_limit sets
// it (0: every wait times out at once — a test-only setting).
constexpr uint32_t kSpinDefault = 1u << 22;
uint32_t spin_limit();
void set_spin_limit(uint32_t polls);

}  // namespace orion
