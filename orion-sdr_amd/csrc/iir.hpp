// iir.hpp — the reference's IIR recurrences (exact per-sample op order) and the
// wave-level state-carry scan that parallelises them on gfx950.
//
// Every recurrence here is affine in its state: s' = A s + B x. A lane runs the
// reference update over C consecutive samples from a zero state (its aggregate),
// the 64 lanes of a wave combine aggregates with a Kogge-Stone scan using the
// precomputed chunk-transition matrices (A^C)^(2^s), and each lane re-runs its
// chunk from the exact incoming state. The re-run is the reference's own
// update, so only the incoming state carries scan rounding (~1 ulp of the state).
#pragma once
#include "hip_common.hpp"

namespace orion {

// dsp/iir.rs:34-40 Biquad::process, TDF-II:
//   y = fma(x,b0,z1); z1 = fma(x,b1,z2) - a1*y; z2 = x*b2 - a2*y.
struct BiquadK {
  float b0, b1, b2, a1, a2;
  __device__ __forceinline__ float step(float& z1, float& z2, float x) const {
    const float y = __builtin_fmaf(x, b0, z1);
    z1 = __builtin_fmaf(x, b1, z2) - a1 * y;
    z2 = x * b2 - a2 * y;
    return y;
  }
};

// dsp/iir.rs:15-41 Biquad::process — one TDF-II biquad; state (z1, z2) = design.cpp biquad_ss.
struct RecBQ {
  static constexpr int S = 2;
  BiquadK bq;
  __device__ __forceinline__ float step(float (&s)[S], float x) const { return bq.step(s[0], s[1], x); }
};

// dsp/iir.rs:79-83 LpCascade::process — two identical biquads. State order
// (z0_1, z0_2, z1_1, z1_2) matches design.cpp lp_cascade_ss.
struct RecLP4 {
  static constexpr int S = 4;
  BiquadK bq;
  __device__ __forceinline__ float step(float (&s)[S], float x) const {
    const float y0 = bq.step(s[0], s[1], x);
    return bq.step(s[2], s[3], y0);
  }
};

// dsp/iir.rs:151-165 LpDcCascade::process: LP4 then y = y1 - x1 + r*y1_prev.
// State (z0_1, z0_2, z1_1, z1_2, dc_x1, dc_y1) = design.cpp lpdc_ss.
struct RecLpDc {
  static constexpr int S = 6;
  BiquadK bq;
  float r;
  __device__ __forceinline__ float step(float (&s)[S], float x) const {
    const float y0 = bq.step(s[0], s[1], x);
    const float y1 = bq.step(s[2], s[3], y0);
    const float y = y1 - s[4] + r * s[5];
    s[4] = y1;
    s[5] = y;
    return y;
  }
};

// dsp/dc.rs:47-51 DcBlocker: y = x - x1 + r*y1; state (x1, y1) = design.cpp dc_ss.
struct RecDC {
  static constexpr int S = 2;
  float r;
  __device__ __forceinline__ float step(float (&s)[S], float x) const {
    const float y = x - s[0] + r * s[1];
    s[0] = x;
    s[1] = y;
    return y;
  }
};

// demodulate/cw.rs:40: y = a*y + (1-a)*mag.
struct RecOnePole {
  static constexpr int S = 1;
  float a;
  __device__ __forceinline__ float step(float (&s)[S], float x) const {
    s[0] = a * s[0] + (1.0f - a) * x;
    return s[0];
  }
};

// acc += Mx * v (S x S row-major). T = double for the scan combine: the chunk
// transition matrices of these near-unit-circle filters have entries ~7 and
// condition ~1e3, so f32 carries lose ~3 digits; f64 keeps the carried state
// at the f32 rounding level of the reference's own update.
__device__ __forceinline__ float fmaT(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
__device__ __forceinline__ double fmaT(double a, double b, double c) { return __builtin_fma(a, b, c); }

template <int S, class T, class MT>
__device__ __forceinline__ void matvec_acc(const MT* __restrict__ Mx, const T (&v)[S], T (&acc)[S]) {
#pragma unroll
  for (int i = 0; i < S; ++i) {
    T a = acc[i];
#pragma unroll
    for (int j = 0; j < S; ++j) a = fmaT(static_cast<T>(Mx[i * S + j]), v[j], a);
    acc[i] = a;
  }
}

// Lane l receives lane l - D's value (lanes l < D: unspecified) without the LDS
// crossbar (ds_bpermute waits ~100 cycles): D = 1 is DPP wave_shr:1; D = 32 is
// v_permlane32_swap; D = 16 moves the odd rows up with v_permlane16_swap and row
// 1 to row 2 with a v_permlane32_swap of the swapped-out even rows; D = 2, 4, 8
// is DPP row_shr:D inside a row and, for a row's first D lanes, DPP row_ror:D of
// the row-shifted copy (the previous row's last D lanes).
template <int D>
__device__ __forceinline__ uint32_t wave_up32(uint32_t x) {
  static_assert(D == 1 || D == 2 || D == 4 || D == 8 || D == 16 || D == 32, "shift");
  if constexpr (D == 1) {
    return static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x138, 0xf, 0xf, false));
  } else if constexpr (D == 32) {
    return __builtin_amdgcn_permlane32_swap(x, x, false, false)[0];
  } else {
    const auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);  // [0] rows 1, 3 <- rows 0, 2
    const auto b = __builtin_amdgcn_permlane32_swap(a[1], a[1], false, false);  // [0] row 2 <- a[1] row 0 = row 1
    const uint32_t s16 = ((threadIdx.x >> 4) & 3) == 2 ? b[0] : a[0];
    if constexpr (D == 16) {
      return s16;
    } else {
      const int in = __builtin_amdgcn_update_dpp(0, static_cast<int>(x), 0x110 + D, 0xf, 0xf, false);
      const int fx = __builtin_amdgcn_update_dpp(0, static_cast<int>(s16), 0x120 + D, 0xf, 0xf, false);
      return static_cast<uint32_t>((threadIdx.x & 15) >= D ? in : fx);
    }
  }
}
template <int D>
__device__ __forceinline__ double wave_up(double v) {
  const unsigned long long u = static_cast<unsigned long long>(__double_as_longlong(v));
  const uint32_t lo = wave_up32<D>(static_cast<uint32_t>(u)), hi = wave_up32<D>(static_cast<uint32_t>(u >> 32));
  return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}
template <int D>
__device__ __forceinline__ float wave_up(float v) {
  return __uint_as_float(wave_up32<D>(__float_as_uint(v)));
}

// Inclusive Kogge-Stone over the 64 lanes of a wave:
//   Q_L = agg_L + A^C * Q_{L-1}, using pw[s] = (A^C)^(2^s) (S*S each, uniform).
template <int S, class T, class MT>
__device__ __forceinline__ void wave_scan_inclusive(T (&q)[S], const MT* __restrict__ pw, int lane) {
#pragma unroll 1
  for (int s = 0; s < 6; ++s) {
    const int d = 1 << s;
    T o[S];
#pragma unroll
    for (int i = 0; i < S; ++i) o[i] = __shfl_up(q[i], d, 64);
    if (lane >= d) matvec_acc<S>(pw + s * S * S, o, q);
  }
}

// The same scan with the lane shifts of wave_up (no LDS round trips). Rolled,
// with a uniform branch per step: unrolled, the compiler hoists the six step
// matrices' scalar loads and the kernel around the scan spills.
template <int S, class T>
__device__ __forceinline__ void wave_up_dyn(int st, const T (&q)[S], T (&o)[S]) {
  switch (st) {
    case 0:
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = wave_up<1>(q[i]);
      break;
    case 1:
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = wave_up<2>(q[i]);
      break;
    case 2:
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = wave_up<4>(q[i]);
      break;
    case 3:
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = wave_up<8>(q[i]);
      break;
    case 4:
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = wave_up<16>(q[i]);
      break;
    default:
#pragma unroll
      for (int i = 0; i < S; ++i) o[i] = wave_up<32>(q[i]);
      break;
  }
}
template <int S, class T, class MT>
__device__ __forceinline__ void wave_scan_inclusive_fast(T (&q)[S], const MT* __restrict__ pw, int lane) {
#pragma unroll 1
  for (int s = 0; s < 6; ++s) {
    T o[S];
    wave_up_dyn<S>(s, q, o);
    if (lane >= (1 << s)) matvec_acc<S>(pw + s * S * S, o, q);
  }
}

}  // namespace orion
