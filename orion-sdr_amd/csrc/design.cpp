// design.cpp — built with -ffp-contract=off (see design.hpp). Host only.
#include "design.hpp"

#include <algorithm>

#include <cfloat>
#include <cmath>
#include <cstring>
#include <unordered_map>

namespace orion {

namespace {
constexpr float kTau = 6.28318530717958647692f;  // core::f32::consts::TAU
constexpr float kPi = 3.14159265358979323846f;   // core::f32::consts::PI
inline float fmax_rs(float a, float b) { return a > b ? a : (b > a ? b : a); }  // f32::max
inline float clamp_rs(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
}  // namespace

std::vector<float> fir_lowpass_taps(float fs, float pass_hz, float trans_hz) {
  // dsp/fir.rs:17-19: clamp the pass band and transition, odd tap count >= 31.
  pass_hz = fmax_rs(pass_hz, 10.0f);
  trans_hz = fmax_rs(trans_hz, pass_hz * 0.2f);
  size_t ntaps = static_cast<size_t>(std::ceil(fs / trans_hz));
  if (ntaps < 31) ntaps = 31;
  ntaps |= 1u;
  std::vector<float> taps(ntaps);
  const float fc = pass_hz / fs;
  const long half = static_cast<long>(ntaps) / 2;
  for (size_t n = 0; n < ntaps; ++n) {
    const long m = static_cast<long>(n) - half;
    float sinc;
    if (m == 0) {
      sinc = 2.0f * fc;
    } else {
      const float x = kPi * static_cast<float>(m);
      const float arg = 2.0f * kPi * fc * static_cast<float>(m);
      sinc = (2.0f * fc) * std::sin(arg) / x;  // fir.rs:29 evaluation order
    }
    const float w = 0.5f - 0.5f * std::cos(2.0f * kPi * static_cast<float>(n) /
                                           (static_cast<float>(ntaps) - 1.0f));
    taps[n] = sinc * w;
  }
  float s = 0.0f;  // Iterator::sum over f32: sequential left fold
  for (float t : taps) s += t;
  for (float& t : taps) t /= s;
  return taps;
}

static float kaiser_beta(float a) {  // fir.rs:74-82
  if (a > 50.0f) return 0.1102f * (a - 8.7f);
  if (a >= 21.0f) return 0.5842f * std::pow(a - 21.0f, 0.4f) + 0.07886f * (a - 21.0f);
  return 0.0f;
}

static float bessel_i0(float x) {  // fir.rs:86-99
  const float half = 0.5f * x;
  float term = 1.0f, sum = 1.0f;
  for (unsigned k = 1; k <= 40; ++k) {
    term *= half / static_cast<float>(k);
    const float t = term * term;
    sum += t;
    if (t < 1e-12f * sum) break;
  }
  return sum;
}

std::vector<float> kaiser_lowpass_taps(size_t num_taps, float cutoff_norm, float stopband_db) {
  const size_t m = (num_taps < 3 ? size_t{3} : num_taps) | 1u;  // fir.rs:114
  const float mid = static_cast<float>(m / 2);
  const float fc = clamp_rs(cutoff_norm, 1e-4f, 0.4999f);
  const float beta = kaiser_beta(stopband_db);
  const float i0b = bessel_i0(beta);
  std::vector<float> taps(m);
  for (size_t n = 0; n < m; ++n) {
    const float d = static_cast<float>(n) - mid;
    const float ideal = (d == 0.0f) ? 2.0f * fc : std::sin(kTau * fc * d) / (kPi * d);
    const float r = d / mid;
    const float w = bessel_i0(beta * std::sqrt(fmax_rs(1.0f - r * r, 0.0f))) / i0b;
    taps[n] = ideal * w;
  }
  float s = 0.0f;
  for (float t : taps) s += t;
  if (std::fabs(s) > FLT_EPSILON)
    for (float& t : taps) t /= s;
  return taps;
}

float kaiser_transition_norm(size_t num_taps, float stopband_db) {  // fir.rs:147-150
  const float m = static_cast<float>((num_taps < 3 ? size_t{3} : num_taps) | 1u);
  return (fmax_rs(stopband_db, 21.0f) - 8.0f) / (14.36f * m);
}

size_t kaiser_num_taps(float transition_norm, float stopband_db) {  // fir.rs:154-157
  const float m = std::ceil((fmax_rs(stopband_db, 21.0f) - 8.0f) /
                            (14.36f * fmax_rs(transition_norm, 1e-4f)));
  return static_cast<size_t>(fmax_rs(m, 3.0f)) | 1u;
}

static BiquadCoeffs rbj_butterworth_lp(float fs, float fc) {  // iir.rs:51-67, 112-121
  const float w0 = kTau * fc / fs;
  const float sn = std::sin(w0), cs = std::cos(w0);
  const float alpha = sn / (2.0f * std::sqrt(0.5f));
  const float b0 = (1.0f - cs) * 0.5f;
  const float b1 = 1.0f - cs;
  const float b2 = (1.0f - cs) * 0.5f;
  const float a0 = 1.0f + alpha;
  const float a1 = -2.0f * cs;
  const float a2 = 1.0f - alpha;
  const float norm = 1.0f / a0;
  return {b0 * norm, b1 * norm, b2 * norm, a1 * norm, a2 * norm};
}

BiquadCoeffs lp_cascade_design(float fs, float fc) { return rbj_butterworth_lp(fs, fc); }

float dc_blocker_pole(float fs, float cut_hz) {  // dc.rs:17, iir.rs:122
  return clamp_rs(1.0f - 2.0f * kPi * (fmax_rs(cut_hz, 0.1f) / fs), 0.0f, 0.9999f);
}

LpDcCoeffs lpdc_design(float fs, float lp_fc, float dc_cut_hz) {
  return {rbj_butterworth_lp(fs, lp_fc), dc_blocker_pole(fs, dc_cut_hz)};
}

float cw_alpha(float fs, float env_bw_hz) {  // cw.rs:17-18
  const float fc = fmax_rs(env_bw_hz, 1.0f);
  return std::exp(-kTau * fc / fs);
}

Oscillator oscillator(float freq_hz, float fs) {  // rotator.rs:17-18
  Oscillator o;
  const float phi = kTau * freq_hz / fs;
  o.w_re = std::cos(phi);
  o.w_im = std::sin(phi);
  o.theta = std::atan2(static_cast<double>(o.w_im), static_cast<double>(o.w_re));
  // theta/2pi in [-0.5, 0.5] -> wrapping Q0.64. Split to keep 64 bits exact.
  long double rev = static_cast<long double>(o.theta) / (2.0L * 3.14159265358979323846264338327950288L);
  if (rev < 0) rev += 1.0L;
  long double scaled = rev * 18446744073709551616.0L;  // 2^64
  if (scaled >= 18446744073709551616.0L) scaled -= 18446744073709551616.0L;
  o.step_q64 = static_cast<uint64_t>(scaled + 0.5L);
  return o;
}

std::vector<float> phasor_table_q64(uint64_t step_q64, size_t n) {
  // the angle of output k reduced exactly (k step mod 2^64, a Q0.64 turn count), then one
  // double sincos: ~20 ns per entry (a long double sin/cos of k theta: ~200)
  std::vector<float> t(2 * n);
  constexpr double kTurn = 6.283185307179586476925286766559 / 18446744073709551616.0;  // 2 pi / 2^64
  for (size_t k = 0; k < n; ++k) {
    const uint64_t ph = static_cast<uint64_t>(k) * step_q64;
    const double a = static_cast<double>(static_cast<int64_t>(ph)) * kTurn;  // (-pi, pi]
    t[2 * k] = static_cast<float>(std::cos(a));
    t[2 * k + 1] = static_cast<float>(std::sin(a));
  }
  return t;
}

std::vector<float> phasor_table(double theta, size_t n) {
  std::vector<float> t(2 * n);
  for (size_t k = 0; k < n; ++k) {
    const long double a = static_cast<long double>(theta) * static_cast<long double>(k);
    t[2 * k] = static_cast<float>(std::cos(a));
    t[2 * k + 1] = static_cast<float>(std::sin(a));
  }
  return t;
}

// ---- the reference's phasor recurrence -----------------------------------------
uint64_t q64_of_angle(long double rad) {
  constexpr long double kTwoPi = 6.283185307179586476925286766559005768L;
  long double rev = std::fmod(rad / kTwoPi, 1.0L);
  if (rev < 0) rev += 1.0L;
  long double scaled = rev * 18446744073709551616.0L;  // 2^64
  if (scaled >= 18446744073709551616.0L) scaled -= 18446744073709551616.0L;
  return static_cast<uint64_t>(scaled);
}

namespace {
// One reference step (rotator.rs:44-62; nco.rs:42-58 is the same): Rust's mul_add is
// a fused multiply-add, the products, the norm and 1/sqrt are plain f32 operations.
template <class Fma>
inline void rec_step(RecState& s, float wr, float wi, Fma fma) {
  const float zr = fma(s.zr, wr, -s.zi * wi);
  const float zi = fma(s.zi, wr, s.zr * wi);
  s.zr = zr;
  s.zi = zi;
  s.ctr += 1u;
  if ((s.ctr & 0x3FFu) == 0) {
    const float r2 = s.zr * s.zr + s.zi * s.zi;
    const float inv = 1.0f / std::sqrt(r2);
    s.zr *= inv;
    s.zi *= inv;
  }
}
inline uint64_t state_key(const RecState& s) {
  uint32_t a, b;
  std::memcpy(&a, &s.zr, 4);
  std::memcpy(&b, &s.zi, 4);
  return (static_cast<uint64_t>(a) << 32) | b;
}
// The run from output k0 to k1 (z holds 2 k1 floats; s is the state after output
// k0 - 1), stopping at the first repeated renorm-point state. Returns the step count
// of the earlier occurrence (cycle start; z cut there) or UINT64_MAX.
template <class Fma>
uint64_t rec_run(float wr, float wi, RecState& s, uint64_t k0, uint64_t k1, std::vector<float>& z,
                 std::unordered_map<uint64_t, uint64_t>& seen, Fma fma) {
  float* __restrict__ zp = z.data();
  for (uint64_t k = k0; k < k1;) {
    // the steps up to the next renorm point: the rotation alone (no per-step tests)
    const uint64_t to_renorm = 1024u - (s.ctr & 0x3FFu);
    const uint64_t m = std::min<uint64_t>(to_renorm - 1, k1 - k);
    float zr = s.zr, zi = s.zi;
    for (uint64_t i = 0; i < m; ++i) {
      const float nr = fma(zr, wr, -zi * wi);
      const float ni = fma(zi, wr, zr * wi);
      zr = nr;
      zi = ni;
      zp[2 * (k + i)] = zr;
      zp[2 * (k + i) + 1] = zi;
    }
    s.zr = zr;
    s.zi = zi;
    s.ctr += static_cast<uint32_t>(m);
    k += m;
    if (k == k1) break;
    rec_step(s, wr, wi, fma);  // the renorm step
    zp[2 * k] = s.zr;
    zp[2 * k + 1] = s.zi;
    ++k;
    if ((s.ctr & 0x3FFu) == 0) {
      const auto ins = seen.emplace(state_key(s), k);
      if (!ins.second) {
        z.resize(static_cast<size_t>(2 * k));
        return ins.first->second;
      }
    }
  }
  return UINT64_MAX;
}
__attribute__((target("fma"))) uint64_t rec_run_hw(float wr, float wi, RecState& s, uint64_t k0, uint64_t k1,
                                                   std::vector<float>& z, std::unordered_map<uint64_t, uint64_t>& seen) {
  return rec_run(wr, wi, s, k0, k1, z, seen, [](float a, float b, float c) { return __builtin_fmaf(a, b, c); });
}
uint64_t rec_run_sw(float wr, float wi, RecState& s, uint64_t k0, uint64_t k1, std::vector<float>& z,
                    std::unordered_map<uint64_t, uint64_t>& seen) {
  return rec_run(wr, wi, s, k0, k1, z, seen, [](float a, float b, float c) { return std::fma(a, b, c); });
}
}  // namespace

RecBuilder::RecBuilder(float wr, float wi, RecState s0, uint64_t budget, uint64_t min_cycle, uint64_t step_q64)
    : wr_(wr), wi_(wi), s_(s0), s0_(s0), budget_(budget), min_cycle_(min_cycle) {
  t_.ctr0 = s0.ctr;
  t_.mstep = step_q64;
  if ((s0.ctr & 0x3FFu) == 0) seen_.emplace(state_key(s0), 0);
  if (budget_ == 0) finish(UINT64_MAX);
}

void RecBuilder::extend(uint64_t want) {
  if (done_) return;
  const uint64_t k1 = std::min(std::max(want, t_.n), budget_);
  if (k1 > t_.n) {
    t_.z.resize(static_cast<size_t>(2 * k1));
    const uint64_t c0 = __builtin_cpu_supports("fma") ? rec_run_hw(wr_, wi_, s_, t_.n, k1, t_.z, seen_)
                                                      : rec_run_sw(wr_, wi_, s_, t_.n, k1, t_.z, seen_);
    t_.n = t_.z.size() / 2;
    if (c0 != UINT64_MAX) {
      finish(c0);
      return;
    }
  }
  if (t_.n >= budget_) finish(UINT64_MAX);
}

void RecBuilder::finish(uint64_t c0) {
  done_ = true;
  std::unordered_map<uint64_t, uint64_t>().swap(seen_);
  RecTable& t = t_;
  if (c0 != UINT64_MAX) {  // outputs c0 .. n-1 repeat forever
    t.cyc_start = c0;
    t.cyc_len = t.n - c0;
    const uint64_t period = t.cyc_len;
    while (t.cyc_len < min_cycle_) {  // unroll
      for (uint64_t k = 0; k < period; ++k) {
        t.z.push_back(t.z[2 * (c0 + k)]);
        t.z.push_back(t.z[2 * (c0 + k) + 1]);
      }
      t.cyc_len += period;
    }
    t.n = t.z.size() / 2;
    return;
  }
  // No cycle within the budget: outputs beyond n follow a model anchored at the last
  // exact output: its phase, plus the mean step fitted (least squares over the renorm
  // points of the run's last half) and the mean magnitude by renorm-counter position
  // (over its last quarter).
  const RecState s0 = s0_;
  if (t.n == 0) {
    t.mbase = q64_of_angle(std::atan2(static_cast<long double>(s0.zi), static_cast<long double>(s0.zr)));
    return;
  }
  const float wr = wr_, wi = wi_;
  const long double th = std::atan2(static_cast<long double>(wi), static_cast<long double>(wr));
  const long double a0 = std::atan2(static_cast<long double>(s0.zi), static_cast<long double>(s0.zr));
  const uint64_t from = t.n / 2, from_mag = t.n - t.n / 4;
  std::vector<double> msum(1024, 0.0);
  std::vector<uint64_t> mcnt(1024, 0);
  long double sx = 0, sy = 0, sxx = 0, sxy = 0;
  uint64_t np = 0;
  constexpr long double kTwoPi = 6.283185307179586476925286766559005768L;
  for (uint64_t k = from_mag; k < t.n; ++k) {
    const double re = t.z[2 * k], im = t.z[2 * k + 1];
    const uint32_t j = (t.ctr0 + static_cast<uint32_t>(k) + 1u) & 1023u;
    msum[j] += std::sqrt(re * re + im * im);
    mcnt[j] += 1;
  }
  // renorm points: (ctr0 + k + 1) & 1023 == 0
  for (uint64_t k = from + ((1023u - ((t.ctr0 + static_cast<uint32_t>(from)) & 1023u)) & 1023u); k < t.n; k += 1024) {
    const double re = t.z[2 * k], im = t.z[2 * k + 1];
    {  // drift of the phase against the closed form at this renorm point
      const long double ideal = std::fmod(a0 + static_cast<long double>(k + 1) * th, kTwoPi);
      long double e = std::atan2(static_cast<long double>(im), static_cast<long double>(re)) - ideal;
      e = std::remainder(e, kTwoPi);
      const long double x = static_cast<long double>(k + 1);
      sx += x;
      sy += e;
      sxx += x * x;
      sxy += x * e;
      ++np;
    }
  }
  {  // least-squares line through the mean magnitude at each renorm position
    double s0m = 0, s1 = 0, s2 = 0, t0 = 0, t1 = 0;
    for (int j = 0; j < 1024; ++j) {
      if (!mcnt[j]) continue;
      const double m = msum[j] / static_cast<double>(mcnt[j]);
      s0m += 1;
      s1 += j;
      s2 += static_cast<double>(j) * j;
      t0 += m;
      t1 += j * m;
    }
    const double den = s0m * s2 - s1 * s1;
    if (s0m >= 2 && den > 0) {
      const double b = (s0m * t1 - s1 * t0) / den;
      t.mag1 = static_cast<float>(b);
      t.mag0 = static_cast<float>((t0 - b * s1) / s0m);
    }
  }
  long double slope = 0;
  if (np >= 8) {
    const long double den = static_cast<long double>(np) * sxx - sx * sx;
    if (den > 0) slope = (static_cast<long double>(np) * sxy - sx * sy) / den;
  }
  t.mstep = q64_of_angle(th + slope);
  const uint64_t l = t.n - 1;
  t.mbase = q64_of_angle(std::atan2(static_cast<long double>(t.z[2 * l + 1]), static_cast<long double>(t.z[2 * l])));
}

double rec_mean_step(float wr, float wi, uint64_t step_q64) {
  const RecTable t = rec_table(wr, wi, RecState{}, 1ull << 18, 0, step_q64);
  constexpr long double kTwoPi = 6.283185307179586476925286766559005768L;
  if (t.cyc_len) {  // the advance around the cycle, increment by increment
    long double sum = 0;
    for (uint64_t i = 0; i < t.cyc_len; ++i) {
      const uint64_t k = t.cyc_start + i, k1 = i + 1 < t.cyc_len ? k + 1 : t.cyc_start;
      const long double ar = t.z[2 * k], ai = t.z[2 * k + 1], br = t.z[2 * k1], bi = t.z[2 * k1 + 1];
      sum += std::atan2(bi * ar - br * ai, br * ar + bi * ai);  // arg(z[k1] conj z[k])
    }
    return static_cast<double>(sum / static_cast<long double>(t.cyc_len));
  }
  long double a = static_cast<long double>(t.mstep) / 18446744073709551616.0L * kTwoPi;
  if (a > kTwoPi / 2) a -= kTwoPi;
  return static_cast<double>(a);
}

RecTable rec_table(float wr, float wi, RecState s0, uint64_t max_out, uint64_t min_cycle, uint64_t step_q64) {
  RecBuilder b(wr, wi, s0, max_out, min_cycle, step_q64);
  b.extend(max_out);
  return b.table();
}

RecState rec_state_after(const RecTable& t, uint64_t k) {
  RecState s;
  s.ctr = t.ctr0 + static_cast<uint32_t>(k) + 1u;
  uint64_t j = k;
  if (t.cyc_len && j >= t.n) j = t.cyc_start + (j - t.cyc_start) % t.cyc_len;
  if (j < t.n) {
    s.zr = t.z[2 * j];
    s.zi = t.z[2 * j + 1];
    return s;
  }
  constexpr long double kTwoPi = 6.283185307179586476925286766559005768L;
  const uint64_t ph = t.mbase + (k + 1 - t.n) * t.mstep;
  const long double a = static_cast<long double>(ph) / 18446744073709551616.0L * kTwoPi;
  const long double m = static_cast<long double>(t.mag0) + static_cast<long double>(t.mag1) * (s.ctr & 1023u);
  s.zr = static_cast<float>(m * std::cos(a));
  s.zi = static_cast<float>(m * std::sin(a));
  return s;
}

// ---- state-space extraction -------------------------------------------------
// Run one exact-arithmetic (f64) step of the reference update with x = 0 on each
// unit state to obtain the columns of A.
template <class Step>
static std::vector<double> extract_A(int S, Step step) {
  std::vector<double> A(S * S);
  for (int c = 0; c < S; ++c) {
    std::vector<double> s(S, 0.0);
    s[c] = 1.0;
    step(s.data(), 0.0);
    for (int r = 0; r < S; ++r) A[r * S + c] = s[r];
  }
  return A;
}
// B: one step from the zero state with x = 1.
template <class Step>
static std::vector<double> extract_B(int S, Step step) {
  std::vector<double> s(S, 0.0);
  step(s.data(), 1.0);
  return s;
}

static double biquad_step(double* z, double x, const BiquadCoeffs& c) {  // iir.rs:34-40
  const double y = x * c.b0 + z[0];
  const double z1 = x * c.b1 + z[1] - c.a1 * y;
  const double z2 = x * c.b2 - c.a2 * y;
  z[0] = z1;
  z[1] = z2;
  return y;
}

StateSpace lp_cascade_ss(const BiquadCoeffs& c) {
  StateSpace ss;
  ss.S = 4;
  const auto step = [&](double* s, double x) {
    const double y0 = biquad_step(s, x, c);
    biquad_step(s + 2, y0, c);
  };
  ss.A = extract_A(4, step);
  ss.B = extract_B(4, step);
  ss.D = 0;
  return ss;
}

StateSpace biquad_ss(const BiquadCoeffs& c) {  // iir.rs:34-40, state (z1, z2)
  StateSpace ss;
  ss.S = 2;
  const auto step = [&](double* s, double x) { biquad_step(s, x, c); };
  ss.A = extract_A(2, step);
  ss.B = extract_B(2, step);
  ss.D = 0;
  return ss;
}

StateSpace lpdc_ss(const LpDcCoeffs& c) {  // iir.rs:151-165, state (z0_1,z0_2,z1_1,z1_2,dc_x1,dc_y1)
  StateSpace ss;
  ss.S = 6;
  const auto step = [&](double* s, double x) {
    const double y0 = biquad_step(s, x, c.bq);
    const double y1 = biquad_step(s + 2, y0, c.bq);
    const double y = y1 - s[4] + static_cast<double>(c.r) * s[5];
    s[4] = y1;
    s[5] = y;
  };
  ss.A = extract_A(6, step);
  ss.B = extract_B(6, step);
  ss.D = 0;
  return ss;
}

StateSpace dc_ss(float r) {  // dc.rs:47-51, state (x1, y1)
  StateSpace ss;
  ss.S = 2;
  const auto step = [&](double* s, double x) {
    const double y = x - s[0] + static_cast<double>(r) * s[1];
    s[0] = x;
    s[1] = y;
  };
  ss.A = extract_A(2, step);
  ss.B = extract_B(2, step);
  ss.D = 0;
  return ss;
}

StateSpace onepole_ss(float a) {  // cw.rs:40, state y
  StateSpace ss;
  ss.S = 1;
  ss.A = {static_cast<double>(a)};
  ss.B = {static_cast<double>(1.0f - a)};  // s = a s + (1 - a) x, (1 - a) in f32 as iir.hpp RecOnePole
  ss.D = 0;
  return ss;
}

std::vector<double> mat_mul(const std::vector<double>& X, const std::vector<double>& Y, int S) {
  std::vector<double> Z(S * S, 0.0);
  for (int i = 0; i < S; ++i)
    for (int k = 0; k < S; ++k)
      for (int j = 0; j < S; ++j) Z[i * S + j] += X[i * S + k] * Y[k * S + j];
  return Z;
}

std::vector<double> mat_pow(const std::vector<double>& A, int S, uint64_t k) {
  std::vector<double> R(S * S, 0.0);
  for (int i = 0; i < S; ++i) R[i * S + i] = 1.0;
  std::vector<double> P = A;
  while (k) {
    if (k & 1) R = mat_mul(R, P, S);
    P = mat_mul(P, P, S);
    k >>= 1;
  }
  return R;
}

// ---- multicarrier/tx_lowpass.rs:96-185 TxLowpass (host-side sizing helpers) ----
TxLowpassSpec tx_lowpass_for_null_band(size_t n_fft, size_t occupied_half, size_t num_taps, float stopband_db) {
  const float occupied_norm = static_cast<float>(occupied_half) / static_cast<float>(std::max<size_t>(n_fft, 1));
  const float half_transition = 0.5f * kaiser_transition_norm(num_taps, stopband_db);
  const float earliest = occupied_norm + half_transition;  // tx_lowpass.rs:125-128
  const float latest = 0.5f - half_transition;
  const float cutoff = earliest <= latest ? earliest : 0.5f * (occupied_norm + 0.5f);
  return {cutoff, num_taps, stopband_db};
}
size_t tx_lowpass_taps_for_null_band(size_t n_fft, size_t occupied_half, float stopband_db) {  // :141-144
  const float occupied_norm = static_cast<float>(occupied_half) / static_cast<float>(std::max<size_t>(n_fft, 1));
  return kaiser_num_taps(0.5f - occupied_norm, stopband_db);
}
size_t tx_lowpass_group_delay(const TxLowpassSpec& t) { return (std::max<size_t>(t.num_taps, 3) | 1) / 2; }  // :148-150
float tx_lowpass_transition_norm(const TxLowpassSpec& t) { return kaiser_transition_norm(t.num_taps, t.stopband_db); }
bool tx_lowpass_transition_fits(const TxLowpassSpec& t, size_t n_fft, size_t occupied_half) {  // :162-165
  const float occupied_norm = static_cast<float>(occupied_half) / static_cast<float>(std::max<size_t>(n_fft, 1));
  return tx_lowpass_transition_norm(t) <= 0.5f - occupied_norm;
}
float tx_lowpass_stopband_edge_norm(const TxLowpassSpec& t) { return t.cutoff_norm + 0.5f * tx_lowpass_transition_norm(t); }
bool tx_lowpass_fits_guard(const TxLowpassSpec& t, size_t cp_len, size_t roll_off, size_t backoff) {  // :179-182
  const size_t slack = std::min(cp_len > backoff ? cp_len - backoff : 0, backoff);
  return roll_off + tx_lowpass_group_delay(t) <= slack;
}

}  // namespace orion
