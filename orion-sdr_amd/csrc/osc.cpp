// osc.cpp — RefOsc (osc.hpp): the reference's phasor recurrence, tabulated per tune.
#include "osc.hpp"

#include <cmath>
#include <stdexcept>
#include <vector>

namespace orion {

namespace {
constexpr float kTauF = 6.28318530717958647692f;  // core::f32::consts::TAU
constexpr long double kTwoPiL = 6.283185307179586476925286766559005768L;

// rotator.rs:17 / nco.rs:21: phi = TAU * f / fs in f32. A non-finite phi (fs = 0)
// gives the reference a NaN step and NaN output forever; the engine rejects it.
Oscillator checked_oscillator(float f, float fs) {
  if (!std::isfinite(kTauF * f / fs)) throw std::invalid_argument("oscillator: TAU * freq / fs is not finite");
  return oscillator(f, fs);
}
}  // namespace

RefOsc::RefOsc(float freq_hz, float fs, uint64_t budget)
    : fs_(fs), budget_(budget > kNcoTableMax ? kNcoTableMax : budget), osc_(checked_oscillator(freq_hz, fs)) {
  build(RecState{}, 0);
}

RecState RefOsc::state() const {
  if (k_ == 0) return org_;
  if (budget_ == 0) {  // closed form: the ideal phasor after k_ steps
    const uint64_t ph = closed_anchor();
    const long double a = static_cast<long double>(ph) / 18446744073709551616.0L * kTwoPiL;
    RecState s;
    s.zr = static_cast<float>(std::cos(a));
    s.zi = static_cast<float>(std::sin(a));
    s.ctr = org_.ctr + static_cast<uint32_t>(k_);
    return s;
  }
  return rec_state_after(tab_, k_ - 1);
}

uint64_t RefOsc::closed_anchor() const {
  if (budget_ == 0) return tab_.mbase + k_ * tab_.mstep;  // phase(k) = mbase + (k + 1) mstep
  const RecState s = state();
  return q64_of_angle(std::atan2(static_cast<long double>(s.zi), static_cast<long double>(s.zr)));
}

void RefOsc::retune(float freq_hz, float fs) {
  const Oscillator o = checked_oscillator(freq_hz, fs);
  const RecState st = state();
  const uint64_t anchor = closed_anchor();
  osc_ = o;
  fs_ = fs;
  build(st, anchor);
}

void RefOsc::reset() { build(RecState{}, 0); }

void RefOsc::set_budget(uint64_t budget) {
  if (budget > kNcoTableMax) throw std::invalid_argument("NCO table budget above 2^28 outputs");
  const RecState st = state();
  const uint64_t anchor = closed_anchor();
  budget_ = budget;
  build(st, anchor);
}

void RefOsc::build(const RecState& st, uint64_t closed_anchor_q64) {
  ORION_HIP(hipDeviceSynchronize());  // kernels in flight may still read the old tables
  org_ = st;
  k_ = 0;
  if (budget_ == 0) {
    tab_ = RecTable{};
    tab_.ctr0 = st.ctr;
    tab_.mbase = closed_anchor_q64;
    tab_.mstep = osc_.step_q64;
  } else {
    tab_ = rec_table(osc_.w_re, osc_.w_im, st, budget_, kOscSpan, osc_.step_q64);
  }
  if (tab_.n) {
    // kOscSpan entries past the table (OscDev: a run reads tab[j + off] unwrapped): the
    // cycle's continuation, or the last entry repeated (never a used value).
    std::vector<float> z(tab_.z);
    z.resize(2 * (tab_.n + kOscSpan));
    for (uint64_t i = 0; i < static_cast<uint64_t>(kOscSpan); ++i) {
      const uint64_t src = tab_.cyc_len ? tab_.cyc_start + i % tab_.cyc_len : tab_.n - 1;
      z[2 * (tab_.n + i)] = tab_.z[2 * src];
      z[2 * (tab_.n + i) + 1] = tab_.z[2 * src + 1];
    }
    dtab_.upload(z.data(), z.size() * sizeof(float));
  }
  const double th = static_cast<double>(static_cast<long double>(tab_.mstep) / 18446744073709551616.0L * kTwoPiL);
  const auto mt = phasor_table(th, kOscSpan);
  dmtab_.upload(mt.data(), mt.size() * sizeof(float));
}

OscDev RefOsc::dev() const {
  OscDev d{};
  d.tab = tab_.n ? dtab_.as<f2>() : nullptr;
  d.mtab = dmtab_.as<f2>();
  d.n_tab = tab_.n;
  d.cyc_start = tab_.cyc_start;
  d.cyc_len = tab_.cyc_len;
  d.mbase = tab_.mbase;
  d.mstep = tab_.mstep;
  d.ctr0 = tab_.ctr0;
  d.mag0 = tab_.mag0;
  d.mag1 = tab_.mag1;
  return d;
}

}  // namespace orion
