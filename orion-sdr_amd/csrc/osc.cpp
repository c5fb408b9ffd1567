// osc.cpp — RefOsc (osc.hpp): the reference's phasor recurrence, tabulated per tune.
#include "osc.hpp"

#include "kernels.hpp"

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

constexpr uint64_t kOscFirst = 4096;   // outputs tabulated at a (re)tune before any call asks
// Outputs tabulated past a call's last one while the table grows: the longest tile a
// kernel forms one cursor for (kRotTile; k_mod's tiles are shorter, the scans' runs lie
// inside the call), so every run of the call is table-only.
constexpr uint64_t kOscMargin = static_cast<uint64_t>(kRotTile);

RefOsc::RefOsc(float freq_hz, float fs, uint64_t budget)
    : fs_(fs), budget_(budget > kNcoTableMax ? kNcoTableMax : budget), osc_(checked_oscillator(freq_hz, fs)) {
  for (auto& e : ev_) ORION_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  reset();
}

RefOsc::~RefOsc() {
  for (auto& e : ev_)
    if (e) (void)hipEventDestroy(e);
}

RecState RefOsc::state() {
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
  rb_.extend(k_);  // no-op unless outputs were advanced past the table
  return rec_state_after(tab(), k_ - 1);
}

uint64_t RefOsc::closed_anchor() {
  if (budget_ == 0) return tab().mbase + k_ * tab().mstep;  // phase(k) = mbase + (k + 1) mstep
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

// Construction and reset_phase tabulate the whole budget at once (a block's setup, outside
// its streaming calls); retune and set_budget tabulate on demand (dev()).
void RefOsc::reset() {
  build(RecState{}, 0);
  rb_.extend(budget_);
}

void RefOsc::set_budget(uint64_t budget) {
  if (budget > kNcoTableMax) throw std::invalid_argument("NCO table budget above 2^28 outputs");
  const RecState st = state();
  const uint64_t anchor = closed_anchor();
  budget_ = budget;
  build(st, anchor);
}

void RefOsc::build(const RecState& st, uint64_t closed_anchor_q64) {
  // leave the current device tables to the kernels that may still read them
  if (used_[cur_] && !multi_[cur_]) ORION_HIP(hipEventRecord(ev_[cur_], last_s_[cur_]));
  cur_ ^= 1;
  if (used_[cur_]) {  // used two tunes ago: wait until that work has drained
    if (multi_[cur_]) ORION_HIP(hipDeviceSynchronize());
    else ORION_HIP(hipEventSynchronize(ev_[cur_]));
  }
  used_[cur_] = multi_[cur_] = false;
  last_s_[cur_] = nullptr;
  up_ = 0;
  mt_up_ = false;
  org_ = st;
  k_ = 0;
  pad_up_ = false;
  {  // the previous tune's host table storage, reused (no page faults on the next extend)
    std::vector<float> z = std::move(rb_.table().z);
    z.clear();
    rb_ = RecBuilder(osc_.w_re, osc_.w_im, st, budget_, kOscSpan, osc_.step_q64);
    if (rb_.table().z.empty()) rb_.table().z.swap(z);
  }
  if (budget_ == 0) {  // the closed form: no table, the model from this phase on
    rb_.table().ctr0 = st.ctr;
    rb_.table().mbase = closed_anchor_q64;
    rb_.table().mstep = osc_.step_q64;
    rb_.table().mag0 = 1.0f;
    rb_.table().mag1 = 0.0f;
  } else {
    rb_.extend(std::min<uint64_t>(kOscFirst, budget_));
  }
}

// New table entries [up_, n) and the kOscSpan entries past n (OscDev: a run reads
// tab[j + off] unwrapped): the cycle's continuation, or the last entry repeated (never
// a used value); once the table is final, the model's step table.
void RefOsc::upload(hipStream_t s) {
  const RecTable& t = tab();
  if (t.n > up_ || (t.n && up_ == 0)) {
    const uint64_t cap = budget_ + 3 * static_cast<uint64_t>(kOscSpan);
    if (dtab_[cur_].size() < cap * sizeof(f2)) {  // first use of this buffer (or a larger budget)
      if (dtab_[cur_].size()) ORION_HIP(hipDeviceSynchronize());
      dtab_[cur_].resize(cap * sizeof(f2));
    }
    const uint64_t n0 = up_ ? up_ : 0;
    char* d = dtab_[cur_].as<char>();
    // pageable sources: the copy has read them when hipMemcpyAsync returns
    ORION_HIP(hipMemcpyAsync(d + n0 * sizeof(f2), t.z.data() + 2 * n0, (t.n - n0) * sizeof(f2),
                             hipMemcpyHostToDevice, s));
    up_ = t.n;
  }
  if (!pad_up_ && rb_.done() && t.cyc_len) {
    // A final table with a cycle: the run past n continues the cycle (runs read tab[j + off]
    // unwrapped). Without a cycle the entries past n are never used (the model serves
    // them; reads there stay inside the allocation), so nothing is uploaded for them.
    std::vector<float> pad(2 * static_cast<size_t>(kOscSpan));
    for (uint64_t i = 0; i < static_cast<uint64_t>(kOscSpan); ++i) {
      const uint64_t src = t.cyc_start + i % t.cyc_len;
      pad[2 * i] = t.z[2 * src];
      pad[2 * i + 1] = t.z[2 * src + 1];
    }
    ORION_HIP(hipMemcpyAsync(dtab_[cur_].as<char>() + t.n * sizeof(f2), pad.data(), pad.size() * sizeof(float),
                             hipMemcpyHostToDevice, s));
    pad_up_ = true;
  }
  if (!mt_up_ && rb_.done()) {
    dmtab_[cur_].resize(2 * static_cast<size_t>(kOscSpan) * sizeof(float));
    launch_phasor_table_q64(dmtab_[cur_].as<f2>(), t.mstep, kOscSpan, s);
    mt_up_ = true;
  }
}

OscDev RefOsc::dev(uint64_t n, hipStream_t s) {
  // the launch's range plus the longest tile past it (every run a kernel forms lies in the table)
  if (!rb_.done()) rb_.extend(k_ + n + kOscMargin);
  upload(s);
  // used_ (not a non-null last stream) says a stream was seen: the null stream is a
  // stream of its own here (null then a non-blocking stream is two streams)
  if (used_[cur_] && last_s_[cur_] != s) multi_[cur_] = true;
  last_s_[cur_] = s;
  used_[cur_] = true;
  const RecTable& t = tab();
  if (!dmtab_[cur_].size()) {  // never read before the table is final (runs lie in the table)
    dmtab_[cur_].resize(2 * kOscSpan * sizeof(float));
    dmtab_[cur_].zero(s);
  }
  OscDev d{};
  d.tab = t.n ? dtab_[cur_].as<f2>() : nullptr;
  d.mtab = dmtab_[cur_].as<f2>();
  d.n_tab = t.n;
  d.cyc_start = t.cyc_start;
  d.cyc_len = t.cyc_len;
  d.mbase = t.mbase;
  d.mstep = t.mstep;
  d.ctr0 = t.ctr0;
  d.mag0 = t.mag0;
  d.mag1 = t.mag1;
  return d;
}

}  // namespace orion
