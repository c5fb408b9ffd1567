// osc.hpp — the reference's phasor oscillator on the device (host side).
//
// Rotator (dsp/rotator.rs:8-95) and Nco (dsp/nco.rs:11-66) advance z <- z w in f32
// and renormalise every 1024 steps; the result drifts from the ideal phasor by its
// own rounding (1.2e-2 rad after 2^20 steps at -1.5 MHz / 10 MHz). RefOsc tracks that
// recurrence instead of the ideal phasor: at every (re)tune the host runs it from the
// current state (design.hpp rec_table) for up to `budget` outputs, detecting the
// cycle the finite-state map falls into. The device reads the reference's own
// phasors from that table — forever when the cycle closed within the budget
// (bit-exact), else for the first `budget` outputs, then the drift model (the fitted
// mean step and a linear magnitude over each renorm period). budget 0: the closed form (the ideal phasor of
// the reference's f32 step w), which is what the engine computed before round 4.
#pragma once
#include <cstdint>

#include "blocks.hpp"

namespace orion {

constexpr uint64_t kNcoTableDefault = 1ull << 20;  // outputs tabulated per (re)tune
constexpr uint64_t kNcoTableMax = 1ull << 28;      // 2 GiB of device table

class RefOsc {
 public:
  RefOsc(float freq_hz, float fs, uint64_t budget = kNcoTableDefault);
  // set_freq (rotator.rs:35-39, nco.rs:33-38): a new step w; z and renorm_ctr carry on.
  void retune(float freq_hz, float fs);
  // reset_phase (rotator.rs:28-31): z = 1 + 0j, renorm_ctr = 0, the step stays.
  void reset();
  // Tabulation budget (orion_block_configure ORION_OPT_NCO_TABLE); the state carries on.
  void set_budget(uint64_t budget);
  uint64_t budget() const { return budget_; }
  // The device view; the next call's output i is oscillator output count() + i.
  OscDev dev() const;
  uint64_t count() const { return k_; }
  void advance(uint64_t n) { k_ += n; }
  const Oscillator& osc() const { return osc_; }
  float fs() const { return fs_; }
  // Every output is the reference's own (a cycle closed within the budget).
  bool exact_forever() const { return tab_.cyc_len != 0; }
  uint64_t exact_outputs() const { return tab_.cyc_len ? UINT64_MAX : tab_.n; }

 private:
  void build(const RecState& st, uint64_t closed_anchor_q64);
  RecState state() const;        // the reference's (z, renorm_ctr) after count() outputs
  uint64_t closed_anchor() const;  // closed form: the Q0.64 phase after count() outputs
  float fs_;
  uint64_t budget_;
  Oscillator osc_{};
  RecTable tab_;
  RecState org_;  // start state of tab_
  uint64_t k_ = 0;
  DevBuf dtab_, dmtab_;
};

}  // namespace orion
