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
  ~RefOsc();
  RefOsc(const RefOsc&) = delete;
  RefOsc& operator=(const RefOsc&) = delete;
  // set_freq (rotator.rs:35-39, nco.rs:33-38): a new step w; z and renorm_ctr carry on.
  void retune(float freq_hz, float fs);
  // reset_phase (rotator.rs:28-31): z = 1 + 0j, renorm_ctr = 0, the step stays.
  void reset();
  // Tabulation budget (orion_block_configure ORION_OPT_NCO_TABLE); the state carries on.
  void set_budget(uint64_t budget);
  uint64_t budget() const { return budget_; }
  // The device view for a launch on stream s whose outputs are count() .. count() + n - 1:
  // tabulates on the host and uploads (stream-ordered on s) whatever of that range the
  // table does not hold yet. Construction and reset tabulate the whole budget up front;
  // a retune only restarts the recurrence, so its tabulation cost follows the samples
  // actually produced after it (a retune used to run 2^20 steps, upload
  // 8 MiB and synchronise the device).
  OscDev dev(uint64_t n, hipStream_t s);
  uint64_t count() const { return k_; }
  void advance(uint64_t n) { k_ += n; }
  void seek(uint64_t k) { k_ = k; }  // the next output index (tabulated on demand by dev())
  const Oscillator& osc() const { return osc_; }
  float fs() const { return fs_; }

 private:
  void build(const RecState& st, uint64_t closed_anchor_q64);
  void upload(hipStream_t s);
  RecState state();                // the reference's (z, renorm_ctr) after count() outputs
  uint64_t closed_anchor();        // closed form: the Q0.64 phase after count() outputs
  const RecTable& tab() const { return rb_.table(); }
  float fs_;
  uint64_t budget_;
  Oscillator osc_{};
  RecBuilder rb_;
  RecState org_;  // start state of the table
  uint64_t k_ = 0;
  // Two device tables, alternating per (re)tune: kernels of the previous tune may still
  // read theirs. A buffer is rewritten only after the work that used it has drained
  // (an event on the stream it was used on; a device sync if several streams used it).
  DevBuf dtab_[2], dmtab_[2];
  hipEvent_t ev_[2] = {nullptr, nullptr};
  bool used_[2] = {false, false}, multi_[2] = {false, false};
  hipStream_t last_s_[2] = {nullptr, nullptr};
  int cur_ = 0;
  uint64_t up_ = 0;       // table entries uploaded to dtab_[cur_] (their padding included)
  bool mt_up_ = false;    // dmtab_[cur_] holds this tune's model steps
  bool pad_up_ = false;   // dtab_[cur_] holds the cycle's continuation past n (final tables with a cycle)
};

}  // namespace orion
