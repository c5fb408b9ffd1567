// design.hpp — host-side filter/oscillator design for the MI355X engine.
//
// These run once at block construction (never on the sample path) and must
// produce the reference's f32 coefficients bit for bit, so design.cpp is built
// with -ffp-contract=off and calls the same libm functions Rust's f32 methods
// lower to. Each routine cites the reference constructor it restates.
#pragma once
#include <cstddef>
#include <cstdint>
#include <unordered_map>
#include <vector>

namespace orion {

// dsp/fir.rs:16-44 FirLowpass::design (sinc x Hann, normalised by the tap sum).
std::vector<float> fir_lowpass_taps(float fs, float pass_hz, float trans_hz);

// dsp/fir.rs:74-141 Kaiser-windowed low-pass; :147-157 sizing helpers.
std::vector<float> kaiser_lowpass_taps(size_t num_taps, float cutoff_norm, float stopband_db);
float kaiser_transition_norm(size_t num_taps, float stopband_db);
size_t kaiser_num_taps(float transition_norm, float stopband_db);

// dsp/iir.rs:49-71 LpCascade::design -> {b0,b1,b2,a1,a2} shared by both biquads.
struct BiquadCoeffs { float b0, b1, b2, a1, a2; };
BiquadCoeffs lp_cascade_design(float fs, float fc);
// dsp/iir.rs:111-137 LpDcCascade::design -> biquad coeffs + DC pole r.
struct LpDcCoeffs { BiquadCoeffs bq; float r; };
LpDcCoeffs lpdc_design(float fs, float lp_fc, float dc_cut_hz);
// dsp/dc.rs:15-21 DcBlocker::new pole.
float dc_blocker_pole(float fs, float cut_hz);
// demodulate/cw.rs:15-25 one-pole alpha.
float cw_alpha(float fs, float env_bw_hz);

// dsp/rotator.rs:16-26: the reference's f32 step phasor w = (cos phi, sin phi),
// phi = f32(TAU*f/fs). The engine generates phasors in closed form from the
// exact angle of that f32 phasor: theta = atan2(w.im, w.re), carried as a
// Q0.64 fraction of a revolution so that phase(n) = n*step mod 2^64 is exact
// integer arithmetic on the device (error <= n * 2^-65 rev).
struct Oscillator {
  float w_re, w_im;     // the reference's f32 step phasor
  double theta;         // its exact angle (rad), in (-pi, pi]
  uint64_t step_q64;    // theta / 2pi as a wrapping Q0.64 fraction of a turn
};
Oscillator oscillator(float freq_hz, float fs);

// Phasor e^{j*theta*k} for k = 0..n-1, computed in f64 and rounded to f32 pairs.
std::vector<float> phasor_table(double theta, size_t n);
// The same for a Q0.64 step (turns): e^{j 2 pi k step / 2^64}, k < n.
std::vector<float> phasor_table_q64(uint64_t step_q64, size_t n);

// ---- the reference's phasor recurrence (rotator.rs:44-62, nco.rs:42-58) ----------
// z <- (fma(z.re, w.re, -(z.im w.im)), fma(z.im, w.re, z.re w.im)) in f32, then when
// (++ctr & 0x3FF) == 0, z *= 1/sqrt(re^2 + im^2). A finite-state map: renormalised,
// z stays in a thin annulus, so the trajectory is eventually periodic. Sampled at
// the renorm points (where the state is z alone), the period is often short
// (-1.5 MHz / 10 MHz: 16 renorms of tail, then a cycle of 5 renorms = 5120 steps),
// and then a table of tail + cycle reproduces the reference bit for bit forever.
struct RecState {
  float zr = 1.0f, zi = 0.0f;  // the phasor (Rotator::z / Nco::z)
  uint32_t ctr = 0;            // renorm_ctr
};
struct RecTable {
  std::vector<float> z;        // exact outputs k < n: the phasor after k + 1 steps (re, im)
  uint64_t n = 0;
  uint64_t cyc_start = 0;      // cyc_len > 0: output k >= n equals output
  uint64_t cyc_len = 0;        //   cyc_start + (k - cyc_start) mod cyc_len
  // beyond n when there is no cycle (a model of the drift, not the reference):
  uint64_t mbase = 0;          // Q0.64 phase of output n - 1 (the last exact one)
  uint64_t mstep = 0;          // fitted mean step: phase(k) = mbase + (k + 1 - n) mstep
  float mag0 = 1.0f, mag1 = 0.0f;  // mean magnitude mag0 + mag1 ((ctr0 + k + 1) & 1023): within a
                                   // renorm period |z| moves linearly to ~1e-8 (|w| != 1 in f32)
  uint32_t ctr0 = 0;           // renorm_ctr of the start state
};
// Runs the recurrence with step (wr, wi) from s0 for at most max_out outputs,
// detecting a cycle at the renorm points; a cycle shorter than min_cycle outputs is
// unrolled (replicated) to at least min_cycle, so a kernel wraps a tile with one
// subtraction. step_q64: the closed-form step (the model's starting estimate).
RecTable rec_table(float wr, float wi, RecState s0, uint64_t max_out, uint64_t min_cycle, uint64_t step_q64);
// The same table built incrementally (osc.hpp RefOsc: a retune tabulates only what the
// next calls use): extend(want) runs the recurrence on to min(want, budget) outputs;
// reaching the budget or closing the cycle finalises it (cycle unrolled / drift model
// fitted), after which table() equals rec_table(..., budget, ...).
class RecBuilder {
 public:
  RecBuilder() = default;
  RecBuilder(float wr, float wi, RecState s0, uint64_t budget, uint64_t min_cycle, uint64_t step_q64);
  void extend(uint64_t want);
  bool done() const { return done_; }
  const RecTable& table() const { return t_; }
  RecTable& table() { return t_; }

 private:
  void finish(uint64_t cycle_start);
  float wr_ = 1.0f, wi_ = 0.0f;
  RecState s_, s0_;
  uint64_t budget_ = 0, min_cycle_ = 0;
  std::unordered_map<uint64_t, uint64_t> seen_;
  RecTable t_;
  bool done_ = false;
};
// The phasor of output k of a table (exact, or the model beyond it) and the state
// after output k (for set_freq: the reference keeps z and renorm_ctr).
RecState rec_state_after(const RecTable& t, uint64_t k);
// The long-run phase step (radians) of the recurrence with step (wr, wi) from z = 1:
// the exact mean over its cycle when it closes within 2^18 outputs, else the slope
// fitted to its renorm points (RecTable mstep). step_q64: the closed-form step.
double rec_mean_step(float wr, float wi, uint64_t step_q64);
// Q0.64 fraction of a turn of an angle in radians.
uint64_t q64_of_angle(long double rad);

// multicarrier/tx_lowpass.rs:88-185 TxLowpass: the spec and its sizing helpers (f32
// arithmetic as the reference). filter() is FirLowpassIq::design(num_taps, cutoff, stopband).
struct TxLowpassSpec { float cutoff_norm; size_t num_taps; float stopband_db; };
TxLowpassSpec tx_lowpass_for_null_band(size_t n_fft, size_t occupied_half, size_t num_taps, float stopband_db);
size_t tx_lowpass_taps_for_null_band(size_t n_fft, size_t occupied_half, float stopband_db);
size_t tx_lowpass_group_delay(const TxLowpassSpec& t);
float tx_lowpass_transition_norm(const TxLowpassSpec& t);
bool tx_lowpass_transition_fits(const TxLowpassSpec& t, size_t n_fft, size_t occupied_half);
float tx_lowpass_stopband_edge_norm(const TxLowpassSpec& t);
bool tx_lowpass_fits_guard(const TxLowpassSpec& t, size_t cp_len, size_t roll_off, size_t backoff);

// ---- linear state-space form of the IIR recurrences (for chunked scans) ----
// A recurrence s' = A s + B x, y = C s + D x with S states. We derive A, B, C, D
// numerically (f64) from the reference per-sample update so that they match it
// exactly in real arithmetic. Matrices are row-major S x S.
struct StateSpace {
  int S;
  std::vector<double> A, B, C;
  double D;
};
StateSpace lp_cascade_ss(const BiquadCoeffs& c);           // S = 4
StateSpace biquad_ss(const BiquadCoeffs& c);               // S = 2 (one TDF-II biquad)
StateSpace lpdc_ss(const LpDcCoeffs& c);                   // S = 6 (LP4 + DC blocker)
StateSpace dc_ss(float r);                                 // S = 2 (x1, y1)
StateSpace onepole_ss(float a);                            // S = 1 (cw)
// (A^k) for k >= 0, row-major, f64.
std::vector<double> mat_pow(const std::vector<double>& A, int S, uint64_t k);
std::vector<double> mat_mul(const std::vector<double>& X, const std::vector<double>& Y, int S);

}  // namespace orion
