// design.hpp — host-side filter/oscillator design for the MI355X engine.
//
// These run once at block construction (never on the sample path) and must
// produce the reference's f32 coefficients bit for bit, so design.cpp is built
// with -ffp-contract=off and calls the same libm functions Rust's f32 methods
// lower to. Each routine cites the reference constructor it restates.
#pragma once
#include <cstddef>
#include <cstdint>
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
