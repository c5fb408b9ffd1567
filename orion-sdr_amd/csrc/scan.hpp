// scan.hpp — chunked state-carry scan for the reference's stateful recurrences.
//
// Blocks whose output depends on an IIR state (LpCascade, LpDcCascade,
// DcBlocker, the CW one-pole, and the demodulators built on them) run as three
// launches per call:
//   agg   : every workgroup (CH = 4096 samples, 16 per lane) runs the reference
//           update from a zero state and reduces its lanes' end states to one
//           workgroup aggregate (wave Kogge-Stone + cross-wave combine);
//   carry : one workgroup per channel scans the aggregates with the carried
//           stream state -> the exact state entering every workgroup;
//   apply : every workgroup recomputes its lane aggregates, derives each lane's
//           exact entering state and re-runs the reference update to produce
//           outputs; the workgroup holding the last sample stores the carried
//           state for the next call.
// Inputs are staged through LDS with coalesced loads; LDS rows are padded one
// slot every 16 so the 16-samples-per-lane reads are bank-conflict free.
#pragma once
#include <cstdint>

#include "hip_common.hpp"
#include "iir.hpp"

namespace orion {

constexpr int kScanC = 16;                 // samples per lane
constexpr int kScanNT = 256;               // lanes per workgroup
constexpr int kScanCH = kScanC * kScanNT;  // samples per workgroup (4096)
constexpr int kScanCarry = 8;              // carried floats per channel: state[<=6], prev[2]

// Front ends (the per-sample map before the recurrence), one per reference block.
enum class Pre : int {
  Real = 0,    // f32 input (LpCascade / DcBlocker blocks)
  Fm = 1,      // demodulate/fm.rs:60-68 (optionally translated, fm.rs:48-58)
  Pm = 2,      // demodulate/pm.rs:54-58
  Ssb = 3,     // demodulate/ssb.rs:33-38 (BFO rotator)
  AmSqrt = 4,  // demodulate/am.rs:201-205, LP stage before the sqrt map
  AmAbs = 5,   // demodulate/am.rs:232-239
  Cw = 6,      // demodulate/cw.rs:38-39
  RealLp = 7,      // f32 input through the LP4 (+ DC) of LpDcCascade::process (iir.rs:151-165)
  RealLpSqrt = 8,  // the same with sqrt between LP4 and DC: process_mapped(x, f32::sqrt) (iir.rs:170-186)
  RealLpAbs = 9,   // the same with abs: process_mapped(x, f32::abs)
};
enum class Post : int { Id = 0, Sqrt = 1, Gain = 2, Abs = 3 };
enum class RecK : int { LP4 = 0, LPDC = 1, DC = 2, ONEPOLE = 3, BQ = 4 };

// Matrices of the chunk transition, all S x S row-major f32, in one device buffer.
struct ScanMatsLayout {
  static constexpr int kPwc = 0;    // (A^C)^(2^s), s = 0..5
  static constexpr int kM64 = 6;    // A^(64C)
  static constexpr int kPch = 7;    // (A^CH)^(2^s), s = 0..7
  static constexpr int kLane = 15;  // A^(C*L), L = 0..63
  static constexpr int kM128 = 79;  // A^(128C): the wave-to-wave step of k_lpdc_sp at 2C samples per lane
  static constexpr int kCount = 80;
};

struct ScanCoef {
  float b0, b1, b2, a1, a2;  // biquad (LP4 / LPDC)
  float r;                   // DC pole (LPDC / DC)
  float a;                   // one-pole (CW)
  float k;                   // discriminator gain (FM: 1/dev, PM: k)
  float k1, k2;              // AM AbsApprox
  float gain;                // CW set_gain
};

struct ScanArgs {
  const void* x;  long long x_stride;  // inputs: cf32 or f32, [ch][x_stride]
  void* y;        long long y_stride;  // outputs: f32, [ch][y_stride]
  long long n;                         // samples this call
  long long k0;                        // oscillator output of sample 0 (translator / BFO)
  int translate;                       // Pre::Fm: apply the fm.rs:48-58 translator
  OscDev osc;                          // the translator's / BFO's Rotator (hip_common.hpp)
  const double* mats;                  // ScanMatsLayout (f64: see iir.hpp matvec_acc)
  const float* zmap;                   // k_scan_sp: [kSpC][S] A^(kSpC-1-i) B, a lane run's zero-state map
  double* aggs;                        // [ch][nblk][S]
  double* sin;                         // [ch][nblk][S] state entering each workgroup
  const float* carry_in;               // [ch][kScanCarry]
  float* carry_out;                    // [ch][kScanCarry]
  ScanCoef c;
  int* err;                            // host-visible error word: a look-back wait timed out (single pass)
  uint32_t spin;                       // polls before a look-back wait times out (hip_common.hpp)
};

void launch_scan(RecK rec, Pre pre, Post post, const ScanArgs& a, int nch, hipStream_t s);
// Single-pass LpDcCascade (Pre::Ssb / Pre::AmAbs): LP4 warm-up of kSpWarm samples
// per chunk (valid when ||A_lp^kSpWarm|| is negligible), DC state by decoupled
// look-back. mats_lp: ScanMatsLayout for the LP4 state space (S = 4); rec:
// lpdc_sp_chunks(n) * nch * 8 u32 look-back records; epoch: this launch's tag.
constexpr int kSpWarm = 256;
long long lpdc_sp_chunks(long long n);
// k_lpdc_sp's own geometry: kSpC samples per lane (2 kScanC: the wave scans and the
// LP4 state folding cost per lane, not per sample, so longer lane runs amortise them),
// chunks of kSpCH samples.
constexpr int kSpC = 2 * kScanC;
constexpr int kSpCH = kSpC * kScanNT;
constexpr int kLpdcSC = 32;  // k_lpdc_sp's samples per lane
long long lpdc_sp_demod_chunks(long long n, int sc, int warm);  // warm: kSpWarm, or 0 for the DcBlocker alone
// SsbPhasingMod in one pass (k_ssb_mod_sp): valid when ||A_lp^kSpWarm|| is
// negligible; mats_lp = the LP4 scan matrices; carry = [I 4][Q 4] floats.
void launch_ssb_mod_sp(const float* x, f2* y, long long n, uint64_t k0, const OscDev& aud, const OscDev& rf,
                       float side, const ScanCoef& c, const double* mats_lp, const float* zmap_lp,
                       const float* carry_in, float* carry_out, hipStream_t s);
void launch_lpdc_sp(Pre pre, const ScanArgs& a, const double* mats_lp, int nch, uint32_t* rec, uint32_t epoch,
                    hipStream_t s);
int scan_state_dim(RecK rec);
// Single-pass scan (k_scan_sp) for LpCascade / FM / PM / AM PowerSqrt / CW when the
// recurrence forgets its state within one kSpCH-sample chunk (the host checks
// ||A^kSpCH|| < 1e-10): chunk c starts from chunk c-1's zero-state end state.
// recs: scan_sp_chunks(n) * nch * 16 u32 records; epoch: this launch's tag.
bool scan_sp_supported(RecK rec, Pre pre, Post post);
long long scan_sp_chunks(long long n);
// trs: 3, 4 or 5 when the stage also forgets within 2^trs lane runs of kSpC samples
// (||A^(2^trs kSpC)|| < 1e-10): the lane scan is truncated to that horizon; 0: full.
void launch_scan_sp(RecK rec, Pre pre, Post post, const ScanArgs& a, int nch, uint32_t* recs, uint32_t epoch,
                    int trs, hipStream_t s);

}  // namespace orion
