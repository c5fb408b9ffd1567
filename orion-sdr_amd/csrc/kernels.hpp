// kernels.hpp — launch interfaces of the gfx950 kernels (host side).
// Every pointer named *_dev is device memory; every launch is asynchronous on
// the given stream and allocation-free (graph-capturable).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hip_common.hpp"

namespace orion {

// ---------------------------------------------------------------- NCO --
// Rotator / Nco kernel tile (k_fir.hip k_rotator): samples per workgroup tile.
constexpr int kRotTile = 4096;
// ---- analog modulators (k_mod.hip; modulate/am.rs, fm.rs, ssb.rs) ----
// Every oscillator: o (hip_common.hpp OscDev), sample i of a call = output k0 + i.
void launch_am_mod(const float* x, f2* y, long long n, uint64_t k0, const OscDev& o, float cl, float mi, float g,
                   bool clamp, hipStream_t s);
// pm.rs:36-47: out = mix_with_nco((cos kp x, sin kp x) * g, rf phasor)
void launch_pm_mod(const float* x, f2* y, long long n, uint64_t k0, const OscDev& o, float kp, float g, hipStream_t s);
// u = [x p.re | x p.im] (planar, 2n floats), p = audio NCO phasor
void launch_ssb_mod_front(const float* x, float* u, long long n, uint64_t k0, const OscDev& o, hipStream_t s);
// y = (v[i], side v[n + i]) * rf phasor
void launch_ssb_mod_back(const float* v, f2* y, long long n, uint64_t k0, const OscDev& o, float side, hipStream_t s);
// FM phase accumulator: sums = fm_mod_chunks(n) uint64 of workspace; carry_in /
// carry_out: the running phase as a Q0.64 turn count (one uint64 each, ping-pong
// between calls; zero = phase 0); o: the RF Nco.
long long fm_mod_chunks(long long n);
// Single-pass form: rec = fm_mod_chunks(n) * 8 u32 look-back records (zeroed when
// allocated), epoch = this launch's tag (never reused while a record may hold it).
// err: the handle's host-visible error word (a look-back wait that timed out).
void launch_fm_mod_sp(const float* x, f2* y, long long n, float kf, float gain, uint32_t* rec, uint32_t epoch,
                      const uint64_t* carry_in, uint64_t* carry_out, uint64_t k0, const OscDev& o, int* err,
                      hipStream_t s);
void launch_fm_mod(const float* x, f2* y, long long n, float kf, float gain, uint64_t* sums,
                   const uint64_t* carry_in, uint64_t* carry_out, uint64_t k0, const OscDev& o, hipStream_t s);
// Oscillator blocks (k_fir.hip k_rotator): output i of a call is oscillator output
// k0 + i. mode: 0 Rotator::rotate_block (rotator.rs:74-85, cf32 -> cf32), 1
// Rotator::mix_usb_block (rotator.rs:88-94, cf32 -> f32), 2 mix_with_nco (nco.rs:63-66,
// cf32 -> cf32, non-FMA), 3 Nco::next_cs / Rotator::next (no input, cf32 phasors out).
void launch_osc(int mode, const f2* x_dev, void* y_dev, long long n, uint64_t k0, const OscDev& o, hipStream_t s);

// ---------------------------------------------------------- FIR family --
// Decimating FIR at the kept outputs only: out[j] = sum_k g[k] * x[M*j - k],
// j < n_out, with x[P<0] from hist (hist_len samples ending at x[-1]).
struct Taps256 { float g[256]; };
void launch_decim(const f2* x_dev, long long n, const f2* hist_dev, int hist_len, f2* out_dev,
                  long long n_out, int M, int K, const Taps256& g, const float* g_dev,
                  hipStream_t s);
// Batched over channels: x[ch*x_stride + i], out[ch*out_stride + j], shared taps.
// hist_out (optional): each channel's next history, written by the launch itself.
void launch_decim_batch(const f2* x_dev, long long x_stride, long long n, const f2* hist_dev,
                        int hist_len, f2* out_dev, long long out_stride, long long n_out, int nch,
                        int M, int K, const Taps256& g, const float* g_dev, hipStream_t s,
                        f2* hist_out = nullptr);
// Real FIR y[i] = sum_k g[k] x[i-k] (x[P<0] from hist).
// hist_out (optional): the next call's history (last hist_len of [hist | x]), written by
// the FIR launch itself (no separate k_hist_update launch).
void launch_fir_real(const float* x_dev, long long n, const float* hist_dev, int hist_len,
                     float* y_dev, int K, const Taps256& g, const float* g_dev, hipStream_t s,
                     float* hist_out = nullptr);
// Complex-sample real-tap FIR y[i] = sum_k g[k] x[i + off - k], i < n_out
// (x[P<0] from hist, x[P>=n] = 0). off = 0: streaming; off = (K-1)/2 with an
// all-zero history: FirLowpassIq::filter_aligned.
// nch > 1: independent channels, channel ch at x + ch x_stride / y + ch y_stride, its
// histories at ch hist_len of hist_dev / hist_out (batched FirLowpassIq).
void launch_fir_iq(const f2* x_dev, long long n, const f2* hist_dev, int hist_len, f2* y_dev,
                   long long n_out, long long off, int K, const Taps256& g, const float* g_dev,
                   hipStream_t s, f2* hist_out = nullptr, int nch = 1, long long x_stride = 0,
                   long long y_stride = 0);
// Copy the last hist_len samples of [old_hist | x[0..n)] into new_hist.
// FirLowpassIq::filter_aligned in place (k_fir_iq8 INPLACE + boundary copies);
// writes the history the reference leaves (last hist_len of [x | 0^d]) to
// hist_out first. false: K > 256 or edges too small (fir_iq_aligned_edges f2).
bool launch_fir_iq_aligned_inplace(f2* io, long long n, long long d, int K, const Taps256& g, f2* edges,
                                   long long edges_cap, f2* hist_out, int hist_len, hipStream_t s);
long long fir_iq_aligned_edges(long long n, int K);
void launch_hist_update_c(const f2* x_dev, long long n, const f2* old_dev, f2* new_dev,
                          int hist_len, hipStream_t s, int nch = 1, long long x_stride = 0);
void launch_hist_update_r(const float* x_dev, long long n, const float* old_dev, float* new_dev,
                          int hist_len, hipStream_t s);
// out[k] = e^{j 2 pi k step / 2^64}, k < n (device-built oscillator model step table)
void launch_phasor_table_q64(f2* out, uint64_t step_q64, int n, hipStream_t s);

// ------------------------------------------------------------ WBFM chain --
// Default: one launch per call (k_wbfm_seg, see k_wbfm.hip). The two-kernel path
// (any IIR design):
//  front: NCO mix -> polyphase decim x8 (<= 128 taps) -> FM discriminator,
//         writing phi (f32, 1/8 rate) — 8 B in, 0.5 B out per input sample;
//  back : LpCascade (wave scan, f64 carries, warm-up across workgroups) ->
//         audio FIR (<= 128 taps) — 0.59 B in, 0.5 B out per input sample.
constexpr int kWbfmM = 8;
constexpr int kWbfmQ = 16;
constexpr int kWbfmT = 512;                          // decimated outputs per front workgroup
constexpr int kWbfmPhi = kWbfmT - 1;                 // discriminator outputs per front workgroup
constexpr int kWbfmNS = kWbfmM * (kWbfmT + kWbfmQ);  // staged input samples per front workgroup
constexpr int kWbfmHist = kWbfmM * kWbfmQ;           // raw input history (128)
constexpr int kBackA = 4096;                         // audio outputs per back workgroup
constexpr int kBackC = 10;                           // IIR samples per lane and half
constexpr int kBackW = 510;                          // zero-state warm-up per half (51 chunks)
constexpr int kBackSpan = 256 * kBackC;              // 2560 = kBackA / 2 + warm-up (+2)
constexpr int kWbfmCarry = 8 + 128;                  // iir[4], prev[2], pad[2], fhist[128]
struct WbfmFrontConst {
  float g[128];  // decimator taps g[8q+c] phase-major at [c*16+q]; quirk-mapped
                 // (g[0]=h[L-1], g[k]=h[k-1], dsp/fir.rs:57-66), zero padded
  float k;       // 1/dev (fm.rs:23)
};
struct WbfmBackConst {
  float a[128];               // audio taps, quirk-mapped, zero padded
  float b0, b1, b2, a1, a2;   // LpCascade biquad (iir.rs:49-71)
  double pw[6 * 16];          // (A^C)^(2^s), s = 0..5 (C = kBackC)
  double mw[16];              // A^(64 C): one wave's span
};
// Segmented single-kernel chain (k_wbfm_seg): sub-range backs of kSgL outputs.
constexpr int kFuTail = 128;                         // IIR outputs handed to the next segment (FIR history)
constexpr int kFuSlot = 144;                         // u32 words of a segment's end-state record
// record layout (u32 words): [2,10) end state of the IIR (4 f64), [16,144) last
// 128 IIR outputs. Flags: 3 u32 per segment (the epoch of the last publish).
struct WbfmFusedConst {
  float b0, b1, b2, a1, a2;   // LpCascade biquad (iir.rs:49-71)
  float tscale;               // audio FIR on the matrix cores: 2^-st (taps scaled by 2^st; f per sub-range)
  // device memory, read with scalar loads where used (kWbfmMats doubles): (A^kSgC)^(2^s)
  // for s = 0..5, then A^(kSgL/2) (one half sub-range, read by iir16 as step 6)
  const double* mats;
};
constexpr int kWbfmMats = 7 * 16;
struct WbfmArgs {
  const f2* x;  long long x_stride;  long long n;
  float* phi;   long long phi_stride;               // workspace [nch][>= n_dec]
  float* y;     long long y_stride;  long long n_dec;
  long long k0;                                     // samples consumed by earlier calls
  const uint64_t* step;                             // [nch] Q0.64 oscillator step
  const f2* tab;                                    // [nch][kWbfmNS] e^{j theta p}
  const float* carry_in; float* carry_out;          // [nch][kWbfmCarry]
  const f2* hist_in; f2* hist_out;                  // [nch][kWbfmHist]
  const double* lanemats;                           // A^(C L), L = 0..63 (16 doubles each; k_wbfm_back)
  // segmented chain only
  uint32_t* hand;                                   // [slots][kSeg4Slot] hand-off records
  uint32_t* flags;                                  // [slots][3] epoch of the last publish
  int* err;                                         // host-visible error word: a hand-off wait timed out
  uint32_t spin;                                    // polls before a wait times out (kernels.hpp kSpinDefault)
  uint32_t epoch;                                   // this launch's tag (never 0)
  long long* trace;                                 // debug: per-wave phase timestamps (or null)
  const void* afrag;                                // audio FIR reversed f16 tap words (k_wbfm.hip sg::back)
};
// The audio FIR's taps as the A operand source: r[m] = a[127 - m] 2^st (zero outside
// [0, 128)) as f16 hi and lo parts, each in two parity copies of 96 words (copy p, word w:
// halves r[2w - 16 - p], r[2w - 15 - p]), so that any 8 consecutive halves are 4 aligned
// words of one copy (k_wbfm.hip sg::back keeps them in LDS).
constexpr int kAudTapWords = 96;
constexpr int kAudFragBytes = 2 * 2 * kAudTapWords * 4;  // (hi, lo) x 2 parity copies
constexpr int kFuTracePoints = 16;
void launch_wbfm(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmBackConst& b, int nch,
                 hipStream_t s);
// Segmented single-kernel chain (k_wbfm_seg): sub-ranges of kSgL outputs, one round
// of waves. Requires ||A^(kSgL - 128)|| negligible (the block checks it).
constexpr int kSgL = 1024;                           // outputs per sub-range
constexpr int kSgC = kSgL / 128;                     // IIR samples per lane and half (8)
constexpr int kSeg4Slot = kFuSlot + kSgL;            // u32 words per segment: end-state record, then sub-range 0's phi
long long wbfm_seg_slots(long long n_dec, int nch);
// max_segments > 0 caps the waves (default: the resident capacity).
void launch_wbfm_seg(const WbfmArgs& a, const WbfmFrontConst& f, const WbfmFusedConst& b, int nch,
                     int max_segments, hipStream_t s);

// On-box bandwidth probe (k_diag.hip): a streaming read of the first
// stream_read_bytes(bytes) bytes of x (16-B aligned) with the WBFM front's load shape.
long long stream_read_bytes(long long bytes);
void launch_stream_read(const void* x, long long bytes, float* sink, hipStream_t s);
// Residency tests: `workgroups` one-wave workgroups holding lds_bytes of LDS each for
// `seconds` of wall clock (bounded; every wave exits).
void launch_spin(int workgroups, int lds_bytes, double seconds, hipStream_t s);
}  // namespace orion
