/*
 * orion_sdr_amd.h — C ABI of the MI355X (gfx950) streaming DSP engine.
 *
 * Drop-in boundary for skynavga/orion-sdr's analog sample-stream path. Every
 * entry point replaces one reference interface (cited file:line, reference
 * v0.0.63). Plain pointers and sizes only: no HIP or torch types cross this
 * boundary (streams are passed as `void*` = hipStream_t, NULL = default stream).
 *
 * Contract (src/core.rs:6-22, trait Block):
 *  - A handle is one stateful Block instance; it keeps its streaming state
 *    (delay lines, oscillator phase, IIR state, discriminator history) across
 *    calls, so k calls on consecutive chunks equal one call on the whole.
 *  - orion_block_process*: 1:1 blocks consume n = min(n_in, out_cap) samples;
 *    FirDecimator and the WBFM chain consume all n_in and write
 *    min(ceil(n_in/m), out_cap) (dsp/decim.rs:66-75). The decimation phase
 *    restarts at every call, as in the reference (decim.rs:68-71).
 *  - Return 0 on success, a negative ORION_E_* code otherwise (the reference
 *    never fails on lengths; errors here are HIP/argument failures only).
 *  - Types: cf32 = interleaved {float re, im} (num_complex::Complex32), f32.
 *  - Multi-channel handles (nch > 1) read in[ch*n_in + i] and write
 *    out[ch*out_cap + j]; channels are independent streams.
 */
#ifndef ORION_SDR_AMD_H
#define ORION_SDR_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORION_OK 0
#define ORION_E_NULL (-1)
#define ORION_E_HIP (-2)
#define ORION_E_ARG (-3)
#define ORION_E_TYPE (-4)
#define ORION_E_UNSUPPORTED (-5)

#define ORION_DT_C32 0
#define ORION_DT_F32 1

/* core.rs:6-10 */
typedef struct {
  size_t in_read;
  size_t out_written;
} orion_work_report;

typedef struct orion_block orion_block;

/* ---- library ---------------------------------------------------------- */
const char* orion_version(void);
const char* orion_last_error(void);          /* thread-local message of the last failure */
int orion_device_count(void);
int orion_set_device(int device);
int orion_synchronize(void* stream);
/* Pinned (page-locked) host memory for the host-buffer path (no reference counterpart):
 * orion_block_process DMAs it without staging copies. NULL on failure. */
void* orion_host_alloc(size_t bytes);
int orion_host_free(void* p);
int orion_device_cus(void);                 /* compute units of the current device (< 0: error) */
/* On-box bandwidth probe (no reference counterpart; bench.py's measured read
 * peak): one streaming read of the first orion_diag_stream_read_bytes(bytes)
 * bytes of the 16-B aligned device buffer `dev`, asynchronous on `stream`. */
size_t orion_diag_stream_read_bytes(size_t bytes);
int orion_diag_stream_read(const void* dev, size_t bytes, void* stream);
/* Residency tests (no reference counterpart): `workgroups` one-wave workgroups that
 * each hold lds_bytes of LDS (256 .. 160 KiB) for `seconds` (<= 10) of wall clock on
 * `stream`, asynchronous; and a stream restricted to the first n_cus CUs (0: an
 * ordinary non-blocking stream), destroyed with orion_diag_stream_destroy. */
int orion_diag_spin(void* stream, uint32_t workgroups, uint32_t lds_bytes, double seconds);
void* orion_diag_stream_create(uint32_t n_cus);
int orion_diag_stream_destroy(void* stream);

/* ---- constructors (one per reference constructor) ---------------------- */
/* dsp/rotator.rs:16-26 Rotator::new(freq_hz, fs); Block-like rotate_block (:74-85). cf32->cf32
 * The oscillator tracks the reference's own f32 recurrence (z <- z w, renormalised
 * every 1024 steps, :44-62), not the ideal phasor it drifts from: at construction and
 * every set_freq / reset_phase the host runs that recurrence from the current state
 * for up to ORION_OPT_NCO_TABLE outputs (default 2^20, a few ms) and the device reads
 * its phasors. The finite-state recurrence falls into a cycle; when the cycle closes
 * within the budget (-1.5 MHz / 10 MHz: after 21504 steps) every output is the
 * reference's, bit for bit, forever. Otherwise outputs past the budget follow a drift
 * model (the fitted mean step and a magnitude linear in the renorm position).
 * Construction fails (NULL, orion_last_error) if TAU * freq_hz / fs is not finite. */
orion_block* orion_rotator_new(float freq_hz, float fs);
/* dsp/rotator.rs:35-39 Rotator::set_freq(freq_hz, fs): a new step phasor; z and the
 * renorm counter carry on (the reference keeps them). Synchronizes the device
 * (kernels in flight read the oscillator table). ORION_E_ARG if TAU * freq_hz / fs is
 * not finite (e.g. fs = 0: the reference would produce NaN forever). */
int orion_rotator_set_freq(orion_block* b, float freq_hz, float fs);
/* dsp/rotator.rs:44-68 Rotator::next / next_cs, n times: out[i] = the phasor after each
 * step (cf32 pairs), advancing the same oscillator as rotate_block. Host buffer
 * (synchronous) / device buffer. */
int orion_rotator_next_cs_block(orion_block* b, void* out, size_t n);
int orion_rotator_next_cs_block_device(orion_block* b, void* out_dev, size_t n, void* stream);
/* dsp/rotator.rs:28-31 Rotator::reset_phase: phasor back to 1 + j0 (the step stays);
 * the same as orion_block_reset on a Rotator. */
int orion_rotator_reset_phase(orion_block* b);
/* dsp/rotator.rs:88-94 Rotator::mix_usb_block(input, out): out[i] = fma(I, cos, Q*sin)
 * with the phasor of the next step, on the same oscillator as rotate_block; n =
 * min(n_in, out_cap). cf32 -> f32. Host buffers (synchronous) / device buffers. */
int orion_rotator_mix_usb_block(orion_block* b, const void* in, size_t n_in, float* out, size_t out_cap,
                                orion_work_report* wr);
int orion_rotator_mix_usb_block_device(orion_block* b, const void* in_dev, size_t n_in, float* out_dev, size_t out_cap,
                                       void* stream, orion_work_report* wr);
/* Host only (no device; tests and diagnostics, no reference counterpart): the first n
 * phasors of Rotator::new(freq_hz, fs) as the engine tabulates them with a budget of
 * max_out outputs (the reference recurrence, its cycle, or the drift model past the
 * budget) into out (cf32); cyc_len = 0 when no cycle closed within the budget. */
int orion_osc_table_phasors(float freq_hz, float fs, uint64_t max_out, void* out, size_t n, uint64_t* cyc_start,
                            uint64_t* cyc_len, uint64_t* n_tab);
/* dsp/nco.rs:20-31 Nco::new(freq_hz, fs) as a block: process = mix_with_nco per sample
 * (nco.rs:63-66, the non-FMA product (x.re c - x.im s, x.re s + x.im c)). cf32->cf32
 * The oscillator tracks the reference recurrence (nco.rs:42-58) as the Rotator's does. */
orion_block* orion_nco_new(float freq_hz, float fs);
/* dsp/nco.rs:33-38 Nco::set_freq(freq_hz) (fs from orion_nco_new): the phase continues.
 * Synchronizes the device. */
int orion_nco_set_freq(orion_block* b, float freq_hz);
/* dsp/nco.rs:42-58 next_cs, n times: out[i] = (cos, sin) of the phasor after each step
 * (cf32 pairs). Host buffer (synchronous) / device buffer. */
int orion_nco_next_cs_block(orion_block* b, void* out, size_t n);
int orion_nco_next_cs_block_device(orion_block* b, void* out_dev, size_t n, void* stream);
/* dsp/decim.rs:24-37 FirDecimator::new(fs, m, cutoff_hz, trans_hz). cf32->cf32 */
orion_block* orion_fir_decimator_new(float fs, size_t m, float cutoff_hz, float trans_hz);
/* Batched FirDecimator: nch independent channels sharing one design. */
orion_block* orion_fir_decimator_batch_new(float fs, size_t m, float cutoff_hz, float trans_hz,
                                           size_t nch);
/* dsp/fir.rs:16-44 FirLowpass::design(fs, pass_hz, trans_hz); process :47-54. f32->f32 */
orion_block* orion_fir_lowpass_new(float fs, float pass_hz, float trans_hz);
/* dsp/fir.rs:186-188 FirLowpassIq::design(num_taps, cutoff_norm, stopband_db). cf32->cf32 */
orion_block* orion_fir_lowpass_iq_design(size_t num_taps, float cutoff_norm, float stopband_db);
/* dsp/fir.rs:193-204 FirLowpassIq::from_taps(taps) (empty -> [1.0]). */
orion_block* orion_fir_lowpass_iq_from_taps(const float* taps, size_t n);
/* Batched FirLowpassIq: nch independent channels sharing the taps (a channel filter in
 * front of a batched demodulator, BASELINE C5), [nch][n] in and out; filter_aligned is
 * single-channel only (ORION_E_ARG here). */
orion_block* orion_fir_lowpass_iq_batch_from_taps(const float* taps, size_t n, size_t nch);
/* dsp/fir.rs:210-212 FirLowpassIq::num_taps, :216-218 group_delay = (num_taps - 1) / 2.
 * ORION_E_TYPE if b is not a FirLowpassIq. */
int orion_fir_lowpass_iq_num_taps(const orion_block* b, size_t* num_taps);
int orion_fir_lowpass_iq_group_delay(const orion_block* b, size_t* group_delay);
/* dsp/fir.rs:260-276 FirLowpassIq::filter_aligned(io) on device memory (resets state). */
int orion_fir_lowpass_iq_filter_aligned_device(orion_block* b, void* io_dev, size_t n, void* stream);
/* Host-memory variant of filter_aligned (synchronous). */
int orion_fir_lowpass_iq_filter_aligned(orion_block* b, void* io, size_t n);
/* dsp/iir.rs:49-71 LpCascade::design(fs, fc) as a f32->f32 block (:79-83). */
orion_block* orion_lp_cascade_new(float fs, float fc);
/* dsp/iir.rs:15-41 Biquad::new(b0, b1, b2, a1, a2) (TDF-II, process :34-40) as an f32->f32
 * block; orion_block_reset = Biquad::reset. Any coefficients: a design whose state
 * decays within 8192 samples runs one pass, any other (a pole near the unit circle)
 * the three-kernel state-carry scan with f64 carries. */
orion_block* orion_biquad_new(float b0, float b1, float b2, float a1, float a2);
/* dsp/iir.rs:111-137 LpDcCascade::design(fs, lp_fc, dc_cut_hz); process :151-165 (LP4 then
 * the DC blocker). f32->f32 */
orion_block* orion_lp_dc_cascade_new(float fs, float lp_fc, float dc_cut_hz);
/* LpDcCascade::process_mapped(x, f) (iir.rs:170-186: f between the LP4 and the DC blocker)
 * instead of process (:151-165), for the maps a C caller can name: ORION_MAP_IDENTITY
 * (|v| v, the same as process), ORION_MAP_SQRT (f32::sqrt, the AM-PowerSqrt use,
 * demodulate/am.rs:55) or ORION_MAP_ABS (f32::abs). Set before the first call.
 * ORION_E_ARG for another value, ORION_E_TYPE for another block. */
#define ORION_MAP_IDENTITY 0
#define ORION_MAP_SQRT 1
#define ORION_MAP_ABS 2
int orion_lp_dc_cascade_set_map(orion_block* b, int map);
/* on = 1: orion_lp_dc_cascade_set_map(b, ORION_MAP_SQRT); on = 0: ORION_MAP_IDENTITY. */
int orion_lp_dc_cascade_set_sqrt_map(orion_block* b, int on);
/* dsp/dc.rs:15-21 DcBlocker::new(fs, cut_hz); Block impl :40-58. f32->f32 */
orion_block* orion_dc_blocker_new(float fs, float cut_hz);
/* demodulate/fm.rs:22-32 FmQuadratureDemod::new(fs, dev_hz, audio_bw_hz). cf32->f32 */
orion_block* orion_fm_quadrature_demod_new(float fs, float dev_hz, float audio_bw_hz);
/* demodulate/fm.rs:34-37 with_translate(freq_hz) (before the first process call). */
int orion_fm_quadrature_demod_with_translate(orion_block* b, float freq_hz);
/* demodulate/pm.rs:22-32 PmQuadratureDemod::new(fs, k, audio_bw_hz). cf32->f32 */
orion_block* orion_pm_quadrature_demod_new(float fs, float k, float audio_bw_hz);
/* demodulate/ssb.rs:15-20 SsbProductDemod::new(fs, bfo_hz, audio_bw_hz). cf32->f32 */
orion_block* orion_ssb_product_demod_new(float fs, float bfo_hz, float audio_bw_hz);
/* Batched SsbProductDemod: nch independent channels. */
orion_block* orion_ssb_product_demod_batch_new(float fs, float bfo_hz, float audio_bw_hz, size_t nch);
/* demodulate/am.rs:24-30 AmEnvelopeDemod::new(fs, audio_bw_hz). cf32->f32 */
orion_block* orion_am_envelope_demod_new(float fs, float audio_bw_hz);
/* demodulate/am.rs:33-36 with_abs_approx(k1, k2). */
int orion_am_envelope_demod_with_abs_approx(orion_block* b, float k1, float k2);
/* demodulate/cw.rs:15-25 CwEnvelopeDemod::new(fs, tone_hz, env_bw_hz); set_gain :26-28. */
orion_block* orion_cw_envelope_demod_new(float fs, float tone_hz, float env_bw_hz);
int orion_cw_envelope_demod_set_gain(orion_block* b, float g);

/* ---- analog modulators: f32 audio -> cf32 IQ ---- */
/* modulate/am.rs:20-30 AmDsbMod::new(fs, rf_hz, carrier_level, modulation_index);
 * set_gain :31-33, set_clamp :34-36 (ORION_E_TYPE on another block). */
orion_block* orion_am_dsb_mod_new(float fs, float rf_hz, float carrier_level, float modulation_index);
/* dsp/agc.rs:20-31 AgcRms::new(fs, attack_ms, release_ms, target_rms); process :48-75. f32->f32 */
orion_block* orion_agc_rms_new(float fs, float attack_ms, float release_ms, float target_rms);
/* dsp/agc.rs:93-106 AgcRmsIq::new(fs, attack_ms, release_ms, target_rms); process :124-150. cf32->cf32 */
orion_block* orion_agc_rms_iq_new(float fs, float attack_ms, float release_ms, float target_rms);
int orion_am_dsb_mod_set_gain(orion_block* b, float g);
int orion_am_dsb_mod_set_clamp(orion_block* b, int on);
/* modulate/fm.rs:21-32 FmPhaseAccumMod::new(sample_rate, deviation_hz, rf_hz);
 * set_deviation :33-35, set_gain :36-38. The running phase is summed on the device as
 * exact Q0.64 turn counts of the reference's own f32 step pairs (associative: any
 * summation order gives the same bits), then the reference's f32 recurrence is re-run
 * over each thread's 16 samples; the RF Nco is the reference's recurrence (tabulated). */
orion_block* orion_fm_phase_accum_mod_new(float fs, float deviation_hz, float rf_hz);
int orion_fm_phase_accum_mod_set_deviation(orion_block* b, float deviation_hz);
int orion_fm_phase_accum_mod_set_gain(orion_block* b, float g);
/* modulate/pm.rs:17-29 PmDirectPhaseMod::new(sample_rate, kp_rad_per_unit, rf_hz); set_gain,
 * set_sensitivity. process :36-47: (cos kp x, sin kp x) * gain, mixed with the RF Nco. */
orion_block* orion_pm_direct_phase_mod_new(float fs, float kp_rad_per_unit, float rf_hz);
int orion_pm_direct_phase_mod_set_gain(orion_block* b, float g);
int orion_pm_direct_phase_mod_set_sensitivity(orion_block* b, float kp_rad_per_unit);
/* modulate/cw.rs:21-41 CwKeyedMod::new(sample_rate, tone_hz, rise_ms, fall_ms); set_gain.
 * process :45-87: keying input clamped to [0, 1], rise/fall one-pole envelope, mixed with
 * the tone Nco. The envelope is a data-dependent recurrence: chunked warm-ups whose
 * exactness is checked bitwise, in-order re-runs where it fails (as AgcRms). */
orion_block* orion_cw_keyed_mod_new(float fs, float tone_hz, float rise_ms, float fall_ms);
int orion_cw_keyed_mod_set_gain(orion_block* b, float g);
/* modulate/ssb.rs:22-35 SsbPhasingMod::new(fs, audio_bw_hz, audio_if_hz, rf_hz, usb). */
orion_block* orion_ssb_phasing_mod_new(float fs, float audio_bw_hz, float audio_if_hz, float rf_hz, int usb);

/* The WBFM chain composed per docs/demodulate.md:128-133 (no single reference
 * type): Rotator(-f_off, fs) -> FirDecimator(fs, m, dec_cutoff, dec_trans) ->
 * FmQuadratureDemod(fs/m, dev_hz, audio_bw) -> FirLowpass(fs/m, audio_pass,
 * audio_trans). Any design the reference's constructors accept. cf32 -> f32 in one
 * gfx950 kernel per call for m = 8 with <= 128 decimator and audio taps and an
 * LpCascade that forgets within 896 outputs (the WBFM defaults): NCO + polyphase
 * decimation + discriminator + LpCascade + audio FIR, intermediates on chip; other
 * designs run the four blocks stage by stage (see configure). */
typedef struct {
  float fs, f_off, dec_cutoff, dec_trans, dev_hz, audio_bw, audio_pass, audio_trans;
  size_t m;
} orion_wbfm_params;
orion_block* orion_wbfm_chain_new(const orion_wbfm_params* p);
/* nch channels sharing the design, each with its own tuning offset f_off[ch]. */
orion_block* orion_wbfm_chain_batch_new(const orion_wbfm_params* p, const float* f_off, size_t nch);
/* Engine tuning and tests (no reference counterpart): the kernel path of a WBFM
 * chain handle, chosen before its first call. ORION_WBFM_AUTO picks the segmented
 * single kernel when the design allows it, else the two-kernel path when its
 * LpCascade warm-up suffices, else the four blocks (ORION_WBFM_GRAPH);
 * max_segments > 0 sets the segmented kernel's segments (waves; more than the
 * resident capacity runs several rounds), 0 = one round at the resident capacity.
 * ORION_E_TYPE if b is not a WBFM chain, ORION_E_ARG if the design cannot run on
 * that path.
 * Residency: the segmented kernel launches one round of waves (at most the
 * device's resident capacity) and each segment waits, bounded, for the end state
 * its predecessor publishes. A predecessor is always the previous workgroup in
 * dispatch order, so the wait ends even when other streams hold most CUs; a wait
 * that still outlasts its bound (~0.5 s) makes the handle report ORION_E_HIP (see
 * orion_block_status) instead of returning the audio as valid. */
#define ORION_WBFM_AUTO 0
#define ORION_WBFM_SEGMENTED 1  /* one kernel, one round of segments (k_wbfm_seg) */
#define ORION_WBFM_SPLIT 3      /* two kernels (front, back): m = 8, <= 128 taps, ||A^510|| < 1e-7 */
#define ORION_WBFM_GRAPH 4      /* Rotator, FirDecimator, FmQuadratureDemod, FirLowpass blocks: any design */
int orion_wbfm_chain_configure(orion_block* b, int path, int max_segments);
/* Time-sharded streams (no reference counterpart): the absolute
 * index of the next input sample, i.e. the NCO phase origin (rotator.rs:44-62
 * advances the phase once per sample from index 0). A shard of one stream is
 * processed by a fresh handle sought to its halo start, fed the halo and then
 * the shard (orion_sdr.stream_shard). ORION_E_TYPE if b is not a WBFM chain. */
int orion_wbfm_chain_seek(orion_block* b, uint64_t index);

/* ---- Block contract (core.rs:12-22) ------------------------------------ */
/* Host buffers (synchronous): the path Block::process with host slices takes.
 * Pinned host memory (orion_host_alloc, or hipHostRegister'ed) moves by DMA directly;
 * pageable memory through the handle's pinned staging buffers, the CPU copy of one
 * chunk overlapping the DMA of the next. Blocks whose output does not depend on how a
 * call is cut (Rotator, Nco, FirLowpass, FirLowpassIq, FirDecimator at multiples of m,
 * the AM / PM / FM modulators, AgcRms(Iq), CwKeyedMod) run calls >= 2^21 samples as a
 * pipeline of chunks on three streams (H2D, kernel, D2H overlapped); the others upload,
 * run one device call and download. Either way the output equals one
 * orion_block_process_device call on the same input, bit for bit. */
int orion_block_process(orion_block* b, const void* in, size_t n_in, void* out, size_t out_cap,
                        orion_work_report* wr);
/* Device buffers (asynchronous on `stream`). Overlapping in/out ranges are
 * ORION_E_ARG, except for AgcRms / AgcRmsIq, which work in place (through an
 * internal copy of the input). */
int orion_block_process_device(orion_block* b, const void* in_dev, size_t n_in, void* out_dev,
                               size_t out_cap, void* stream, orion_work_report* wr);
/* The batched entry SURVEY §8(b) names (no reference counterpart: the reference runs one
 * channel per Block): n_ch channels of n_per_ch samples laid out [n_ch][n_per_ch] on the
 * device, outputs [n_ch][out_cap]; the handle must have been built for n_ch channels
 * (the *_batch_new constructors), else ORION_E_ARG. Equals orion_block_process_device
 * on the same buffers; wr reports per-channel counts. */
int orion_batch_process(orion_block* b, const void* in_dev, size_t n_ch, size_t n_per_ch, void* out_dev,
                        size_t out_cap, void* stream, orion_work_report* wr);
/* Device-side failures (no reference counterpart; the reference never fails on the
 * path, core.rs:12-22): kernels that wait on other workgroups (the WBFM segment
 * hand-off, the single-pass scans' decoupled look-back, FmPhaseAccumMod's phase
 * look-back) bound every wait and flag a timeout in the handle's host-visible
 * error word instead of hanging. orion_block_status returns ORION_E_HIP once if a
 * kernel of this handle flagged one since the last check (non-blocking; it sees
 * every kernel that has finished: orion_synchronize(stream) first to cover all).
 * orion_block_process checks after its own sync; orion_block_process_device
 * checks at entry, so an error of call k fails call k+1 at the latest. */
int orion_block_status(orion_block* b);
/* Test-only: polls a cross-workgroup wait makes before it times out (process-wide;
 * default 1 << 22; 0 makes every such wait time out at once). */
void orion_debug_set_spin_limit(uint32_t polls);
uint32_t orion_debug_spin_limit(void);
int orion_block_reset(orion_block* b);
void orion_block_free(orion_block* b);
int orion_block_in_type(const orion_block* b);
int orion_block_out_type(const orion_block* b);
size_t orion_block_out_len(const orion_block* b, size_t n_in);
size_t orion_block_channels(const orion_block* b);
const char* orion_block_name(const orion_block* b);
/* Engine options (no reference counterpart; tests and timing comparisons).
 * ORION_E_TYPE if the block has no such option, ORION_E_ARG for a bad value. */
#define ORION_OPT_SCAN_PATH 1   /* IIR-based blocks (LpCascade, DcBlocker, Biquad, LpDcCascade, the FM/PM/SSB/
                                   AM/CW demods): 0 single pass where the design allows (default), 1 the
                                   three-kernel scan */
#define ORION_OPT_MOD_PASSES 2  /* FmPhaseAccumMod, SsbPhasingMod: 0 single pass (default), 3 three passes */
#define ORION_OPT_NCO_TABLE 3   /* Rotator, Nco: outputs of the reference recurrence tabulated per (re)tune,
                                   0 .. 2^28 (default 2^20; 0 = the closed-form ideal phasor of the f32 step).
                                   The oscillator state carries on across the change. */
int orion_block_configure(orion_block* b, int option, long long value);
/* Designed coefficients, for parity tests: which = 0 primary taps, 1 audio taps. */
int orion_block_taps(const orion_block* b, int which, float* out, size_t cap, size_t* n);

/* ---- designs (host only; bit-exact with the reference constructors) ----- */
size_t orion_fir_lowpass_design(float fs, float pass_hz, float trans_hz, float* taps, size_t cap); /* fir.rs:16-44 */
size_t orion_kaiser_lowpass_taps(size_t num_taps, float cutoff_norm, float stopband_db, float* taps,
                                 size_t cap);                                                     /* fir.rs:113-141 */
float orion_kaiser_transition_norm(size_t num_taps, float stopband_db);                           /* fir.rs:147-150 */
size_t orion_kaiser_num_taps(float transition_norm, float stopband_db);                           /* fir.rs:154-157 */
void orion_lp_cascade_design(float fs, float fc, float out5[5]);                                  /* iir.rs:49-71 */

/* ---- multicarrier/tx_lowpass.rs:88-195 TxLowpass (the TX mask) ----
 * The spec and its host-side sizing helpers (the reference's f32 arithmetic); the
 * filter itself is FirLowpassIq::design(num_taps, cutoff_norm, stopband_db), applied
 * by filter_aligned (TxLowpass::apply = orion_tx_lowpass_filter +
 * orion_fir_lowpass_iq_filter_aligned[_device]). */
typedef struct {
  float cutoff_norm;
  size_t num_taps;
  float stopband_db;
} orion_tx_lowpass;
orion_tx_lowpass orion_tx_lowpass_for_null_band(size_t n_fft, size_t occupied_half, size_t num_taps,
                                                float stopband_db);                              /* :118-134 */
size_t orion_tx_lowpass_taps_for_null_band(size_t n_fft, size_t occupied_half, float stopband_db); /* :141-144 */
size_t orion_tx_lowpass_group_delay(const orion_tx_lowpass* t);                                  /* :148-150 */
float orion_tx_lowpass_transition_norm(const orion_tx_lowpass* t);                               /* :154-156 */
int orion_tx_lowpass_transition_fits(const orion_tx_lowpass* t, size_t n_fft, size_t occupied_half); /* :162-165 */
float orion_tx_lowpass_stopband_edge_norm(const orion_tx_lowpass* t);                            /* :171-173 */
int orion_tx_lowpass_fits_guard(const orion_tx_lowpass* t, size_t cp_len, size_t roll_off, size_t backoff); /* :179-182 */
orion_block* orion_tx_lowpass_filter(const orion_tx_lowpass* t);                                 /* :185-187 */

#ifdef __cplusplus
}
#endif
#endif /* ORION_SDR_AMD_H */
