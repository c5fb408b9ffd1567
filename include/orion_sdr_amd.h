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
/* On-box bandwidth probe (no reference counterpart; bench.py's measured read
 * peak): one streaming read of the first orion_diag_stream_read_bytes(bytes)
 * bytes of the 16-B aligned device buffer `dev`, asynchronous on `stream`. */
size_t orion_diag_stream_read_bytes(size_t bytes);
int orion_diag_stream_read(const void* dev, size_t bytes, void* stream);

/* ---- constructors (one per reference constructor) ---------------------- */
/* dsp/rotator.rs:16-26 Rotator::new(freq_hz, fs); Block-like rotate_block (:74-85). cf32->cf32 */
orion_block* orion_rotator_new(float freq_hz, float fs);
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
/* dsp/fir.rs:260-276 FirLowpassIq::filter_aligned(io) on device memory (resets state). */
int orion_fir_lowpass_iq_filter_aligned_device(orion_block* b, void* io_dev, size_t n, void* stream);
/* Host-memory variant of filter_aligned (synchronous). */
int orion_fir_lowpass_iq_filter_aligned(orion_block* b, void* io, size_t n);
/* dsp/iir.rs:49-71 LpCascade::design(fs, fc) as a f32->f32 block (:79-83). */
orion_block* orion_lp_cascade_new(float fs, float fc);
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
 * set_deviation :33-35, set_gain :36-38. The phase is summed in f64 on the
 * device (the reference multiplies f32 phasors, renormalised every 1024). */
orion_block* orion_fm_phase_accum_mod_new(float fs, float deviation_hz, float rf_hz);
int orion_fm_phase_accum_mod_set_deviation(orion_block* b, float deviation_hz);
int orion_fm_phase_accum_mod_set_gain(orion_block* b, float g);
/* modulate/ssb.rs:22-35 SsbPhasingMod::new(fs, audio_bw_hz, audio_if_hz, rf_hz, usb). */
orion_block* orion_ssb_phasing_mod_new(float fs, float audio_bw_hz, float audio_if_hz, float rf_hz, int usb);

/* The WBFM chain composed per docs/demodulate.md:128-133 (no single reference
 * type): Rotator(-f_off, fs) -> FirDecimator(fs, m, dec_cutoff, dec_trans) ->
 * FmQuadratureDemod(fs/m, dev_hz, audio_bw) -> FirLowpass(fs/m, audio_pass,
 * audio_trans). cf32 -> f32 in one gfx950 kernel per call (m must be 8): NCO +
 * polyphase decimation + discriminator + LpCascade + audio FIR, intermediates on
 * chip (two kernels for IIR designs that decay too slowly; see configure). */
typedef struct {
  float fs, f_off, dec_cutoff, dec_trans, dev_hz, audio_bw, audio_pass, audio_trans;
  size_t m;
} orion_wbfm_params;
orion_block* orion_wbfm_chain_new(const orion_wbfm_params* p);
/* nch channels sharing the design, each with its own tuning offset f_off[ch]. */
orion_block* orion_wbfm_chain_batch_new(const orion_wbfm_params* p, const float* f_off, size_t nch);
/* Engine tuning and tests (no reference counterpart): the kernel path of a WBFM
 * chain handle. ORION_WBFM_AUTO picks the segmented single kernel when the
 * LpCascade decays fast enough for it (the WBFM defaults), else two kernels;
 * max_segments > 0 caps the segmented kernel's waves (0 = the resident
 * capacity). ORION_E_TYPE if b is not a WBFM chain, ORION_E_ARG if the design
 * cannot run on that path. */
#define ORION_WBFM_AUTO 0
#define ORION_WBFM_SEGMENTED 1  /* one kernel, one round of segments, FIR spread over tiles */
#define ORION_WBFM_RANGES 2     /* one kernel, one wave per 2048-output range */
#define ORION_WBFM_SPLIT 3      /* two kernels (front, back), any IIR design */
#define ORION_WBFM_SEGMENTED_V1 4
#define ORION_WBFM_SPECIALIZED 5  /* one kernel, streaming and back waves per CU */
#define ORION_WBFM_SEGMENTED3 6   /* one kernel, three waves per SIMD, burst back */
#define ORION_WBFM_SEGMENTED4 7   /* k_wbfm_seg with the four-group decimator tile */
int orion_wbfm_chain_configure(orion_block* b, int path, int max_segments);
/* Time-sharded streams (no reference counterpart): the absolute
 * index of the next input sample, i.e. the NCO phase origin (rotator.rs:44-62
 * advances the phase once per sample from index 0). A shard of one stream is
 * processed by a fresh handle sought to its halo start, fed the halo and then
 * the shard (orion_sdr.stream_shard). ORION_E_TYPE if b is not a WBFM chain. */
int orion_wbfm_chain_seek(orion_block* b, uint64_t index);

/* ---- Block contract (core.rs:12-22) ------------------------------------ */
/* Host buffers (synchronous). */
int orion_block_process(orion_block* b, const void* in, size_t n_in, void* out, size_t out_cap,
                        orion_work_report* wr);
/* Device buffers (asynchronous on `stream`). Overlapping in/out ranges are
 * ORION_E_ARG, except for AgcRms / AgcRmsIq, which work in place (through an
 * internal copy of the input). */
int orion_block_process_device(orion_block* b, const void* in_dev, size_t n_in, void* out_dev,
                               size_t out_cap, void* stream, orion_work_report* wr);
int orion_block_reset(orion_block* b);
void orion_block_free(orion_block* b);
int orion_block_in_type(const orion_block* b);
int orion_block_out_type(const orion_block* b);
size_t orion_block_out_len(const orion_block* b, size_t n_in);
size_t orion_block_channels(const orion_block* b);
const char* orion_block_name(const orion_block* b);
/* Designed coefficients, for parity tests: which = 0 primary taps, 1 audio taps. */
int orion_block_taps(const orion_block* b, int which, float* out, size_t cap, size_t* n);

/* ---- designs (host only; bit-exact with the reference constructors) ----- */
size_t orion_fir_lowpass_design(float fs, float pass_hz, float trans_hz, float* taps, size_t cap); /* fir.rs:16-44 */
size_t orion_kaiser_lowpass_taps(size_t num_taps, float cutoff_norm, float stopband_db, float* taps,
                                 size_t cap);                                                     /* fir.rs:113-141 */
float orion_kaiser_transition_norm(size_t num_taps, float stopband_db);                           /* fir.rs:147-150 */
size_t orion_kaiser_num_taps(float transition_norm, float stopband_db);                           /* fir.rs:154-157 */
void orion_lp_cascade_design(float fs, float fc, float out5[5]);                                  /* iir.rs:49-71 */

#ifdef __cplusplus
}
#endif
#endif /* ORION_SDR_AMD_H */
