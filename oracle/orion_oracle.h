/*
 * orion_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * Scalar CPU restatement of the skynavga/orion-sdr analog sample-stream path
 * (reference v0.0.63 at /root/reference, Rust, f32 everywhere). Every routine
 * cites the reference file:line it follows. It is the parity CHECKER for the
 * MI355X engine in ../orion-sdr_amd and the "port" CPU baseline of bench.py.
 * Product code never links, loads or calls it.
 *
 * Parity pinning: the reference Rust cannot be built here (no cargo/rustc, no
 * crates.io) and ships no golden vectors. This restatement is pinned by
 * (1) every property / known-answer test the reference holds for this path
 *     (tests/unit/{dsp,fm,ssb,pm,chains,am}.rs, tests/roundtrip/{fm,am,ssb,pm,cw}.rs,
 *     python/tests/test_{unit,roundtrip}.py), re-run against this oracle in tests/;
 * (2) an independently written numpy restatement (tests/np_ref.py) that must agree
 *     bit-for-bit (or to 1 ulp where libm differs) on the committed fixtures in
 *     tests/golden/.
 * Bit-level parity with the Rust binary itself is therefore "partially pinned":
 * the arithmetic is restated op-for-op (fmaf exactly where Rust uses mul_add,
 * -ffp-contract=off elsewhere, glibc sinf/cosf/expf/powf/sqrtf as Rust's libm
 * calls on Linux), but no output of the Rust build itself was available.
 */
#ifndef ORION_ORACLE_H
#define ORION_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float re, im; } oc32;
typedef struct { size_t in_read, out_written; } o_work_report;

/* ---- util.rs:305-322 ---- */
float o_atan2_approx(float y, float x);

/* ---- dsp/rotator.rs:8-95 ---- */
typedef struct { oc32 z, w; uint32_t renorm_ctr; } o_rotator;
void o_rotator_init(o_rotator *r, float freq_hz, float fs);
oc32 o_rotator_next(o_rotator *r);
void o_rotator_set_freq(o_rotator *r, float freq_hz, float fs);
void o_rotator_rotate_block(o_rotator *r, const oc32 *in, oc32 *out, size_t n);
void o_rotator_mix_usb_block(o_rotator *r, const oc32 *in, float *out, size_t n);

/* ---- dsp/nco.rs:11-66 ---- */
typedef struct { float fs, freq_hz; oc32 z, w; uint32_t renorm_ctr; } o_nco;
void o_nco_init(o_nco *n, float freq_hz, float fs);
void o_nco_set_freq(o_nco *n, float freq_hz);
void o_nco_next_cs(o_nco *n, float *c, float *s);
oc32 o_mix_with_nco(oc32 x, o_nco *n);

/* ---- dsp/fir.rs:7-67 (FirLowpass, real) ---- */
typedef struct { float *taps; float *delay; size_t len, idx; } o_fir;
size_t o_fir_design_taps(float fs, float pass_hz, float trans_hz, float *taps_out, size_t cap);
void o_fir_init(o_fir *f, float fs, float pass_hz, float trans_hz);
void o_fir_free(o_fir *f);
void o_fir_process(o_fir *f, const float *in, float *out, size_t n);

/* ---- dsp/fir.rs:74-157 (Kaiser design) ---- */
float o_kaiser_beta(float a_db);
float o_bessel_i0(float x);
size_t o_kaiser_lowpass_taps(size_t num_taps, float cutoff_norm, float stopband_db,
                             float *taps_out, size_t cap);
float o_kaiser_transition_norm(size_t num_taps, float stopband_db);
size_t o_kaiser_num_taps(float transition_norm, float stopband_db);

/* ---- dsp/fir.rs:176-297 (FirLowpassIq) ---- */
typedef struct { float *taps; oc32 *delay; size_t len, idx; } o_firiq;
void o_firiq_from_taps(o_firiq *f, const float *taps, size_t len);
void o_firiq_free(o_firiq *f);
void o_firiq_reset(o_firiq *f);
oc32 o_firiq_push(o_firiq *f, oc32 s);
o_work_report o_firiq_process(o_firiq *f, const oc32 *in, size_t n_in, oc32 *out, size_t n_out);
void o_firiq_filter_aligned(o_firiq *f, oc32 *io, size_t n);

/* ---- dsp/decim.rs:10-77 (FirDecimator) ---- */
typedef struct { size_t m; o_fir lp_i, lp_q; float *ri, *rq, *yi, *yq; size_t cap; } o_decim;
void o_decim_init(o_decim *d, float fs, size_t m, float cutoff_hz, float trans_hz);
void o_decim_free(o_decim *d);
o_work_report o_decim_process(o_decim *d, const oc32 *in, size_t n, oc32 *out, size_t out_len);

/* ---- dsp/iir.rs:4-84 (Biquad, LpCascade) ---- */
typedef struct { float b0, b1, b2, a1, a2, z1, z2; } o_biquad;
float o_biquad_process(o_biquad *b, float x);
typedef struct { o_biquad s[2]; } o_lp_cascade;
void o_lp_cascade_design(o_lp_cascade *c, float fs, float fc);
float o_lp_cascade_process(o_lp_cascade *c, float x);

/* ---- dsp/iir.rs:86-187 (LpDcCascade) ---- */
typedef struct { float z0_1, z0_2, z1_1, z1_2, dc_x1, dc_y1, b0, b1, b2, a1, a2, r; } o_lpdc;
void o_lpdc_design(o_lpdc *c, float fs, float lp_fc, float dc_cut_hz);
float o_lpdc_process(o_lpdc *c, float x);
float o_lpdc_process_mapped_sqrt(o_lpdc *c, float x);
float o_lpdc_process_mapped(o_lpdc *c, float x, int map);

/* ---- dsp/dc.rs:8-59 (DcBlocker) ---- */
typedef struct { float r, x1, y1; } o_dc;
void o_dc_init(o_dc *d, float fs, float cut_hz);
o_work_report o_dc_process(o_dc *d, const float *in, float *out, size_t n);

/* ---- demodulate/fm.rs:11-78 ---- */
typedef struct { float fs, k; int has_xf; o_rotator xf; oc32 prev; o_lp_cascade post_lp; } o_fm_demod;
void o_fm_demod_init(o_fm_demod *d, float fs, float dev_hz, float audio_bw_hz);
void o_fm_demod_with_translate(o_fm_demod *d, float freq_hz);
o_work_report o_fm_demod_process(o_fm_demod *d, const oc32 *in, float *out, size_t n);

/* ---- demodulate/pm.rs:12-67 ---- */
typedef struct { float fs, k; o_lp_cascade post_lp; oc32 prev; } o_pm_demod;
void o_pm_demod_init(o_pm_demod *d, float fs, float k, float audio_bw_hz);
o_work_report o_pm_demod_process(o_pm_demod *d, const oc32 *in, float *out, size_t n);

/* ---- demodulate/ssb.rs:9-72 ---- */
typedef struct { o_lpdc filt; o_rotator rot; } o_ssb_demod;
void o_ssb_demod_init(o_ssb_demod *d, float fs, float bfo_hz, float audio_bw_hz);
o_work_report o_ssb_demod_process(o_ssb_demod *d, const oc32 *in, float *out, size_t n);

/* ---- demodulate/am.rs:18-130 ---- */
typedef struct { o_lpdc filt; int abs_approx; float k1, k2; } o_am_demod;
void o_am_demod_init(o_am_demod *d, float fs, float audio_bw_hz);
void o_am_demod_with_abs_approx(o_am_demod *d, float k1, float k2);
o_work_report o_am_demod_process(o_am_demod *d, const oc32 *in, float *out, size_t n);

/* ---- demodulate/cw.rs:8-47 ---- */
typedef struct { float alpha, y, gain; } o_cw_demod;
void o_cw_demod_init(o_cw_demod *d, float fs, float tone_hz, float env_bw_hz);
o_work_report o_cw_demod_process(o_cw_demod *d, const oc32 *in, float *out, size_t n);

/* ---- modulate/fm.rs:11-75 ---- */
typedef struct { float fs, kf_hz_per_unit; oc32 z; o_nco rf_nco; float gain; uint32_t renorm_ctr; } o_fm_mod;
void o_fm_mod_init(o_fm_mod *m, float fs, float deviation_hz, float rf_hz);
o_work_report o_fm_mod_process(o_fm_mod *m, const float *in, oc32 *out, size_t n);

/* ---- modulate/pm.rs:8-49 ---- */
typedef struct { float kp; o_nco rf_nco; float gain; } o_pm_mod;
void o_pm_mod_init(o_pm_mod *m, float fs, float kp, float rf_hz);
o_work_report o_pm_mod_process(o_pm_mod *m, const float *in, oc32 *out, size_t n);

/* ---- modulate/ssb.rs:9-114 ---- */
typedef struct { int usb; o_lp_cascade lp_i, lp_q; o_rotator aud_nco, rf_nco; } o_ssb_mod;
void o_ssb_mod_init(o_ssb_mod *m, float fs, float audio_bw_hz, float audio_if_hz, float rf_hz, int usb);
o_work_report o_ssb_mod_process(o_ssb_mod *m, const float *in, oc32 *out, size_t n);

/* ---- modulate/am.rs:9-120 ---- */
typedef struct { float gain, carrier_level, modulation_index; int clamp; o_rotator rf_nco; } o_am_mod;
void o_am_mod_init(o_am_mod *m, float fs, float rf_hz, float carrier_level, float modulation_index);
o_work_report o_am_mod_process(o_am_mod *m, const float *in, oc32 *out, size_t n);

/* ---- modulate/cw.rs:8-87 ---- */
typedef struct { o_nco nco; float env, alpha_rise, alpha_fall, gain; } o_cw_mod;
void o_cw_mod_init(o_cw_mod *m, float fs, float tone_hz, float rise_ms, float fall_ms);
o_work_report o_cw_mod_process(o_cw_mod *m, const float *in, oc32 *out, size_t n);

/* ---- tests/common/mod.rs:27-48 ---- */
void o_add_awgn(oc32 *iq, size_t n, float noise_power, uint64_t seed);

/* ======================================================================
 * Flat "run" entry points for ctypes (one object lifetime per call set).
 * Each allocates a block, streams `n` samples through it in chunks of
 * `chunk` (0 = one call), and frees it; streaming state crosses chunks
 * exactly like repeated Block::process calls on one Rust instance.
 * ====================================================================== */
size_t o_run_rotator(float freq_hz, float fs, const oc32 *in, oc32 *out, size_t n, size_t chunk);
size_t o_run_rotator_retune(float f1, float fs, int mode, const oc32 *in, void *out, size_t n, size_t n_switch,
                            float f2, float fs2, int reset_at_switch);
size_t o_run_nco(float f1, float fs, int mode, const oc32 *in, oc32 *out, size_t n, size_t n_switch, float f2);
size_t o_run_biquad(float b0, float b1, float b2, float a1, float a2, const float *in, float *out, size_t n);
size_t o_run_lpdc(float fs, float lp_fc, float dc_cut, int map, const float *in, float *out, size_t n);
size_t o_run_fir(float fs, float pass_hz, float trans_hz, const float *in, float *out, size_t n, size_t chunk);
size_t o_run_firiq(const float *taps, size_t ntaps, const oc32 *in, oc32 *out, size_t n, size_t chunk);
void   o_run_firiq_aligned(const float *taps, size_t ntaps, oc32 *io, size_t n);
size_t o_run_decim(float fs, size_t m, float cutoff_hz, float trans_hz, const oc32 *in, size_t n,
                   oc32 *out, size_t out_cap, size_t chunk);
size_t o_run_lp_cascade(float fs, float fc, const float *in, float *out, size_t n);
size_t o_run_dc(float fs, float cut_hz, const float *in, float *out, size_t n, size_t chunk);
size_t o_run_fm_demod(float fs, float dev_hz, float audio_bw_hz, float translate_hz, int has_translate,
                      const oc32 *in, float *out, size_t n, size_t chunk);
size_t o_run_pm_demod(float fs, float k, float audio_bw_hz, const oc32 *in, float *out, size_t n, size_t chunk);
size_t o_run_ssb_demod(float fs, float bfo_hz, float audio_bw_hz, const oc32 *in, float *out, size_t n, size_t chunk);
size_t o_run_am_demod(float fs, float audio_bw_hz, int abs_approx, float k1, float k2,
                      const oc32 *in, float *out, size_t n, size_t chunk);
size_t o_run_cw_demod(float fs, float tone_hz, float env_bw_hz, float gain, const oc32 *in, float *out,
                      size_t n, size_t chunk);
size_t o_run_fm_mod(float fs, float dev_hz, float rf_hz, const float *in, oc32 *out, size_t n, size_t chunk);
size_t o_run_pm_mod(float fs, float kp, float rf_hz, const float *in, oc32 *out, size_t n);
size_t o_run_ssb_mod(float fs, float bw, float if_hz, float rf_hz, int usb, const float *in, oc32 *out, size_t n);
size_t o_run_am_mod(float fs, float rf_hz, float cl, float mi, float gain, int clamp, const float *in,
                    oc32 *out, size_t n);
size_t o_run_cw_mod(float fs, float tone_hz, float rise_ms, float fall_ms, const float *in, oc32 *out, size_t n);
void   o_lp_cascade_coeffs(float fs, float fc, float out5[5]);
void   o_lpdc_coeffs(float fs, float lp_fc, float dc_cut_hz, float out6[6]);

/* The WBFM chain (SURVEY §3 stack 2, docs/demodulate.md:128-133): Rotator(-f_off)
 * -> FirDecimator(fs, m, cutoff, trans) -> FmQuadratureDemod(fs/m, dev, audio_bw)
 * -> FirLowpass(fs/m, audio_pass, audio_trans). Streams `n` samples in calls of
 * `chunk` samples; returns the number of audio samples written. */
typedef struct {
    float fs, f_off, dec_cutoff, dec_trans, dev_hz, audio_bw, audio_pass, audio_trans;
    size_t m;
} o_wbfm_params;
size_t o_run_wbfm(const o_wbfm_params *p, const oc32 *in, size_t n, float *out, size_t out_cap, size_t chunk);
/* Multi-channel CPU baseline: `nch` independent channels laid out [ch][n], one
 * std thread per channel up to `nthreads` (pthreads). f_off per channel. */
size_t o_run_wbfm_channels(const o_wbfm_params *p, const float *f_off, size_t nch, const oc32 *in,
                           size_t n, float *out, size_t nthreads);
size_t o_run_ssb_demod_channels(float fs, float bfo_hz, float audio_bw_hz, size_t nch, const oc32 *in,
                                size_t n, float *out, size_t nthreads);
size_t o_run_decim_channels(float fs, size_t m, float cutoff_hz, float trans_hz, size_t nch,
                            const oc32 *in, size_t n, oc32 *out, size_t nthreads);
/* dsp/agc.rs AgcRms (iq = 0, f32) / AgcRmsIq (iq = 1, cf32 interleaved); returns the end env. */
float o_run_agc(int iq, float fs, float attack_ms, float release_ms, float target_rms,
                const float *in, float *out, size_t n, size_t chunk);

#ifdef __cplusplus
}
#endif
#endif
