/*
 * orion_oracle.c — TEST INFRASTRUCTURE ONLY (see orion_oracle.h header for scope
 * and pinning status). Scalar restatement of skynavga/orion-sdr v0.0.63.
 *
 * Build: gcc -O3 -ffp-contract=off -fno-fast-math (oracle/Makefile). Rust never
 * contracts a*b+c into an FMA; it only fuses where the source says mul_add, which
 * is restated here as fmaf(). All constants are the f32 values of Rust's
 * core::f32::consts.
 */
#include "orion_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define O_TAU 6.28318530717958647692f      /* core::f32::consts::TAU */
#define O_PI 3.14159265358979323846f       /* core::f32::consts::PI */
#define O_FRAC_PI_2 1.57079632679489661923f
#define O_FRAC_PI_4 0.78539816339744830962f

static inline float o_maxf(float a, float b) { return a > b ? a : (b > a ? b : a); }
static inline float o_clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* util.rs:305-322 — 5th-order "minimax" atan2; restated op for op. */
float o_atan2_approx(float y, float x) {
    float ax = fabsf(x), ay = fabsf(y);
    float mn, mx;
    if (ax < ay) { mn = ax; mx = ay; } else { mn = ay; mx = ax; }
    float r = mn / (mx + FLT_EPSILON);
    float r2 = r * r;
    float phi = r * (O_FRAC_PI_4 + r2 * (-0.2447f + r2 * 0.0663f));
    if (ax < ay) phi = O_FRAC_PI_2 - phi;
    if (x < 0.0f) return (O_PI - phi) * (y < 0.0f ? -1.0f : 1.0f);
    return phi * (y < 0.0f ? -1.0f : 1.0f);
}

/* ------------------------------------------------------------------ */
/* dsp/rotator.rs:16-26 new; :44-62 next; :74-85 rotate_block; :88-94 */
void o_rotator_init(o_rotator *r, float freq_hz, float fs) {
    float phi = O_TAU * freq_hz / fs;
    r->z.re = 1.0f; r->z.im = 0.0f;
    r->w.re = cosf(phi); r->w.im = sinf(phi);
    r->renorm_ctr = 0;
}
/* rotator.rs:35-39 set_freq: recompute w only (z and the renorm counter stay). */
void o_rotator_set_freq(o_rotator *r, float freq_hz, float fs) {
    float phi = O_TAU * freq_hz / fs;
    r->w.re = cosf(phi); r->w.im = sinf(phi);
}
oc32 o_rotator_next(o_rotator *r) {
    float zr = fmaf(r->z.re, r->w.re, -(r->z.im * r->w.im));
    float zi = fmaf(r->z.im, r->w.re, r->z.re * r->w.im);
    r->z.re = zr; r->z.im = zi;
    r->renorm_ctr += 1u;
    if ((r->renorm_ctr & 0x3FFu) == 0) {
        float r2 = r->z.re * r->z.re + r->z.im * r->z.im;
        float inv = 1.0f / sqrtf(r2);
        r->z.re *= inv; r->z.im *= inv;
    }
    return r->z;
}
void o_rotator_rotate_block(o_rotator *r, const oc32 *in, oc32 *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        oc32 p = o_rotator_next(r);
        float a = in[i].re, b = in[i].im;
        out[i].re = fmaf(a, p.re, -(b * p.im));
        out[i].im = fmaf(b, p.re, a * p.im);
    }
}
void o_rotator_mix_usb_block(o_rotator *r, const oc32 *in, float *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        oc32 p = o_rotator_next(r);
        out[i] = fmaf(in[i].re, p.re, in[i].im * p.im);
    }
}

/* ------------------------------------------------------------------ */
/* dsp/nco.rs:20-31 new; :33-38 set_freq; :42-58 next_cs; :63-66 mix  */
void o_nco_init(o_nco *n, float freq_hz, float fs) {
    float dphi = O_TAU * freq_hz / fs;
    n->fs = fs; n->freq_hz = freq_hz;
    n->z.re = 1.0f; n->z.im = 0.0f;
    n->w.re = cosf(dphi); n->w.im = sinf(dphi);
    n->renorm_ctr = 0;
}
void o_nco_set_freq(o_nco *n, float freq_hz) {
    n->freq_hz = freq_hz;
    float dphi = O_TAU * freq_hz / n->fs;
    n->w.re = cosf(dphi); n->w.im = sinf(dphi);
}
void o_nco_next_cs(o_nco *n, float *c, float *s) {
    float zr = fmaf(n->z.re, n->w.re, -(n->z.im * n->w.im));
    float zi = fmaf(n->z.im, n->w.re, n->z.re * n->w.im);
    n->z.re = zr; n->z.im = zi;
    n->renorm_ctr += 1u;
    if ((n->renorm_ctr & 0x3FFu) == 0) {
        float inv = 1.0f / sqrtf(n->z.re * n->z.re + n->z.im * n->z.im);
        n->z.re *= inv; n->z.im *= inv;
    }
    *c = n->z.re; *s = n->z.im;
}
oc32 o_mix_with_nco(oc32 x, o_nco *n) {
    float c, s;
    o_nco_next_cs(n, &c, &s);
    oc32 o = { x.re * c - x.im * s, x.re * s + x.im * c };
    return o;
}

/* ------------------------------------------------------------------ */
/* dsp/fir.rs:16-44 FirLowpass::design (sinc x Hann, sum-normalised)   */
static size_t o_fir_ntaps(float fs, float pass_hz, float trans_hz) {
    pass_hz = o_maxf(pass_hz, 10.0f);
    trans_hz = o_maxf(trans_hz, pass_hz * 0.2f);
    size_t nt = (size_t)ceilf(fs / trans_hz);
    if (nt < 31) nt = 31;
    return nt | 1u;
}
size_t o_fir_design_taps(float fs, float pass_hz, float trans_hz, float *taps, size_t cap) {
    size_t ntaps = o_fir_ntaps(fs, pass_hz, trans_hz);
    if (!taps || cap < ntaps) return ntaps;
    pass_hz = o_maxf(pass_hz, 10.0f);
    float fc = pass_hz / fs;
    long m0 = (long)ntaps / 2;
    for (size_t n = 0; n < ntaps; n++) {
        long m = (long)n - m0;
        float sinc;
        if (m == 0) {
            sinc = 2.0f * fc;
        } else {
            float x = O_PI * (float)m;
            sinc = (2.0f * fc) * sinf(2.0f * O_PI * fc * (float)m) / x;
        }
        float w = 0.5f - 0.5f * cosf(2.0f * O_PI * (float)n / ((float)ntaps - 1.0f));
        taps[n] = sinc * w;
    }
    float s = 0.0f;
    for (size_t n = 0; n < ntaps; n++) s += taps[n];
    for (size_t n = 0; n < ntaps; n++) taps[n] /= s;
    return ntaps;
}
void o_fir_init(o_fir *f, float fs, float pass_hz, float trans_hz) {
    f->len = o_fir_ntaps(fs, pass_hz, trans_hz);
    f->taps = (float *)malloc(f->len * sizeof(float));
    f->delay = (float *)calloc(f->len, sizeof(float));
    o_fir_design_taps(fs, pass_hz, trans_hz, f->taps, f->len);
    f->idx = 0;
}
void o_fir_free(o_fir *f) { free(f->taps); free(f->delay); f->taps = NULL; f->delay = NULL; }
/* dsp/fir.rs:57-66 dot: taps[t] pairs with delay[(idx+len-1-t) % len]; the
 * reference's integer modulo per tap is kept on purpose (it is what the CPU
 * baseline costs). */
static inline float o_fir_dot(const o_fir *f) {
    size_t len = f->len;
    float acc = 0.0f;
    for (size_t t = 0; t < len; t++) {
        size_t d_idx = (f->idx + len - 1 - t) % len;
        acc += f->delay[d_idx] * f->taps[t];
    }
    return acc;
}
/* dsp/fir.rs:47-54 process */
void o_fir_process(o_fir *f, const float *in, float *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        f->delay[f->idx] = in[i];
        out[i] = o_fir_dot(f);
        f->idx = (f->idx + 1) % f->len;
    }
}

/* ------------------------------------------------------------------ */
/* dsp/fir.rs:74-82 kaiser_beta; :86-99 bessel_i0; :113-141 taps;
 * :147-150 transition_norm; :154-157 num_taps                          */
float o_kaiser_beta(float a_db) {
    if (a_db > 50.0f) return 0.1102f * (a_db - 8.7f);
    if (a_db >= 21.0f) return 0.5842f * powf(a_db - 21.0f, 0.4f) + 0.07886f * (a_db - 21.0f);
    return 0.0f;
}
float o_bessel_i0(float x) {
    float half = 0.5f * x;
    float term = 1.0f, sum = 1.0f;
    for (unsigned k = 1; k <= 40; k++) {
        term *= half / (float)k;
        float t = term * term;
        sum += t;
        if (t < 1e-12f * sum) break;
    }
    return sum;
}
size_t o_kaiser_lowpass_taps(size_t num_taps, float cutoff_norm, float stopband_db, float *taps, size_t cap) {
    size_t m = (num_taps < 3 ? 3 : num_taps) | 1u;
    if (!taps || cap < m) return m;
    float mid = (float)(m / 2);
    float fc = o_clampf(cutoff_norm, 1e-4f, 0.4999f);
    float beta = o_kaiser_beta(stopband_db);
    float i0_beta = o_bessel_i0(beta);
    for (size_t n = 0; n < m; n++) {
        float d = (float)n - mid;
        float ideal = (d == 0.0f) ? 2.0f * fc : sinf(O_TAU * fc * d) / (O_PI * d);
        float r = d / mid;
        float w = o_bessel_i0(beta * sqrtf(o_maxf(1.0f - r * r, 0.0f))) / i0_beta;
        taps[n] = ideal * w;
    }
    float s = 0.0f;
    for (size_t n = 0; n < m; n++) s += taps[n];
    if (fabsf(s) > FLT_EPSILON)
        for (size_t n = 0; n < m; n++) taps[n] /= s;
    return m;
}
float o_kaiser_transition_norm(size_t num_taps, float stopband_db) {
    float m = (float)((num_taps < 3 ? 3 : num_taps) | 1u);
    return (o_maxf(stopband_db, 21.0f) - 8.0f) / (14.36f * m);
}
size_t o_kaiser_num_taps(float transition_norm, float stopband_db) {
    float m = ceilf((o_maxf(stopband_db, 21.0f) - 8.0f) / (14.36f * o_maxf(transition_norm, 1e-4f)));
    return ((size_t)o_maxf(m, 3.0f)) | 1u;
}

/* ------------------------------------------------------------------ */
/* dsp/fir.rs:193-204 from_taps; :221-224 reset; :229-247 push;
 * :260-276 filter_aligned; :287-296 Block::process                      */
void o_firiq_from_taps(o_firiq *f, const float *taps, size_t len) {
    if (len == 0) {
        f->len = 1;
        f->taps = (float *)malloc(sizeof(float));
        f->taps[0] = 1.0f;
    } else {
        f->len = len;
        f->taps = (float *)malloc(len * sizeof(float));
        memcpy(f->taps, taps, len * sizeof(float));
    }
    f->delay = (oc32 *)calloc(f->len, sizeof(oc32));
    f->idx = 0;
}
void o_firiq_free(o_firiq *f) { free(f->taps); free(f->delay); }
void o_firiq_reset(o_firiq *f) { memset(f->delay, 0, f->len * sizeof(oc32)); f->idx = 0; }
oc32 o_firiq_push(o_firiq *f, oc32 s) {
    size_t len = f->len, idx = f->idx;
    f->delay[idx] = s;
    float re = 0.0f, im = 0.0f;
    for (size_t j = 0; j <= idx; j++) {
        oc32 d = f->delay[idx - j];
        float t = f->taps[j];
        re = fmaf(d.re, t, re);
        im = fmaf(d.im, t, im);
    }
    for (size_t k = 0; k + idx + 1 < len; k++) {
        oc32 d = f->delay[len - 1 - k];
        float t = f->taps[idx + 1 + k];
        re = fmaf(d.re, t, re);
        im = fmaf(d.im, t, im);
    }
    f->idx = (idx + 1 == len) ? 0 : idx + 1;
    oc32 o = { re, im };
    return o;
}
o_work_report o_firiq_process(o_firiq *f, const oc32 *in, size_t n_in, oc32 *out, size_t n_out) {
    size_t n = n_in < n_out ? n_in : n_out;
    for (size_t i = 0; i < n; i++) out[i] = o_firiq_push(f, in[i]);
    o_work_report w = { n, n };
    return w;
}
void o_firiq_filter_aligned(o_firiq *f, oc32 *io, size_t n) {
    size_t d = (f->len - 1) / 2;
    o_firiq_reset(f);
    for (size_t i = 0; i < d; i++) {
        oc32 x = { 0.0f, 0.0f };
        if (i < n) x = io[i];
        o_firiq_push(f, x);
    }
    for (size_t i = 0; i < n; i++) {
        oc32 x = { 0.0f, 0.0f };
        if (i + d < n) x = io[i + d];
        io[i] = o_firiq_push(f, x);
    }
}

/* ------------------------------------------------------------------ */
/* dsp/decim.rs:24-37 new; :44-76 process (full-rate filter, keep j*m) */
void o_decim_init(o_decim *d, float fs, size_t m, float cutoff_hz, float trans_hz) {
    d->m = m < 1 ? 1 : m;
    o_fir_init(&d->lp_i, fs, cutoff_hz, trans_hz);
    o_fir_init(&d->lp_q, fs, cutoff_hz, trans_hz);
    d->ri = d->rq = d->yi = d->yq = NULL;
    d->cap = 0;
}
void o_decim_free(o_decim *d) {
    o_fir_free(&d->lp_i); o_fir_free(&d->lp_q);
    free(d->ri); free(d->rq); free(d->yi); free(d->yq);
}
o_work_report o_decim_process(o_decim *d, const oc32 *in, size_t n, oc32 *out, size_t out_len) {
    if (d->cap < n) {
        d->ri = (float *)realloc(d->ri, n * sizeof(float));
        d->rq = (float *)realloc(d->rq, n * sizeof(float));
        d->yi = (float *)realloc(d->yi, n * sizeof(float));
        d->yq = (float *)realloc(d->yq, n * sizeof(float));
        d->cap = n;
    }
    for (size_t k = 0; k < n; k++) { d->ri[k] = in[k].re; d->rq[k] = in[k].im; }
    o_fir_process(&d->lp_i, d->ri, d->yi, n);
    o_fir_process(&d->lp_q, d->rq, d->yq, n);
    size_t m = d->m;
    size_t n_out = (n + m - 1) / m;
    size_t n_write = n_out < out_len ? n_out : out_len;
    for (size_t j = 0; j < n_write; j++) {
        out[j].re = d->yi[j * m];
        out[j].im = d->yq[j * m];
    }
    o_work_report w = { n, n_write };
    return w;
}

/* ------------------------------------------------------------------ */
/* dsp/iir.rs:34-40 Biquad::process (TDF-II with mul_add)              */
float o_biquad_process(o_biquad *b, float x) {
    float y = fmaf(x, b->b0, b->z1);
    b->z1 = fmaf(x, b->b1, b->z2) - b->a1 * y;
    b->z2 = x * b->b2 - b->a2 * y;
    return y;
}
/* dsp/iir.rs:49-71 LpCascade::design (RBJ Butterworth, Q=1/sqrt2, x2) */
void o_lp_cascade_design(o_lp_cascade *c, float fs, float fc) {
    float w0 = O_TAU * fc / fs;
    float sn = sinf(w0), cs = cosf(w0);
    float alpha = sn / (2.0f * sqrtf(0.5f));
    float b0 = (1.0f - cs) * 0.5f;
    float b1 = 1.0f - cs;
    float b2 = (1.0f - cs) * 0.5f;
    float a0 = 1.0f + alpha;
    float a1 = -2.0f * cs;
    float a2 = 1.0f - alpha;
    float norm = 1.0f / a0;
    o_biquad st = { b0 * norm, b1 * norm, b2 * norm, a1 * norm, a2 * norm, 0.0f, 0.0f };
    c->s[0] = st; c->s[1] = st;
}
/* dsp/iir.rs:79-83 */
float o_lp_cascade_process(o_lp_cascade *c, float x) {
    x = o_biquad_process(&c->s[0], x);
    return o_biquad_process(&c->s[1], x);
}
void o_lp_cascade_coeffs(float fs, float fc, float out5[5]) {
    o_lp_cascade c;
    o_lp_cascade_design(&c, fs, fc);
    out5[0] = c.s[0].b0; out5[1] = c.s[0].b1; out5[2] = c.s[0].b2; out5[3] = c.s[0].a1; out5[4] = c.s[0].a2;
}

/* dsp/iir.rs:111-137 LpDcCascade::design */
void o_lpdc_design(o_lpdc *c, float fs, float lp_fc, float dc_cut_hz) {
    float w0 = O_TAU * lp_fc / fs;
    float sn = sinf(w0), cs = cosf(w0);
    float alpha = sn / (2.0f * sqrtf(0.5f));
    float b0r = (1.0f - cs) * 0.5f, b1r = 1.0f - cs, b2r = (1.0f - cs) * 0.5f;
    float a0 = 1.0f + alpha, a1r = -2.0f * cs, a2r = 1.0f - alpha;
    float norm = 1.0f / a0;
    float r = o_clampf(1.0f - 2.0f * O_PI * (o_maxf(dc_cut_hz, 0.1f) / fs), 0.0f, 0.9999f);
    memset(c, 0, sizeof(*c));
    c->b0 = b0r * norm; c->b1 = b1r * norm; c->b2 = b2r * norm;
    c->a1 = a1r * norm; c->a2 = a2r * norm; c->r = r;
}
/* dsp/iir.rs:151-165 process */
float o_lpdc_process(o_lpdc *c, float x) {
    float y0 = fmaf(x, c->b0, c->z0_1);
    c->z0_1 = fmaf(x, c->b1, c->z0_2) - c->a1 * y0;
    c->z0_2 = x * c->b2 - c->a2 * y0;
    float y1 = fmaf(y0, c->b0, c->z1_1);
    c->z1_1 = fmaf(y0, c->b1, c->z1_2) - c->a1 * y1;
    c->z1_2 = y0 * c->b2 - c->a2 * y1;
    float y = y1 - c->dc_x1 + c->r * c->dc_y1;
    c->dc_x1 = y1;
    c->dc_y1 = y;
    return y;
}
/* dsp/iir.rs:170-186 process_mapped with f = f32::sqrt (am.rs:54) */
/* iir.rs:170-186 process_mapped(x, f) for the maps the engine exposes (ORION_MAP_*):
 * 0 identity (|v| v: the same as process), 1 f32::sqrt, 2 f32::abs. */
float o_lpdc_process_mapped(o_lpdc *c, float x, int map) {
    float y0 = fmaf(x, c->b0, c->z0_1);
    c->z0_1 = fmaf(x, c->b1, c->z0_2) - c->a1 * y0;
    c->z0_2 = x * c->b2 - c->a2 * y0;
    float y1 = fmaf(y0, c->b0, c->z1_1);
    c->z1_1 = fmaf(y0, c->b1, c->z1_2) - c->a1 * y1;
    c->z1_2 = y0 * c->b2 - c->a2 * y1;
    float mapped = map == 1 ? sqrtf(y1) : map == 2 ? fabsf(y1) : y1;
    float y = mapped - c->dc_x1 + c->r * c->dc_y1;
    c->dc_x1 = mapped;
    c->dc_y1 = y;
    return y;
}
float o_lpdc_process_mapped_sqrt(o_lpdc *c, float x) {
    float y0 = fmaf(x, c->b0, c->z0_1);
    c->z0_1 = fmaf(x, c->b1, c->z0_2) - c->a1 * y0;
    c->z0_2 = x * c->b2 - c->a2 * y0;
    float y1 = fmaf(y0, c->b0, c->z1_1);
    c->z1_1 = fmaf(y0, c->b1, c->z1_2) - c->a1 * y1;
    c->z1_2 = y0 * c->b2 - c->a2 * y1;
    float mapped = sqrtf(y1);
    float y = mapped - c->dc_x1 + c->r * c->dc_y1;
    c->dc_x1 = mapped;
    c->dc_y1 = y;
    return y;
}
void o_lpdc_coeffs(float fs, float lp_fc, float dc_cut_hz, float out6[6]) {
    o_lpdc c;
    o_lpdc_design(&c, fs, lp_fc, dc_cut_hz);
    out6[0] = c.b0; out6[1] = c.b1; out6[2] = c.b2; out6[3] = c.a1; out6[4] = c.a2; out6[5] = c.r;
}

/* ------------------------------------------------------------------ */
/* dsp/dc.rs:15-21 new; :40-58 process                                 */
void o_dc_init(o_dc *d, float fs, float cut_hz) {
    d->r = o_clampf(1.0f - 2.0f * O_PI * (o_maxf(cut_hz, 0.1f) / fs), 0.0f, 0.9999f);
    d->x1 = 0.0f; d->y1 = 0.0f;
}
o_work_report o_dc_process(o_dc *d, const float *in, float *out, size_t n) {
    float x1 = d->x1, y1 = d->y1, r = d->r;
    for (size_t i = 0; i < n; i++) {
        float x = in[i];
        float y = x - x1 + r * y1;
        out[i] = y;
        x1 = x; y1 = y;
    }
    d->x1 = x1; d->y1 = y1;
    o_work_report w = { n, n };
    return w;
}

/* ------------------------------------------------------------------ */
/* demodulate/fm.rs:22-32 new; :34-37 with_translate; :45-77 process   */
void o_fm_demod_init(o_fm_demod *d, float fs, float dev_hz, float audio_bw_hz) {
    d->fs = fs;
    d->k = 1.0f / o_maxf(dev_hz, 1.0f);
    d->has_xf = 0;
    d->prev.re = 1.0f; d->prev.im = 0.0f;
    o_lp_cascade_design(&d->post_lp, fs, audio_bw_hz * 0.9f);
}
void o_fm_demod_with_translate(o_fm_demod *d, float freq_hz) {
    d->has_xf = 1;
    o_rotator_init(&d->xf, freq_hz, d->fs);
}
o_work_report o_fm_demod_process(o_fm_demod *d, const oc32 *in, float *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        oc32 z = in[i];
        if (d->has_xf) {
            /* num-complex Mul (a+bi)(c+di) = (ac - bd) + (ad + bc)i with the
             * conjugated rotator phasor, fm.rs:49 */
            oc32 p = o_rotator_next(&d->xf);
            float c = p.re, dd = -p.im;
            oc32 t = { z.re * c - z.im * dd, z.re * dd + z.im * c };
            z = t;
        }
        float pr = z.re * d->prev.re + z.im * d->prev.im;
        float pi = z.im * d->prev.re - z.re * d->prev.im;
        out[i] = o_lp_cascade_process(&d->post_lp, o_atan2_approx(pi, pr) * d->k);
        d->prev = z;
    }
    o_work_report w = { n, n };
    return w;
}

/* demodulate/pm.rs:22-32 new; :39-66 process (num-complex z*conj(prev)) */
void o_pm_demod_init(o_pm_demod *d, float fs, float k, float audio_bw_hz) {
    d->fs = fs; d->k = k;
    o_lp_cascade_design(&d->post_lp, fs, audio_bw_hz * 0.9f);
    d->prev.re = 1.0f; d->prev.im = 0.0f;
}
o_work_report o_pm_demod_process(o_pm_demod *d, const oc32 *in, float *out, size_t n) {
    oc32 prev = d->prev;
    for (size_t i = 0; i < n; i++) {
        oc32 z = in[i];
        float c = prev.re, dd = -prev.im;
        float wr = z.re * c - z.im * dd;
        float wi = z.re * dd + z.im * c;
        out[i] = o_lp_cascade_process(&d->post_lp, d->k * o_atan2_approx(wi, wr));
        prev = z;
    }
    d->prev = prev;
    o_work_report w = { n, n };
    return w;
}

/* demodulate/ssb.rs:15-20 new; :28-71 process                         */
void o_ssb_demod_init(o_ssb_demod *d, float fs, float bfo_hz, float audio_bw_hz) {
    o_lpdc_design(&d->filt, fs, audio_bw_hz * 0.9f, 2.0f);
    o_rotator_init(&d->rot, bfo_hz, fs);
}
o_work_report o_ssb_demod_process(o_ssb_demod *d, const oc32 *in, float *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        oc32 p = o_rotator_next(&d->rot);
        float y = fmaf(in[i].re, p.re, in[i].im * p.im);
        out[i] = o_lpdc_process(&d->filt, y);
    }
    o_work_report w = { n, n };
    return w;
}

/* demodulate/am.rs:24-30 new; :33-36 with_abs_approx; :44-129 process  */
void o_am_demod_init(o_am_demod *d, float fs, float audio_bw_hz) {
    o_lpdc_design(&d->filt, fs, audio_bw_hz * 0.9f, 2.0f);
    d->abs_approx = 0; d->k1 = 0.0f; d->k2 = 0.0f;
}
void o_am_demod_with_abs_approx(o_am_demod *d, float k1, float k2) { d->abs_approx = 1; d->k1 = k1; d->k2 = k2; }
o_work_report o_am_demod_process(o_am_demod *d, const oc32 *in, float *out, size_t n) {
    if (!d->abs_approx) {
        for (size_t i = 0; i < n; i++) {
            float p = fmaf(in[i].re, in[i].re, in[i].im * in[i].im);
            out[i] = o_lpdc_process_mapped_sqrt(&d->filt, p);
        }
    } else {
        for (size_t i = 0; i < n; i++) {
            float e = fmaf(d->k1, fabsf(in[i].re), d->k2 * fabsf(in[i].im));
            out[i] = o_lpdc_process(&d->filt, e);
        }
    }
    o_work_report w = { n, n };
    return w;
}

/* demodulate/cw.rs:15-25 new; :34-46 process                          */
void o_cw_demod_init(o_cw_demod *d, float fs, float tone_hz, float env_bw_hz) {
    (void)tone_hz;
    float fc = o_maxf(env_bw_hz, 1.0f);
    d->alpha = expf(-O_TAU * fc / fs);
    d->y = 0.0f; d->gain = 1.0f;
}
o_work_report o_cw_demod_process(o_cw_demod *d, const oc32 *in, float *out, size_t n) {
    float a = d->alpha;
    for (size_t i = 0; i < n; i++) {
        float mag = sqrtf(in[i].re * in[i].re + in[i].im * in[i].im);
        d->y = a * d->y + (1.0f - a) * mag;
        out[i] = d->y * d->gain;
    }
    o_work_report w = { n, n };
    return w;
}

/* ------------------------------------------------------------------ */
/* modulate/fm.rs:22-31 new; :45-74 process                            */
void o_fm_mod_init(o_fm_mod *m, float fs, float deviation_hz, float rf_hz) {
    m->fs = fs; m->kf_hz_per_unit = deviation_hz;
    m->z.re = 1.0f; m->z.im = 0.0f;
    o_nco_init(&m->rf_nco, rf_hz, fs);
    m->gain = 1.0f; m->renorm_ctr = 0;
}
o_work_report o_fm_mod_process(o_fm_mod *m, const float *in, oc32 *out, size_t n) {
    float kf = O_TAU * m->kf_hz_per_unit / m->fs;
    for (size_t i = 0; i < n; i++) {
        float dphi = kf * in[i];
        float ds = sinf(dphi), dc = cosf(dphi);
        float zr = fmaf(m->z.re, dc, -(m->z.im * ds));
        float zi = fmaf(m->z.im, dc, m->z.re * ds);
        m->z.re = zr; m->z.im = zi;
        m->renorm_ctr += 1u;
        if ((m->renorm_ctr & 0x3FFu) == 0) {
            float inv = 1.0f / sqrtf(m->z.re * m->z.re + m->z.im * m->z.im);
            m->z.re *= inv; m->z.im *= inv;
        }
        oc32 base = { m->z.re * m->gain, m->z.im * m->gain };
        out[i] = o_mix_with_nco(base, &m->rf_nco);
    }
    o_work_report w = { n, n };
    return w;
}

/* modulate/pm.rs:15-22 new; :36-47 process                             */
void o_pm_mod_init(o_pm_mod *m, float fs, float kp, float rf_hz) {
    m->kp = kp; o_nco_init(&m->rf_nco, rf_hz, fs); m->gain = 1.0f;
}
o_work_report o_pm_mod_process(o_pm_mod *m, const float *in, oc32 *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        float phi = m->kp * in[i];
        oc32 base = { cosf(phi) * m->gain, sinf(phi) * m->gain };
        out[i] = o_mix_with_nco(base, &m->rf_nco);
    }
    o_work_report w = { n, n };
    return w;
}

/* modulate/ssb.rs:23-35 new; :43-114 process                           */
void o_ssb_mod_init(o_ssb_mod *m, float fs, float audio_bw_hz, float audio_if_hz, float rf_hz, int usb) {
    float fc = audio_bw_hz * 0.9f;
    m->usb = usb;
    o_lp_cascade_design(&m->lp_i, fs, fc);
    o_lp_cascade_design(&m->lp_q, fs, fc);
    o_rotator_init(&m->aud_nco, audio_if_hz, fs);
    o_rotator_init(&m->rf_nco, rf_hz, fs);
}
o_work_report o_ssb_mod_process(o_ssb_mod *m, const float *in, oc32 *out, size_t n) {
    float side = m->usb ? 1.0f : -1.0f;
    for (size_t i = 0; i < n; i++) {
        oc32 p = o_rotator_next(&m->aud_nco);
        float ii = o_lp_cascade_process(&m->lp_i, in[i] * p.re);
        float qq = o_lp_cascade_process(&m->lp_q, in[i] * p.im);
        oc32 z = { ii, side * qq };
        oc32 r = o_rotator_next(&m->rf_nco);
        out[i].re = fmaf(z.re, r.re, -(z.im * r.im));
        out[i].im = fmaf(z.im, r.re, z.re * r.im);
    }
    o_work_report w = { n, n };
    return w;
}

/* modulate/am.rs:21-32 new; :44-120 process                            */
void o_am_mod_init(o_am_mod *m, float fs, float rf_hz, float carrier_level, float modulation_index) {
    m->gain = 1.0f; m->carrier_level = carrier_level; m->modulation_index = modulation_index;
    m->clamp = 0; o_rotator_init(&m->rf_nco, rf_hz, fs);
}
o_work_report o_am_mod_process(o_am_mod *m, const float *in, oc32 *out, size_t n) {
    float mi = m->modulation_index, cl = m->carrier_level, g = m->gain;
    for (size_t i = 0; i < n; i++) {
        float v = cl + mi * in[i];
        if (m->clamp) v = o_clampf(v, -1.0f, 1.0f);
        float mm = v * g;
        oc32 r = o_rotator_next(&m->rf_nco);
        out[i].re = mm * r.re; out[i].im = mm * r.im;
    }
    o_work_report w = { n, n };
    return w;
}

/* modulate/cw.rs:22-36 new; :45-87 process                             */
void o_cw_mod_init(o_cw_mod *m, float fs, float tone_hz, float rise_ms, float fall_ms) {
    float tau_r = (o_maxf(rise_ms, 0.1f) * 1e-3f) * fs;
    float tau_f = (o_maxf(fall_ms, 0.1f) * 1e-3f) * fs;
    o_nco_init(&m->nco, tone_hz, fs);
    m->env = 0.0f;
    m->alpha_rise = expf(-1.0f / tau_r);
    m->alpha_fall = expf(-1.0f / tau_f);
    m->gain = 1.0f;
}
o_work_report o_cw_mod_process(o_cw_mod *m, const float *in, oc32 *out, size_t n) {
    for (size_t i = 0; i < n; i++) {
        float tgt = o_clampf(in[i], 0.0f, 1.0f);
        if (tgt >= m->env) m->env = m->alpha_rise * m->env + (1.0f - m->alpha_rise) * tgt;
        else m->env = m->alpha_fall * m->env + (1.0f - m->alpha_fall) * tgt;
        oc32 base = { m->env * m->gain, 0.0f };
        out[i] = o_mix_with_nco(base, &m->nco);
    }
    o_work_report w = { n, n };
    return w;
}

/* ------------------------------------------------------------------ */
/* tests/common/mod.rs:27-48 add_awgn: xorshift64 (13,7,17), 12-uniform sum */
static inline float o_awgn_next(uint64_t *s) {
    float sum = 0.0f;
    for (int k = 0; k < 12; k++) {
        *s ^= *s << 13;
        *s ^= *s >> 7;
        *s ^= *s << 17;
        sum += (float)(*s) / (float)UINT64_MAX - 0.5f;
    }
    return sum;
}
void o_add_awgn(oc32 *iq, size_t n, float noise_power, uint64_t seed) {
    uint64_t state = seed ^ 0xDEADBEEFCAFE0000ull;
    float scale = sqrtf(noise_power / 2.0f);
    for (size_t i = 0; i < n; i++) {
        float ni = o_awgn_next(&state) * scale;
        float nq = o_awgn_next(&state) * scale;
        iq[i].re += ni;
        iq[i].im += nq;
    }
}

/* ================================================================== */
/* Flat entry points                                                   */
static inline size_t o_step(size_t chunk, size_t left) { return (chunk == 0 || chunk > left) ? left : chunk; }

size_t o_run_rotator(float freq_hz, float fs, const oc32 *in, oc32 *out, size_t n, size_t chunk) {
    o_rotator r; o_rotator_init(&r, freq_hz, fs);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_rotator_rotate_block(&r, in + i, out + i, c); i += c; }
    return n;
}
/* Rotator with a retune mid-stream (rotator.rs:35-39: w changes, z stays): mode 0
 * rotate_block (out: cf32), 1 mix_usb_block (out: f32, rotator.rs:88-94); set_freq(f2,
 * fs2) after the first n_switch samples; reset_phase (rotator.rs:28-31) instead when
 * reset_at_switch. */
size_t o_run_rotator_retune(float f1, float fs, int mode, const oc32 *in, void *out, size_t n, size_t n_switch,
                            float f2, float fs2, int reset_at_switch) {
    o_rotator r; o_rotator_init(&r, f1, fs);
    for (int part = 0; part < 2; part++) {
        size_t a = part ? n_switch : 0, b = part ? n : (n_switch < n ? n_switch : n);
        if (part) {
            if (reset_at_switch) { r.z.re = 1.0f; r.z.im = 0.0f; r.renorm_ctr = 0; }
            else o_rotator_set_freq(&r, f2, fs2);
        }
        if (b <= a) continue;
        if (mode == 0) o_rotator_rotate_block(&r, in + a, (oc32 *)out + a, b - a);
        else o_rotator_mix_usb_block(&r, in + a, (float *)out + a, b - a);
    }
    return n;
}
/* Nco (nco.rs): mode 0 mix_with_nco per sample (nco.rs:63-66), 1 next_cs (nco.rs:42-58)
 * as (cos, sin) pairs (in unused); set_freq(f2) after n_switch samples. */
size_t o_run_nco(float f1, float fs, int mode, const oc32 *in, oc32 *out, size_t n, size_t n_switch, float f2) {
    o_nco q; o_nco_init(&q, f1, fs);
    for (size_t i = 0; i < n; i++) {
        if (i == n_switch) o_nco_set_freq(&q, f2);
        if (mode == 0) out[i] = o_mix_with_nco(in[i], &q);
        else { float cc, ss; o_nco_next_cs(&q, &cc, &ss); out[i].re = cc; out[i].im = ss; }
    }
    return n;
}
/* Biquad::new(b0, b1, b2, a1, a2) (iir.rs:15-41) over a stream. */
size_t o_run_biquad(float b0, float b1, float b2, float a1, float a2, const float *in, float *out, size_t n) {
    o_biquad b = {b0, b1, b2, a1, a2, 0.0f, 0.0f};
    for (size_t i = 0; i < n; i++) out[i] = o_biquad_process(&b, in[i]);
    return n;
}
/* LpDcCascade::design(fs, lp_fc, dc_cut) (iir.rs:111-137): process (:151-165), or
 * process_mapped(x, f32::sqrt) (:170-186) when sqrt_map. */
/* map: -1 process (:151-165), else process_mapped with map 0 identity, 1 sqrt, 2 abs */
size_t o_run_lpdc(float fs, float lp_fc, float dc_cut, int map, const float *in, float *out, size_t n) {
    o_lpdc c; o_lpdc_design(&c, fs, lp_fc, dc_cut);
    for (size_t i = 0; i < n; i++) out[i] = map < 0 ? o_lpdc_process(&c, in[i]) : o_lpdc_process_mapped(&c, in[i], map);
    return n;
}
size_t o_run_fir(float fs, float pass_hz, float trans_hz, const float *in, float *out, size_t n, size_t chunk) {
    o_fir f; o_fir_init(&f, fs, pass_hz, trans_hz);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_fir_process(&f, in + i, out + i, c); i += c; }
    o_fir_free(&f);
    return n;
}
size_t o_run_firiq(const float *taps, size_t ntaps, const oc32 *in, oc32 *out, size_t n, size_t chunk) {
    o_firiq f; o_firiq_from_taps(&f, taps, ntaps);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_firiq_process(&f, in + i, c, out + i, c); i += c; }
    o_firiq_free(&f);
    return n;
}
void o_run_firiq_aligned(const float *taps, size_t ntaps, oc32 *io, size_t n) {
    o_firiq f; o_firiq_from_taps(&f, taps, ntaps);
    o_firiq_filter_aligned(&f, io, n);
    o_firiq_free(&f);
}
size_t o_run_decim(float fs, size_t m, float cutoff_hz, float trans_hz, const oc32 *in, size_t n,
                   oc32 *out, size_t out_cap, size_t chunk) {
    o_decim d; o_decim_init(&d, fs, m, cutoff_hz, trans_hz);
    size_t w = 0;
    for (size_t i = 0; i < n;) {
        size_t c = o_step(chunk, n - i);
        o_work_report r = o_decim_process(&d, in + i, c, out + w, out_cap - w);
        w += r.out_written; i += c;
    }
    o_decim_free(&d);
    return w;
}
size_t o_run_lp_cascade(float fs, float fc, const float *in, float *out, size_t n) {
    o_lp_cascade c; o_lp_cascade_design(&c, fs, fc);
    for (size_t i = 0; i < n; i++) out[i] = o_lp_cascade_process(&c, in[i]);
    return n;
}
size_t o_run_dc(float fs, float cut_hz, const float *in, float *out, size_t n, size_t chunk) {
    o_dc d; o_dc_init(&d, fs, cut_hz);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_dc_process(&d, in + i, out + i, c); i += c; }
    return n;
}
size_t o_run_fm_demod(float fs, float dev_hz, float audio_bw_hz, float translate_hz, int has_translate,
                      const oc32 *in, float *out, size_t n, size_t chunk) {
    o_fm_demod d; o_fm_demod_init(&d, fs, dev_hz, audio_bw_hz);
    if (has_translate) o_fm_demod_with_translate(&d, translate_hz);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_fm_demod_process(&d, in + i, out + i, c); i += c; }
    return n;
}
size_t o_run_pm_demod(float fs, float k, float audio_bw_hz, const oc32 *in, float *out, size_t n, size_t chunk) {
    o_pm_demod d; o_pm_demod_init(&d, fs, k, audio_bw_hz);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_pm_demod_process(&d, in + i, out + i, c); i += c; }
    return n;
}
size_t o_run_ssb_demod(float fs, float bfo_hz, float audio_bw_hz, const oc32 *in, float *out, size_t n, size_t chunk) {
    o_ssb_demod d; o_ssb_demod_init(&d, fs, bfo_hz, audio_bw_hz);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_ssb_demod_process(&d, in + i, out + i, c); i += c; }
    return n;
}
size_t o_run_am_demod(float fs, float audio_bw_hz, int abs_approx, float k1, float k2,
                      const oc32 *in, float *out, size_t n, size_t chunk) {
    o_am_demod d; o_am_demod_init(&d, fs, audio_bw_hz);
    if (abs_approx) o_am_demod_with_abs_approx(&d, k1, k2);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_am_demod_process(&d, in + i, out + i, c); i += c; }
    return n;
}
size_t o_run_cw_demod(float fs, float tone_hz, float env_bw_hz, float gain, const oc32 *in, float *out,
                      size_t n, size_t chunk) {
    o_cw_demod d; o_cw_demod_init(&d, fs, tone_hz, env_bw_hz); d.gain = gain;
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_cw_demod_process(&d, in + i, out + i, c); i += c; }
    return n;
}
size_t o_run_fm_mod(float fs, float dev_hz, float rf_hz, const float *in, oc32 *out, size_t n, size_t chunk) {
    o_fm_mod m; o_fm_mod_init(&m, fs, dev_hz, rf_hz);
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_fm_mod_process(&m, in + i, out + i, c); i += c; }
    return n;
}
size_t o_run_pm_mod(float fs, float kp, float rf_hz, const float *in, oc32 *out, size_t n) {
    o_pm_mod m; o_pm_mod_init(&m, fs, kp, rf_hz); o_pm_mod_process(&m, in, out, n); return n;
}
size_t o_run_ssb_mod(float fs, float bw, float if_hz, float rf_hz, int usb, const float *in, oc32 *out, size_t n) {
    o_ssb_mod m; o_ssb_mod_init(&m, fs, bw, if_hz, rf_hz, usb); o_ssb_mod_process(&m, in, out, n); return n;
}
size_t o_run_am_mod(float fs, float rf_hz, float cl, float mi, float gain, int clamp, const float *in,
                    oc32 *out, size_t n) {
    o_am_mod m; o_am_mod_init(&m, fs, rf_hz, cl, mi); m.gain = gain; m.clamp = clamp;
    o_am_mod_process(&m, in, out, n); return n;
}
size_t o_run_cw_mod(float fs, float tone_hz, float rise_ms, float fall_ms, const float *in, oc32 *out, size_t n) {
    o_cw_mod m; o_cw_mod_init(&m, fs, tone_hz, rise_ms, fall_ms); o_cw_mod_process(&m, in, out, n); return n;
}

/* ------------------------------------------------------------------ */
/* WBFM chain as composed by docs/demodulate.md:128-133 */
typedef struct { o_rotator rot; o_decim dec; o_fm_demod fm; o_fir audio; oc32 *mixed; oc32 *dec_out; float *disc; size_t cap; } o_wbfm;
static void o_wbfm_init(o_wbfm *w, const o_wbfm_params *p, float f_off) {
    o_rotator_init(&w->rot, -f_off, p->fs);
    o_decim_init(&w->dec, p->fs, p->m, p->dec_cutoff, p->dec_trans);
    float fs2 = p->fs / (float)p->m;
    o_fm_demod_init(&w->fm, fs2, p->dev_hz, p->audio_bw);
    o_fir_init(&w->audio, fs2, p->audio_pass, p->audio_trans);
    w->mixed = NULL; w->dec_out = NULL; w->disc = NULL; w->cap = 0;
}
static void o_wbfm_free(o_wbfm *w) {
    o_decim_free(&w->dec); o_fir_free(&w->audio);
    free(w->mixed); free(w->dec_out); free(w->disc);
}
static size_t o_wbfm_call(o_wbfm *w, const oc32 *in, size_t n, float *out, size_t out_cap) {
    if (w->cap < n) {
        w->mixed = (oc32 *)realloc(w->mixed, n * sizeof(oc32));
        w->dec_out = (oc32 *)realloc(w->dec_out, n * sizeof(oc32));
        w->disc = (float *)realloc(w->disc, n * sizeof(float));
        w->cap = n;
    }
    o_rotator_rotate_block(&w->rot, in, w->mixed, n);
    o_work_report r = o_decim_process(&w->dec, w->mixed, n, w->dec_out, n);
    size_t nd = r.out_written < out_cap ? r.out_written : out_cap;
    o_fm_demod_process(&w->fm, w->dec_out, w->disc, nd);
    o_fir_process(&w->audio, w->disc, out, nd);
    return nd;
}
size_t o_run_wbfm(const o_wbfm_params *p, const oc32 *in, size_t n, float *out, size_t out_cap, size_t chunk) {
    o_wbfm w; o_wbfm_init(&w, p, p->f_off);
    size_t wr = 0;
    for (size_t i = 0; i < n;) {
        size_t c = o_step(chunk, n - i);
        wr += o_wbfm_call(&w, in + i, c, out + wr, out_cap - wr);
        i += c;
    }
    o_wbfm_free(&w);
    return wr;
}

/* Multi-channel: independent channels on a pthread pool. */
typedef struct {
    int kind;
    const o_wbfm_params *p; const float *f_off; size_t nch, n; const oc32 *in; void *out;
    float fs, bfo, bw, cutoff, trans; size_t m;
    size_t next; pthread_mutex_t mu;
} o_pool;
static void *o_pool_worker(void *arg) {
    o_pool *P = (o_pool *)arg;
    for (;;) {
        pthread_mutex_lock(&P->mu);
        size_t ch = P->next++;
        pthread_mutex_unlock(&P->mu);
        if (ch >= P->nch) break;
        const oc32 *x = P->in + ch * P->n;
        if (P->kind == 0) {
            size_t nout = (P->n + P->p->m - 1) / P->p->m;
            o_wbfm w; o_wbfm_init(&w, P->p, P->f_off[ch]);
            o_wbfm_call(&w, x, P->n, (float *)P->out + ch * nout, nout);
            o_wbfm_free(&w);
        } else if (P->kind == 1) {
            o_ssb_demod d; o_ssb_demod_init(&d, P->fs, P->bfo, P->bw);
            o_ssb_demod_process(&d, x, (float *)P->out + ch * P->n, P->n);
        } else {
            size_t nout = (P->n + P->m - 1) / P->m;
            o_decim d; o_decim_init(&d, P->fs, P->m, P->cutoff, P->trans);
            o_decim_process(&d, x, P->n, (oc32 *)P->out + ch * nout, nout);
            o_decim_free(&d);
        }
    }
    return NULL;
}
static void o_pool_run(o_pool *P, size_t nthreads) {
    if (nthreads < 1) nthreads = 1;
    if (nthreads > P->nch) nthreads = P->nch;
    P->next = 0;
    pthread_mutex_init(&P->mu, NULL);
    pthread_t *th = (pthread_t *)malloc(nthreads * sizeof(pthread_t));
    for (size_t t = 0; t < nthreads; t++) pthread_create(&th[t], NULL, o_pool_worker, P);
    for (size_t t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    pthread_mutex_destroy(&P->mu);
}
size_t o_run_wbfm_channels(const o_wbfm_params *p, const float *f_off, size_t nch, const oc32 *in,
                           size_t n, float *out, size_t nthreads) {
    o_pool P; memset(&P, 0, sizeof(P));
    P.kind = 0; P.p = p; P.f_off = f_off; P.nch = nch; P.n = n; P.in = in; P.out = out;
    o_pool_run(&P, nthreads);
    return nch * ((n + p->m - 1) / p->m);
}
size_t o_run_ssb_demod_channels(float fs, float bfo_hz, float audio_bw_hz, size_t nch, const oc32 *in,
                                size_t n, float *out, size_t nthreads) {
    o_pool P; memset(&P, 0, sizeof(P));
    P.kind = 1; P.fs = fs; P.bfo = bfo_hz; P.bw = audio_bw_hz; P.nch = nch; P.n = n; P.in = in; P.out = out;
    o_pool_run(&P, nthreads);
    return nch * n;
}
size_t o_run_decim_channels(float fs, size_t m, float cutoff_hz, float trans_hz, size_t nch,
                            const oc32 *in, size_t n, oc32 *out, size_t nthreads) {
    o_pool P; memset(&P, 0, sizeof(P));
    P.kind = 2; P.fs = fs; P.m = m; P.cutoff = cutoff_hz; P.trans = trans_hz; P.nch = nch; P.n = n;
    P.in = in; P.out = out;
    o_pool_run(&P, nthreads);
    return nch * ((n + m - 1) / m);
}

/* ------------------------------------------------------------------ */
/* dsp/agc.rs:20-31 AgcRms::new / :93-106 AgcRmsIq::new; update_env    */
/* :32-41 / :108-116; process :48-75 / :124-150. iq != 0: cf32 input.  */
/* Rust's f32 ops: no FMA contraction (-ffp-contract=off), expf/sqrtf. */
typedef struct { float attack_a, release_a, target_rms, min_gain, max_gain, env; } o_agc;
static void o_agc_init(o_agc *a, float fs, float attack_ms, float release_ms, float target_rms) {
    a->attack_a = expf(-1.0f / (fs * (o_maxf(attack_ms, 1e-3f) / 1000.0f)));
    a->release_a = expf(-1.0f / (fs * (o_maxf(release_ms, 1e-3f) / 1000.0f)));
    a->target_rms = o_maxf(target_rms, 1e-6f);
    a->min_gain = 0.05f;
    a->max_gain = 20.0f;
    a->env = 0.0f;
}
static void o_agc_process(o_agc *a, int iq, const float *in, float *out, size_t n) {
    if (n == 0) return;
    if (a->env == 0.0f) {  /* agc.rs:57-60 / :133-136 seed */
        float x2 = iq ? in[0] * in[0] + in[1] * in[1] : in[0] * in[0];
        a->env = o_maxf(x2, 1e-12f);
    }
    float env = a->env;
    for (size_t i = 0; i < n; i++) {
        float re = iq ? in[2 * i] : in[i], im = iq ? in[2 * i + 1] : 0.0f;
        float x2 = iq ? re * re + im * im : re * re;
        float k = x2 > env ? a->attack_a : a->release_a;
        env = k * env + (1.0f - k) * x2;
        float rms = o_maxf(sqrtf(env), 1e-6f);
        float g = a->target_rms / rms;
        g = g < a->min_gain ? a->min_gain : (g > a->max_gain ? a->max_gain : g);
        if (iq) { out[2 * i] = g * re; out[2 * i + 1] = g * im; } else out[i] = g * re;
    }
    a->env = env;
}
/* Streams n samples through one AGC in calls of `chunk` (0 = one call); returns the end env. */
float o_run_agc(int iq, float fs, float attack_ms, float release_ms, float target_rms,
                const float *in, float *out, size_t n, size_t chunk) {
    o_agc a; o_agc_init(&a, fs, attack_ms, release_ms, target_rms);
    const size_t w = iq ? 2 : 1;
    for (size_t i = 0; i < n;) { size_t c = o_step(chunk, n - i); o_agc_process(&a, iq, in + w * i, out + w * i, c); i += c; }
    return a.env;
}
