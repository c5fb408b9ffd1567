"""CPU: the oracle against the committed golden vectors and against every
property / threshold test the reference holds for this path.

These pin the oracle before any GPU result is compared with it.
"""
import math
import os

import numpy as np
import pytest

from conftest import FS, complex_tone, real_tone, snr_db, tail

GOLD = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden.npz"))
SEED = 0x1234_5678_ABCD_EF00


def _eq(a, b):
    assert a.shape == b.shape
    assert np.array_equal(a.view(np.uint32) if a.dtype == np.float32 else a.view(np.uint64),
                          b.view(np.uint32) if b.dtype == np.float32 else b.view(np.uint64))


# ---- golden vectors: the oracle reproduces them bit for bit -------------------------
@pytest.mark.parametrize("key,args", [("taps_c2_dec", (10e6, 200e3, 79e3)), ("taps_c2_audio", (1.25e6, 15e3, 10e3)),
                                      ("taps_c3_dec", (10e6, 190e3, 39370.0)), ("taps_small", (48e3, 3000.0, 800.0))])
def test_golden_fir_taps(oracle, key, args):
    _eq(oracle.fir_lowpass_taps(*args), GOLD[key])


def test_golden_blocks(oracle):
    x, xr = GOLD["x_c"], GOLD["x_r"]
    _eq(oracle.rotator(x, -1.5e6, 10e6), GOLD["rotator_out"])
    _eq(oracle.fir_lowpass(xr, 1.25e6, 15e3, 10e3), GOLD["fir_lowpass_out"])
    _eq(oracle.fir_decimator(x, 10e6, 8, 200e3, 79e3), GOLD["decim_out"])
    _eq(oracle.lp_cascade(xr, 1.25e6, 13.5e3), GOLD["lp_cascade_out"])
    _eq(oracle.fm_demod(GOLD["fm_iq"], 48e3, 2500.0, 5000.0), GOLD["fm_demod_out"])
    _eq(oracle.pm_demod(GOLD["fm_iq"], 48e3, 0.9, 5000.0), GOLD["pm_demod_out"])
    _eq(oracle.ssb_demod(GOLD["ssb_iq"], 48e3, 1500.0, 2800.0), GOLD["ssb_demod_out"])
    _eq(oracle.am_demod(GOLD["am_iq"], 48e3, 5000.0), GOLD["am_demod_out"])
    _eq(oracle.am_demod(GOLD["am_iq"], 48e3, 5000.0, abs_approx=(0.9482, 0.3920)), GOLD["am_abs_demod_out"])
    _eq(oracle.cw_demod(GOLD["am_iq"], 48e3, 700.0, 300.0), GOLD["cw_demod_out"])
    _eq(oracle.dc_blocker(xr, 48e3, 2.0), GOLD["dc_out"])
    _eq(oracle.fir_lowpass_iq(x, GOLD["kaiser_31"]), GOLD["firiq_out"])
    _eq(oracle.fir_lowpass_iq_aligned(x, GOLD["kaiser_31"]), GOLD["firiq_aligned_out"])
    _eq(oracle.add_awgn(np.zeros(300, np.complex64), 0.01, SEED), GOLD["awgn_p001"])
    _eq(oracle.wbfm(GOLD["wbfm_iq"]), GOLD["wbfm_out"])
    _eq(oracle.rotator_retune(x, 1500.0, 48e3, len(x), 0.0, usb=True), GOLD["mix_usb_out"])
    _eq(oracle.nco(x, 12e3, 48e3), GOLD["nco_mix_out"])
    _eq(oracle.biquad(xr, *GOLD["biquad_coeffs"]), GOLD["biquad_out"])
    _eq(oracle.lp_dc_cascade(xr, 48e3, 2520.0, 2.0), GOLD["lpdc_out"])
    _eq(oracle.lp_dc_cascade(GOLD["lpdc_sqrt_in"], 48e3, 2520.0, 2.0, True), GOLD["lpdc_sqrt_out"])
    _eq(oracle.pm_mod(_golden_audio(), 48e3, 0.9, 12e3), GOLD["pm_mod_out"])
    _eq(oracle.cw_mod(GOLD["cw_key"], 48e3, 700.0, 2.0, 8.0), GOLD["cw_mod_out"])


def _golden_audio():
    t = np.arange(3000, dtype=np.float32) / 48e3
    return (0.5 * np.sin(2 * np.pi * 1000 * t)).astype(np.float32)


def test_np_ref_reproduces_every_golden_output():
    """The independent numpy restatement (tests/np_ref.py, correctly rounded FMA
    emulation) recomputes every recorded output from the recorded inputs bit for
    bit: each fixture is agreed by two restatements of the reference source."""
    import np_ref as R

    x, xr, aud = GOLD["x_c"], GOLD["x_r"], _golden_audio()
    checks = {
        "rotator_out": lambda: R.rotator(x, -1.5e6, 10e6),
        "fir_lowpass_out": lambda: R.fir_lowpass(xr, R.fir_lowpass_taps(1.25e6, 15e3, 10e3)),
        "decim_out": lambda: R.fir_decimator(x, 10e6, 8, 200e3, 79e3),
        "lp_cascade_out": lambda: R.lp_cascade(xr, 1.25e6, 13.5e3),
        "fm_iq": lambda: R.fm_mod(aud, 48e3, 2500.0),
        "fm_demod_out": lambda: R.fm_demod(GOLD["fm_iq"], 48e3, 2500.0, 5000.0),
        "pm_demod_out": lambda: R.pm_demod(GOLD["fm_iq"], 48e3, 0.9, 5000.0),
        "ssb_demod_out": lambda: R.ssb_demod(GOLD["ssb_iq"], 48e3, 1500.0, 2800.0),
        "am_iq": lambda: R.am_mod(aud, 48e3, 0.0, 0.8, 0.5),
        "am_demod_out": lambda: R.am_demod(GOLD["am_iq"], 48e3, 5000.0),
        "am_abs_demod_out": lambda: R.am_demod(GOLD["am_iq"], 48e3, 5000.0, (0.9482, 0.3920)),
        "cw_demod_out": lambda: R.cw_demod(GOLD["am_iq"], 48e3, 700.0, 300.0),
        "dc_out": lambda: R.dc_blocker(xr, 48e3, 2.0),
        "firiq_out": lambda: R.fir_lowpass_iq(x, GOLD["kaiser_31"]),
        "firiq_aligned_out": lambda: R.fir_lowpass_iq_aligned(x, GOLD["kaiser_31"]),
        "kaiser_127": lambda: R.kaiser_lowpass_taps(127, 0.2, 60.0),
        "mix_usb_out": lambda: R.rotator_mix_usb(x, 1500.0, 48e3),
        "nco_mix_out": lambda: R.nco_mix(x, 12e3, 48e3),
        "biquad_out": lambda: R.biquad(xr, *GOLD["biquad_coeffs"]),
        "lpdc_out": lambda: R.lp_dc_cascade(xr, 48e3, 2520.0, 2.0),
        "lpdc_sqrt_out": lambda: R.lp_dc_cascade(GOLD["lpdc_sqrt_in"], 48e3, 2520.0, 2.0, True),
        "pm_mod_out": lambda: R.pm_mod(aud, 48e3, 0.9, 12e3),
        "cw_mod_out": lambda: R.cw_mod(GOLD["cw_key"], 48e3, 700.0, 2.0, 8.0),
        "wbfm_out": lambda: R.wbfm(GOLD["wbfm_iq"]),
        "awgn_p001": lambda: R.add_awgn(np.zeros(300, np.complex64), 0.01, SEED),
    }
    for key, fn in checks.items():
        got = np.asarray(fn())
        _eq(got.astype(GOLD[key].dtype), GOLD[key])


def test_np_ref_fma_is_correctly_rounded():
    """np_ref._fma against exact rational arithmetic, including a double-rounding
    tie that a plain f64 a*b + c rounded to f32 gets wrong."""
    from fractions import Fraction

    import np_ref as R

    rng = np.random.default_rng(3)
    for _ in range(3000):
        a, b, c = (np.float32(v) for v in rng.standard_normal(3) * np.exp(rng.uniform(-20, 20, 3)))
        ex = Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))
        r = R._fma(a, b, c)
        for q in (np.nextafter(r, np.float32(np.inf)), np.nextafter(r, np.float32(-np.inf))):
            assert abs(Fraction(float(r)) - ex) <= abs(Fraction(float(q)) - ex)
    a, b, c = np.float32(1 - 2 ** -23), np.float32(64 + 2 ** -17), np.float32(2 ** 30 + 128)
    assert R._fma(a, b, c) == np.float32(2 ** 30 + 128)  # exact: 2^30 + 192 - 2^-40
    assert np.float32(np.float64(a) * np.float64(b) + np.float64(c)) == np.float32(2 ** 30 + 256)


def test_golden_atan2(oracle):
    got = np.array([oracle.atan2_approx(float(y), float(x)) for y, x in zip(GOLD["atan2_y"], GOLD["atan2_x"])],
                   np.float32)
    _eq(got, GOLD["atan2_out"])


def test_np_ref_agrees_on_fresh_vectors(oracle):
    """Independent restatement (tests/np_ref.py) vs oracle on new seeded inputs."""
    import np_ref as R

    rng = np.random.default_rng(11)
    x = (rng.standard_normal(1200) + 1j * rng.standard_normal(1200)).astype(np.complex64)
    _eq(oracle.rotator(x, 1234.5, 48e3), R.rotator(x, 1234.5, 48e3))
    _eq(oracle.fir_decimator(x, 96e3, 4, 10.8e3, 2.4e3), R.fir_decimator(x, 96e3, 4, 10.8e3, 2.4e3))
    _eq(oracle.fm_demod(x, 48e3, 3000.0, 4000.0), R.fm_demod(x, 48e3, 3000.0, 4000.0))


# ---- streaming ("resume") semantics ------------------------------------------------
def test_chunking_invariance_oracle(oracle):
    x = GOLD["x_c"]
    _eq(oracle.rotator(x, -1.5e6, 10e6, chunk=333), GOLD["rotator_out"])
    _eq(oracle.fir_lowpass(GOLD["x_r"], 1.25e6, 15e3, 10e3, chunk=100), GOLD["fir_lowpass_out"])
    _eq(oracle.fm_demod(GOLD["fm_iq"], 48e3, 2500.0, 5000.0, chunk=257), GOLD["fm_demod_out"])
    # FirDecimator restarts its decimation phase per call (decim.rs:66-71): equal
    # only when every chunk is a multiple of m.
    _eq(oracle.fir_decimator(x, 10e6, 8, 200e3, 79e3, chunk=800), GOLD["decim_out"])
    assert not np.array_equal(oracle.fir_decimator(x, 10e6, 8, 200e3, 79e3, chunk=333), GOLD["decim_out"])


# ---- reference unit tests (tests/unit/dsp.rs) ----------------------------------------
def test_decimator_reduces_length(oracle):  # dsp.rs:12-27
    fs, m = 96_000.0, 4
    tone = complex_tone(fs, 2000.0, 4096)
    out = oracle.fir_decimator(tone, fs, m, fs / m * 0.45, fs / m * 0.10)
    assert len(out) == 4096 // m


def _response_db(taps, f):
    n = np.arange(len(taps))
    h = np.sum(taps.astype(np.float64) * np.exp(-2j * np.pi * f * n))
    return 20 * np.log10(max(abs(h), 1e-12))


@pytest.mark.parametrize("req", [3, 16, 31, 64, 101])
def test_kaiser_linear_phase_unit_dc(oracle, req):  # dsp.rs:44-60
    t = oracle.kaiser_lowpass_taps(req, 0.2, 60.0)
    assert len(t) == (max(req, 3) | 1)
    assert np.all(np.abs(t - t[::-1]) < 1e-6)
    assert abs(float(np.sum(t)) - 1.0) < 1e-5


def test_kaiser_stopband(oracle):  # dsp.rs:63-91
    t = oracle.kaiser_lowpass_taps(101, 0.2, 60.0)
    half = 0.5 * oracle.kaiser_transition_norm(101, 60.0)
    for f in (0.0, 0.05, 0.1, 0.2 - half):
        assert abs(_response_db(t, f)) < 0.5
    assert abs(_response_db(t, 0.2) + 6.0) < 1.0
    for f in (0.2 + half, 0.3, 0.4, 0.5):
        assert _response_db(t, f) < -55.0


@pytest.mark.parametrize("tr,a", [(0.02, 60.0), (0.05, 40.0), (0.084, 60.0)])
def test_kaiser_num_taps_inverse(oracle, tr, a):  # dsp.rs:94-112
    m = oracle.kaiser_num_taps(tr, a)
    assert m % 2 == 1
    assert oracle.kaiser_transition_norm(m, a) <= tr * 1.001
    assert oracle.kaiser_transition_norm(max(m - 2, 0), a) > tr * 0.999


def test_fir_iq_in_and_out_of_band(oracle):  # dsp.rs:115-144
    taps = oracle.kaiser_lowpass_taps(81, 0.2, 60.0)
    n = 2048

    def amp(f):
        i = np.arange(n)
        x = np.exp(1j * (2 * np.pi * f * i).astype(np.float32)).astype(np.complex64)
        y = oracle.fir_lowpass_iq(x, taps)
        return float(np.max(np.abs(y[2 * 81 + 1:])))

    ib, ob = amp(0.1), amp(0.35)
    assert abs(ib - 1.0) < 0.02
    assert 20 * np.log10(max(ob, 1e-12) / ib) < -55.0


def test_filter_aligned_equals_streamed_shift(oracle):  # dsp.rs:147-199
    taps = oracle.kaiser_lowpass_taps(31, 0.2, 60.0)
    n = 512
    i = np.arange(n, dtype=np.float32)
    env = np.exp(-((i - 200.0) / 60.0) ** 2)
    x = (env * np.exp(1j * 2 * np.pi * 0.03 * i)).astype(np.complex64)
    d = (len(taps) - 1) // 2
    streamed = oracle.fir_lowpass_iq(np.concatenate([x, np.zeros(d, np.complex64)]), taps)
    aligned = oracle.fir_lowpass_iq_aligned(x, taps)
    assert len(aligned) == n
    assert np.max(np.abs(aligned - streamed[d:d + n])) < 1e-5
    assert abs(int(np.argmax(np.abs(aligned))) - int(np.argmax(np.abs(x)))) <= 1


# ---- reference demod unit tests ---------------------------------------------------------
def test_fm_demod_recovers_tone(oracle):  # tests/unit/fm.rs:10-28
    n, fmod, dev = 16384, 1000.0, 2500.0
    k = np.arange(n, dtype=np.float32)
    f_inst = (dev * np.sin((2 * np.pi * fmod * (k / np.float32(FS))).astype(np.float32))).astype(np.float32)
    phi = np.cumsum((2 * np.pi * f_inst / FS).astype(np.float32), dtype=np.float32)
    iq = np.exp(1j * phi).astype(np.complex64)
    assert snr_db(oracle.fm_demod(iq, FS, dev, 5000.0), FS, fmod) > 20.0


def test_ssb_demod_strong_tone_low_dc(oracle):  # tests/unit/ssb.rs:10-36
    iq = complex_tone(FS, 1000.0, 16384)
    y = oracle.ssb_demod(iq, FS, 0.0, 2800.0)
    assert abs(float(np.mean(y))) < 1e-3
    n = len(y)
    k = np.arange(n)

    def p(f):
        return abs(np.dot(y, np.exp(-2j * np.pi * f / FS * k))) ** 2 / n / n

    assert 10 * np.log10(p(1000.0) / (p(700.0) + 1e-20)) > 25.0


def test_pm_demod_recovers_tone(oracle):  # tests/unit/pm.rs:10-26
    n, fmod, beta = 16384, 1000.0, 0.8
    t = np.arange(n, dtype=np.float32) / np.float32(FS)
    phi = (beta * np.sin(2 * np.pi * fmod * t)).astype(np.float32)
    iq = np.exp(1j * phi).astype(np.complex64)
    assert snr_db(oracle.pm_demod(iq, FS, beta, 5000.0), FS, fmod) > 20.0


def test_chain_lengths(oracle):  # tests/unit/chains.rs:10-33
    tone = complex_tone(FS, 1000.0, 4096)
    assert len(oracle.cw_demod(tone, FS, 700.0, 300.0)) == 4096
    assert len(oracle.am_demod(tone, FS, 5000.0)) == 4096
    assert len(oracle.ssb_demod(tone, FS, 0.0, 2800.0)) == 4096


# ---- reference roundtrips (tests/roundtrip/*.rs, python/tests/test_roundtrip.py) --------
def test_roundtrip_fm(oracle):
    a = real_tone(FS, 1000.0, 32768, 0.5)
    y = oracle.fm_demod(oracle.fm_mod(a, FS, 2500.0), FS, 2500.0, 5000.0)
    assert snr_db(tail(y), FS, 1000.0) > 20.0


def test_roundtrip_am(oracle):
    a = real_tone(FS, 1000.0, 32768, 0.5)
    iq = oracle.am_mod(a, FS, 0.0, 0.8, 0.5)
    assert snr_db(tail(oracle.am_demod(iq, FS, 5000.0)), FS, 1000.0) > 24.0
    assert snr_db(tail(oracle.am_demod(iq, FS, 5000.0, abs_approx=(0.9482, 0.3920))), FS, 1000.0) > 20.0


def test_roundtrip_ssb(oracle):
    a = real_tone(FS, 1200.0, 32768, 0.4)
    y = oracle.ssb_demod(oracle.ssb_mod(a, FS, 2800.0, 1500.0), FS, 1500.0, 2800.0)
    assert snr_db(y[int(0.120 * FS):], FS, 1200.0) > 18.0


def test_roundtrip_pm(oracle):
    a = real_tone(FS, 900.0, 32768, 0.5)
    y = oracle.pm_demod(oracle.pm_mod(a, FS, 0.9), FS, 0.9, 5000.0)
    assert snr_db(tail(y), FS, 900.0) > 18.0


def test_roundtrip_cw(oracle):  # tests/roundtrip/cw.rs:11-38
    n = 24000
    key = ((np.arange(n) * 5.0 / FS) % 1.0 < 0.5).astype(np.float32)
    y = oracle.cw_demod(oracle.cw_mod(key, FS, 700.0, 3.0, 3.0), FS, 700.0, 300.0)
    skip = int(0.1 * FS)
    a, k = y[skip:], key[skip:]
    on = np.sqrt(np.mean(a[k > 0.5] ** 2))
    off = np.sqrt(np.mean(a[k < 0.5] ** 2)) + 1e-12
    assert 20 * np.log10(on / off) > 14.0


def test_wbfm_chain_recovers_audio(oracle):
    """C2 configuration at 2^20 samples: the 1 kHz and 7 kHz
    components come through the oracle chain; output RMS ~2e-6 (fm.rs:23 k=1/dev)."""
    from conftest import wbfm_input

    y = oracle.wbfm(wbfm_input(1 << 20))
    assert len(y) == (1 << 20) // 8
    assert snr_db(tail(y), 1.25e6, 1000.0) > 30.0
    assert 5e-7 < float(np.sqrt(np.mean(tail(y) ** 2))) < 5e-6


# ---- AGC (dsp/agc.rs) ---------------------------------------------
def _agc_py(x, fs, attack_ms, release_ms, target):
    """Pure-Python f32 restatement of agc.rs:20-75 / :93-150 (small n only)."""
    f = np.float32
    coef = lambda ms: f(math.exp(float(f(-1.0) / (f(fs) * (f(max(ms, 1e-3)) / f(1000.0))))))  # expf, rounded once
    att, rel, tgt = coef(attack_ms), coef(release_ms), f(max(target, 1e-6))
    iq = np.iscomplexobj(x)
    x2s = [(f(v.real) * f(v.real) + f(v.imag) * f(v.imag)) if iq else f(v) * f(v) for v in x]
    env = max(x2s[0], f(1e-12))
    out = np.empty_like(x)
    for i, (v, x2) in enumerate(zip(x, x2s)):
        a = att if x2 > env else rel
        env = f(f(a * env) + f(f(f(1.0) - a) * x2))
        g = min(max(f(tgt / max(f(np.sqrt(env)), f(1e-6))), f(0.05)), f(20.0))
        out[i] = (f(g * f(v.real)) + 1j * f(g * f(v.imag))) if iq else f(g * v)
    return out


def test_agc_reference_threshold(oracle):
    """tests/unit/agc.rs:9-32: AgcRmsIq(48k, 0.2, 5.0, 0.2), steps 0.02 -> 1.0, tail RMS 0.2 +- 0.03."""
    n = 8000
    x = np.where(np.arange(n) < n // 2, 0.02, 1.0).astype(np.complex64)
    y, _ = oracle.agc(x, 48e3, 0.2, 5.0, 0.2)
    rms = float(np.sqrt(np.mean(np.abs(y[-1000:]) ** 2)))
    assert abs(rms - 0.2) < 0.03, rms


@pytest.mark.parametrize("iq", [False, True])
def test_agc_oracle_vs_python(oracle, iq):
    rng = np.random.default_rng(7)
    n = 3000
    a = np.where(np.arange(n) < 1500, 0.05, 0.8)
    x = (a * rng.standard_normal(n)).astype(np.float32)
    if iq:
        x = (x + 1j * a * rng.standard_normal(n)).astype(np.complex64)
    y, _ = oracle.agc(x, 48e3, 1.0, 20.0, 0.3)
    _eq(y.view(np.float32), _agc_py(x, 48e3, 1.0, 20.0, 0.3).view(np.float32))
    ys, _ = oracle.agc(x, 48e3, 1.0, 20.0, 0.3, chunk=777)
    _eq(ys.view(np.float32), y.view(np.float32))
