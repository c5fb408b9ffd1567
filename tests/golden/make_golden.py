"""Generate tests/golden/golden.npz — small input/output vectors for the hot path.

No reference binary can run here (no cargo/rustc; the PyO3 module is not
built), and the reference ships no golden vectors. The expected outputs below
are produced by the scalar C oracle (oracle/orion_oracle.c) and — for every
block it covers — independently by tests/np_ref.py; this script refuses to
write the fixture unless the two agree bit for bit (max |diff| == 0), so a
fixture only records a value two separate restatements of the reference
source agree on. Since round 3 every recorded output is agreed this way (every
§8(a) row, the modulators, the WBFM composition); the inputs are seeded noise,
tones, or the oracle's own modulator outputs (themselves agreed).

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import np_ref as R  # noqa: E402
import oracle as O  # noqa: E402

SEED = 0x1234_5678_ABCD_EF00


def same(name, a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    d = np.max(np.abs(a.astype(np.complex128) - b.astype(np.complex128))) if a.size else 0.0
    assert d == 0.0, f"{name}: oracle and np_ref disagree (max |diff| {d})"
    print(f"  {name}: oracle == np_ref ({a.size} values)")


def main():
    g = {}
    rng = np.random.default_rng(7)
    # ---- designs -----------------------------------------------------------
    for key, args in {"taps_c2_dec": (10e6, 200e3, 79e3), "taps_c2_audio": (1.25e6, 15e3, 10e3),
                      "taps_c3_dec": (10e6, 190e3, 39370.0), "taps_small": (48e3, 3000.0, 800.0)}.items():
        t = O.fir_lowpass_taps(*args)
        same(key, t, R.fir_lowpass_taps(*args))
        g[key] = t
    for nt in (3, 31, 81, 127):
        g[f"kaiser_{nt}"] = O.kaiser_lowpass_taps(nt, 0.2, 60.0)
        same(f"kaiser_{nt}", g[f"kaiser_{nt}"], R.kaiser_lowpass_taps(nt, 0.2, 60.0))
    g["lp_coeffs_c2"] = O.lp_cascade_coeffs(1.25e6, 13.5e3)
    same("lp_coeffs_c2", g["lp_coeffs_c2"], np.array(R.lp_cascade_coeffs(1.25e6, 13.5e3), np.float32))
    g["lpdc_coeffs_ssb"] = O.lpdc_coeffs(48e3, 2520.0, 2.0)
    same("lpdc_coeffs_ssb", g["lpdc_coeffs_ssb"], np.array(R.lpdc_coeffs(48e3, 2520.0, 2.0), np.float32))
    # ---- atan2_approx incl. signed zeros / axes / octant boundaries ----------
    ys = np.array([0.0, -0.0, 1.0, -1.0, 1.0, -1.0, 0.5, -0.5, 1e-30, 3.0, -2.0, 0.0], np.float32)
    xs = np.array([0.0, 1.0, 1.0, 1.0, -1.0, -1.0, -0.0, -2.0, -1.0, 3.0, 2.0, -1.0], np.float32)
    ys = np.concatenate([ys, rng.standard_normal(500).astype(np.float32)])
    xs = np.concatenate([xs, rng.standard_normal(500).astype(np.float32)])
    at = np.array([O.atan2_approx(float(y), float(x)) for y, x in zip(ys, xs)], np.float32)
    same("atan2_approx", at, R.atan2_approx(ys, xs))
    g["atan2_y"], g["atan2_x"], g["atan2_out"] = ys, xs, at
    # ---- AWGN (tests/common/mod.rs:27-48) ------------------------------------
    z = np.zeros(300, np.complex64)
    aw = O.add_awgn(z, 0.01, SEED)
    same("add_awgn", aw, R.add_awgn(z, 0.01, SEED))
    g["awgn_p001"] = aw
    # ---- Rotator (crosses two renormalisations) -----------------------------
    x = (rng.standard_normal(2600) + 1j * rng.standard_normal(2600)).astype(np.complex64)
    g["x_c"] = x
    ro = O.rotator(x, -1.5e6, 10e6)
    same("rotator", ro, R.rotator(x, -1.5e6, 10e6))
    g["rotator_out"] = ro
    # ---- FirLowpass (real) ----------------------------------------------------
    xr = rng.standard_normal(1500).astype(np.float32)
    g["x_r"] = xr
    fo = O.fir_lowpass(xr, 1.25e6, 15e3, 10e3)
    same("fir_lowpass", fo, R.fir_lowpass(xr, R.fir_lowpass_taps(1.25e6, 15e3, 10e3)))
    g["fir_lowpass_out"] = fo
    # ---- FirDecimator ---------------------------------------------------------
    do = O.fir_decimator(x, 10e6, 8, 200e3, 79e3)
    same("fir_decimator", do, R.fir_decimator(x, 10e6, 8, 200e3, 79e3))
    g["decim_out"] = do
    # ---- LpCascade ------------------------------------------------------------
    lo = O.lp_cascade(xr, 1.25e6, 13.5e3)
    same("lp_cascade", lo, R.lp_cascade(xr, 1.25e6, 13.5e3))
    g["lp_cascade_out"] = lo
    # ---- FmQuadratureDemod ------------------------------------------------------
    t = np.arange(3000, dtype=np.float32) / 48e3
    aud = (0.5 * np.sin(2 * np.pi * 1000 * t)).astype(np.float32)
    fm_iq = O.fm_mod(aud, 48e3, 2500.0)
    g["fm_iq"] = fm_iq
    fmo = O.fm_demod(fm_iq, 48e3, 2500.0, 5000.0)
    same("fm_demod", fmo, R.fm_demod(fm_iq, 48e3, 2500.0, 5000.0))
    g["fm_demod_out"] = fmo
    # ---- demodulators, DC blocker, complex FIR -----------------------------------
    pm = O.pm_demod(fm_iq, 48e3, 0.9, 5000.0)
    same("pm_demod", pm, R.pm_demod(fm_iq, 48e3, 0.9, 5000.0))
    g["pm_demod_out"] = pm
    a4 = (0.4 * np.sin(2 * np.pi * 1200 * t)).astype(np.float32)
    ssb_iq = O.ssb_mod(a4, 48e3, 2800.0, 1500.0)
    same("ssb_mod", ssb_iq, R.ssb_mod(a4, 48e3, 2800.0, 1500.0))
    g["ssb_iq"] = ssb_iq
    g["ssb_demod_out"] = O.ssb_demod(ssb_iq, 48e3, 1500.0, 2800.0)
    same("ssb_demod", g["ssb_demod_out"], R.ssb_demod(ssb_iq, 48e3, 1500.0, 2800.0))
    am_iq = O.am_mod(aud, 48e3, 0.0, 0.8, 0.5)
    same("am_mod", am_iq, R.am_mod(aud, 48e3, 0.0, 0.8, 0.5))
    g["am_iq"] = am_iq
    g["am_demod_out"] = O.am_demod(am_iq, 48e3, 5000.0)
    same("am_demod", g["am_demod_out"], R.am_demod(am_iq, 48e3, 5000.0))
    g["am_abs_demod_out"] = O.am_demod(am_iq, 48e3, 5000.0, abs_approx=(0.9482, 0.3920))
    same("am_abs_demod", g["am_abs_demod_out"], R.am_demod(am_iq, 48e3, 5000.0, (0.9482, 0.3920)))
    g["cw_demod_out"] = O.cw_demod(am_iq, 48e3, 700.0, 300.0)
    same("cw_demod", g["cw_demod_out"], R.cw_demod(am_iq, 48e3, 700.0, 300.0))
    g["dc_out"] = O.dc_blocker(xr, 48e3, 2.0)
    same("dc_blocker", g["dc_out"], R.dc_blocker(xr, 48e3, 2.0))
    g["firiq_out"] = O.fir_lowpass_iq(x, g["kaiser_31"])
    same("fir_lowpass_iq", g["firiq_out"], R.fir_lowpass_iq(x, g["kaiser_31"]))
    g["firiq_aligned_out"] = O.fir_lowpass_iq_aligned(x, g["kaiser_31"])
    same("fir_lowpass_iq_aligned", g["firiq_aligned_out"], R.fir_lowpass_iq_aligned(x, g["kaiser_31"]))
    # ---- Rotator mix_usb / Nco / Biquad / LpDcCascade (round 3 API rows) ---------
    g["mix_usb_out"] = O.rotator_retune(x, 1500.0, 48e3, len(x), 0.0, usb=True)
    same("rotator_mix_usb", g["mix_usb_out"], R.rotator_mix_usb(x, 1500.0, 48e3))
    g["nco_mix_out"] = O.nco(x, 12e3, 48e3)
    same("nco_mix", g["nco_mix_out"], R.nco_mix(x, 12e3, 48e3))
    bq = (np.float32(0.01), np.float32(0.02), np.float32(0.01), np.float32(-1.9), np.float32(0.92))
    g["biquad_coeffs"] = np.array(bq, np.float32)
    g["biquad_out"] = O.biquad(xr, *bq)
    same("biquad", g["biquad_out"], R.biquad(xr, *bq))
    g["lpdc_out"] = O.lp_dc_cascade(xr, 48e3, 2520.0, 2.0)
    same("lp_dc_cascade", g["lpdc_out"], R.lp_dc_cascade(xr, 48e3, 2520.0, 2.0))
    pw = (np.abs(x) ** 2).astype(np.float32)
    g["lpdc_sqrt_in"] = pw
    g["lpdc_sqrt_out"] = O.lp_dc_cascade(pw, 48e3, 2520.0, 2.0, True)
    same("lp_dc_cascade sqrt", g["lpdc_sqrt_out"], R.lp_dc_cascade(pw, 48e3, 2520.0, 2.0, True))
    # ---- modulators -----------------------------------------------------------------
    same("fm_mod", fm_iq, R.fm_mod(aud, 48e3, 2500.0))
    g["pm_mod_out"] = O.pm_mod(aud, 48e3, 0.9, 12e3)
    same("pm_mod", g["pm_mod_out"], R.pm_mod(aud, 48e3, 0.9, 12e3))
    key = np.repeat(np.array([1.0, 0.0, 0.6, 1.4, -0.2, 1.0, 0.0], np.float32), 430)[:3000]
    g["cw_key"] = key
    g["cw_mod_out"] = O.cw_mod(key, 48e3, 700.0, 2.0, 8.0)
    same("cw_mod", g["cw_mod_out"], R.cw_mod(key, 48e3, 700.0, 2.0, 8.0))
    # ---- WBFM chain (C2 parameters, 2^14 samples) -------------------------------
    fs = 10e6
    tt = np.arange(1 << 14) / fs
    a2 = (0.5 * np.sin(2 * np.pi * 1e3 * tt) + 0.3 * np.sin(2 * np.pi * 7e3 * tt)).astype(np.float32)
    fm_rf = O.fm_mod(a2, fs, 75e3, 1.5e6)
    same("fm_mod rf", fm_rf, R.fm_mod(a2, fs, 75e3, 1.5e6))
    wiq = O.add_awgn(fm_rf, 0.0025, SEED)
    same("add_awgn wbfm", wiq, R.add_awgn(fm_rf, 0.0025, SEED))
    g["wbfm_iq"] = wiq
    g["wbfm_out"] = O.wbfm(wiq)
    same("wbfm chain", g["wbfm_out"], R.wbfm(wiq))
    out = os.path.join(HERE, "golden.npz")
    np.savez_compressed(out, **g)
    print(f"wrote {out} ({os.path.getsize(out)} bytes, {len(g)} arrays)")


if __name__ == "__main__":
    main()
