"""TEST INFRASTRUCTURE ONLY — ctypes view of the scalar C oracle (orion_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline; the MI355X product path in
orion-sdr_amd/ never touches it. See orion_oracle.h for what it restates
(skynavga/orion-sdr v0.0.63, file:line per routine) and its pinning status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liborion_oracle.so")

_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
_c64p = np.ctypeslib.ndpointer(np.complex64, flags="C_CONTIGUOUS")
_sz = C.c_size_t
_f = C.c_float


class WbfmParams(C.Structure):
    _fields_ = [
        ("fs", _f), ("f_off", _f), ("dec_cutoff", _f), ("dec_trans", _f), ("dev_hz", _f),
        ("audio_bw", _f), ("audio_pass", _f), ("audio_trans", _f), ("m", _sz),
    ]


def build() -> str:
    """Compile the oracle with its Makefile (gcc, -ffp-contract=off)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = C.CDLL(_LIB_PATH)
    sig = {
        "o_atan2_approx": (_f, [_f, _f]),
        "o_fir_design_taps": (_sz, [_f, _f, _f, _f32p, _sz]),
        "o_kaiser_lowpass_taps": (_sz, [_sz, _f, _f, _f32p, _sz]),
        "o_kaiser_transition_norm": (_f, [_sz, _f]),
        "o_kaiser_num_taps": (_sz, [_f, _f]),
        "o_kaiser_beta": (_f, [_f]),
        "o_bessel_i0": (_f, [_f]),
        "o_run_rotator": (_sz, [_f, _f, _c64p, _c64p, _sz, _sz]),
        "o_run_rotator_retune": (_sz, [_f, _f, C.c_int, _c64p, C.c_void_p, _sz, _sz, _f, _f, C.c_int]),
        "o_run_nco": (_sz, [_f, _f, C.c_int, _c64p, _c64p, _sz, _sz, _f]),
        "o_run_biquad": (_sz, [_f, _f, _f, _f, _f, _f32p, _f32p, _sz]),
        "o_run_lpdc": (_sz, [_f, _f, _f, C.c_int, _f32p, _f32p, _sz]),
        "o_run_fir": (_sz, [_f, _f, _f, _f32p, _f32p, _sz, _sz]),
        "o_run_firiq": (_sz, [_f32p, _sz, _c64p, _c64p, _sz, _sz]),
        "o_run_firiq_aligned": (None, [_f32p, _sz, _c64p, _sz]),
        "o_run_decim": (_sz, [_f, _sz, _f, _f, _c64p, _sz, _c64p, _sz, _sz]),
        "o_run_lp_cascade": (_sz, [_f, _f, _f32p, _f32p, _sz]),
        "o_run_dc": (_sz, [_f, _f, _f32p, _f32p, _sz, _sz]),
        "o_run_fm_demod": (_sz, [_f, _f, _f, _f, C.c_int, _c64p, _f32p, _sz, _sz]),
        "o_run_pm_demod": (_sz, [_f, _f, _f, _c64p, _f32p, _sz, _sz]),
        "o_run_ssb_demod": (_sz, [_f, _f, _f, _c64p, _f32p, _sz, _sz]),
        "o_run_am_demod": (_sz, [_f, _f, C.c_int, _f, _f, _c64p, _f32p, _sz, _sz]),
        "o_run_cw_demod": (_sz, [_f, _f, _f, _f, _c64p, _f32p, _sz, _sz]),
        "o_run_fm_mod": (_sz, [_f, _f, _f, _f32p, _c64p, _sz, _sz]),
        "o_run_pm_mod": (_sz, [_f, _f, _f, _f32p, _c64p, _sz]),
        "o_run_ssb_mod": (_sz, [_f, _f, _f, _f, C.c_int, _f32p, _c64p, _sz]),
        "o_run_am_mod": (_sz, [_f, _f, _f, _f, _f, C.c_int, _f32p, _c64p, _sz]),
        "o_run_cw_mod": (_sz, [_f, _f, _f, _f, _f32p, _c64p, _sz]),
        "o_lp_cascade_coeffs": (None, [_f, _f, _f32p]),
        "o_lpdc_coeffs": (None, [_f, _f, _f, _f32p]),
        "o_run_wbfm": (_sz, [C.POINTER(WbfmParams), _c64p, _sz, _f32p, _sz, _sz]),
        "o_run_wbfm_channels": (_sz, [C.POINTER(WbfmParams), _f32p, _sz, _c64p, _sz, _f32p, _sz]),
        "o_run_ssb_demod_channels": (_sz, [_f, _f, _f, _sz, _c64p, _sz, _f32p, _sz]),
        "o_run_decim_channels": (_sz, [_f, _sz, _f, _f, _sz, _c64p, _sz, _c64p, _sz]),
        "o_add_awgn": (None, [_c64p, _sz, _f, C.c_uint64]),
        "o_run_agc": (_f, [C.c_int, _f, _f, _f, _f, C.c_void_p, C.c_void_p, _sz, _sz]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _c64(x):
    return np.ascontiguousarray(x, dtype=np.complex64)


def _f32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


# ---- designs -------------------------------------------------------------
def atan2_approx(y: float, x: float) -> float:
    return lib().o_atan2_approx(y, x)


def fir_lowpass_taps(fs, pass_hz, trans_hz) -> np.ndarray:
    n = lib().o_fir_design_taps(fs, pass_hz, trans_hz, np.zeros(1, np.float32), 0)
    t = np.zeros(n, np.float32)
    lib().o_fir_design_taps(fs, pass_hz, trans_hz, t, n)
    return t


def kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db) -> np.ndarray:
    n = lib().o_kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db, np.zeros(1, np.float32), 0)
    t = np.zeros(n, np.float32)
    lib().o_kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db, t, n)
    return t


def kaiser_transition_norm(num_taps, stopband_db) -> float:
    return lib().o_kaiser_transition_norm(num_taps, stopband_db)


def kaiser_num_taps(transition_norm, stopband_db) -> int:
    return lib().o_kaiser_num_taps(transition_norm, stopband_db)


def lp_cascade_coeffs(fs, fc) -> np.ndarray:
    o = np.zeros(5, np.float32)
    lib().o_lp_cascade_coeffs(fs, fc, o)
    return o


def lpdc_coeffs(fs, lp_fc, dc_cut) -> np.ndarray:
    o = np.zeros(6, np.float32)
    lib().o_lpdc_coeffs(fs, lp_fc, dc_cut, o)
    return o


# ---- blocks (streamed in `chunk`-sample calls; 0 = one call) ---------------
def rotator(x, freq_hz, fs, chunk=0):
    x = _c64(x)
    y = np.empty_like(x)
    lib().o_run_rotator(freq_hz, fs, x, y, len(x), chunk)
    return y


def rotator_retune(x, f1, fs, n_switch, f2, fs2=None, usb=False, reset=False):
    """Rotator(f1, fs): rotate_block (usb: mix_usb_block, f32 out) over x with
    set_freq(f2, fs2) (reset: reset_phase) after the first n_switch samples."""
    x = _c64(x)
    out = np.zeros(len(x), np.float32 if usb else np.complex64)
    lib().o_run_rotator_retune(f1, fs, 1 if usb else 0, x, out.ctypes.data, len(x), n_switch, f2,
                               fs if fs2 is None else fs2, 1 if reset else 0)
    return out


def nco(x, f1, fs, n_switch=None, f2=0.0, gen=False):
    """Nco(f1, fs): mix_with_nco per sample (gen: next_cs pairs; x gives the length),
    set_freq(f2) after n_switch samples."""
    x = _c64(x)
    out = np.zeros(len(x), np.complex64)
    lib().o_run_nco(f1, fs, 1 if gen else 0, x, out, len(x), len(x) if n_switch is None else n_switch, f2)
    return out


def biquad(x, b0, b1, b2, a1, a2):
    x = _f32(x)
    out = np.zeros_like(x)
    lib().o_run_biquad(b0, b1, b2, a1, a2, x, out, len(x))
    return out


_LPDC_MAPS = {None: -1, "identity": 0, "sqrt": 1, "abs": 2}


def lp_dc_cascade(x, fs, lp_fc, dc_cut, sqrt_map=False, map=None):
    """iir.rs:151-165 process, or :170-186 process_mapped(x, f) with map "identity" /
    "sqrt" / "abs" (sqrt_map=True: "sqrt")."""
    x = _f32(x)
    out = np.zeros_like(x)
    lib().o_run_lpdc(fs, lp_fc, dc_cut, _LPDC_MAPS["sqrt" if sqrt_map else map], x, out, len(x))
    return out


def fir_lowpass(x, fs, pass_hz, trans_hz, chunk=0):
    x = _f32(x)
    y = np.empty_like(x)
    lib().o_run_fir(fs, pass_hz, trans_hz, x, y, len(x), chunk)
    return y


def fir_lowpass_iq(x, taps, chunk=0):
    x = _c64(x)
    t = _f32(taps) if len(taps) else np.zeros(1, np.float32)
    y = np.empty_like(x)
    lib().o_run_firiq(t, len(taps), x, y, len(x), chunk)
    return y


def fir_lowpass_iq_aligned(x, taps):
    y = _c64(x).copy()
    t = _f32(taps) if len(taps) else np.zeros(1, np.float32)
    lib().o_run_firiq_aligned(t, len(taps), y, len(y))
    return y


def fir_decimator(x, fs, m, cutoff_hz, trans_hz, chunk=0):
    x = _c64(x)
    cap = len(x) + 8 * max(1, (len(x) // max(chunk, 1)) if chunk else 1)
    y = np.empty(cap, np.complex64)
    w = lib().o_run_decim(fs, m, cutoff_hz, trans_hz, x, len(x), y, cap, chunk)
    return y[:w].copy()


def lp_cascade(x, fs, fc):
    x = _f32(x)
    y = np.empty_like(x)
    lib().o_run_lp_cascade(fs, fc, x, y, len(x))
    return y


def dc_blocker(x, fs, cut_hz, chunk=0):
    x = _f32(x)
    y = np.empty_like(x)
    lib().o_run_dc(fs, cut_hz, x, y, len(x), chunk)
    return y


def agc(x, fs, attack_ms, release_ms, target_rms, chunk=0):
    """dsp/agc.rs AgcRms (real input) / AgcRmsIq (complex input). Returns (out, end env)."""
    iq = np.iscomplexobj(x)
    x = _c64(x) if iq else _f32(x)
    y = np.empty_like(x)
    env = lib().o_run_agc(int(iq), fs, attack_ms, release_ms, target_rms,
                          x.ctypes.data, y.ctypes.data, len(x), chunk)
    return y, env


def fm_demod(x, fs, dev_hz, audio_bw_hz, translate_hz=None, chunk=0):
    x = _c64(x)
    y = np.empty(len(x), np.float32)
    lib().o_run_fm_demod(fs, dev_hz, audio_bw_hz, translate_hz or 0.0, translate_hz is not None, x, y,
                         len(x), chunk)
    return y


def pm_demod(x, fs, k, audio_bw_hz, chunk=0):
    x = _c64(x)
    y = np.empty(len(x), np.float32)
    lib().o_run_pm_demod(fs, k, audio_bw_hz, x, y, len(x), chunk)
    return y


def ssb_demod(x, fs, bfo_hz, audio_bw_hz, chunk=0):
    x = _c64(x)
    y = np.empty(len(x), np.float32)
    lib().o_run_ssb_demod(fs, bfo_hz, audio_bw_hz, x, y, len(x), chunk)
    return y


def am_demod(x, fs, audio_bw_hz, abs_approx=None, chunk=0):
    x = _c64(x)
    y = np.empty(len(x), np.float32)
    k1, k2 = abs_approx if abs_approx else (0.0, 0.0)
    lib().o_run_am_demod(fs, audio_bw_hz, 1 if abs_approx else 0, k1, k2, x, y, len(x), chunk)
    return y


def cw_demod(x, fs, tone_hz, env_bw_hz, gain=1.0, chunk=0):
    x = _c64(x)
    y = np.empty(len(x), np.float32)
    lib().o_run_cw_demod(fs, tone_hz, env_bw_hz, gain, x, y, len(x), chunk)
    return y


def fm_mod(a, fs, dev_hz, rf_hz=0.0, chunk=0):
    a = _f32(a)
    y = np.empty(len(a), np.complex64)
    lib().o_run_fm_mod(fs, dev_hz, rf_hz, a, y, len(a), chunk)
    return y


def pm_mod(a, fs, kp, rf_hz=0.0):
    a = _f32(a)
    y = np.empty(len(a), np.complex64)
    lib().o_run_pm_mod(fs, kp, rf_hz, a, y, len(a))
    return y


def ssb_mod(a, fs, bw, if_hz, rf_hz=0.0, usb=True):
    a = _f32(a)
    y = np.empty(len(a), np.complex64)
    lib().o_run_ssb_mod(fs, bw, if_hz, rf_hz, 1 if usb else 0, a, y, len(a))
    return y


def am_mod(a, fs, rf_hz, carrier_level, mod_index, gain=1.0, clamp=False):
    a = _f32(a)
    y = np.empty(len(a), np.complex64)
    lib().o_run_am_mod(fs, rf_hz, carrier_level, mod_index, gain, 1 if clamp else 0, a, y, len(a))
    return y


def cw_mod(a, fs, tone_hz, rise_ms, fall_ms):
    a = _f32(a)
    y = np.empty(len(a), np.complex64)
    lib().o_run_cw_mod(fs, tone_hz, rise_ms, fall_ms, a, y, len(a))
    return y


def add_awgn(iq, noise_power, seed):
    """In place on a copy; tests/common/mod.rs:27-48."""
    y = _c64(iq).copy()
    lib().o_add_awgn(y, len(y), noise_power, seed & 0xFFFFFFFFFFFFFFFF)
    return y


# ---- WBFM chain (docs/demodulate.md:128-133) --------------------------------
WBFM_C2 = dict(fs=10e6, f_off=1.5e6, dec_cutoff=200e3, dec_trans=79e3, dev_hz=75e3, audio_bw=15e3,
               audio_pass=15e3, audio_trans=10e3, m=8)


def wbfm_params(**kw) -> WbfmParams:
    d = dict(WBFM_C2)
    d.update(kw)
    return WbfmParams(**d)


def wbfm(x, chunk=0, **kw):
    p = wbfm_params(**kw)
    x = _c64(x)
    cap = len(x) // p.m + 64 + (len(x) // chunk if chunk else 0)
    y = np.empty(cap, np.float32)
    w = lib().o_run_wbfm(C.byref(p), x, len(x), y, cap, chunk)
    return y[:w].copy()


def wbfm_channels(x2d, f_offs, nthreads, **kw):
    p = wbfm_params(**kw)
    x2d = _c64(x2d)
    nch, n = x2d.shape
    nout = (n + p.m - 1) // p.m
    y = np.empty((nch, nout), np.float32)
    lib().o_run_wbfm_channels(C.byref(p), _f32(f_offs), nch, x2d, n, y, nthreads)
    return y


def ssb_demod_channels(x2d, fs, bfo_hz, audio_bw_hz, nthreads):
    x2d = _c64(x2d)
    nch, n = x2d.shape
    y = np.empty((nch, n), np.float32)
    lib().o_run_ssb_demod_channels(fs, bfo_hz, audio_bw_hz, nch, x2d, n, y, nthreads)
    return y


def decim_channels(x2d, fs, m, cutoff, trans, nthreads):
    x2d = _c64(x2d)
    nch, n = x2d.shape
    nout = (n + m - 1) // m
    y = np.empty((nch, nout), np.complex64)
    lib().o_run_decim_channels(fs, m, cutoff, trans, nch, x2d, n, y, nthreads)
    return y
