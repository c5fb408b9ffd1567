"""TEST INFRASTRUCTURE — a second, independently written restatement of the
reference algorithms in numpy float32 (no shared code with oracle/orion_oracle.c).

It exists to cross-check the C oracle: both must agree bit for bit on the
committed fixtures (tests/golden/). Where the reference uses ``mul_add`` this
file uses a correctly rounded f32 FMA emulation (``_fma``: the f64 product of two
f32 values is exact; the sum is carried as an f64 pair (TwoSum) and rounded to
f32 once, the f64 rounding's direction breaking an exact f32 tie), elsewhere
plain float32 numpy arithmetic (one rounding per op, no contraction).
Sequential recurrences are Python loops: keep inputs small (<= 1e4 samples).
"""
import ctypes
import math

import numpy as np

f32 = np.float32

# Rust's f32::sin/cos lower to the platform libm sinf/cosf (glibc on Linux),
# which is not correctly rounded in every case: call it, don't emulate it.
_libm = ctypes.CDLL("libm.so.6")
for _fn in ("sinf", "cosf"):
    getattr(_libm, _fn).restype = ctypes.c_float
    getattr(_libm, _fn).argtypes = [ctypes.c_float]


for _fn in ("expf", "sqrtf"):
    getattr(_libm, _fn).restype = ctypes.c_float
    getattr(_libm, _fn).argtypes = [ctypes.c_float]
_libm.powf.restype = ctypes.c_float
_libm.powf.argtypes = [ctypes.c_float, ctypes.c_float]


def sinf(x):
    return f32(_libm.sinf(float(x)))


def expf(x):
    return f32(_libm.expf(float(x)))


def cosf(x):
    return f32(_libm.cosf(float(x)))
TAU = f32(2.0 * math.pi)
PI = f32(math.pi)


def _fma(a, b, c):
    """Correctly rounded f32 fma(a, b, c) (scalars or arrays). a*b is exact in f64
    (24 + 24 bits); s = fl64(a*b + c) with its TwoSum error e gives the exact sum
    s + e. Rounding s to f32 is then exact unless s sits exactly on an f32 midpoint
    with e != 0 (|e| is far below half an f32 ulp, and every f32 midpoint is an f64
    number, so s + e cannot cross any other rounding boundary); there the sign of e
    decides the tie. Plain f64 a*b + c rounded to f32 would round twice."""
    scalar = not isinstance(a, np.ndarray) and not isinstance(b, np.ndarray) and not isinstance(c, np.ndarray)
    p = np.float64(a) * np.float64(b)
    cc = np.float64(c)
    s = p + cc
    bb = s - p
    e = (p - (s - bb)) + (cc - bb)
    r = np.asarray(s).astype(np.float32)
    rd = r.astype(np.float64)
    toward = np.nextafter(r, np.where(np.asarray(s) > rd, np.float32(np.inf), np.float32(-np.inf)).astype(np.float32))
    mid = (rd + toward.astype(np.float64)) * 0.5
    tie = (np.asarray(e) != 0.0) & (rd != np.asarray(s)) & (np.asarray(s) == mid)
    if np.any(tie):
        up = (toward.astype(np.float64) - np.asarray(s)) * np.asarray(e) > 0  # e points at `toward`
        r = np.where(tie & up, toward, r).astype(np.float32)
    return f32(r) if scalar else r.astype(np.float32)


def atan2_approx(y, x):
    """util.rs:305-322, vectorised."""
    y = np.asarray(y, f32)
    x = np.asarray(x, f32)
    ax, ay = np.abs(x), np.abs(y)
    sw = ax < ay
    mn = np.where(sw, ax, ay)
    mx = np.where(sw, ay, ax)
    r = (mn / (mx + f32(np.finfo(np.float32).eps))).astype(f32)
    r2 = (r * r).astype(f32)
    inner = (f32(-0.2447) + (r2 * f32(0.0663)).astype(f32)).astype(f32)
    phi = (r * (f32(math.pi / 4) + (r2 * inner).astype(f32)).astype(f32)).astype(f32)
    phi = np.where(sw, (f32(math.pi / 2) - phi).astype(f32), phi)
    sgn = np.where(y < 0, f32(-1.0), f32(1.0))
    return np.where(x < 0, ((PI - phi).astype(f32) * sgn).astype(f32), (phi * sgn).astype(f32)).astype(f32)


def fir_lowpass_taps(fs, pass_hz, trans_hz):
    """dsp/fir.rs:16-44."""
    fs, pass_hz, trans_hz = f32(fs), f32(pass_hz), f32(trans_hz)
    pass_hz = max(pass_hz, f32(10.0))
    trans_hz = max(trans_hz, f32(pass_hz * f32(0.2)))
    ntaps = max(int(math.ceil(float(f32(fs / trans_hz)))), 31) | 1
    fc = f32(pass_hz / fs)
    m0 = ntaps // 2
    taps = np.zeros(ntaps, f32)
    for n in range(ntaps):
        m = n - m0
        if m == 0:
            sinc = f32(f32(2.0) * fc)
        else:
            x = f32(PI * f32(m))
            arg = f32(f32(f32(f32(2.0) * PI) * fc) * f32(m))
            sinc = f32(f32(f32(f32(2.0) * fc) * sinf(arg)) / x)
        warg = f32(f32(f32(f32(2.0) * PI) * f32(n)) / f32(f32(ntaps) - f32(1.0)))
        w = f32(f32(0.5) - f32(f32(0.5) * cosf(warg)))
        taps[n] = f32(sinc * w)
    s = f32(0.0)
    for t in taps:
        s = f32(s + t)
    return (taps / s).astype(f32)


def fir_lowpass(x, taps):
    """dsp/fir.rs:47-66: y[n] = sum_t taps[t]*x[n-1-t] (t < L-1) + taps[L-1]*x[n],
    accumulated sequentially over t in f32 (no FMA)."""
    x = np.asarray(x, f32)
    L = len(taps)
    xp = np.concatenate([np.zeros(L, f32), x])
    n = len(x)
    acc = np.zeros(n, f32)
    for t in range(L):
        k = -1 - t if t < L - 1 else 0  # sample offset relative to n
        seg = xp[L + k: L + k + n]
        acc = (acc + (seg * taps[t]).astype(f32)).astype(f32)
    return acc


def fir_decimator(x, fs, m, cutoff, trans):
    """dsp/decim.rs:44-76 (one call from zero state)."""
    taps = fir_lowpass_taps(fs, cutoff, trans)
    yi = fir_lowpass(np.real(x).astype(f32), taps)
    yq = fir_lowpass(np.imag(x).astype(f32), taps)
    return (yi[::m] + 1j * yq[::m]).astype(np.complex64)


def rotator(x, freq_hz, fs):
    """dsp/rotator.rs:16-26, 44-62, 74-85."""
    phi = f32(f32(TAU * f32(freq_hz)) / f32(fs))
    wr, wi = cosf(phi), sinf(phi)
    zr, zi = f32(1.0), f32(0.0)
    out = np.zeros(len(x), np.complex64)
    ctr = 0
    for i, s in enumerate(np.asarray(x, np.complex64)):
        nzr = _fma(zr, wr, -f32(zi * wi))
        nzi = _fma(zi, wr, f32(zr * wi))
        zr, zi = nzr, nzi
        ctr = (ctr + 1) & 0xFFFFFFFF
        if ctr & 0x3FF == 0:
            inv = f32(f32(1.0) / f32(np.sqrt(f32(f32(zr * zr) + f32(zi * zi)))))
            zr, zi = f32(zr * inv), f32(zi * inv)
        a, b = f32(s.real), f32(s.imag)
        out[i] = complex(_fma(a, zr, -f32(b * zi)), _fma(b, zr, f32(a * zi)))
    return out


def lp_cascade_coeffs(fs, fc):
    """dsp/iir.rs:49-71."""
    w0 = f32(f32(TAU * f32(fc)) / f32(fs))
    sn, cs = sinf(w0), cosf(w0)
    alpha = f32(sn / f32(f32(2.0) * f32(np.sqrt(f32(0.5)))))
    b0 = f32(f32(f32(1.0) - cs) * f32(0.5))
    b1 = f32(f32(1.0) - cs)
    b2 = f32(f32(f32(1.0) - cs) * f32(0.5))
    a0 = f32(f32(1.0) + alpha)
    a1 = f32(f32(-2.0) * cs)
    a2 = f32(f32(1.0) - alpha)
    norm = f32(f32(1.0) / a0)
    return [f32(b0 * norm), f32(b1 * norm), f32(b2 * norm), f32(a1 * norm), f32(a2 * norm)]


def lp_cascade(x, fs, fc):
    b0, b1, b2, a1, a2 = lp_cascade_coeffs(fs, fc)
    z = [f32(0.0)] * 4
    out = np.zeros(len(x), f32)
    for i, v in enumerate(np.asarray(x, f32)):
        for s in (0, 2):
            y = _fma(v, b0, z[s])
            z[s] = f32(_fma(v, b1, z[s + 1]) - f32(a1 * y))
            z[s + 1] = f32(f32(v * b2) - f32(a2 * y))
            v = y
        out[i] = v
    return out


def fm_demod(x, fs, dev_hz, audio_bw_hz):
    """demodulate/fm.rs:22-32, 60-70 (no translate)."""
    z = np.asarray(x, np.complex64)
    prev = np.concatenate([np.array([1 + 0j], np.complex64), z[:-1]])
    zr, zi = z.real.astype(f32), z.imag.astype(f32)
    pr, pi = prev.real.astype(f32), prev.imag.astype(f32)
    qr = ((zr * pr).astype(f32) + (zi * pi).astype(f32)).astype(f32)
    qi = ((zi * pr).astype(f32) - (zr * pi).astype(f32)).astype(f32)
    k = f32(f32(1.0) / max(f32(dev_hz), f32(1.0)))
    d = (atan2_approx(qi, qr) * k).astype(f32)
    return lp_cascade(d, fs, f32(f32(audio_bw_hz) * f32(0.9)))


def add_awgn(iq, noise_power, seed):
    """tests/common/mod.rs:27-48, xorshift64 in Python integers."""
    M = 0xFFFFFFFFFFFFFFFF
    st = (seed ^ 0xDEADBEEFCAFE0000) & M
    scale = f32(np.sqrt(f32(f32(noise_power) / f32(2.0))))
    umax = f32(float(M))
    out = np.array(iq, np.complex64)

    def nxt():
        nonlocal st
        s = f32(0.0)
        for _ in range(12):
            st ^= (st << 13) & M
            st ^= st >> 7
            st ^= (st << 17) & M
            s = f32(s + f32(f32(_u64_to_f32(st) / umax) - f32(0.5)))
        return s

    for i in range(len(out)):
        ni = f32(nxt() * scale)
        nq = f32(nxt() * scale)
        out[i] = complex(f32(f32(out[i].real) + ni), f32(f32(out[i].imag) + nq))
    return out


def _u64_to_f32(v: int) -> np.float32:
    """Round-to-nearest-even u64 -> f32 (LLVM uitofp)."""
    if v == 0:
        return f32(0.0)
    e = v.bit_length() - 24
    if e <= 0:
        return f32(v)
    mant = v >> e
    rem = v & ((1 << e) - 1)
    half = 1 << (e - 1)
    if rem > half or (rem == half and (mant & 1)):
        mant += 1
    return f32(float(mant) * float(2 ** e))


# ---- multicarrier/tx_lowpass.rs:96-185 TxLowpass sizing helpers (f32 arithmetic) ----
def kaiser_transition_norm(num_taps, stopband_db):
    """fir.rs:147-150: (max(A, 21) - 8) / (14.36 m), m = (max(num_taps, 3) | 1) as f32."""
    m = f32(max(int(num_taps), 3) | 1)
    return f32(f32(max(f32(stopband_db), f32(21.0)) - f32(8.0)) / f32(f32(14.36) * m))


def kaiser_num_taps(transition_norm, stopband_db):
    """fir.rs:154-157: ceil((max(A, 21) - 8) / (14.36 max(tn, 1e-4))), max 3, | 1."""
    m = np.ceil(f32(f32(max(f32(stopband_db), f32(21.0)) - f32(8.0)) /
                    f32(f32(14.36) * max(f32(transition_norm), f32(1e-4)))))
    return int(max(m, f32(3.0))) | 1


def tx_lowpass_for_null_band(n_fft, occupied_half, num_taps, stopband_db):
    occ = f32(f32(occupied_half) / f32(max(n_fft, 1)))
    half = f32(f32(0.5) * kaiser_transition_norm(num_taps, stopband_db))
    earliest = f32(occ + half)
    latest = f32(f32(0.5) - half)
    cutoff = earliest if earliest <= latest else f32(f32(0.5) * f32(occ + f32(0.5)))
    return cutoff, int(num_taps), f32(stopband_db)


def tx_lowpass_group_delay(num_taps):
    return (max(int(num_taps), 3) | 1) // 2


def tx_lowpass_fits_guard(num_taps, cp_len, roll_off, backoff):
    slack = min(max(cp_len - backoff, 0), backoff)
    return roll_off + tx_lowpass_group_delay(num_taps) <= slack


def tx_lowpass_taps_for_null_band(n_fft, occupied_half, stopband_db):
    occ = f32(f32(occupied_half) / f32(max(n_fft, 1)))
    return kaiser_num_taps(f32(f32(0.5) - occ), stopband_db)



# ---- second restatements of the remaining §8(a) rows (round 3) ------------------------
def _vsin(x):
    return np.array([sinf(v) for v in np.asarray(x, f32)], f32)


def _vcos(x):
    return np.array([cosf(v) for v in np.asarray(x, f32)], f32)


class _Osc:
    """The reference's phasor recurrence (rotator.rs:44-62 / nco.rs:42-58: the same
    update): z <- z w with mul_add, renormalised every 1024 steps; next() returns the
    post-multiply phasor."""

    def __init__(self, freq_hz, fs):
        self.fs = f32(fs)
        self.z = (f32(1.0), f32(0.0))
        self.ctr = 0
        self.set_freq(freq_hz, fs)

    def set_freq(self, freq_hz, fs=None):
        phi = f32(f32(TAU * f32(freq_hz)) / f32(self.fs if fs is None else fs))
        self.w = (cosf(phi), sinf(phi))

    def next(self):
        zr, zi = self.z
        wr, wi = self.w
        zr, zi = _fma(zr, wr, -f32(zi * wi)), _fma(zi, wr, f32(zr * wi))
        self.ctr = (self.ctr + 1) & 0xFFFFFFFF
        if self.ctr & 0x3FF == 0:
            inv = f32(f32(1.0) / f32(np.sqrt(f32(f32(zr * zr) + f32(zi * zi)))))
            zr, zi = f32(zr * inv), f32(zi * inv)
        self.z = (zr, zi)
        return zr, zi

    def phasors(self, n):
        out = np.zeros(n, np.complex64)
        for i in range(n):
            c, s_ = self.next()
            out[i] = complex(c, s_)
        return out


def rotator_mix_usb(x, freq_hz, fs):
    """rotator.rs:88-94: y = fma(I, cos, Q sin)."""
    p = _Osc(freq_hz, fs).phasors(len(x))
    x = np.asarray(x, np.complex64)
    return _fma(x.real.astype(f32), p.real.astype(f32), (x.imag.astype(f32) * p.imag.astype(f32)).astype(f32))


def nco_mix(x, freq_hz, fs):
    """nco.rs:63-66 mix_with_nco: (x.re c - x.im s, x.re s + x.im c), no FMA."""
    p = _Osc(freq_hz, fs).phasors(len(x))
    x = np.asarray(x, np.complex64)
    a, b = x.real.astype(f32), x.imag.astype(f32)
    c, d = p.real.astype(f32), p.imag.astype(f32)
    re = ((a * c).astype(f32) - (b * d).astype(f32)).astype(f32)
    im = ((a * d).astype(f32) + (b * c).astype(f32)).astype(f32)
    return (re + 1j * im).astype(np.complex64)


def biquad(x, b0, b1, b2, a1, a2):
    """iir.rs:34-40 TDF-II: y = fma(x, b0, z1); z1 = fma(x, b1, z2) - a1 y; z2 = x b2 - a2 y."""
    b0, b1, b2, a1, a2 = (f32(v) for v in (b0, b1, b2, a1, a2))
    z1 = z2 = f32(0.0)
    out = np.zeros(len(x), f32)
    for i, v in enumerate(np.asarray(x, f32)):
        y = _fma(v, b0, z1)
        z1 = f32(_fma(v, b1, z2) - f32(a1 * y))
        z2 = f32(f32(v * b2) - f32(a2 * y))
        out[i] = y
    return out


def lpdc_coeffs(fs, lp_fc, dc_cut):
    """iir.rs:111-137 (the biquad as LpCascade::design) and the DC pole
    r = clamp(1 - 2 PI (max(cut, 0.1) / fs), 0, 0.9999)."""
    b = lp_cascade_coeffs(fs, lp_fc)
    r = f32(f32(1.0) - f32(f32(f32(2.0) * PI) * f32(max(f32(dc_cut), f32(0.1)) / f32(fs))))
    r = min(max(r, f32(0.0)), f32(0.9999))
    return b + [r]


def lp_dc_cascade(x, fs, lp_fc, dc_cut, sqrt_map=False):
    """iir.rs:151-186: two TDF-II biquads, optional f32::sqrt, then the DC blocker
    y = y1 - x1 + r y1_prev."""
    b0, b1, b2, a1, a2, r = lpdc_coeffs(fs, lp_fc, dc_cut)
    z = [f32(0.0)] * 4
    x1 = y1 = f32(0.0)
    out = np.zeros(len(x), f32)
    for i, v in enumerate(np.asarray(x, f32)):
        for s_ in (0, 2):
            y = _fma(v, b0, z[s_])
            z[s_] = f32(_fma(v, b1, z[s_ + 1]) - f32(a1 * y))
            z[s_ + 1] = f32(f32(v * b2) - f32(a2 * y))
            v = y
        if sqrt_map:
            v = f32(np.sqrt(v))
        y = f32(f32(v - x1) + f32(r * y1))
        x1, y1 = v, y
        out[i] = y
    return out


def dc_blocker(x, fs, cut_hz):
    """dsp/dc.rs:15-58."""
    r = f32(f32(1.0) - f32(f32(f32(2.0) * PI) * f32(max(f32(cut_hz), f32(0.1)) / f32(fs))))
    r = min(max(r, f32(0.0)), f32(0.9999))
    x1 = y1 = f32(0.0)
    out = np.zeros(len(x), f32)
    for i, v in enumerate(np.asarray(x, f32)):
        y = f32(f32(v - x1) + f32(r * y1))
        out[i] = y
        x1, y1 = v, y
    return out


def ssb_demod(x, fs, bfo_hz, audio_bw_hz):
    """demodulate/ssb.rs:15-71: y = fma(I, p.re, Q p.im) with the BFO Rotator, then
    LpDcCascade(fs, 0.9 bw, 2 Hz)."""
    y = rotator_mix_usb(x, bfo_hz, fs)
    return lp_dc_cascade(y, fs, f32(f32(audio_bw_hz) * f32(0.9)), 2.0)


def am_demod(x, fs, audio_bw_hz, abs_approx=None):
    """demodulate/am.rs:44-129: PowerSqrt p = fma(I, I, Q Q) -> process_mapped(p, sqrt);
    AbsApprox e = fma(k1, |I|, k2 |Q|) -> process."""
    x = np.asarray(x, np.complex64)
    re, im = x.real.astype(f32), x.imag.astype(f32)
    lp = f32(f32(audio_bw_hz) * f32(0.9))
    if abs_approx is None:
        p = _fma(re, re, (im * im).astype(f32))
        return lp_dc_cascade(p, fs, lp, 2.0, sqrt_map=True)
    k1, k2 = f32(abs_approx[0]), f32(abs_approx[1])
    e = _fma(np.full(len(x), k1, f32), np.abs(re), (k2 * np.abs(im)).astype(f32))
    return lp_dc_cascade(e, fs, lp, 2.0)


def pm_demod(x, fs, k, audio_bw_hz):
    """demodulate/pm.rs:22-66: w = z conj(prev) (num-complex: re = a c - b (-d),
    im = a (-d) + b c), k atan2_approx(w.im, w.re), LpCascade(fs, 0.9 bw)."""
    z = np.asarray(x, np.complex64)
    prev = np.concatenate([np.array([1 + 0j], np.complex64), z[:-1]])
    a, b = z.real.astype(f32), z.imag.astype(f32)
    c, nd = prev.real.astype(f32), (-prev.imag).astype(f32)
    wr = ((a * c).astype(f32) - (b * nd).astype(f32)).astype(f32)
    wi = ((a * nd).astype(f32) + (b * c).astype(f32)).astype(f32)
    d = (f32(k) * atan2_approx(wi, wr)).astype(f32)
    return lp_cascade(d, fs, f32(f32(audio_bw_hz) * f32(0.9)))


def cw_demod(x, fs, tone_hz, env_bw_hz, gain=1.0):
    """demodulate/cw.rs:15-46: alpha = exp(-TAU fc / fs), fc = max(bw, 1);
    y = a y + (1 - a) sqrt(I I + Q Q); out = y gain."""
    fc = max(f32(env_bw_hz), f32(1.0))
    a = expf(f32(f32(-TAU * fc) / f32(fs)))
    oma = f32(f32(1.0) - a)
    x = np.asarray(x, np.complex64)
    mag = np.sqrt(((x.real.astype(f32) * x.real.astype(f32)).astype(f32) +
                   (x.imag.astype(f32) * x.imag.astype(f32)).astype(f32)).astype(f32)).astype(f32)
    y = f32(0.0)
    out = np.zeros(len(x), f32)
    for i, m in enumerate(mag):
        y = f32(f32(a * y) + f32(oma * m))
        out[i] = f32(y * f32(gain))
    return out


def fir_lowpass_iq(x, taps):
    """dsp/fir.rs:229-247 push (from a zero delay line): re/im = fma(d, taps[j], acc)
    for j = 0 .. L-1, taps[0] with the newest sample, in that order."""
    taps = np.asarray(taps, f32) if len(taps) else np.array([1.0], f32)
    x = np.asarray(x, np.complex64)
    L, n = len(taps), len(x)
    xr = np.concatenate([np.zeros(L, f32), x.real.astype(f32)])
    xi = np.concatenate([np.zeros(L, f32), x.imag.astype(f32)])
    re = np.zeros(n, f32)
    im = np.zeros(n, f32)
    for j in range(L):
        t = np.full(n, taps[j], f32)
        re = _fma(xr[L - j: L - j + n], t, re)
        im = _fma(xi[L - j: L - j + n], t, im)
    return (re + 1j * im).astype(np.complex64)


def fir_lowpass_iq_aligned(x, taps):
    """dsp/fir.rs:260-276 filter_aligned: reset, push io[0..d), then io[i + d] (0
    past the end) for every i: the streamed filter of [io | 0^d] from index d."""
    L = len(taps) if len(taps) else 1
    d = (L - 1) // 2
    x = np.asarray(x, np.complex64)
    y = fir_lowpass_iq(np.concatenate([x, np.zeros(d, np.complex64)]), taps)
    return y[d: d + len(x)]


def fm_mod(a, fs, dev_hz, rf_hz=0.0, gain=1.0):
    """modulate/fm.rs:45-74: kf = TAU dev / fs; z *= (cos, sin)(kf x) with mul_add,
    renormalised every 1024; out = mix_with_nco(z gain, rf)."""
    kf = f32(f32(TAU * f32(dev_hz)) / f32(fs))
    rf = _Osc(rf_hz, fs)
    zr, zi = f32(1.0), f32(0.0)
    ctr = 0
    out = np.zeros(len(a), np.complex64)
    g = f32(gain)
    for i, v in enumerate(np.asarray(a, f32)):
        dphi = f32(kf * v)
        ds, dc = sinf(dphi), cosf(dphi)
        zr, zi = _fma(zr, dc, -f32(zi * ds)), _fma(zi, dc, f32(zr * ds))
        ctr = (ctr + 1) & 0xFFFFFFFF
        if ctr & 0x3FF == 0:
            inv = f32(f32(1.0) / f32(np.sqrt(f32(f32(zr * zr) + f32(zi * zi)))))
            zr, zi = f32(zr * inv), f32(zi * inv)
        br, bi = f32(zr * g), f32(zi * g)
        c, s_ = rf.next()
        out[i] = complex(f32(f32(br * c) - f32(bi * s_)), f32(f32(br * s_) + f32(bi * c)))
    return out


def am_mod(a, fs, rf_hz, carrier_level, mod_index, gain=1.0, clamp=False):
    """modulate/am.rs:44-120: m = (cl + mi x) [clamp(-1, 1)] g; out = (m r.re, m r.im)."""
    r = _Osc(rf_hz, fs)
    cl, mi, g = f32(carrier_level), f32(mod_index), f32(gain)
    out = np.zeros(len(a), np.complex64)
    for i, v in enumerate(np.asarray(a, f32)):
        m = f32(cl + f32(mi * v))
        if clamp:
            m = f32(-1.0) if m < -1.0 else (f32(1.0) if m > 1.0 else m)
        m = f32(m * g)
        c, s_ = r.next()
        out[i] = complex(f32(m * c), f32(m * s_))
    return out


def ssb_mod(a, fs, audio_bw_hz, audio_if_hz, rf_hz=0.0, usb=True):
    """modulate/ssb.rs:43-114: LpCascade(x p.re), LpCascade(x p.im) with the audio
    Rotator, z = (I, side Q), out = z r in rotate_block's FMA form."""
    fc = f32(f32(audio_bw_hz) * f32(0.9))
    p = _Osc(audio_if_hz, fs).phasors(len(a))
    r = _Osc(rf_hz, fs).phasors(len(a))
    a = np.asarray(a, f32)
    ii = lp_cascade((a * p.real.astype(f32)).astype(f32), fs, fc)
    qq = lp_cascade((a * p.imag.astype(f32)).astype(f32), fs, fc)
    side = f32(1.0 if usb else -1.0)
    zr, zi = ii, (side * qq).astype(f32)
    rr, ri = r.real.astype(f32), r.imag.astype(f32)
    re = _fma(zr, rr, -(zi * ri).astype(f32))
    im = _fma(zi, rr, (zr * ri).astype(f32))
    return (re + 1j * im).astype(np.complex64)


def pm_mod(a, fs, kp, rf_hz=0.0, gain=1.0):
    """modulate/pm.rs:36-47: (cos kp x, sin kp x) gain, mix_with_nco with the RF Nco."""
    phi = (f32(kp) * np.asarray(a, f32)).astype(f32)
    base = ((_vcos(phi) * f32(gain)).astype(f32) + 1j * (_vsin(phi) * f32(gain)).astype(f32)).astype(np.complex64)
    return nco_mix(base, rf_hz, fs)


def cw_mod(a, fs, tone_hz, rise_ms, fall_ms, gain=1.0):
    """modulate/cw.rs:21-87: tau = (max(ms, 0.1) 1e-3) fs, alpha = exp(-1 / tau);
    tgt = clamp(x, 0, 1); env = a env + (1 - a) tgt (rise when tgt >= env, else fall);
    out = mix_with_nco((env gain, 0), nco)."""
    def alpha(ms):
        tau = f32(f32(max(f32(ms), f32(0.1)) * f32(1e-3)) * f32(fs))
        return expf(f32(f32(-1.0) / tau))
    ar, af = alpha(rise_ms), alpha(fall_ms)
    env = f32(0.0)
    m = np.zeros(len(a), f32)
    for i, v in enumerate(np.asarray(a, f32)):
        t = f32(0.0) if v < 0.0 else (f32(1.0) if v > 1.0 else v)
        if t >= env:
            env = f32(f32(ar * env) + f32(f32(f32(1.0) - ar) * t))
        else:
            env = f32(f32(af * env) + f32(f32(f32(1.0) - af) * t))
        m[i] = f32(env * f32(gain))
    return nco_mix(m.astype(np.complex64), tone_hz, fs)


def wbfm(x, f_off=1.5e6, fs=10e6, m=8, dec_cutoff=200e3, dec_trans=79e3, dev_hz=75e3, audio_bw=15e3,
         audio_pass=15e3, audio_trans=10e3):
    """The WBFM chain of docs/demodulate.md:128-133, one call: Rotator(-f_off) ->
    FirDecimator -> FmQuadratureDemod(fs/m) -> FirLowpass(fs/m)."""
    fs2 = f32(f32(fs) / f32(m))
    mixed = rotator(x, -f32(f_off), fs)
    dec = fir_decimator(mixed, fs, m, dec_cutoff, dec_trans)
    ph = fm_demod(dec, fs2, dev_hz, audio_bw)
    return fir_lowpass(ph, fir_lowpass_taps(fs2, audio_pass, audio_trans))



def kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db):
    """dsp/fir.rs:74-141: Kaiser-windowed sinc, f32 throughout, sum-normalised."""
    a_db = f32(stopband_db)
    if a_db > 50.0:
        beta = f32(f32(0.1102) * f32(a_db - f32(8.7)))
    elif a_db >= 21.0:
        beta = f32(f32(f32(0.5842) * f32(_libm.powf(float(f32(a_db - f32(21.0))), 0.4))) +
                   f32(f32(0.07886) * f32(a_db - f32(21.0))))
    else:
        beta = f32(0.0)

    def i0(xv):
        half = f32(f32(0.5) * f32(xv))
        term = f32(1.0)
        sm = f32(1.0)
        for k in range(1, 41):
            term = f32(term * f32(half / f32(k)))
            t = f32(term * term)
            sm = f32(sm + t)
            if t < f32(f32(1e-12) * sm):
                break
        return sm

    m = max(int(num_taps), 3) | 1
    mid = f32(m // 2)
    fc = min(max(f32(cutoff_norm), f32(1e-4)), f32(0.4999))
    i0b = i0(beta)
    taps = np.zeros(m, f32)
    for n in range(m):
        d = f32(f32(n) - mid)
        if d == 0.0:
            ideal = f32(f32(2.0) * fc)
        else:
            ideal = f32(sinf(f32(f32(TAU * fc) * d)) / f32(PI * d))
        r = f32(d / mid)
        arg = f32(np.sqrt(max(f32(f32(1.0) - f32(r * r)), f32(0.0))))
        w = f32(i0(f32(beta * arg)) / i0b)
        taps[n] = f32(ideal * w)
    sm = f32(0.0)
    for v in taps:
        sm = f32(sm + v)
    if abs(sm) > np.finfo(np.float32).eps:
        taps = (taps / sm).astype(f32)
    return taps
