"""TEST INFRASTRUCTURE — a second, independently written restatement of the
reference algorithms in numpy float32 (no shared code with oracle/orion_oracle.c).

It exists to cross-check the C oracle: both must agree bit for bit on the
committed fixtures (tests/golden/). Where the reference uses ``mul_add`` this
file uses an exact-product f32 FMA emulation (``_fma``: the f64 product of two
f32 values is exact; one rounding to f32 after the add), elsewhere plain
float32 numpy arithmetic (one rounding per op, no contraction).
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


def sinf(x):
    return f32(_libm.sinf(float(x)))


def cosf(x):
    return f32(_libm.cosf(float(x)))
TAU = f32(2.0 * math.pi)
PI = f32(math.pi)


def _fma(a, b, c):
    return (np.float64(a) * np.float64(b) + np.float64(c)).astype(np.float32) if isinstance(a, np.ndarray) \
        else f32(float(np.float64(a) * np.float64(b) + np.float64(c)))


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
