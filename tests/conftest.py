"""Shared test setup.

* Registers the ``gpu`` marker: ``-m gpu`` tests need an MI355X and exercise the
  HIP kernels through the C ABI; ``-m "not gpu"`` tests run anywhere (oracle vs
  golden vectors, host-side designs, library load/exports).
* Puts ``oracle/`` (test infrastructure: the scalar C restatement of the
  reference) and ``orion-sdr_amd/`` (the product's Python mirror) on sys.path.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "oracle"), os.path.join(ROOT, "orion-sdr_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

FS = 48_000.0  # python/tests/conftest.py:8


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


def real_tone(fs, f_hz, n, amp=1.0):
    """python/tests/conftest.py:11-14."""
    t = np.arange(n, dtype=np.float32) / fs
    return (amp * np.sin(2.0 * np.pi * f_hz * t)).astype(np.float32)


def complex_tone(fs, f_hz, n, amp=1.0):
    """python/tests/conftest.py:17-20."""
    t = np.arange(n, dtype=np.float32) / fs
    return (amp * np.exp(1j * 2.0 * np.pi * f_hz * t)).astype(np.complex64)


def snr_db(x, fs, f_hz):
    """python/tests/conftest.py:23-38 (single-bin DFT: f vs 0.73 f)."""
    x = np.asarray(x, np.float64)
    n = len(x)
    k = np.arange(n, dtype=np.float64)

    def p(f):
        w = -2.0 * np.pi * f / fs * k
        return float(abs(np.dot(np.cos(w) + 1j * np.sin(w), x)) ** 2) / (n * n)

    return 10.0 * np.log10(p(f_hz) / (p(f_hz * 0.73) + 1e-20))


def tail(x, fraction=0.75):
    return x[int(len(x) * (1.0 - fraction)):]


def report(name, v, tol):
    """Print a measured parity figure and assert it is within tol."""
    print(f"[parity] {name}: {v:.3e} (tol {tol:.1e})")
    assert v <= tol, f"{name}: {v:.3e} > {tol:.1e}"


def nrmse(got, ref):
    got = np.asarray(got, np.complex128 if np.iscomplexobj(got) else np.float64)
    ref = np.asarray(ref, got.dtype)
    den = np.sqrt(np.mean(np.abs(ref) ** 2))
    return float(np.sqrt(np.mean(np.abs(got - ref) ** 2)) / (den if den > 0 else 1.0))


def wbfm_input(n, f_off=1.5e6, fs=10e6, noise=0.0025, seed=0x1234_5678_ABCD_EF00, amp=1.0, dev=75e3):
    """C2 synthetic IQ: FM dev 75 kHz of amp (0.5 sin(1k) + 0.3 sin(7k)),
    up-converted to f_off by FmPhaseAccumMod's RF NCO, plus add_awgn."""
    import oracle as O

    t = np.arange(n) / fs
    aud = (amp * (0.5 * np.sin(2 * np.pi * 1e3 * t) + 0.3 * np.sin(2 * np.pi * 7e3 * t))).astype(np.float32)
    iq = O.fm_mod(aud, fs, dev, f_off)
    if noise > 0:
        iq = O.add_awgn(iq, noise, seed)
    return iq


@pytest.fixture(scope="session")
def oracle():
    import oracle as O

    O.lib()
    return O


@pytest.fixture(scope="session")
def gpu_lib():
    """The product library on a real device; skips nothing on a GPU box (fails loud)."""
    import orion_sdr

    if orion_sdr.device_count() < 1:
        pytest.fail("gpu test selected but no HIP device is visible")
    return orion_sdr
