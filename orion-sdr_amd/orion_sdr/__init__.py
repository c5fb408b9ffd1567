"""orion_sdr (MI355X engine) — Python mirror of skynavga/orion-sdr's analog API.

Same class names, constructor arguments and ``process(ndarray) -> ndarray``
contract as the reference PyO3 module (``python/orion_sdr/__init__.pyi:18-79``,
``src/python/demodulate.rs:9-148``): IQ arrays are ``numpy.complex64``, audio
``numpy.float32``, inputs must be 1-D and C-contiguous (else ``ValueError`` /
``TypeError``), every call returns a new array, and instances keep their
streaming state between calls.

Every class runs on the GPU through ``lib/liborion_sdr_amd.so`` (gfx950 HIP
kernels behind the C ABI in ``include/orion_sdr_amd.h``). There is no CPU
fallback: importing without the built library, or calling without a visible
device, raises.

``process`` also accepts torch CUDA tensors (device path, no host copies): the
output is a new torch tensor on the same device, computed asynchronously on
torch's current stream.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

__all__ = [
    "Rotator", "Nco", "Biquad", "LpDcCascade", "PmDirectPhaseMod", "CwKeyedMod", "TxLowpass", "FirDecimator", "FirLowpass", "FirLowpassIq", "LpCascade", "DcBlocker",
    "FmQuadratureDemod", "PmQuadratureDemod", "SsbProductDemod", "AmEnvelopeDemod",
    "CwEnvelopeDemod", "WbfmChain", "AgcRms", "AgcRmsIq", "AmDsbMod", "FmPhaseAccumMod", "SsbPhasingMod",
    "fir_lowpass_design", "kaiser_lowpass_taps",
    "kaiser_transition_norm", "kaiser_num_taps", "lp_cascade_design", "lib_path", "OrionError", "diag_stream_read",
    "AudioToIqChain", "IqToIqChain", "IqToAudioChain", "Graph", "stream_shard", "STREAM_HALO",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# ORION_SDR_LIB: an alternative build of the same library (timing experiments)
_LIB = os.environ.get("ORION_SDR_LIB") or os.path.join(os.path.dirname(_HERE), "lib", "liborion_sdr_amd.so")


def lib_path() -> str:
    return _LIB


class OrionError(RuntimeError):
    """A failure reported by the C ABI (HIP error, bad argument, ...)."""


class WorkReport(C.Structure):
    _fields_ = [("in_read", C.c_size_t), ("out_written", C.c_size_t)]


class TxLowpassSpec(C.Structure):
    _fields_ = [("cutoff_norm", C.c_float), ("num_taps", C.c_size_t), ("stopband_db", C.c_float)]


class WbfmParams(C.Structure):
    _fields_ = [("fs", C.c_float), ("f_off", C.c_float), ("dec_cutoff", C.c_float),
                ("dec_trans", C.c_float), ("dev_hz", C.c_float), ("audio_bw", C.c_float),
                ("audio_pass", C.c_float), ("audio_trans", C.c_float), ("m", C.c_size_t)]


def _load():
    if not os.path.exists(_LIB):
        raise ImportError(
            f"orion_sdr: native library {_LIB} is missing — build it with "
            "`make -C orion-sdr_amd` (hipcc, gfx950). There is no CPU fallback.")
    # The library and torch both need libamdhip64.so.7 (one soname: the first one
    # loaded serves the process). Load torch's first, as bench.py does, so torch's
    # own device path keeps the runtime it was built against whatever the import order.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(_LIB)
    vp, sz, f, i = C.c_void_p, C.c_size_t, C.c_float, C.c_int
    fp = C.POINTER(C.c_float)
    sig = {
        "orion_version": (C.c_char_p, []), "orion_last_error": (C.c_char_p, []),
        "orion_device_count": (i, []), "orion_set_device": (i, [i]), "orion_synchronize": (i, [vp]),
        "orion_rotator_new": (vp, [f, f]),
        "orion_rotator_set_freq": (i, [vp, f, f]), "orion_rotator_reset_phase": (i, [vp]),
        "orion_rotator_mix_usb_block": (i, [vp, vp, sz, vp, sz, C.POINTER(WorkReport)]),
        "orion_rotator_mix_usb_block_device": (i, [vp, vp, sz, vp, sz, vp, C.POINTER(WorkReport)]),
        "orion_nco_new": (vp, [f, f]), "orion_nco_set_freq": (i, [vp, f]),
        "orion_nco_next_cs_block": (i, [vp, vp, sz]), "orion_nco_next_cs_block_device": (i, [vp, vp, sz, vp]),
        "orion_rotator_next_cs_block": (i, [vp, vp, sz]),
        "orion_rotator_next_cs_block_device": (i, [vp, vp, sz, vp]),
        "orion_osc_table_phasors": (i, [f, f, C.c_uint64, vp, sz, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64),
                                        C.POINTER(C.c_uint64)]),
        "orion_fir_lowpass_iq_num_taps": (i, [vp, C.POINTER(sz)]),
        "orion_fir_lowpass_iq_group_delay": (i, [vp, C.POINTER(sz)]),
        "orion_biquad_new": (vp, [f, f, f, f, f]),
        "orion_lp_dc_cascade_new": (vp, [f, f, f]), "orion_lp_dc_cascade_set_sqrt_map": (i, [vp, i]),
        "orion_lp_dc_cascade_set_map": (i, [vp, i]),
        "orion_pm_direct_phase_mod_new": (vp, [f, f, f]), "orion_pm_direct_phase_mod_set_gain": (i, [vp, f]),
        "orion_pm_direct_phase_mod_set_sensitivity": (i, [vp, f]),
        "orion_cw_keyed_mod_new": (vp, [f, f, f, f]), "orion_cw_keyed_mod_set_gain": (i, [vp, f]),
        "orion_tx_lowpass_for_null_band": (TxLowpassSpec, [sz, sz, sz, f]),
        "orion_tx_lowpass_taps_for_null_band": (sz, [sz, sz, f]),
        "orion_tx_lowpass_group_delay": (sz, [C.POINTER(TxLowpassSpec)]),
        "orion_tx_lowpass_transition_norm": (f, [C.POINTER(TxLowpassSpec)]),
        "orion_tx_lowpass_transition_fits": (i, [C.POINTER(TxLowpassSpec), sz, sz]),
        "orion_tx_lowpass_stopband_edge_norm": (f, [C.POINTER(TxLowpassSpec)]),
        "orion_tx_lowpass_fits_guard": (i, [C.POINTER(TxLowpassSpec), sz, sz, sz]),
        "orion_tx_lowpass_filter": (vp, [C.POINTER(TxLowpassSpec)]),
        "orion_fir_decimator_new": (vp, [f, sz, f, f]),
        "orion_fir_decimator_batch_new": (vp, [f, sz, f, f, sz]),
        "orion_fir_lowpass_new": (vp, [f, f, f]),
        "orion_fir_lowpass_iq_design": (vp, [sz, f, f]),
        "orion_fir_lowpass_iq_from_taps": (vp, [fp, sz]),
        "orion_fir_lowpass_iq_batch_from_taps": (vp, [fp, sz, sz]),
        "orion_fir_lowpass_iq_filter_aligned_device": (i, [vp, vp, sz, vp]),
        "orion_fir_lowpass_iq_filter_aligned": (i, [vp, vp, sz]),
        "orion_lp_cascade_new": (vp, [f, f]),
        "orion_dc_blocker_new": (vp, [f, f]),
        "orion_fm_quadrature_demod_new": (vp, [f, f, f]),
        "orion_fm_quadrature_demod_with_translate": (i, [vp, f]),
        "orion_pm_quadrature_demod_new": (vp, [f, f, f]),
        "orion_ssb_product_demod_new": (vp, [f, f, f]),
        "orion_ssb_product_demod_batch_new": (vp, [f, f, f, sz]),
        "orion_am_envelope_demod_new": (vp, [f, f]),
        "orion_am_envelope_demod_with_abs_approx": (i, [vp, f, f]),
        "orion_cw_envelope_demod_new": (vp, [f, f, f]),
        "orion_cw_envelope_demod_set_gain": (i, [vp, f]),
        "orion_am_dsb_mod_new": (vp, [f, f, f, f]),
        "orion_agc_rms_new": (vp, [f, f, f, f]),
        "orion_agc_rms_iq_new": (vp, [f, f, f, f]),
        "orion_am_dsb_mod_set_gain": (i, [vp, f]),
        "orion_am_dsb_mod_set_clamp": (i, [vp, i]),
        "orion_fm_phase_accum_mod_new": (vp, [f, f, f]),
        "orion_fm_phase_accum_mod_set_deviation": (i, [vp, f]),
        "orion_fm_phase_accum_mod_set_gain": (i, [vp, f]),
        "orion_ssb_phasing_mod_new": (vp, [f, f, f, f, i]),
        "orion_wbfm_chain_new": (vp, [C.POINTER(WbfmParams)]),
        "orion_wbfm_chain_batch_new": (vp, [C.POINTER(WbfmParams), fp, sz]),
        "orion_wbfm_chain_configure": (i, [vp, i, i]),
        "orion_wbfm_chain_seek": (i, [vp, C.c_uint64]),
        "orion_block_process": (i, [vp, vp, sz, vp, sz, C.POINTER(WorkReport)]),
        "orion_block_process_device": (i, [vp, vp, sz, vp, sz, vp, C.POINTER(WorkReport)]),
        "orion_batch_process": (i, [vp, vp, sz, sz, vp, sz, vp, C.POINTER(WorkReport)]),
        "orion_block_reset": (i, [vp]), "orion_block_free": (None, [vp]),
        "orion_block_configure": (i, [vp, i, C.c_longlong]),
        "orion_block_status": (i, [vp]),
        "orion_debug_set_spin_limit": (None, [C.c_uint32]), "orion_debug_spin_limit": (C.c_uint32, []),
        "orion_block_in_type": (i, [vp]), "orion_block_out_type": (i, [vp]),
        "orion_block_out_len": (sz, [vp, sz]), "orion_block_channels": (sz, [vp]),
        "orion_block_name": (C.c_char_p, [vp]),
        "orion_block_taps": (i, [vp, i, fp, sz, C.POINTER(sz)]),
        "orion_fir_lowpass_design": (sz, [f, f, f, fp, sz]),
        "orion_kaiser_lowpass_taps": (sz, [sz, f, f, fp, sz]),
        "orion_kaiser_transition_norm": (f, [sz, f]),
        "orion_kaiser_num_taps": (sz, [f, f]),
        "orion_lp_cascade_design": (None, [f, f, fp]),
        "orion_diag_stream_read_bytes": (sz, [sz]),
        "orion_diag_stream_read": (i, [vp, sz, vp]),
        "orion_diag_spin": (i, [vp, C.c_uint32, C.c_uint32, C.c_double]),
        "orion_diag_stream_create": (vp, [C.c_uint32]), "orion_diag_stream_destroy": (i, [vp]),
        "orion_device_cus": (i, []),
        "orion_host_alloc": (vp, [sz]), "orion_host_free": (i, [vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


_L = _load()


def _err() -> str:
    return (_L.orion_last_error() or b"").decode()


def _check(rc: int):
    if rc != 0:
        raise OrionError(f"orion_sdr: error {rc}: {_err()}")


def _fptr(a: np.ndarray):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _taps_of(h, which: int) -> np.ndarray:
    n = C.c_size_t(0)
    _check(_L.orion_block_taps(h, which, None, 0, C.byref(n)))
    out = np.zeros(n.value, np.float32)
    _check(_L.orion_block_taps(h, which, _fptr(out), n.value, C.byref(n)))
    return out


_DT = {0: np.complex64, 1: np.float32}


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


class _Block:
    """Shared Block contract (reference src/core.rs:12-22)."""

    def __init__(self, handle):
        if not handle:
            raise OrionError(f"orion_sdr: construction failed: {_err()}")
        self._h = handle
        self._in = _DT[_L.orion_block_in_type(handle)]
        self._out = _DT[_L.orion_block_out_type(handle)]
        self._nch = _L.orion_block_channels(handle)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _L is not None:  # at interpreter exit the module globals may already be gone
            _L.orion_block_free(h)
            self._h = None

    @property
    def name(self) -> str:
        return _L.orion_block_name(self._h).decode()

    def out_len(self, n: int) -> int:
        return _L.orion_block_out_len(self._h, n)

    def reset(self):
        _check(_L.orion_block_reset(self._h))

    def _validate(self, x: np.ndarray) -> np.ndarray:
        # python/tests/test_unit.py:86-127: wrong dtype / ndim / non-contiguous -> error
        if not isinstance(x, np.ndarray):
            raise TypeError(f"{type(self).__name__}.process expects a numpy array")
        if x.dtype != self._in:
            raise TypeError(f"{type(self).__name__}.process expects {np.dtype(self._in).name}, got {x.dtype}")
        want_ndim = 1 if self._nch == 1 else 2
        if x.ndim != want_ndim:
            raise ValueError(f"{type(self).__name__}.process expects a {want_ndim}-D array, got {x.ndim}-D")
        if not x.flags["C_CONTIGUOUS"]:
            raise ValueError("array is not C-contiguous")
        if self._nch > 1 and x.shape[0] != self._nch:
            raise ValueError(f"expected {self._nch} channels, got {x.shape[0]}")
        return x

    def process_into(self, x: np.ndarray, out: np.ndarray) -> WorkReport:
        """Preallocated path (core.rs:19-21 process_into): honours out capacity."""
        x = self._validate(x)
        n = x.shape[-1]
        wr = WorkReport()
        _check(_L.orion_block_process(self._h, x.ctypes.data, n, out.ctypes.data, out.shape[-1], C.byref(wr)))
        return wr

    def process(self, x):
        if _is_torch(x):
            return self.process_device(x)
        x = self._validate(x)
        n = x.shape[-1]
        cap = self.out_len(n)
        out = np.empty((cap,) if self._nch == 1 else (self._nch, cap), self._out)
        wr = WorkReport()
        _check(_L.orion_block_process(self._h, x.ctypes.data, n, out.ctypes.data, cap, C.byref(wr)))
        if wr.out_written != cap:
            out = out[..., : wr.out_written].copy()
        return out

    def process_device(self, x, out=None, stream=None):
        """Device buffers (torch CUDA tensors). Asynchronous on `stream`
        (default: torch's current stream). Returns out (its first out_written samples)."""
        import torch

        if not x.is_cuda or not x.is_contiguous():
            raise ValueError("process_device needs a contiguous CUDA tensor")
        want = torch.complex64 if self._in is np.complex64 else torch.float32
        if x.dtype != want:
            raise TypeError(f"expected {want}, got {x.dtype}")
        n = x.shape[-1]
        cap = self.out_len(n)
        odt = torch.complex64 if self._out is np.complex64 else torch.float32
        if out is None:
            out = torch.empty((cap,) if self._nch == 1 else (self._nch, cap), dtype=odt, device=x.device)
        else:
            cap = out.shape[-1]
        s = stream if stream is not None else torch.cuda.current_stream(x.device).cuda_stream
        wr = WorkReport()
        _check(_L.orion_block_process_device(self._h, x.data_ptr(), n, out.data_ptr(), cap, s, C.byref(wr)))
        return out if wr.out_written == cap else out[..., : wr.out_written]

    def taps(self, which: int = 0) -> np.ndarray:
        return _taps_of(self._h, which)

    _OPTS = {"scan_path": 1, "mod_passes": 2, "nco_table": 3}

    def configure_option(self, option: str, value: int):
        """Engine options (no reference counterpart; include/orion_sdr_amd.h
        orion_block_configure): scan_path 0/1 (single pass / three-kernel scan),
        mod_passes 0/3, nco_table 0..2^28 (outputs of the reference's oscillator
        recurrence tabulated per tune; 0 = the closed-form ideal phasor)."""
        _check(_L.orion_block_configure(self._h, self._OPTS[option], int(value)))
        return self

    def status(self):
        """Raise OrionError if a kernel of this handle flagged a device-side failure
        (a cross-workgroup wait that timed out) since the last check (non-blocking;
        include/orion_sdr_amd.h orion_block_status)."""
        _check(_L.orion_block_status(self._h))


# ---- DSP primitives (src/dsp) -------------------------------------------------
class Rotator(_Block):
    """dsp/rotator.rs:16 Rotator::new(freq_hz, fs); process = rotate_block (:74-85)."""

    def __init__(self, freq_hz: float, fs: float):
        super().__init__(_L.orion_rotator_new(freq_hz, fs))

    def set_freq(self, freq_hz: float, fs: float):
        """rotator.rs:35-39: a new step; the phase continues (synchronizes the device)."""
        _check(_L.orion_rotator_set_freq(self._h, freq_hz, fs))

    def reset_phase(self):
        """rotator.rs:28-31: phasor back to 1 + j0."""
        _check(_L.orion_rotator_reset_phase(self._h))

    def next_cs_block(self, n: int) -> np.ndarray:
        """rotator.rs:44-68 next / next_cs, n times: complex64 phasors, advancing the
        same oscillator as process / mix_usb_block."""
        out = np.empty(int(n), np.complex64)
        _check(_L.orion_rotator_next_cs_block(self._h, out.ctypes.data, out.size))
        return out

    def mix_usb_block(self, x):
        """rotator.rs:88-94: I*cos + Q*sin on the same oscillator (complex64 -> float32).
        A torch CUDA tensor runs on the device path (torch's current stream)."""
        wr = WorkReport()
        if _is_torch(x):
            import torch

            if not x.is_cuda or not x.is_contiguous() or x.dtype != torch.complex64:
                raise ValueError("mix_usb_block needs a contiguous complex64 CUDA tensor")
            out = torch.empty(x.shape[-1], dtype=torch.float32, device=x.device)
            s = torch.cuda.current_stream(x.device).cuda_stream
            _check(_L.orion_rotator_mix_usb_block_device(self._h, x.data_ptr(), x.shape[-1], out.data_ptr(),
                                                        out.shape[0], s, C.byref(wr)))
            return out
        x = self._validate(x)
        out = np.empty(x.shape[-1], np.float32)
        _check(_L.orion_rotator_mix_usb_block(self._h, x.ctypes.data, x.shape[-1], out.ctypes.data, out.size,
                                              C.byref(wr)))
        return out


class Nco(_Block):
    """dsp/nco.rs:20 Nco::new(freq_hz, fs) as a block: process = mix_with_nco per
    sample (nco.rs:63-66, the non-FMA product)."""

    def __init__(self, freq_hz: float, fs: float):
        super().__init__(_L.orion_nco_new(freq_hz, fs))

    def set_freq(self, freq_hz: float):
        """nco.rs:33-38 (fs from the constructor); the phase continues."""
        _check(_L.orion_nco_set_freq(self._h, freq_hz))

    def next_cs_block(self, n: int) -> np.ndarray:
        """nco.rs:42-58 next_cs, n times: complex64 (cos, sin) of each step's phasor."""
        out = np.empty(int(n), np.complex64)
        _check(_L.orion_nco_next_cs_block(self._h, out.ctypes.data, out.size))
        return out


class Biquad(_Block):
    """dsp/iir.rs:15-41 Biquad::new(b0, b1, b2, a1, a2) (TDF-II); reset() = Biquad::reset."""

    def __init__(self, b0: float, b1: float, b2: float, a1: float, a2: float):
        super().__init__(_L.orion_biquad_new(b0, b1, b2, a1, a2))


class LpDcCascade(_Block):
    """dsp/iir.rs:111 LpDcCascade::design(fs, lp_fc, dc_cut_hz); process (:151-165), or
    process_mapped(x, f) (:170-186) with map "identity" / "sqrt" / "abs"
    (sqrt_map=True: "sqrt", the AM-PowerSqrt use)."""

    MAPS = {"identity": 0, "sqrt": 1, "abs": 2}

    def __init__(self, fs: float, lp_fc: float, dc_cut_hz: float, sqrt_map: bool = False, map: str | None = None):
        super().__init__(_L.orion_lp_dc_cascade_new(fs, lp_fc, dc_cut_hz))
        if sqrt_map:
            _check(_L.orion_lp_dc_cascade_set_sqrt_map(self._h, 1))
        if map is not None:
            self.set_map(map)

    def set_map(self, map: str):
        """process_mapped's f from the next call on (before the first call)."""
        if map not in self.MAPS:
            raise ValueError(f"LpDcCascade map must be one of {sorted(self.MAPS)}, got {map!r}")
        _check(_L.orion_lp_dc_cascade_set_map(self._h, self.MAPS[map]))
        return self


class FirDecimator(_Block):
    """dsp/decim.rs:24 FirDecimator::new(fs, m, cutoff_hz, trans_hz). channels>1: batched
    [nch, n] input (independent streams)."""

    def __init__(self, fs: float, m: int, cutoff_hz: float, trans_hz: float, channels: int = 1):
        h = (_L.orion_fir_decimator_new(fs, m, cutoff_hz, trans_hz) if channels == 1
             else _L.orion_fir_decimator_batch_new(fs, m, cutoff_hz, trans_hz, channels))
        super().__init__(h)


class FirLowpass(_Block):
    """dsp/fir.rs:16 FirLowpass::design(fs, pass_hz, trans_hz) (real f32 stream)."""

    def __init__(self, fs: float, pass_hz: float, trans_hz: float):
        super().__init__(_L.orion_fir_lowpass_new(fs, pass_hz, trans_hz))


class FirLowpassIq(_Block):
    """dsp/fir.rs:176-297. Use FirLowpassIq.design(...) or FirLowpassIq.from_taps(...)."""

    def __init__(self, handle):
        super().__init__(handle)

    @classmethod
    def design(cls, num_taps: int, cutoff_norm: float, stopband_db: float, channels: int = 1) -> "FirLowpassIq":
        """fir.rs:186-188; channels > 1: a batch of independent [channels, n] streams."""
        if channels == 1:
            return cls(_L.orion_fir_lowpass_iq_design(num_taps, cutoff_norm, stopband_db))
        return cls.from_taps(cls.design(num_taps, cutoff_norm, stopband_db).taps(), channels)

    @classmethod
    def from_taps(cls, taps, channels: int = 1) -> "FirLowpassIq":
        t = np.ascontiguousarray(taps, np.float32)
        if channels == 1:
            return cls(_L.orion_fir_lowpass_iq_from_taps(_fptr(t) if t.size else None, t.size))
        return cls(_L.orion_fir_lowpass_iq_batch_from_taps(_fptr(t) if t.size else None, t.size, channels))

    def num_taps(self) -> int:
        """fir.rs:210-212."""
        n = C.c_size_t(0)
        _check(_L.orion_fir_lowpass_iq_num_taps(self._h, C.byref(n)))
        return int(n.value)

    def group_delay(self) -> int:
        """fir.rs:216-218: (num_taps - 1) / 2."""
        d = C.c_size_t(0)
        _check(_L.orion_fir_lowpass_iq_group_delay(self._h, C.byref(d)))
        return int(d.value)

    def filter_aligned(self, io: np.ndarray) -> np.ndarray:
        """fir.rs:260-276, returns the filtered copy (time-aligned, same length)."""
        x = np.array(self._validate(io), copy=True)
        _check(_L.orion_fir_lowpass_iq_filter_aligned(self._h, x.ctypes.data, x.size))
        return x

    def filter_aligned_device(self, io, stream=None):
        """fir.rs:260-276 in place on a contiguous complex64 CUDA tensor (as the
        reference's `&mut [C32]`), asynchronous on `stream`. Returns io."""
        import torch

        if not io.is_cuda or not io.is_contiguous() or io.dtype != torch.complex64 or io.dim() != 1:
            raise ValueError("filter_aligned_device needs a contiguous 1-D complex64 CUDA tensor")
        s = stream if stream is not None else torch.cuda.current_stream(io.device).cuda_stream
        _check(_L.orion_fir_lowpass_iq_filter_aligned_device(self._h, io.data_ptr(), io.shape[0], s))
        return io


class LpCascade(_Block):
    """dsp/iir.rs:49 LpCascade::design(fs, fc) as an f32 stream block."""

    def __init__(self, fs: float, fc: float):
        super().__init__(_L.orion_lp_cascade_new(fs, fc))


class DcBlocker(_Block):
    """dsp/dc.rs:15 DcBlocker::new(fs, cut_hz)."""

    def __init__(self, fs: float, cut_hz: float):
        super().__init__(_L.orion_dc_blocker_new(fs, cut_hz))


# ---- demodulators (src/demodulate; PyO3 signatures src/python/demodulate.rs) ---
class CwEnvelopeDemod(_Block):
    def __init__(self, sample_rate: float, tone_hz: float, env_bw_hz: float):
        super().__init__(_L.orion_cw_envelope_demod_new(sample_rate, tone_hz, env_bw_hz))

    def set_gain(self, g: float):
        _check(_L.orion_cw_envelope_demod_set_gain(self._h, g))


class AmEnvelopeDemod(_Block):
    """abs_approx=True uses k1=0.9482, k2=0.3920 (src/python/demodulate.rs:46-53)."""

    def __init__(self, fs: float, audio_bw_hz: float, abs_approx: bool = False):
        super().__init__(_L.orion_am_envelope_demod_new(fs, audio_bw_hz))
        if abs_approx:
            _check(_L.orion_am_envelope_demod_with_abs_approx(self._h, 0.9482, 0.3920))

    def with_abs_approx(self, k1: float, k2: float) -> "AmEnvelopeDemod":
        _check(_L.orion_am_envelope_demod_with_abs_approx(self._h, k1, k2))
        return self


class SsbProductDemod(_Block):
    def __init__(self, fs: float, bfo_hz: float, audio_bw_hz: float, channels: int = 1):
        h = (_L.orion_ssb_product_demod_new(fs, bfo_hz, audio_bw_hz) if channels == 1
             else _L.orion_ssb_product_demod_batch_new(fs, bfo_hz, audio_bw_hz, channels))
        super().__init__(h)


class FmQuadratureDemod(_Block):
    def __init__(self, fs: float, dev_hz: float, audio_bw_hz: float):
        super().__init__(_L.orion_fm_quadrature_demod_new(fs, dev_hz, audio_bw_hz))

    def with_translate(self, freq_hz: float) -> "FmQuadratureDemod":
        _check(_L.orion_fm_quadrature_demod_with_translate(self._h, freq_hz))
        return self


class PmQuadratureDemod(_Block):
    def __init__(self, fs: float, k: float, audio_bw_hz: float):
        super().__init__(_L.orion_pm_quadrature_demod_new(fs, k, audio_bw_hz))


# ---- analog modulators (src/modulate): f32 audio -> complex64 IQ ----
class AgcRms(_Block):
    """dsp/agc.rs:20-31 AgcRms::new(fs, attack_ms, release_ms, target_rms): real audio AGC."""

    def __init__(self, fs: float, attack_ms: float, release_ms: float, target_rms: float):
        super().__init__(_L.orion_agc_rms_new(fs, attack_ms, release_ms, target_rms))


class AgcRmsIq(_Block):
    """dsp/agc.rs:93-106 AgcRmsIq::new(fs, attack_ms, release_ms, target_rms): one gain on I and Q."""

    def __init__(self, fs: float, attack_ms: float, release_ms: float, target_rms: float):
        super().__init__(_L.orion_agc_rms_iq_new(fs, attack_ms, release_ms, target_rms))


class AmDsbMod(_Block):
    """modulate/am.rs:20-36: carrier_level 1 -> full carrier (A3E), 0 -> DSB-SC."""

    def __init__(self, fs: float, rf_hz: float, carrier_level: float, modulation_index: float):
        super().__init__(_L.orion_am_dsb_mod_new(fs, rf_hz, carrier_level, modulation_index))

    def set_gain(self, g: float):
        _check(_L.orion_am_dsb_mod_set_gain(self._h, g))

    def set_clamp(self, on: bool):
        _check(_L.orion_am_dsb_mod_set_clamp(self._h, 1 if on else 0))


class FmPhaseAccumMod(_Block):
    """modulate/fm.rs:21-38 (deviation in Hz per unit input; rf_hz 0 for baseband)."""

    def __init__(self, sample_rate: float, deviation_hz: float, rf_hz: float = 0.0):
        super().__init__(_L.orion_fm_phase_accum_mod_new(sample_rate, deviation_hz, rf_hz))

    def set_deviation(self, deviation_hz: float):
        _check(_L.orion_fm_phase_accum_mod_set_deviation(self._h, deviation_hz))

    def set_gain(self, g: float):
        _check(_L.orion_fm_phase_accum_mod_set_gain(self._h, g))


class PmDirectPhaseMod(_Block):
    """modulate/pm.rs:17-47 (phase kp * x in radians; rf_hz 0 for baseband)."""

    def __init__(self, sample_rate: float, kp_rad_per_unit: float, rf_hz: float = 0.0):
        super().__init__(_L.orion_pm_direct_phase_mod_new(sample_rate, kp_rad_per_unit, rf_hz))

    def set_gain(self, g: float):
        _check(_L.orion_pm_direct_phase_mod_set_gain(self._h, g))

    def set_sensitivity(self, kp_rad_per_unit: float):
        _check(_L.orion_pm_direct_phase_mod_set_sensitivity(self._h, kp_rad_per_unit))


class CwKeyedMod(_Block):
    """modulate/cw.rs:21-87: keying envelope (0..1) -> keyed tone IQ."""

    def __init__(self, sample_rate: float, tone_hz: float, rise_ms: float, fall_ms: float):
        super().__init__(_L.orion_cw_keyed_mod_new(sample_rate, tone_hz, rise_ms, fall_ms))

    def set_gain(self, g: float):
        _check(_L.orion_cw_keyed_mod_set_gain(self._h, g))


class TxLowpass:
    """multicarrier/tx_lowpass.rs:88-195: the TX spectral-mask spec, its sizing helpers
    (the reference's f32 arithmetic, in the library) and apply() = filter_aligned of
    FirLowpassIq::design(num_taps, cutoff_norm, stopband_db) on the GPU."""

    def __init__(self, cutoff_norm: float, num_taps: int, stopband_db: float):
        self.cutoff_norm, self.num_taps, self.stopband_db = float(np.float32(cutoff_norm)), int(num_taps), \
            float(np.float32(stopband_db))

    def _spec(self):
        return C.byref(TxLowpassSpec(self.cutoff_norm, self.num_taps, self.stopband_db))

    @classmethod
    def for_null_band(cls, n_fft: int, occupied_half: int, num_taps: int, stopband_db: float) -> "TxLowpass":
        s = _L.orion_tx_lowpass_for_null_band(n_fft, occupied_half, num_taps, stopband_db)
        return cls(s.cutoff_norm, s.num_taps, s.stopband_db)

    @staticmethod
    def taps_for_null_band(n_fft: int, occupied_half: int, stopband_db: float) -> int:
        return int(_L.orion_tx_lowpass_taps_for_null_band(n_fft, occupied_half, stopband_db))

    def group_delay(self) -> int:
        return int(_L.orion_tx_lowpass_group_delay(self._spec()))

    def transition_norm(self) -> float:
        return float(_L.orion_tx_lowpass_transition_norm(self._spec()))

    def transition_fits(self, n_fft: int, occupied_half: int) -> bool:
        return bool(_L.orion_tx_lowpass_transition_fits(self._spec(), n_fft, occupied_half))

    def stopband_edge_norm(self) -> float:
        return float(_L.orion_tx_lowpass_stopband_edge_norm(self._spec()))

    def fits_guard(self, cp_len: int, roll_off: int, backoff: int) -> bool:
        return bool(_L.orion_tx_lowpass_fits_guard(self._spec(), cp_len, roll_off, backoff))

    def filter(self) -> "FirLowpassIq":
        return FirLowpassIq(_L.orion_tx_lowpass_filter(self._spec()))

    def apply(self, stream):
        """tx_lowpass.rs:192-195: filter_aligned across the whole stream. A numpy array
        is returned filtered (a copy); a contiguous complex64 CUDA tensor is filtered
        in place on the device."""
        f = self.filter()
        return f.filter_aligned_device(stream) if _is_torch(stream) else f.filter_aligned(stream)


class SsbPhasingMod(_Block):
    """modulate/ssb.rs:22-35."""

    def __init__(self, fs: float, audio_bw_hz: float, audio_if_hz: float, rf_hz: float = 0.0, usb: bool = True):
        super().__init__(_L.orion_ssb_phasing_mod_new(fs, audio_bw_hz, audio_if_hz, rf_hz, 1 if usb else 0))


class WbfmChain(_Block):
    """The WBFM chain of docs/demodulate.md:128-133, fused on the GPU.
    f_off: a float (one channel) or a sequence (one channel each; input [nch, n])."""

    def __init__(self, fs=10e6, f_off=1.5e6, m=8, dec_cutoff=200e3, dec_trans=79e3, dev_hz=75e3,
                 audio_bw=15e3, audio_pass=15e3, audio_trans=10e3):
        offs = np.atleast_1d(np.asarray(f_off, np.float32))
        p = WbfmParams(fs, float(offs[0]), dec_cutoff, dec_trans, dev_hz, audio_bw, audio_pass,
                       audio_trans, m)
        if np.ndim(f_off) == 0:
            h = _L.orion_wbfm_chain_new(C.byref(p))
        else:
            offs = np.ascontiguousarray(offs)
            h = _L.orion_wbfm_chain_batch_new(C.byref(p), _fptr(offs), offs.size)
        super().__init__(h)
        self.m = int(m)

    _PATHS = {"auto": 0, "segmented": 1, "split": 3, "graph": 4}

    def configure(self, path: str = "auto", max_segments: int = 0):
        """Engine tuning / tests (no reference counterpart): the kernel path and a
        cap on the segmented kernel's waves (include/orion_sdr_amd.h)."""
        _check(_L.orion_wbfm_chain_configure(self._h, self._PATHS[path], int(max_segments)))
        return self

    def seek(self, index: int):
        """Absolute index of the next input sample (the NCO phase origin);
        no reference counterpart (include/orion_sdr_amd.h orion_wbfm_chain_seek)."""
        _check(_L.orion_wbfm_chain_seek(self._h, int(index)))
        return self

    def process_shard(self, x_halo, start: int, halo_start: int):
        """One time shard of a stream (stream_shard): x_halo holds input
        samples [halo_start, stop). The handle is reset and sought to halo_start,
        runs the halo (which settles the decimator history, the discriminator's
        previous sample, the LpCascade state and the audio FIR history), and the
        audio of [start, stop) is returned: the same samples a single handle
        produces for the whole stream, up to the halo's settling residual."""
        self.reset()
        self.seek(halo_start)
        y = self.process(x_halo)
        return y[(start - halo_start) // self.m:]


# ---- time-sharded streams ----------------------------------------------
# Halo before a shard: 1024 audio samples at M = 8. The LpCascade forgets its
# zero start state within ~560 samples (||A^560|| < 1e-10 at 1.25 MHz, the host's
# own check uses ||A^896|| ~ 1e-16), the audio FIR then needs 124 settled
# samples, and the decimator 126 raw inputs; the rest is margin.
STREAM_HALO = 8192


def stream_shard(n: int, rank: int, world: int, m: int = 8, halo: int = STREAM_HALO):
    """Rank `rank` of `world`'s time slice of ONE n-sample stream: (start, stop,
    halo_start). Cuts fall on multiples of m (the decimator keeps inputs 0, m,
    2m, ... of every call, decim.rs:66-71), so the shards' outputs concatenate
    to the single-stream output; halo_start = max(0, start - halo)."""
    if not (0 <= rank < world) or n < 0 or halo % m:
        raise ValueError("stream_shard: bad rank/world/n/halo")
    units = n // m
    start = (units * rank // world) * m
    stop = n if rank == world - 1 else (units * (rank + 1) // world) * m
    return start, stop, max(0, start - halo)


# ---- chains (src/core.rs:24-109) and block graphs -------------------------------
class _Chain:
    """core.rs:24-109: a chain wraps one block and returns a new array per call.
    Deliberate divergence from the reference: the reference returns out[..n]
    (n = input length) even when the block wrote fewer samples (a decimator
    then leaks stale samples, core.rs:70-77); here the result is
    out[:out_written]."""

    _in = _out = None

    def __init__(self, block: _Block):
        if block._in is not self._in or block._out is not self._out:
            raise TypeError(f"{type(self).__name__} needs a {np.dtype(self._in).name} -> "
                            f"{np.dtype(self._out).name} block, got {block.name}")
        self.block = block

    def process(self, x):
        return self.block.process(x)

    process_ref = process

    def process_into(self, x: np.ndarray, out: np.ndarray) -> WorkReport:
        return self.block.process_into(x, out)


class AudioToIqChain(_Chain):
    """core.rs:24-53 (f32 -> cf32)."""
    _in, _out = np.float32, np.complex64


class IqToIqChain(_Chain):
    """core.rs:55-80 (cf32 -> cf32)."""
    _in, _out = np.complex64, np.complex64


class IqToAudioChain(_Chain):
    """core.rs:82-109 (cf32 -> f32)."""
    _in, _out = np.complex64, np.float32


class Graph:
    """A linear graph of blocks run back to back on the device: the input is
    staged to HBM once, every intermediate stays there (each stage's output is
    the next one's input, honouring out_written), and only the last output
    returns to the host. The user-composed chains of docs/demodulate.md:128-133
    (e.g. Rotator -> FirDecimator -> FmQuadratureDemod -> FirLowpass) run this
    way; blocks keep their streaming state across calls as usual."""

    def __init__(self, *blocks: _Block):
        if not blocks:
            raise ValueError("Graph needs at least one block")
        for a, b in zip(blocks, blocks[1:]):
            if a._out is not b._in:
                raise TypeError(f"{a.name} outputs {np.dtype(a._out).name}, {b.name} takes {np.dtype(b._in).name}")
        self.blocks = list(blocks)

    def process(self, x):
        import torch

        host = not _is_torch(x)
        if host:
            x = self.blocks[0]._validate(x)
            cur = torch.from_numpy(np.ascontiguousarray(x)).to("cuda")
        else:
            cur = x
        for b in self.blocks:
            cur = b.process_device(cur)
        return cur.cpu().numpy() if host else cur


# ---- designs (host) ----------------------------------------------------------
def fir_lowpass_design(fs: float, pass_hz: float, trans_hz: float) -> np.ndarray:
    n = _L.orion_fir_lowpass_design(fs, pass_hz, trans_hz, None, 0)
    t = np.zeros(n, np.float32)
    _L.orion_fir_lowpass_design(fs, pass_hz, trans_hz, _fptr(t), n)
    return t


def kaiser_lowpass_taps(num_taps: int, cutoff_norm: float, stopband_db: float) -> np.ndarray:
    n = _L.orion_kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db, None, 0)
    t = np.zeros(n, np.float32)
    _L.orion_kaiser_lowpass_taps(num_taps, cutoff_norm, stopband_db, _fptr(t), n)
    return t


def kaiser_transition_norm(num_taps: int, stopband_db: float) -> float:
    return _L.orion_kaiser_transition_norm(num_taps, stopband_db)


def kaiser_num_taps(transition_norm: float, stopband_db: float) -> int:
    return _L.orion_kaiser_num_taps(transition_norm, stopband_db)


def lp_cascade_design(fs: float, fc: float) -> np.ndarray:
    o = np.zeros(5, np.float32)
    _L.orion_lp_cascade_design(fs, fc, _fptr(o))
    return o


def diag_stream_read(x, stream: int = 0) -> int:
    """On-box bandwidth probe (no reference counterpart): one streaming read of the
    leading bytes of the device tensor x on `stream`; returns the bytes read."""
    nb = _L.orion_diag_stream_read_bytes(x.numel() * x.element_size())
    _check(_L.orion_diag_stream_read(C.c_void_p(x.data_ptr()), nb, C.c_void_p(stream)))
    return int(nb)


def diag_spin(stream: int, workgroups: int, lds_bytes: int, seconds: float):
    """Residency tests (no reference counterpart): `workgroups` one-wave workgroups each
    holding lds_bytes of LDS for `seconds` of wall clock, asynchronous on `stream`."""
    _check(_L.orion_diag_spin(C.c_void_p(stream), int(workgroups), int(lds_bytes), float(seconds)))


def diag_stream_create(n_cus: int = 0) -> int:
    """A HIP stream restricted to the first n_cus CUs (0: unrestricted); free it with
    diag_stream_destroy."""
    s = _L.orion_diag_stream_create(int(n_cus))
    if not s:
        raise OrionError(f"orion_sdr: stream creation failed: {_err()}")
    return int(s)


def diag_stream_destroy(stream: int):
    _check(_L.orion_diag_stream_destroy(C.c_void_p(stream)))


def device_cus() -> int:
    """Compute units of the current device."""
    return int(_L.orion_device_cus())


def set_spin_limit(polls: int):
    """Test-only: polls a cross-workgroup wait makes before it times out (process-wide;
    0 makes every such wait time out at once). include/orion_sdr_amd.h."""
    _L.orion_debug_set_spin_limit(int(polls))


def spin_limit() -> int:
    return int(_L.orion_debug_spin_limit())


def osc_table_phasors(freq_hz: float, fs: float, n: int, budget: int = 1 << 20):
    """Host only: the first n phasors of Rotator(freq_hz, fs) as the engine tabulates
    them (include/orion_sdr_amd.h orion_osc_table_phasors). Returns (phasors,
    cyc_start, cyc_len, n_tab)."""
    out = np.empty(int(n), np.complex64)
    cs, cl, nt = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
    _check(_L.orion_osc_table_phasors(freq_hz, fs, int(budget), out.ctypes.data, out.size, C.byref(cs),
                                      C.byref(cl), C.byref(nt)))
    return out, int(cs.value), int(cl.value), int(nt.value)


def pinned_empty(shape, dtype) -> np.ndarray:
    """A numpy array in pinned host memory (orion_host_alloc): the host-buffer path
    (orion_block_process) DMAs it without staging copies. Freed with the array."""
    import weakref

    dt = np.dtype(dtype)
    nbytes = int(np.prod(shape)) * dt.itemsize
    p = _L.orion_host_alloc(max(1, nbytes))
    if not p:
        raise OrionError(f"orion_sdr: pinned allocation failed: {_err()}")
    buf = (C.c_char * max(1, nbytes)).from_address(p)
    weakref.finalize(buf, _L.orion_host_free, C.c_void_p(p))
    return np.frombuffer(buf, dt, count=int(np.prod(shape))).reshape(shape)


def device_count() -> int:
    return _L.orion_device_count()


def version() -> str:
    return _L.orion_version().decode()
