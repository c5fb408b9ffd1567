"""CPU: TxLowpass (multicarrier/tx_lowpass.rs:88-195) sizing
helpers in the library (C ABI) equal the independent numpy f32 restatement
(tests/np_ref.py) bit for bit, over DVB-T-like and COFDM-like layouts. No kernel is
launched (filter()/apply() run in test_gpu_parity.py::test_tx_lowpass_apply)."""
import numpy as np
import pytest

import np_ref as R

LAYOUTS = [(2048, 852, 45, 60.0), (2048, 852, 89, 60.0), (64, 26, 31, 50.0), (256, 100, 15, 40.0),
           (1024, 500, 401, 80.0), (512, 255, 21, 30.0), (0, 0, 3, 10.0)]


@pytest.mark.parametrize("n_fft,occ,taps,a_db", LAYOUTS)
def test_for_null_band_and_helpers(n_fft, occ, taps, a_db):
    import orion_sdr

    t = orion_sdr.TxLowpass.for_null_band(n_fft, occ, taps, a_db)
    cut, nt, sb = R.tx_lowpass_for_null_band(n_fft, occ, taps, a_db)
    assert np.float32(t.cutoff_norm).view(np.uint32) == np.float32(cut).view(np.uint32)
    assert t.num_taps == nt and np.float32(t.stopband_db) == sb
    assert t.group_delay() == R.tx_lowpass_group_delay(taps)
    tn = R.kaiser_transition_norm(taps, a_db)
    assert np.float32(t.transition_norm()).view(np.uint32) == np.float32(tn).view(np.uint32)
    occ_n = np.float32(np.float32(occ) / np.float32(max(n_fft, 1)))
    assert t.transition_fits(n_fft, occ) == bool(tn <= np.float32(np.float32(0.5) - occ_n))
    edge = np.float32(np.float32(cut) + np.float32(np.float32(0.5) * tn))
    assert np.float32(t.stopband_edge_norm()).view(np.uint32) == edge.view(np.uint32)
    for cp, ro, bo in [(512, 0, 256), (512, 100, 256), (64, 0, 32), (64, 8, 0), (16, 0, 64), (2048, 16, 1024)]:
        assert t.fits_guard(cp, ro, bo) == R.tx_lowpass_fits_guard(taps, cp, ro, bo)
    assert orion_sdr.TxLowpass.taps_for_null_band(n_fft, occ, a_db) == R.tx_lowpass_taps_for_null_band(n_fft, occ, a_db)


def test_sizing_loop():
    """The reference's own sizing loop: the shortest length whose transition fits."""
    import orion_sdr

    for n_fft, occ in [(2048, 852), (64, 26), (256, 100)]:
        n = orion_sdr.TxLowpass.taps_for_null_band(n_fft, occ, 60.0)
        assert orion_sdr.TxLowpass.for_null_band(n_fft, occ, n, 60.0).transition_fits(n_fft, occ)
