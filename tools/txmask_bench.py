"""the OFDM/DVB-T TX mask (multicarrier/tx_lowpass.rs:188-195,
TxLowpass::apply = FirLowpassIq::design(num_taps, cutoff, stopband).filter_aligned)
timed on one MI355X at the reference's 45- and 89-tap masks, on a 2^24-sample cf32
stream resident in HBM: in-place filter_aligned on device memory, and the same FIR
as a streaming block. Algorithmic bytes: 8 in + 8 out per sample.
  python tools/txmask_bench.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import orion_sdr  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream(dev)
n, steps = 1 << 24, 10
g = torch.Generator(device=dev)
g.manual_seed(5)
x = torch.randn(n, dtype=torch.complex64, device=dev, generator=g)
y = torch.empty_like(x)


def timed(call):
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        call()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


for taps in (45, 89):
    f = orion_sdr.FirLowpassIq.design(taps, 0.2, 60.0)
    io = x.clone()
    ms = timed(lambda: orion_sdr._check(orion_sdr._L.orion_fir_lowpass_iq_filter_aligned_device(
        f._h, io.data_ptr(), n, st.cuda_stream)))
    ms_s = timed(lambda: f.process_device(x, y, st.cuda_stream))
    for mode, t in (("filter_aligned (in place)", ms), ("streaming process", ms_s)):
        print(json.dumps({"case": f"FirLowpassIq {taps} taps, {mode}", "n": n, "ms_per_call": round(t, 4),
                          "Msamples_per_s": round(n / t / 1e3, 1), "achieved_GBs": round(16 * n / t / 1e6, 1),
                          "frac_of_8TBs": round(16 * n / t / 1e6 / 8000, 3)}), flush=True)
