"""A/B timing of the FIR blocks at 2^24 samples (FirLowpassIq 127 taps, FirLowpass 125
taps): ms per process_device call, HIP events around 20 back-to-back calls, on whatever
library ORION_SDR_LIB points at (experiment variants, scripts/variants.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import orion_sdr  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 24
xc = torch.randn(n, dtype=torch.complex64, device=dev)
xr = torch.randn(n, dtype=torch.float32, device=dev)
s = torch.cuda.current_stream()
for name, blk, x in (("FirLowpassIq127", orion_sdr.FirLowpassIq.design(127, 0.2, 60.0), xc),
                     ("FirLowpass125", orion_sdr.FirLowpass(1.25e6, 15e3, 10e3), xr)):
    y = torch.empty_like(x)
    for _ in range(3):
        blk.process_device(x, y)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        blk.process_device(x, y)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"{name} ms/call {e0.elapsed_time(e1) / 20:.4f}")
