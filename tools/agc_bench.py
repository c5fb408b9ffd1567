"""Times AgcRms / AgcRmsIq (dsp/agc.rs) on device-resident synthetic input (one JSON line per case).
Algorithmic bytes: 16 B per cf32 sample (8 in + 8 out), 8 B per f32 sample."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "orion-sdr_amd"))
import orion_sdr  # noqa: E402


def run(iq, fs, at, rl, tg, n, reps=10, steps=False):
    g = torch.Generator(device="cuda").manual_seed(5)
    dt = torch.complex64 if iq else torch.float32
    x = torch.randn(n, device="cuda", dtype=dt, generator=g)
    if steps:  # constant-envelope stretches (the serial re-run's worst case)
        lv = torch.tensor([1.0, 0.5, 0.8, 0.02], device="cuda")
        x = lv.repeat_interleave(n // 4 + 1)[:n].to(dt)
    blk = (orion_sdr.AgcRmsIq if iq else orion_sdr.AgcRms)(fs, at, rl, tg)
    out = blk.process_device(x)
    for _ in range(3):
        blk.process_device(x, out)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        blk.process_device(x, out)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    b = (16 if iq else 8) * n
    print(json.dumps({"case": f"{'AgcRmsIq' if iq else 'AgcRms'} fs={fs} attack={at}ms release={rl}ms"
                      + (" DC steps" if steps else " noise"),
                      "n": n, "warmup_W": int(blk.taps()[3]), "chunk_L": int(blk.taps(1)[0]),
                      "ms_per_call": round(ms, 4),
                      "Msamples_per_s": round(n / ms / 1e3, 1), "GB_per_s": round(b / ms / 1e6, 1),
                      "frac_hbm_8TBps": round(b / ms / 1e6 / 8000, 4)}), flush=True)


if __name__ == "__main__":
    n = 1 << 24
    for iq in (True, False):
        run(iq, 48e3, 0.2, 5.0, 0.2, n)
        run(iq, 48e3, 1.0, 20.0, 0.3, n)
        run(iq, 48e3, 1.0, 500.0, 0.3, n, reps=3)
        run(iq, 10e6, 0.2, 5.0, 0.5, n, reps=3)
    run(True, 48e3, 1.0, 20.0, 0.3, 1 << 20, reps=2, steps=True)
