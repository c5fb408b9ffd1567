"""Throughput of the on-device analog modulators and of
the reference's own published kind of figure, a modulate -> demodulate round
trip, on one MI355X with inputs resident in HBM. One JSON line per case:
Msamples/s, per-launch kernel time from one HIP event pair around K
back-to-back calls on the launch stream, and the algorithmic bytes per sample
against the 8 TB/s HBM peak (4 B audio in + 8 B IQ out for a modulator).
  python tools/mod_bench.py [--n 67108864] [--steps 10]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import orion_sdr  # noqa: E402

PEAK = 8000.0


def timed(call, steps, stream):
    call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(steps):
        call()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps  # ms per call


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--only", default="", help="run only the cases whose name starts with this (no round trip)")
    ap.add_argument("--passes", type=int, default=0, help="orion_block_configure MOD_PASSES (0 single pass, 3)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    n = args.n
    t = torch.arange(n, device=dev, dtype=torch.float64)
    aud10 = (0.5 * torch.sin(2 * np.pi * 1e3 * t / 10e6) + 0.3 * torch.sin(2 * np.pi * 7e3 * t / 10e6)).float()
    aud48 = (0.5 * torch.sin(2 * np.pi * 1200.0 * t / 48e3)).float()
    del t
    iq = torch.empty(n, dtype=torch.complex64, device=dev)
    audio = torch.empty(n, dtype=torch.float32, device=dev)
    cases = [
        ("FmPhaseAccumMod(10e6, 75e3, 1.5e6)", orion_sdr.FmPhaseAccumMod(10e6, 75e3, 1.5e6), aud10, iq, 12.0),
        ("AmDsbMod(48e3, 12e3, 1.0, 0.8)", orion_sdr.AmDsbMod(48e3, 12e3, 1.0, 0.8), aud48, iq, 12.0),
        ("SsbPhasingMod(48e3, 2800, 1500, 0, usb)", orion_sdr.SsbPhasingMod(48e3, 2800.0, 1500.0), aud48, iq, 12.0),
    ]
    for name, blk, x, y, bps in cases:
        if args.only and not name.startswith(args.only):
            continue
        if args.passes and not name.startswith("Am"):
            blk.configure_option("mod_passes", args.passes)
        ms = timed(lambda: blk.process_device(x, y, sh), args.steps, st)
        print(json.dumps({"case": name, "n": n, "ms_per_call": round(ms, 4), "Msamples_per_s": round(n / ms / 1e3, 1),
                          "achieved_GBs": round(n * bps / ms / 1e6, 1), "frac_of_8TBs": round(n * bps / ms / 1e6 / PEAK, 3),
                          "bytes_per_sample": bps}), flush=True)
    if args.only:
        return
    # round trip (the reference's published kind of metric): FM mod -> WBFM chain
    mod = orion_sdr.FmPhaseAccumMod(10e6, 75e3, 1.5e6)
    chain = orion_sdr.WbfmChain(f_off=1.5e6)
    out = torch.empty(chain.out_len(n), dtype=torch.float32, device=dev)

    def rt():
        mod.process_device(aud10, iq, sh)
        chain.process_device(iq, out, sh)

    ms = timed(rt, args.steps, st)
    print(json.dumps({"case": "FmPhaseAccumMod -> WBFM chain round trip (10 Msps, dev 75 kHz, RF 1.5 MHz)", "n": n,
                      "ms_per_call": round(ms, 4), "Msamples_per_s": round(n / ms / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
