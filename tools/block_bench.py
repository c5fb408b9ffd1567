"""Per-block throughput of every SURVEY §8(a) row on one MI355X, inputs resident
in HBM, beside the scalar oracle (1 thread, bounded prefix) on this host.

One JSON line per block: Msamples/s (input samples), ms per call from one HIP
event pair around K back-to-back process_device calls on the launch stream,
the algorithmic bytes per input sample (input + output, nothing else) and the
fraction of the 8 TB/s HBM peak they imply; for the FIR blocks also the
algorithmic FP32 flops per input sample (2 per real multiply-add: 2 x taps for a
real FIR, 4 x taps for real taps on complex data, divided by the decimation) and
the fraction of the packed-FP32 peak (157.3 TFLOP/s) they imply, with "bound" the
larger of the two fractions' resources; and the oracle's single-thread
Msamples/s on the first `--cpu-n` samples of the same input ("port" of the
reference Rust, which is single-threaded). The oracle is test infrastructure:
it is timed here as the CPU baseline only, never as the measured path.
  python tools/block_bench.py [--n 16777216] [--steps 10] [--cpu-n 1048576]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import orion_sdr  # noqa: E402
import oracle as O  # noqa: E402  (CPU baseline only)

PEAK = 8000.0      # GB/s, HBM3E
PEAK_FP32 = 157.3  # TFLOP/s, packed FP32 (v_pk_fma_f32), MI355X_MICROARCH.md


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


def cpu_rate(fn, x):
    t0 = time.perf_counter()
    fn(x)
    return len(x) / (time.perf_counter() - t0) / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 24)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--cpu-n", type=int, default=1 << 20)
    ap.add_argument("--rows", default="", help="comma-separated rows to run (default: all)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the oracle timing")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    n = args.n
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    t = torch.arange(n, device=dev, dtype=torch.float64)
    tone = torch.polar(torch.ones_like(t), 2 * np.pi * 0.03 * t).to(torch.complex64)
    iq = (0.5 * tone + 0.1 * torch.randn(n, dtype=torch.complex64, device=dev, generator=g)).contiguous()
    real = (0.5 * torch.sin(2 * np.pi * 0.01 * t) + 0.1 * torch.randn(n, dtype=torch.float64, device=dev,
                                                                       generator=g)).float().contiguous()
    del t, tone
    iq_h = iq[: args.cpu_n].cpu().numpy()
    real_h = real[: args.cpu_n].cpu().numpy()
    taps127 = O.kaiser_lowpass_taps(127, 0.2, 60.0)
    # (row, constructor text, block, input, bytes per input sample, oracle call[, flops per input sample])
    cases = [
        ("a1", "Rotator(-1.5e6, 10e6)", orion_sdr.Rotator(-1.5e6, 10e6), iq, 16.0,
         lambda x: O.rotator(x, -1.5e6, 10e6)),
        ("a3", "FirLowpass(1.25e6, 15e3, 10e3) [125 taps]", orion_sdr.FirLowpass(1.25e6, 15e3, 10e3), real, 8.0,
         lambda x: O.fir_lowpass(x, 1.25e6, 15e3, 10e3), 2.0 * 125),
        ("a4", "FirDecimator(10e6, 8, 200e3, 79e3) [127 taps]", orion_sdr.FirDecimator(10e6, 8, 200e3, 79e3), iq,
         9.0, lambda x: O.fir_decimator(x, 10e6, 8, 200e3, 79e3), 4.0 * 127 / 8),
        ("a5", "FirLowpassIq.design(127, 0.2, 60)", orion_sdr.FirLowpassIq.design(127, 0.2, 60.0), iq, 16.0,
         lambda x: O.fir_lowpass_iq(x, taps127), 4.0 * 127),
        ("a6", "LpCascade(1.25e6, 13.5e3)", orion_sdr.LpCascade(1.25e6, 13.5e3), real, 8.0,
         lambda x: O.lp_cascade(x, 1.25e6, 13.5e3)),
        ("a7", "DcBlocker(48e3, 2)", orion_sdr.DcBlocker(48e3, 2.0), real, 8.0,
         lambda x: O.dc_blocker(x, 48e3, 2.0)),
        ("a9", "FmQuadratureDemod(1.25e6, 75e3, 15e3)", orion_sdr.FmQuadratureDemod(1.25e6, 75e3, 15e3), iq, 12.0,
         lambda x: O.fm_demod(x, 1.25e6, 75e3, 15e3)),
        ("a10", "SsbProductDemod(48e3, 1500, 2800)", orion_sdr.SsbProductDemod(48e3, 1500.0, 2800.0), iq, 12.0,
         lambda x: O.ssb_demod(x, 48e3, 1500.0, 2800.0)),
        ("a11", "AmEnvelopeDemod(48e3, 5e3) PowerSqrt", orion_sdr.AmEnvelopeDemod(48e3, 5e3), iq, 12.0,
         lambda x: O.am_demod(x, 48e3, 5e3)),
        ("a11", "AmEnvelopeDemod(48e3, 5e3) AbsApprox", orion_sdr.AmEnvelopeDemod(48e3, 5e3, abs_approx=True), iq,
         12.0, lambda x: O.am_demod(x, 48e3, 5e3, abs_approx=(0.9482, 0.3920))),
        ("a12", "PmQuadratureDemod(48e3, 1.0, 5e3)", orion_sdr.PmQuadratureDemod(48e3, 1.0, 5e3), iq, 12.0,
         lambda x: O.pm_demod(x, 48e3, 1.0, 5e3)),
        ("a12", "CwEnvelopeDemod(48e3, 700, 100)", orion_sdr.CwEnvelopeDemod(48e3, 700.0, 100.0), iq, 12.0,
         lambda x: O.cw_demod(x, 48e3, 700.0, 100.0)),
    ]
    rows = set(args.rows.split(",")) if args.rows else None
    for row, name, blk, x, bps, ref, *fl in cases:
        if rows and row not in rows:
            continue
        out = torch.empty(blk.out_len(n), dtype=torch.complex64 if blk._out is np.complex64 else torch.float32,
                          device=dev)
        ms = timed(lambda: blk.process_device(x, out, sh), args.steps, st)
        xh = iq_h if x is iq else real_h
        cpu = 0.0 if args.no_cpu else cpu_rate(ref, xh)
        rec = {"row": row, "block": name, "n": n, "ms_per_call": round(ms, 4),
               "Msamples_per_s": round(n / ms / 1e3, 1), "bytes_per_sample": bps,
               "achieved_GBs": round(n * bps / ms / 1e6, 1),
               "frac_of_8TBs": round(n * bps / ms / 1e6 / PEAK, 3)}
        if fl:
            tf = n * fl[0] / ms / 1e9
            rec.update({"flop_per_sample": fl[0], "achieved_TFLOPs": round(tf, 2),
                        "frac_of_157TF": round(tf / PEAK_FP32, 3),
                        "bound": "fp32" if tf / PEAK_FP32 > rec["frac_of_8TBs"] else "hbm"})
        rec.update({"cpu_oracle_Msamples_per_s": round(cpu, 2), "cpu_sample": len(xh), "cpu_threads": 1})
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
