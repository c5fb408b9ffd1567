"""The reference's own published analog figures (docs/performance.md:18-23, "Analog modes
(65536 samples x 30 passes)") reproduced on one MI355X: a modulate -> demodulate round
trip per mode, in the harness shape of tests/performance/throughput/{cw,am,pm,ssb,fm}.rs
(fs 48 kHz, n = 65536 per pass, 30 passes (SSB 20), Msps = n * passes / wall time):

  host      AudioToIqChain(mod).process(host audio) -> IqToAudioChain(demod).process(host iq),
            i.e. orion_block_process on host slices twice per pass (the drop-in's path:
            what a Rust `impl Block` would call; H2D + kernel + D2H each);
  device    the same 65536-sample calls on HBM-resident tensors (no PCIe);
  batched   one 1024 x 65536 = 2^26-sample call per block and pass (HBM-resident): the
            device's throughput when the call is large enough to fill it;
  cpu       the oracle (scalar C restatement of the reference, 1 thread) on the same passes.

Each line also carries the round trip's nrmse against the oracle on the first pass.
  python tools/roundtrip_bench.py [--modes CW,FM] [--batched-n 67108864]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-sdr_amd"), os.path.join(ROOT, "oracle")]
import orion_sdr as O  # noqa: E402

FS = 48_000.0
N = 65_536
REF_MSPS = {"CW": 137, "AM-PowerSqrt": 107, "PM": 125, "SSB-USB": 138, "FM": 103, "AM-AbsApprox": 79}  # M2 Pro


def real_tone(f_hz, n, amp):
    """tests/performance/throughput/mod.rs:7-11 (f32 phase, as the reference)."""
    k = np.arange(n, dtype=np.float32)
    return (np.float32(amp) * np.sin(np.float32(2 * np.pi) * np.float32(f_hz) * k / np.float32(FS))).astype(np.float32)


def key_square(key_hz, n):
    """mod.rs:13-17."""
    k = np.arange(n, dtype=np.float32)
    return (np.modf(k * np.float32(key_hz) / np.float32(FS))[0] < 0.5).astype(np.float32)


def modes():
    """(name, audio, passes, make tx, make rx, oracle round trip) per reference harness."""
    import oracle as R

    return [
        ("CW", key_square(5.0, N), 30, lambda: O.CwKeyedMod(FS, 700.0, 3.0, 3.0),
         lambda: O.CwEnvelopeDemod(FS, 700.0, 300.0),
         lambda a: R.cw_demod(R.cw_mod(a, FS, 700.0, 3.0, 3.0), FS, 700.0, 300.0)),
        ("AM-PowerSqrt", real_tone(1000.0, N, 0.5), 30, lambda: O.AmDsbMod(FS, 0.0, 0.8, 0.5),
         lambda: O.AmEnvelopeDemod(FS, 5000.0),
         lambda a: R.am_demod(R.am_mod(a, FS, 0.0, 0.8, 0.5), FS, 5000.0)),
        ("PM", real_tone(900.0, N, 0.5), 30, lambda: O.PmDirectPhaseMod(FS, 0.9, 0.0),
         lambda: O.PmQuadratureDemod(FS, 0.9, 5000.0),
         lambda a: R.pm_demod(R.pm_mod(a, FS, 0.9), FS, 0.9, 5000.0)),
        ("SSB-USB", real_tone(1200.0, N, 0.4), 20, lambda: O.SsbPhasingMod(FS, 2800.0, 1500.0, 0.0, True),
         lambda: O.SsbProductDemod(FS, 0.0, 2800.0),
         lambda a: R.ssb_demod(R.ssb_mod(a, FS, 2800.0, 1500.0, 0.0, True), FS, 0.0, 2800.0)),
        ("FM", real_tone(1000.0, N, 0.5), 30, lambda: O.FmPhaseAccumMod(FS, 2500.0, 0.0),
         lambda: O.FmQuadratureDemod(FS, 2500.0, 5000.0),
         lambda a: R.fm_demod(R.fm_mod(a, FS, 2500.0), FS, 2500.0, 5000.0)),
        ("AM-AbsApprox", real_tone(1000.0, N, 0.5), 30, lambda: O.AmDsbMod(FS, 0.0, 0.8, 0.5),
         lambda: O.AmEnvelopeDemod(FS, 5000.0).with_abs_approx(0.9475, 0.3925),
         lambda a: R.am_demod(R.am_mod(a, FS, 0.0, 0.8, 0.5), FS, 5000.0, abs_approx=(0.9475, 0.3925))),
    ]


def nrmse(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.sqrt(np.mean((a - b) ** 2)) / max(np.sqrt(np.mean(b ** 2)), 1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="")
    ap.add_argument("--batched-n", type=int, default=1024 * N)
    ap.add_argument("--batched-passes", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    sh = st.cuda_stream
    want = set(args.modes.split(",")) if args.modes else None
    for name, audio, passes, mk_tx, mk_rx, oracle_rt in modes():
        if want and name not in want:
            continue
        line = {"case": f"{name} round trip", "fs": FS, "n": N, "passes": passes, "reference_msps_m2pro": REF_MSPS[name]}
        # host slices, the reference's harness shape
        tx, rx = O.AudioToIqChain(mk_tx()), O.IqToAudioChain(mk_rx())
        first = rx.process(tx.process(audio.copy()))
        line["nrmse_vs_oracle_first_pass"] = nrmse(first, oracle_rt(audio))
        tx, rx = O.AudioToIqChain(mk_tx()), O.IqToAudioChain(mk_rx())
        rx.process(tx.process(audio.copy()))  # warm-up (allocations, tables)
        t0 = time.perf_counter()
        for _ in range(passes):
            out = rx.process(tx.process(audio.copy()))
        dt = time.perf_counter() - t0
        assert len(out) == N
        line["host_msps"] = round(N * passes / dt / 1e6, 2)
        # device-resident, same call size
        tx, rx = mk_tx(), mk_rx()
        a_d = torch.from_numpy(audio).to(dev)
        iq = torch.empty(N, dtype=torch.complex64, device=dev)
        y = torch.empty(N, dtype=torch.float32, device=dev)
        tx.process_device(a_d, iq, sh)
        rx.process_device(iq, y, sh)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(passes):
            tx.process_device(a_d, iq, sh)
            rx.process_device(iq, y, sh)
        torch.cuda.synchronize()
        line["device_msps"] = round(N * passes / (time.perf_counter() - t0) / 1e6, 2)
        # batched: 2^26-sample calls (the same tone, tiled)
        nb = args.batched_n
        tx, rx = mk_tx(), mk_rx()
        ab = a_d.repeat(nb // N)
        iqb = torch.empty(nb, dtype=torch.complex64, device=dev)
        yb = torch.empty(nb, dtype=torch.float32, device=dev)
        tx.process_device(ab, iqb, sh)
        rx.process_device(iqb, yb, sh)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(args.batched_passes):
            tx.process_device(ab, iqb, sh)
            rx.process_device(iqb, yb, sh)
        e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.batched_passes
        line["batched_n"] = nb
        line["batched_msps"] = round(nb / ms / 1e3, 1)
        line["batched_ms_per_pass"] = round(ms, 4)
        del ab, iqb, yb
        # the oracle, 1 thread, the reference's passes
        t0 = time.perf_counter()
        for _ in range(passes):
            oracle_rt(audio)
        line["cpu_oracle_msps_1thread"] = round(N * passes / (time.perf_counter() - t0) / 1e6, 2)
        line["host_vs_reference"] = round(line["host_msps"] / REF_MSPS[name], 2)
        line["batched_vs_reference"] = round(line["batched_msps"] / REF_MSPS[name], 1)
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
