"""Paired in-process A/B of library variants on one workload: every variant
(orion-sdr_amd/exp/<name>/liborion_sdr_amd.so, built by scripts/build_variant.sh; "base"
= lib/) is loaded as its own module, launches are interleaved A B C, B C A, ... so the
chip's clock state hits every variant alike, one HIP event pair per launch.
  python tools/ab_variants.py --case c5 --rounds 4 --k 10 base v1 v2
A name may carry engine options for its block: base@scan_path=2 (orion_block_configure),
base@wbfm_path=split (WbfmChain.configure).
Cases: c1 (FirLowpassIq 127 taps 2^20), c2 (WBFM 2^26), c3 (FirDecimator 255 taps, 256 x 2^20), c4 (WBFM 8 x 2^24), c5 (SSB 128 x 2^20; c5b: bench.py's tone + noise input), a4 (FirDecimator 127 taps 2^24), a10 (SSB 2^24), a11 / a11abs (AM PowerSqrt / AbsApprox 2^24), a7 (DcBlocker
2^24), a6 (LpCascade 2^24), a9 (FM demod 2^24), a3 (FirLowpass 125 taps 2^24), fmmod (FmPhaseAccumMod 2^26), a5 (FirLowpassIq 127 taps 2^24), c5fir (batched
FirLowpassIq 128 x 2^20)."""
import argparse
import importlib.util
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name):
    os.environ["ORION_SDR_LIB"] = (os.path.join(ROOT, "orion-sdr_amd", "lib", "liborion_sdr_amd.so") if name == "base"
                                   else os.path.join(ROOT, "orion-sdr_amd", "exp", name, "liborion_sdr_amd.so"))
    spec = importlib.util.spec_from_file_location(f"orion_sdr_{name}",
                                                  os.path.join(ROOT, "orion-sdr_amd", "orion_sdr", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def case(m, name, dev):
    g = torch.Generator(device=dev).manual_seed(1)
    if name == "c2":
        return m.WbfmChain(f_off=0.0), torch.randn(1 << 26, dtype=torch.complex64, device=dev, generator=g)
    if name == "c4":
        return m.WbfmChain(f_off=[0.0] * 8), torch.randn(8, 1 << 24, dtype=torch.complex64, device=dev, generator=g)
    if name == "c5":
        return (m.SsbProductDemod(48e3, 1500.0, 2800.0, channels=128),
                torch.randn(128, 1 << 20, dtype=torch.complex64, device=dev, generator=g))
    if name == "c5b":  # C5 with bench.py's input (a 2.7 kHz USB tone + noise per channel)
        t = torch.arange(1 << 20, device=dev, dtype=torch.float64) / 48e3
        tone = torch.polar(torch.ones_like(t), 2 * 3.141592653589793 * 2700.0 * t).to(torch.complex64) * 0.4
        x = tone + 0.03 * torch.randn(128, 1 << 20, dtype=torch.complex64, device=dev, generator=g)
        return m.SsbProductDemod(48e3, 1500.0, 2800.0, channels=128), x.contiguous()
    if name == "c3":
        return (m.FirDecimator(10e6, 8, 190e3, 39370.0, channels=256),
                torch.randn(256, 1 << 20, dtype=torch.complex64, device=dev, generator=g))
    if name == "a4":
        return (m.FirDecimator(10e6, 8, 200e3, 79e3),
                torch.randn(1 << 24, dtype=torch.complex64, device=dev, generator=g))
    if name == "c1":  # BASELINE configs[0]: FirLowpassIq 127 taps on 2^20 samples
        return (m.FirLowpassIq.design(127, 0.2, 60.0),
                torch.randn(1 << 20, dtype=torch.complex64, device=dev, generator=g))
    if name == "fmmod":  # FmPhaseAccumMod (10 MHz, 75 kHz, RF 1.5 MHz) on 2^26 audio samples
        return m.FmPhaseAccumMod(10e6, 75e3, 1.5e6), torch.randn(1 << 26, dtype=torch.float32, device=dev, generator=g) * 0.5
    if name == "a5":  # FirLowpassIq 127 taps on 2^24 samples
        return (m.FirLowpassIq.design(127, 0.2, 60.0),
                torch.randn(1 << 24, dtype=torch.complex64, device=dev, generator=g))
    if name == "c5fir":  # C5F's channel filter: batched FirLowpassIq 127 taps, 128 x 2^20
        return (m.FirLowpassIq.from_taps(m.FirLowpassIq.design(127, 3000.0 / 48e3, 60.0).taps(), channels=128),
                torch.randn(128, 1 << 20, dtype=torch.complex64, device=dev, generator=g))
    if name == "a3":
        return m.FirLowpass(1.25e6, 15e3, 10e3), torch.randn(1 << 24, dtype=torch.float32, device=dev, generator=g)
    if name == "a10":
        return m.SsbProductDemod(48e3, 1500.0, 2800.0), torch.randn(1 << 24, dtype=torch.complex64, device=dev, generator=g)
    if name == "a11":
        return m.AmEnvelopeDemod(48e3, 5e3), torch.randn(1 << 24, dtype=torch.complex64, device=dev, generator=g)
    if name == "a11abs":
        return (m.AmEnvelopeDemod(48e3, 5e3, abs_approx=True),
                torch.randn(1 << 24, dtype=torch.complex64, device=dev, generator=g))
    if name == "a7":
        return m.DcBlocker(48e3, 2.0), torch.randn(1 << 24, dtype=torch.float32, device=dev, generator=g)
    if name == "a6":
        return m.LpCascade(1.25e6, 13.5e3), torch.randn(1 << 24, dtype=torch.float32, device=dev, generator=g)
    if name == "a9":
        return (m.FmQuadratureDemod(48e3, 2500.0, 5000.0),
                torch.randn(1 << 24, dtype=torch.complex64, device=dev, generator=g))
    raise SystemExit(f"unknown case {name}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="+")
    ap.add_argument("--case", default="c2")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--w", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev)
    libs = {}
    work = {}
    for nm in a.names:
        lib, *opts = nm.split("@")
        if lib not in libs:
            libs[lib] = load(lib)
        m = libs[lib]
        blk, x = case(m, a.case, dev) if not work else (case(m, a.case, dev)[0], next(iter(work.values()))[1])
        for o in opts:
            k, v = o.split("=")
            if k == "wbfm_path":  # WbfmChain kernel path: segmented / split / graph
                blk.configure(v)
            elif k == "wbfm_segs":  # the segmented kernel with this many segments (waves)
                blk.configure("segmented", int(v))
            else:
                blk.configure_option(k, int(v))
        out = blk.process_device(x)
        work[nm] = (blk, x, out)
    for nm in a.names:
        blk, x, out = work[nm]
        for _ in range(a.w):
            blk.process_device(x, out, s.cuda_stream)
    for r in range(a.rounds):
        ev = {nm: [] for nm in a.names}
        for it in range(a.k):
            order = a.names[it % len(a.names):] + a.names[:it % len(a.names)]
            for nm in order:
                blk, x, out = work[nm]
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                blk.process_device(x, out, s.cuda_stream)
                e1.record(s)
                ev[nm].append((e0, e1))
        torch.cuda.synchronize()
        print(f"-- round {r}", flush=True)
        for nm in a.names:
            t = sorted(e0.elapsed_time(e1) * 1e3 for e0, e1 in ev[nm])
            print(f"{nm:12s} med {t[len(t) // 2]:7.1f} p25 {t[len(t) // 4]:7.1f} min {t[0]:7.1f} "
                  f"mean {sum(t) / len(t):7.1f} us", flush=True)


if __name__ == "__main__":
    main()
