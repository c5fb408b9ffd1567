"""A/B of k_wbfm_seg build variants (orion-sdr_amd/exp/<name>/liborion_sdr_amd.so,
built by scripts/build_variant.sh from a git revision) on the C2 workload: each variant runs in its own
process (ORION_SDR_LIB), rounds interleaved so that clock drift hits every variant
alike; per process W warm-up and K timed launches, HIP events around each launch
on the launch stream. Prints per-variant medians over rounds.
  python tools/wbfm_exp.py [--rounds R] [--k K] name ...     ("base" = lib/)"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(k, w, nch, n):
    import torch
    sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
    import orion_sdr
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn((nch, n) if nch > 1 else (n,), dtype=torch.complex64, device=dev, generator=g)
    out = torch.empty((nch, n // 8) if nch > 1 else (n // 8,), dtype=torch.float32, device=dev)
    blk = orion_sdr.WbfmChain(f_off=[0.0] * nch if nch > 1 else 0.0)
    s = torch.cuda.current_stream(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
    for _ in range(w):
        blk.process_device(x, out, s.cuda_stream)
    for a, b in ev:
        a.record(s)
        blk.process_device(x, out, s.cuda_stream)
        b.record(s)
    torch.cuda.synchronize()
    t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
    print(json.dumps({"med": t[len(t) // 2], "min": t[0], "mean": sum(t) / len(t)}))


def multi(names, k, w, nch, n, maxseg=0):
    """All variants in ONE process (each library loaded as its own module), launches
    interleaved A B C, B C A, ... so that the chip's clock state hits every variant
    alike; HIP events around each launch."""
    import importlib.util
    import torch
    mods = {}
    for nm in names:  # "lib" or "lib@segments" (the segmented kernel's segment count)
        lib = nm.split("@")[0]
        if lib in {k.split("@")[0]: 0 for k in mods}:
            mods[nm] = next(v for k, v in mods.items() if k.split("@")[0] == lib)
            continue
        os.environ["ORION_SDR_LIB"] = (os.path.join(ROOT, "orion-sdr_amd", "lib", "liborion_sdr_amd.so") if lib == "base"
                                       else os.path.join(ROOT, "orion-sdr_amd", "exp", lib, "liborion_sdr_amd.so"))
        spec = importlib.util.spec_from_file_location(f"orion_sdr_{lib}",
                                                      os.path.join(ROOT, "orion-sdr_amd", "orion_sdr", "__init__.py"))
        m = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(m)
        mods[nm] = m
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn((nch, n) if nch > 1 else (n,), dtype=torch.complex64, device=dev, generator=g)
    out = torch.empty((nch, n // 8) if nch > 1 else (n // 8,), dtype=torch.float32, device=dev)
    blks = {nm: m.WbfmChain(f_off=[0.0] * nch if nch > 1 else 0.0) for nm, m in mods.items()}
    for nm, b in blks.items():
        segs = int(nm.split("@")[1]) if "@" in nm else maxseg
        if segs:
            b.configure("segmented", segs)
    s = torch.cuda.current_stream(dev)
    for _ in range(w):
        for b in blks.values():
            b.process_device(x, out, s.cuda_stream)
    ev = {nm: [] for nm in names}
    for it in range(k):
        order = names[it % len(names):] + names[:it % len(names)]
        for nm in order:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            blks[nm].process_device(x, out, s.cuda_stream)
            b.record(s)
            ev[nm].append((a, b))
    torch.cuda.synchronize()
    for nm in names:
        t = sorted(a.elapsed_time(b) * 1e3 for a, b in ev[nm])
        print(f"{nm:12s} med {t[len(t) // 2]:7.1f} p25 {t[len(t) // 4]:7.1f} min {t[0]:7.1f} mean {sum(t) / len(t):7.1f} us",
              flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("names", nargs="*")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--w", type=int, default=5)
    ap.add_argument("--nch", type=int, default=1)
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--multi", action="store_true", help="all variants in one process, launches interleaved")
    ap.add_argument("--maxseg", type=int, default=0, help="cap on the segmented kernel's waves")
    a = ap.parse_args()
    if a.child:
        return child(a.k, a.w, a.nch, a.n)
    if a.multi:
        for r in range(a.rounds):
            print(f"-- round {r}", flush=True)
            multi(a.names, a.k, a.w, a.nch, a.n, a.maxseg)
        return None
    res = {nm: [] for nm in a.names}
    for r in range(a.rounds):
        for nm in (a.names if r % 2 == 0 else a.names[::-1]):
            env = dict(os.environ)
            if nm != "base":
                env["ORION_SDR_LIB"] = os.path.join(ROOT, "orion-sdr_amd", "exp", nm, "liborion_sdr_amd.so")
            p = subprocess.run([sys.executable, __file__, "--child", "--k", str(a.k), "--w", str(a.w),
                                "--nch", str(a.nch), "--n", str(a.n)], env=env, capture_output=True, text=True,
                               timeout=300)
            if p.returncode != 0:
                print(nm, "FAILED", p.returncode, p.stderr[-2000:], flush=True)
                sys.exit(1)
            v = json.loads(p.stdout.strip().splitlines()[-1])
            res[nm].append(v)
            print(f"round {r} {nm:12s} med {v['med']:7.1f} min {v['min']:7.1f} mean {v['mean']:7.1f} us", flush=True)
    for nm, v in res.items():
        meds = sorted(x["med"] for x in v)
        print(f"{nm:12s} median-of-medians {meds[len(meds) // 2]:7.1f} us  (all {' '.join(f'{m:.1f}' for m in meds)})")


if __name__ == "__main__":
    main()
