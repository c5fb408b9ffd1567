"""Where two builds of the WBFM chain differ: runs lib/ ("base") and an experiment build
(orion-sdr_amd/exp/<name>) on the tests' C2-like input, default and many-segment
configurations, and prints the pairwise nrmse and the largest differences with their
positions inside tiles (128 outputs), sub-ranges (1024) and segments.
  python tools/wbfm_diff.py NAME [--n LOG2] [--segs S]"""
import argparse
import importlib.util
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def load(lib):
    os.environ["ORION_SDR_LIB"] = (os.path.join(ROOT, "orion-sdr_amd", "lib", "liborion_sdr_amd.so") if lib == "base"
                                   else os.path.join(ROOT, "orion-sdr_amd", "exp", lib, "liborion_sdr_amd.so"))
    spec = importlib.util.spec_from_file_location(f"orion_sdr_{lib}", os.path.join(ROOT, "orion-sdr_amd", "orion_sdr", "__init__.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def nrmse(a, b):
    return float(np.sqrt(np.mean((a - b) ** 2)) / np.sqrt(np.mean(b ** 2)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("name")
    ap.add_argument("--n", type=int, default=25)
    ap.add_argument("--segs", type=int, default=4096)
    ap.add_argument("--oracle", action="store_true")
    args = ap.parse_args()
    import torch
    from conftest import wbfm_input
    x = wbfm_input(1 << args.n)
    xd = torch.from_numpy(x).cuda()
    out = {}
    for lib in ("base", args.name):
        m = load(lib)
        out[lib] = m.WbfmChain().process_device(xd).cpu().numpy()
        out[lib + "#2"] = m.WbfmChain().process_device(xd).cpu().numpy()
        out[lib + "@segs"] = m.WbfmChain().configure("segmented", args.segs).process_device(xd).cpu().numpy()
    if args.oracle:
        import oracle as O
        out["oracle"] = O.wbfm(x)
    keys = list(out)
    for i in range(len(keys)):
        for j in range(i + 1, len(keys)):
            print(f"{keys[i]:>16s} vs {keys[j]:<16s} nrmse {nrmse(out[keys[i]], out[keys[j]]):.3e}")
    for a, b in ((f"{args.name}", "base"), ("base@segs", "base"), (f"{args.name}@segs", args.name)):
        d = np.abs(out[a] - out[b])
        top = np.argsort(d)[-12:][::-1]
        rms = np.sqrt(np.mean(out[b] ** 2))
        print(f"-- {a} - {b}: largest |diff| / rms, index, index mod 128 / 1024")
        for t in top:
            print(f"   {d[t] / rms:.3e} at {t} ({t % 128}, {t % 1024})")
        # error energy by position in the sub-range
        e = (out[a] - out[b]) ** 2
        prof = e[: len(e) // 1024 * 1024].reshape(-1, 1024).mean(axis=0)
        q = np.argsort(prof)[-6:][::-1]
        print("   worst sub-range positions:", [(int(p), f"{prof[p] / np.mean(e):.1f}x") for p in q])


if __name__ == "__main__":
    main()
