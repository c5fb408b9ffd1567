"""Run-to-run spread of the streamed LpDcCascade parity figure (the DC look-back combines
a predecessor's prefix or its aggregates, whichever has been published: f64 rounding that
depends on timing). Same input as tests/test_gpu_parity.py::test_lp_dc_cascade.
  python tools/lpdc_repeat.py [--reps 6]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "orion-sdr_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=6)
    args = ap.parse_args()
    import oracle as O
    import orion_sdr as G

    O.lib()
    rng = np.random.default_rng(1234)
    n = 150_001
    x = (rng.standard_normal(n) + 0.25).astype(np.float32)
    fs, lp, dc = 48000.0, 2520.0, 2.0
    ref = O.lp_dc_cascade(x, fs, lp, dc, False)
    nr = lambda a: float(np.sqrt(np.mean((a - ref) ** 2)) / np.sqrt(np.mean(ref ** 2)))  # noqa: E731
    for rep in range(args.reps):
        one = G.LpDcCascade(fs, lp, dc).process(x)
        blk = G.LpDcCascade(fs, lp, dc)
        st = np.concatenate([blk.process(x[i:i + 33_333]) for i in range(0, n, 33_333)])
        print(f"rep {rep}: one call {nr(one):.4e}  streamed {nr(st):.4e}", flush=True)


if __name__ == "__main__":
    main()
