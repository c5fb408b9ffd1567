"""Summarise a k_wbfm_fused phase trace (ORION_WBFM_TRACE=<file> dump).

Each wave (range) records s_memrealtime (100 MHz) at:
  0 start, 1 front done, 2 zero-state pass + scan done, 3 hand-off done,
  4 pass 2 done, 5 FIR done.
Prints the per-phase duration distribution (microseconds), the dispatch
timeline (how many rounds of waves), and the kernel span.

  python scripts/trace_summary.py gpurun_out/trace.bin
"""
import sys

import numpy as np

PTS = 10
NAMES = ["front (N tiles)", "zero-state pass + scan", "publish + wait", "pass 2 + pair image",
         "audio FIR + store"]


SEG_NAMES = ["front + sub-range backs", "wait for predecessor", "sub-range 0 back"]


def main(path):
    global NAMES
    t = np.fromfile(path, dtype=np.int64)
    t = t[: len(t) // PTS * PTS].reshape(-1, PTS)
    if (t[:, 4] == 0).all():  # k_wbfm_seg: 4 points
        t, NAMES = t[:, :4], SEG_NAMES
    else:
        t = t[:, :6]
    t = t[(t > 0).all(axis=1)]
    if len(t) == 0:
        raise SystemExit("no complete wave records")
    us = (t - t[:, :1].min()) / 100.0  # 100 MHz ticks -> us from the first wave start
    E = t.shape[1] - 1
    print(f"waves: {len(t)}   kernel span: {us[:, E].max():.1f} us   (first start 0, last start "
          f"{us[:, 0].max():.1f} us)")
    d = np.diff(us, axis=1)
    print(f"{'phase':28s} {'mean':>8s} {'p10':>8s} {'p50':>8s} {'p90':>8s} {'max':>8s}  (us)")
    for i, n in enumerate(NAMES):
        c = d[:, i]
        print(f"{n:28s} {c.mean():8.2f} {np.percentile(c, 10):8.2f} {np.percentile(c, 50):8.2f} "
              f"{np.percentile(c, 90):8.2f} {c.max():8.2f}")
    tot = us[:, E] - us[:, 0]
    print(f"{'whole wave':28s} {tot.mean():8.2f} {np.percentile(tot, 10):8.2f} {np.percentile(tot, 50):8.2f} "
          f"{np.percentile(tot, 90):8.2f} {tot.max():8.2f}")
    starts = np.sort(us[:, 0])
    h, e = np.histogram(starts, bins=12)
    print("wave start histogram (us):")
    for k in range(len(h)):
        print(f"  {e[k]:8.1f} - {e[k + 1]:8.1f}: {h[k]}")


if __name__ == "__main__":
    main(sys.argv[1])
