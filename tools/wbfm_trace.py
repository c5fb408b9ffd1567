"""Per-wave phase timing of k_wbfm_seg (debug timestamps, s_memrealtime at 100 MHz):
runs the C2 workload with ORION_WBFM_TRACE set (the library then records, per segment,
the kernel start, sub-ranges 1-3's back start/end, the IIR / plane / FIR split of
sub-range 1's back, the end of the main loop, the end of the predecessor wait and the
end) and prints medians over the segments of the last launch.
  python tools/wbfm_trace.py [--n 67108864] [--launches 6]"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1 << 26)
    ap.add_argument("--launches", type=int, default=6)
    a = ap.parse_args()
    path = os.path.join("/tmp", f"wbfm_trace_{os.getpid()}.bin")
    os.environ["ORION_WBFM_TRACE"] = path
    sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
    import torch
    import orion_sdr

    dev = torch.device("cuda", 0)
    x = torch.randn(a.n, dtype=torch.complex64, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    blk = orion_sdr.WbfmChain(f_off=0.0)
    for _ in range(a.launches):
        blk.process_device(x)
    torch.cuda.synchronize()
    t = np.fromfile(path, dtype=np.int64).reshape(-1, 16).astype(np.float64) * 10e-3  # us
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    med = lambda v: float(np.median(v))  # noqa: E731
    rows = [
        ("start offset (segment start - first start)", t[:, 0] - t0),
        ("sub-range 1: IIR (iir16)", t[:, 10] - t[:, 4]),
        ("sub-range 1: f32 recurrence + f16 planes", t[:, 11] - t[:, 10]),
        ("sub-range 1: audio FIR (MFMA) + stores", t[:, 12] - t[:, 11]),
        ("  FIR: to step 0's MFMAs issued (frags, planes)", t[:, 13] - t[:, 11]),
        ("  FIR: steps 1-4 issued", t[:, 14] - t[:, 13]),
        ("  FIR: results, scale, stores issued", t[:, 12] - t[:, 14]),
        ("sub-range 1: whole back", t[:, 7] - t[:, 4]),
        ("sub-range 2: 8 front tiles", t[:, 5] - t[:, 7]),
        ("sub-range 3: 8 front tiles", t[:, 6] - t[:, 8]),
        ("main loop end -> predecessor's record", t[:, 2] - t[:, 1]),
        ("deferred back", t[:, 3] - t[:, 2]),
        ("segment total", t[:, 3] - t[:, 0]),
        ("kernel span (first start -> last end)", np.array([t[:, 3].max() - t0])),
    ]
    print(f"segments {len(t)}; n {a.n}")
    end = t[:, 3] - t0
    seg = np.arange(len(t))
    print("end time by XCD (blockIdx mod 8):", " ".join(f"{np.median(end[seg % 8 == x]):.1f}" for x in range(8)))
    print("end time by blockIdx decile:     ", " ".join(f"{np.median(end[(seg * 10) // len(t) == d]):.1f}"
                                                        for d in range(10)))
    print("segment total by decile:         ", " ".join(f"{np.median((t[:, 3] - t[:, 0])[(seg * 10) // len(t) == d]):.1f}"
                                                        for d in range(10)))
    print("end-time percentiles 50/90/99/max:", " ".join(f"{np.percentile(end, q):.1f}" for q in (50, 90, 99, 100)))
    for name, v in rows:
        print(f"{name:48s} median {med(v):8.2f} us  p10 {np.percentile(v, 10):8.2f}  p90 {np.percentile(v, 90):8.2f}")
    os.remove(path)


if __name__ == "__main__":
    main()
