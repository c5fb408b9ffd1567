"""Debug: phase timestamps of k_wbfm_seg (the debug-only ORION_WBFM_TRACE dump) on
the C2 workload. Points per wave (s_memrealtime, 100 MHz): 0 start, 1 sub-range loop
done, 2 predecessor's record received, 3 end; 3 + s: sub-range s's tiles done,
6 + s: its back done (s = 1..3); 10, 11, 12: sub-range 1's zero-state pass + scan,
states + pass 2, audio FIR done.
  python tools/wbfm_trace.py [out.bin]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/wbfm_trace.bin"
os.environ["ORION_WBFM_TRACE"] = path
import orion_sdr  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 26
x = torch.randn(n, dtype=torch.complex64, device=dev)
out = torch.empty(n // 8, dtype=torch.float32, device=dev)
blk = orion_sdr.WbfmChain().configure("segmented", 0)
for _ in range(5):  # the last launch's trace is kept
    blk.process_device(x, out, torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize()
t = np.fromfile(path, dtype=np.int64).reshape(-1, 16)
t = t[(t[:, [0, 1, 3, 4, 5, 6, 7, 8, 9]] > 0).all(axis=1)]
us = (t - t[:, 0].min()) / 100.0
print(f"waves {len(t)}  span {us[:, 3].max():.1f} us  last start {us[:, 0].max():.1f} us")
ph = {
    "sub0+sub1 tiles": us[:, 4] - us[:, 0],
    "IIR sub1": us[:, 7] - us[:, 4],
    "sub2 tiles (+FIR1)": us[:, 5] - us[:, 7],
    "IIR sub2": us[:, 8] - us[:, 5],
    "sub3 tiles (+FIR2)": us[:, 6] - us[:, 8],
    "IIR sub3": us[:, 9] - us[:, 6],
    "loop end": us[:, 1] - us[:, 9],
    "wait succ": us[:, 2] - us[:, 1],
    "tail (IIR + 2 FIR)": us[:, 3] - us[:, 2],
    "whole": us[:, 3] - us[:, 0],
}
if (t[:, 10] > 0).all():  # sub-range 1's back split
    ph["  sub1 zero-state+scan"] = us[:, 10] - us[:, 4]
    ph["  sub1 states+pass2"] = us[:, 11] - us[:, 10]
    ph["  sub1 audio FIR"] = us[:, 12] - us[:, 11]
print(f"{'phase':22s} {'mean':>7s} {'p10':>7s} {'p50':>7s} {'p90':>7s} {'max':>7s}")
for k, v in ph.items():
    v = v[np.isfinite(v)]
    print(f"{k:22s} {v.mean():7.2f} {np.percentile(v, 10):7.2f} {np.percentile(v, 50):7.2f} "
          f"{np.percentile(v, 90):7.2f} {v.max():7.2f}")
r = np.nonzero((np.fromfile(path, dtype=np.int64).reshape(-1, 16)[:, [0, 1, 3, 4, 5, 6, 7, 8, 9]] > 0).all(axis=1))[0]
half = (r.max() + 1) // 2
for nm, m in (("early (r < grid/2)", r < half), ("late", r >= half)):
    e = us[m, 3]
    print(f"{nm:20s} end p10 {np.percentile(e, 10):.1f} p50 {np.median(e):.1f} max {e.max():.1f}")
for q in (4, 7, 5, 8, 6, 9, 1, 3):
    print(f"pt{q}: start-to-point p10/p50/p90 {np.percentile(us[:, q], 10):.1f} {np.percentile(us[:, q], 50):.1f} "
          f"{np.percentile(us[:, q], 90):.1f}")
# slowest waves: which phase is long, and where they sit
end = us[:, 3]
slow = end >= np.percentile(end, 95)
print(f"slowest 5% ({slow.sum()} waves, end >= {np.percentile(end, 95):.1f} us): phase means vs all")
for k, v in ph.items():
    print(f"  {k:22s} {v[slow].mean():7.2f} vs {v.mean():7.2f}")
rr = r[: len(us)]
print("end p50 by XCD (blockIdx % 8):", " ".join(f"{np.median(end[rr % 8 == x]):.1f}" for x in range(8)))
print("slow waves per XCD:", " ".join(str(int(slow[rr % 8 == x].sum())) for x in range(8)))
print("slow waves' start p50 / all:", f"{np.median(us[slow, 0]):.2f} / {np.median(us[:, 0]):.2f}")
raw = np.fromfile(path, dtype=np.int64).reshape(-1, 16)
if (raw[:, 14] > 0).any():  # segment geometry
    Lr = raw[r, 14]
    print("segment lengths: min/p50/max", Lr.min(), int(np.median(Lr)), Lr.max(),
          " by XCD (mean):", " ".join(f"{Lr[rr % 8 == x].mean():.0f}" for x in range(8)))
    sl = raw[r, 14][slow]
    print("slow waves' lengths:", np.unique(sl, return_counts=True))
