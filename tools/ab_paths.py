"""A/B timing of the WBFM kernel paths in ONE process, interleaved rounds
(guide rule 24): per round and path, 10 back-to-back launches between HIP
events; prints the median and min per-launch time per path."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import bench  # noqa: E402

paths = sys.argv[1].split(",") if len(sys.argv) > 1 else ["segmented", "segmented_v1", "ranges"]
cfg = sys.argv[2] if len(sys.argv) > 2 else "c2"
dev = torch.device("cuda", 0)
blk, x, n, bps, desc = bench.make_workload(cfg, 0, dev)
out = torch.empty(x.shape[:-1] + (x.shape[-1] // 8,), dtype=torch.float32, device=dev)
s = torch.cuda.current_stream(dev)
res = {p: [] for p in paths}
for rnd in range(int(os.environ.get("AB_ROUNDS", "6"))):
    for p in paths:
        spec, _, xv = p.partition("@")  # "@<bits>": k_wbfm_seg4's alternate variant (ORION_SEG4_X_LIVE)
        os.environ["ORION_SEG4_X_LIVE"] = xv or "-1"
        name, _, ms = spec.partition(":")
        blk.configure(name, int(ms or 0))
        blk.process_device(x, out, s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            blk.process_device(x, out, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        res[p].append(1e3 * e0.elapsed_time(e1) / 10)
base = np.array(res[paths[0]][1:])
for p in paths:
    v = np.array(res[p][1:])
    d = np.median(v - base)  # paired with the first path's same round (the clock drifts between rounds)
    print(f"{p:14s} median {np.median(v):7.1f} us  min {v.min():7.1f} us  paired diff {d:+6.1f} us  "
          f"({' '.join(f'{t:.0f}' for t in res[p])})")
