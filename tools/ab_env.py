"""A/B timing of one BASELINE config under alternating environment settings that
the engine reads per launch (e.g. ORION_DW4_LIVE for the C3 decimator), in ONE
process with interleaved rounds: per round and setting, 10 back-to-back launches
between HIP events; prints the median per-launch time and the median difference
paired with the first setting's same round (the clock drifts between rounds).

    python tools/ab_env.py c3 ORION_DW4_LIVE=0 ORION_DW4_LIVE=1
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import bench  # noqa: E402

cfg, settings = sys.argv[1], sys.argv[2:]
dev = torch.device("cuda", 0)
blk, x, n, bps, desc = bench.make_workload(cfg, 0, dev)
nout = blk.out_len(x.shape[-1])  # as bench.py
out = torch.empty(x.shape[:-1] + (nout,), dtype=torch.complex64 if cfg == "c3" else torch.float32, device=dev)
s = torch.cuda.current_stream(dev)
res = {k: [] for k in settings}
for rnd in range(int(os.environ.get("AB_ROUNDS", "12"))):
    for kv in settings:
        k, _, v = kv.partition("=")
        os.environ[k] = v
        blk.process_device(x, out, s.cuda_stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(10):
            blk.process_device(x, out, s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        res[kv].append(1e3 * e0.elapsed_time(e1) / 10)
base = np.array(res[settings[0]][1:])
for kv in settings:
    v = np.array(res[kv][1:])
    print(f"{kv:24s} median {np.median(v):8.1f} us  paired diff {np.median(v - base):+6.1f} us  "
          f"({' '.join(f'{t:.0f}' for t in res[kv])})")
