"""Diagnostic: host enqueue time per WBFM launch vs GPU time per launch (events),
for K back-to-back launches, and the same through a captured HIP graph."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
blk, x, n, bps, desc = bench.make_workload("c2", 0, dev)
out = torch.empty(n // 8, dtype=torch.float32, device=dev)
s = torch.cuda.current_stream(dev)
for _ in range(3):
    blk.process_device(x, out, s.cuda_stream)
torch.cuda.synchronize()
for K in (10, 50):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(s)
    for _ in range(K):
        blk.process_device(x, out, s.cuda_stream)
    e1.record(s)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"K={K}: host enqueue {1e6 * (t1 - t0) / K:.1f} us/launch, wall {1e6 * (t2 - t0) / K:.1f} us/launch, "
          f"events {1e3 * e0.elapsed_time(e1) / K:.1f} us/launch", flush=True)
