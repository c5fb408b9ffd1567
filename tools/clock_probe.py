"""Diagnostic: per-launch time over a long back-to-back run, for the C2 WBFM launch
and for a pure streaming read of the same input (torch sum over 512 MiB), to see
whether the slowdown after ~10 launches follows the kernel's own work (clock held
down under VALU load) or any HBM-saturating stream.

    python tools/clock_probe.py [K]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import bench  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 60
dev = torch.device("cuda", 0)
blk, x, n, bps, desc = bench.make_workload("c2", 0, dev)
out = torch.empty(n // 8, dtype=torch.float32, device=dev)
s = torch.cuda.current_stream(dev)
xf = torch.view_as_real(x).reshape(-1) if x.is_complex() else x.view(torch.float32)


def series(name, fn):
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(K + 1)]
    torch.cuda.synchronize()
    ev[0].record(s)
    for i in range(K):
        fn()
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    us = [1e3 * ev[i].elapsed_time(ev[i + 1]) for i in range(K)]
    groups = [sum(us[i:i + 10]) / len(us[i:i + 10]) for i in range(0, K, 10)]
    print(f"{name}: per-10-launch means (us): " + " ".join(f"{g:.1f}" for g in groups), flush=True)


acc = torch.empty((), dtype=torch.float32, device=dev)
for rep in range(2):
    series("wbfm", lambda: blk.process_device(x, out, s.cuda_stream))
    torch.cuda._sleep(int(2e8))  # ~0.1 s idle on the device
    torch.cuda.synchronize()
    series("sum ", lambda: torch.sum(xf, dim=0, out=acc))
    torch.cuda._sleep(int(2e8))
    torch.cuda.synchronize()
