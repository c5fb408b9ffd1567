"""Experiment: does the WBFM kernel's per-wave speed depend on where the input
sits in device memory? Runs the C2 chain with the phase trace on the same IQ
placed (a) as generated, (b) at the start and (c) at the end of a fresh 1 GiB
buffer, (d) in a fresh buffer allocated after a 2 GiB spacer, and prints the
front-phase mean per eighth of the channel."""
import os
import shutil
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import bench  # noqa: E402
import orion_sdr  # noqa: E402

tr = os.environ["ORION_WBFM_TRACE"]
dev = torch.device("cuda", 0)
n = 1 << 26
x0 = bench.wbfm_iq(n, 1.5e6, dev, 0x1234)
out = torch.empty(n // 8, dtype=torch.float32, device=dev)
blk = orion_sdr.WbfmChain(f_off=1.5e6)
s = torch.cuda.current_stream(dev)


def run(x, tag):
    for _ in range(3):
        blk.process_device(x, out, s.cuda_stream)
    torch.cuda.synchronize()
    t = np.fromfile(tr, dtype=np.int64).reshape(-1, 10)[:2048, :4]
    us = (t - t[:, :1].min()) / 100.0
    d = us[:, 1] - us[:, 0]
    e8 = [round(float(d[k * 256:(k + 1) * 256].mean()), 1) for k in range(8)]
    print(f"{tag:10s} span {us[:, 3].max():6.1f}  front by eighth {e8}  addr {x.data_ptr():#x}", flush=True)


run(x0, "as-is")
big = torch.empty(2 * n, dtype=torch.complex64, device=dev)
big[:n] = x0
run(big[:n], "big-lo")
big[n:] = x0
run(big[n:], "big-hi")
sp = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
x2 = x0.clone()
run(x2, "after-2G")
