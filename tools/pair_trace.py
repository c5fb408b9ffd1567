"""Debug: per-pair wait totals of k_wbfm_pair (ORION_WBFM_TRACE dump) on the C2 workload,
with the library variant in ORION_SDR_LIB. Words per pair r (s_memrealtime, 100 MHz):
A: 0 start, 1 staging total, 2 post total (no waits), 3 wait u_free, 4 wait f_ready, 5 wait p_free,
6 IIR total, 7 HW_ID;
B: 8 start, 9 loop done, 10 end, 11 wait u_ready, 12 wait f_free, 13 wait p_ready, 14 FIR, 15 HW_ID."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/pair_trace.bin"
os.environ["ORION_WBFM_TRACE"] = path
import orion_sdr  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 26
x = torch.randn(n, dtype=torch.complex64, device=dev)
out = torch.empty(n // 8, dtype=torch.float32, device=dev)
blk = orion_sdr.WbfmChain()
for _ in range(5):
    blk.process_device(x, out, torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize()
t = np.fromfile(path, dtype=np.int64).reshape(-1, 16)
t = t[(t[:, 0] > 0) & (t[:, 8] > 0)]
t0 = min(t[:, 0].min(), t[:, 8].min())
us = lambda v: v / 100.0  # noqa: E731
print(f"pairs {len(t)}  span {us(t[:, 10].max() - t0):.1f} us")
def row(name, v):
    print(f"  {name:28s} mean {v.mean():7.2f} p10 {np.percentile(v, 10):7.2f} p50 {np.median(v):7.2f} "
          f"p90 {np.percentile(v, 90):7.2f} max {v.max():7.2f}")
print("A:")
row("staging (sum)", us(t[:, 1]))
row("post (sum, no waits)", us(t[:, 2]))
row("IIR (sum)", us(t[:, 6]))
row("wait u_free", us(t[:, 3]))
row("wait f_ready", us(t[:, 4]))
row("wait p_free", us(t[:, 5]))
print("B:")
row("tile loop", us(t[:, 9] - t[:, 8]))
row("end", us(t[:, 10] - t0))
row("wait u_ready", us(t[:, 11]))
row("wait f_free", us(t[:, 12]))
row("wait p_ready", us(t[:, 13]))
row("in-loop FIR", us(t[:, 14]))
ha, hb = t[:, 7], t[:, 15]
simd = lambda h: (h >> 4) & 3  # noqa: E731
cu = lambda h: (h >> 8) & 15  # noqa: E731
se = lambda h: (h >> 13) & 7  # noqa: E731
same = (simd(ha) == simd(hb)) & (cu(ha) == cu(hb)) & (se(ha) == se(hb))
print(f"A and B on the same SIMD: {same.mean():.3f}; same CU: {((cu(ha) == cu(hb)) & (se(ha) == se(hb))).mean():.3f}")
print("A simd ids:", np.bincount(simd(ha), minlength=4), " B simd ids:", np.bincount(simd(hb), minlength=4))
