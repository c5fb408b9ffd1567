"""Debug: phase timestamps of one WBFM launch on a given kernel path
(ORION_WBFM_TRACE), summarised by scripts/trace_summary.py.
  python tools/ws_trace.py specialized [out.bin]"""
import os
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
path = sys.argv[2] if len(sys.argv) > 2 else "/tmp/wbfm_trace.bin"
os.environ["ORION_WBFM_TRACE"] = path
import orion_sdr  # noqa: E402

dev = torch.device("cuda", 0)
n = 1 << 26
x = torch.randn(n, dtype=torch.complex64, device=dev)
out = torch.empty(n // 8, dtype=torch.float32, device=dev)
blk = orion_sdr.WbfmChain().configure(sys.argv[1] if len(sys.argv) > 1 else "specialized", 0)
for _ in range(5):  # the last launch's trace is kept
    blk.process_device(x, out, torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize()
sys.exit(subprocess.call([sys.executable, os.path.join(ROOT, "scripts", "trace_summary.py"), path]))
