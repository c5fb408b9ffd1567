"""Quick check of a WBFM library variant (ORION_SDR_LIB) against the oracle, with a
short hand-off spin limit so that a protocol bug times out instead of hanging:
  ORION_SDR_LIB=... python tools/wbfm_smoke_lib.py [log2 n] [spin]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "orion-sdr_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401
import orion_sdr  # noqa: E402
import oracle as O  # noqa: E402
from conftest import nrmse, wbfm_input  # noqa: E402

n = 1 << (int(sys.argv[1]) if len(sys.argv) > 1 else 22)
orion_sdr.set_spin_limit(int(sys.argv[2]) if len(sys.argv) > 2 else 20000)
x = wbfm_input(n, f_off=150e3, seed=7)
blk = orion_sdr.WbfmChain(f_off=150e3)
y = blk.process(x)
st = blk.status()
ref = O.wbfm(x, f_off=150e3)
print(f"n={n} status={st} nrmse={nrmse(y, ref):.3e} len {len(y)} vs {len(ref)}", flush=True)
# streamed in two calls
ok = not st and nrmse(y, ref) < 1e-5
for cut in (n // 3 & ~7,):
    blk2 = orion_sdr.WbfmChain(f_off=150e3)
    y2 = np.concatenate([blk2.process(x[:cut]), blk2.process(x[cut:])])
    e = nrmse(y2[: len(ref)], ref) if len(y2) >= len(ref) else float("nan")
    print(f"two calls at {cut}: status={blk2.status()} len {len(y2)} nrmse={e:.3e}", flush=True)
    ok = ok and not blk2.status() and e < 1e-5
sys.exit(0 if ok else 1)
