"""Cost of retuning an oscillator between calls (an AFC or a scanning
receiver calls set_freq per block). A Rotator runs calls of n samples on
HBM-resident buffers, with set_freq before every call (alternating
between two tunings, so every call starts a new tune) and without; wall time per
call after a stream sync, median of many calls. The retune is lazy
(osc.cpp RefOsc::retune): the next call tabulates the reference recurrence on the
host for that call's outputs only (incrementally, ~n steps: one dependent f32 rotation
per output, ~5 ns on the host core) and uploads them; with nco_table 0 (the closed form,
<= 1e-6 from the exact rotation) a retune costs nothing.
  python tools/retune_bench.py [--calls 200]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import orion_sdr as O  # noqa: E402


def per_call(blk, x, y, calls, retune):
    st = torch.cuda.current_stream()
    tunes = (1.234e6, -0.987e6)
    ts = []
    for i in range(calls):
        t0 = time.perf_counter()
        if retune:
            blk.set_freq(tunes[i & 1], 10e6)
        blk.process_device(x, y, st.cuda_stream)
        st.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    return ts[len(ts) // 2] * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for n in (4096, 65536, 1 << 20):
        x = torch.randn(n, dtype=torch.complex64, device=dev)
        y = torch.empty_like(x)
        blk = O.Rotator(1.234e6, 10e6)
        per_call(blk, x, y, 20, False)
        base = per_call(blk, x, y, a.calls, False)
        blk = O.Rotator(1.234e6, 10e6)
        per_call(blk, x, y, 20, True)
        ret = per_call(blk, x, y, a.calls, True)
        blk = O.Rotator(1.234e6, 10e6).configure_option("nco_table", 0)  # the closed form
        per_call(blk, x, y, 20, True)
        cf = per_call(blk, x, y, a.calls, True)
        print(json.dumps({"case": "Rotator set_freq before every call", "n": n, "us_per_call_no_retune": round(base, 1),
                          "us_per_call_retune": round(ret, 1), "retune_cost_us": round(ret - base, 1),
                          "retune_cost_per_output_ns": round((ret - base) * 1e3 / n, 2),
                          "us_per_call_retune_closed_form": round(cf, 1)}), flush=True)


if __name__ == "__main__":
    main()
