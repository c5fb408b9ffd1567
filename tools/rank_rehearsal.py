"""Rehearsal of the driver's multi-GPU bench ranks on a one-GPU box (no N > 1 run is
possible there): builds the C2 stream-shard workload of the LAST rank of an N-GPU job
(its halo-sought handle and its input slice: the largest stream offsets and phase
indices), runs it, checks the output is finite and that a second handle sought to the
same halo start reproduces it bit for bit (the shard-vs-one-call parity itself is
tests/test_gpu_parity.py::test_wbfm_stream_shards); and prints the C3 / C4 / C5 channel
plans of the last rank.
  python tools/rank_rehearsal.py [--world 8]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
import bench  # noqa: E402
import orion_sdr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    W = args.world
    r = W - 1
    # C2, one stream of W x 2^26 samples cut in time: the last rank's shard
    blk, x, samples, bps, desc = bench.make_workload("c2", r, dev, None, W, "stream")
    out = torch.empty(blk.out_len(x.shape[-1]), dtype=torch.float32, device=dev)
    blk.process_device(x, out, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    o = out.cpu().numpy()
    assert np.isfinite(o).all(), "non-finite output"
    start, stop, h = orion_sdr.stream_shard(W * (1 << 26), r, W)
    # the same rank's audio from a handle sought to the halo start over the same input
    ref = orion_sdr.WbfmChain(f_off=bench.OFFSETS[0]).seek(h)
    out2 = torch.empty_like(out)
    ref.process_device(x, out2, torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    same = np.array_equal(o.view(np.uint32), out2.cpu().numpy().view(np.uint32))
    print(f"[rehearsal] c2 stream rank {r}/{W}: samples [{start}, {stop}) halo {start - h}, "
          f"{samples} per step, out {o.size} finite, repeat bit-identical {same}, rms {float(np.sqrt(np.mean(o ** 2))):.3e}")
    assert same
    del blk, x, out, out2, ref
    torch.cuda.empty_cache()
    for cfg in ("c3", "c4", "c5"):
        plan = bench.channel_plan(cfg, r, W)
        print(f"[rehearsal] {cfg} rank {r}/{W}: {len(plan)} channels, first {plan[0]}, last {plan[-1]}")
    print("[rehearsal] ok")


if __name__ == "__main__":
    main()
