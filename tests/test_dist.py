"""Multi-rank path on CPU (gloo, world_size 2): the bench's channel sharding and
its max-over-ranks timing, with the oracle standing in for the per-rank compute.
Sharding has no data-path collective: each rank's channels are
disjoint and processed independently, so the union of the ranks' outputs must
equal the single-process result channel for channel."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

N = 4096


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _channel_input(f_off, seed):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import conftest
    return conftest.wbfm_input(N, f_off=f_off, seed=seed)


def _channel_out(cfg, param, seed):
    """One channel's output through the oracle (the per-rank stand-in for the GPU)."""
    import bench
    import oracle as O
    if cfg == "c4":
        return O.wbfm(_channel_input(param, seed), f_off=param)
    x = bench.channel_input(cfg, N, seed, torch.device("cpu")).numpy()[None, :]
    if cfg == "c3":
        return O.decim_channels(x, 10e6, 8, 190e3, 39370.0, 1)[0]
    return O.ssb_demod_channels(x, 48e3, 1500.0, 2800.0, 1)[0]


def _rank_main(rank, world, port, q, cfg, sub):
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = bench.channel_plan(cfg, rank, world)
    outs = [_channel_out(cfg, p, s) for p, s in plan[:sub]]
    elapsed = bench.max_over_ranks(0.5 + rank, dist, torch.device("cpu"))
    gathered = [None] * world
    dist.all_gather_object(gathered, (plan, [o.tolist() for o in outs], elapsed))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg,per_rank,sub", [("c4", 8, 8), ("c3", 256, 3), ("c5", 128, 3)])
def test_sharded_channels_match_single_process(cfg, per_rank, sub):
    """C4 (8 WBFM channels per GPU), C3 (256 decimator channels per GPU) and C5 (128
    SSB channels per GPU): disjoint channel ranges, whole-job time = max over ranks,
    and each rank's outputs (the first `sub` channels of its plan, computed in its own
    process) equal the single-process outputs of the same channels."""
    import bench
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, cfg, sub)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = [s for plan, _, _ in gathered for _, s in plan]
    assert len(seeds) == world * per_rank and len(set(seeds)) == len(seeds), "ranks own disjoint channels"
    if cfg != "c4":  # contiguous global channel ranges
        idx = [p for plan, _, _ in gathered for p, _ in plan]
        assert idx == list(range(world * per_rank))
    assert all(e == pytest.approx(1.5) for _, _, e in gathered), "whole-job time is the max over ranks"
    for rank, (plan, outs, _) in enumerate(gathered):
        assert plan == bench.channel_plan(cfg, rank, world)
        for (p, s), o in zip(plan[:sub], outs):
            ref = _channel_out(cfg, p, s)
            np.testing.assert_array_equal(np.asarray(o, ref.dtype), ref)
