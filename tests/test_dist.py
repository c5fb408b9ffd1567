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


def _rank_main(rank, world, port, q):
    import bench
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = bench.channel_plan("c4", rank, world)
    outs = [O.wbfm(_channel_input(f, s), f_off=f) for f, s in plan]
    elapsed = bench.max_over_ranks(0.5 + rank, dist, torch.device("cpu"))
    gathered = [None] * world
    dist.all_gather_object(gathered, (plan, [o.tolist() for o in outs], elapsed))
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_channels_match_single_process():
    import bench
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    seeds = [s for plan, _, _ in gathered for _, s in plan]
    assert len(seeds) == 16 and len(set(seeds)) == 16, "ranks own disjoint channels"
    assert all(e == pytest.approx(1.5) for _, _, e in gathered), "whole-job time is the max over ranks"
    for rank, (plan, outs, _) in enumerate(gathered):
        assert plan == bench.channel_plan("c4", rank, world)
        for (f, s), o in zip(plan, outs):
            ref = O.wbfm(_channel_input(f, s), f_off=f)
            np.testing.assert_array_equal(np.asarray(o, np.float32), ref)
