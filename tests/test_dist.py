"""Multi-rank path (gloo, world_size 2): the bench's channel sharding and its
max-over-ranks timing. On CPU the oracle stands in for the per-rank compute; with a
GPU visible (`-m gpu`) both ranks run the HIP blocks on device 0 and are checked
against the oracle. Sharding has no data-path collective: each rank's
channels are disjoint and processed independently, so the union of the ranks'
outputs must equal the single-process result channel for channel."""
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


def _cpu_input(cfg, seed):
    """A channel's input on the host, from its seed (C3 complex noise; C5 the oracle's
    SsbPhasingMod of 1.2 kHz plus AWGN: the bench builds the same shape on the device)."""
    import oracle as O
    rng = np.random.default_rng(seed)
    w = (rng.standard_normal(N) + 1j * rng.standard_normal(N)).astype(np.complex64)
    if cfg == "c3":
        return w
    a = (0.5 * np.sin(2 * np.pi * 1200.0 * np.arange(N) / 48e3)).astype(np.float32)
    return (O.ssb_mod(a, 48e3, 2800.0, 1500.0) + np.float32(np.sqrt(1e-3 / 2)) * w).astype(np.complex64)


def _channel_out(cfg, param, seed):
    """One channel's output through the oracle (the per-rank stand-in for the GPU)."""
    import bench
    import oracle as O
    if cfg == "c4":
        return O.wbfm(_channel_input(param, seed), f_off=param)
    x = _cpu_input(cfg, seed)[None, :]
    if cfg == "c3":
        return O.decim_channels(x, *bench.C3_DESIGN, 1)[0]
    return O.ssb_demod_channels(x, 48e3, 1500.0, 2800.0, 1)[0]


def _hip_outs(cfg, plan):
    """The rank's channels through the HIP blocks on device 0 (the bench's own inputs and
    batched blocks), each channel beside the oracle's output on the same input: returns
    [(nrmse, tol)] per channel."""
    import bench
    import oracle as O
    sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
    import orion_sdr
    dev = torch.device("cuda", 0)
    if cfg == "c4":
        x = torch.stack([bench.wbfm_iq(N * 16, f, dev, s) for f, s in plan]).contiguous()
        got = orion_sdr.WbfmChain(f_off=[f for f, _ in plan]).process_device(x).cpu().numpy()
        xh = x.cpu().numpy()
        refs = [O.wbfm(xh[c], f_off=f) for c, (f, _) in enumerate(plan)]
        tol = 1e-5
    else:
        x = torch.stack([bench.channel_input(cfg, N, s, dev) for _, s in plan]).contiguous()
        blk = (orion_sdr.FirDecimator(*bench.C3_DESIGN, channels=len(plan)) if cfg == "c3"
               else orion_sdr.SsbProductDemod(48e3, 1500.0, 2800.0, channels=len(plan)))
        got = blk.process_device(x).cpu().numpy()
        xh = x.cpu().numpy()
        refs = list(O.decim_channels(xh, *bench.C3_DESIGN, 1) if cfg == "c3"
                    else O.ssb_demod_channels(xh, 48e3, 1500.0, 2800.0, 1))
        tol = 1e-6 if cfg == "c3" else 2e-5
    out = []
    for g, r in zip(got, refs):
        d = np.asarray(g, np.complex128) - r
        out.append((float(np.sqrt(np.mean(np.abs(d) ** 2)) / np.sqrt(np.mean(np.abs(r.astype(np.complex128)) ** 2))),
                    tol))
    return out


def _rank_main(rank, world, port, q, cfg, sub, hip=False):
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    plan = bench.channel_plan(cfg, rank, world)
    if hip:
        outs = _hip_outs(cfg, plan[:sub])
        elapsed = bench.max_over_ranks(0.5 + rank, dist, torch.device("cpu"))
        gathered = [None] * world
        dist.all_gather_object(gathered, (plan, outs, elapsed))
        if rank == 0:
            q.put(gathered)
        dist.barrier()
        dist.destroy_process_group()
        return
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


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,sub", [("c4", 2), ("c3", 8), ("c5", 8)])
def test_sharded_channels_on_the_gpu(cfg, sub):
    """the same two-rank sharding with each rank's channels through
    the HIP blocks (both ranks on device 0, gloo for the barrier / max), each rank's
    channels against the oracle on the same input."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q, cfg, sub, True)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(e == pytest.approx(1.5) for _, _, e in gathered), "whole-job time is the max over ranks"
    for rank, (plan, errs, _) in enumerate(gathered):
        for (param, _), (err, tol) in zip(plan[:sub], errs):
            print(f"[parity] {cfg} rank {rank} channel {param} HIP vs oracle nrmse {err:.3e} (tol {tol:.0e})")
            assert err <= tol
