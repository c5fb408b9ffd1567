"""SURVEY §8e, C2 over several GPUs: ONE WBFM stream cut in time, each shard
processed from a halo of STREAM_HALO earlier samples. CPU only: the shard
arithmetic, the halo-settling property on the oracle (shards run from a fresh
state reproduce the single-call output), and the world_size-2 gloo path (each
rank runs its own shard, rank 0 concatenates). The GPU form of the same check
is test_gpu_parity.py::test_wbfm_stream_shards."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orion-sdr_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

from conftest import nrmse, report, wbfm_input  # noqa: E402
from orion_sdr import STREAM_HALO, stream_shard  # noqa: E402

N = 3 * (1 << 16) + 44  # ragged: not a multiple of 8


@pytest.mark.parametrize("n", [0, 7, 8, 8200, N, 1 << 26])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shards_cover_the_stream(n, world):
    prev = 0
    for r in range(world):
        start, stop, h = stream_shard(n, r, world)
        assert start == prev and start <= stop and start % 8 == 0
        assert 0 <= h <= start and start - h <= STREAM_HALO and h % 8 == 0
        assert h == max(0, start - STREAM_HALO)
        prev = stop
    assert prev == n


def test_bench_generates_a_shard_of_the_same_stream():
    """bench.py's rank slice (t0 = halo start) continues the stream's FM phase."""
    sys.path.insert(0, ROOT)
    import bench
    n, h = 40_000, 12_344
    full = bench.wbfm_iq(n, 1.5e6, torch.device("cpu"), 1, noise=0)[h:]
    part = bench.wbfm_iq(n - h, 1.5e6, torch.device("cpu"), 1, t0=h, noise=0)
    assert torch.max(torch.abs(full - part)).item() < 1e-5


def test_shard_arguments():
    with pytest.raises(ValueError):
        stream_shard(100, 2, 2)
    with pytest.raises(ValueError):
        stream_shard(100, 0, 1, halo=12)


def _shard_oracle(x, r, world):
    import oracle as O
    start, stop, h = stream_shard(len(x), r, world)
    # a fresh oracle chain on the halo + shard: its NCO starts at a different
    # phase, a constant factor the discriminator (z conj(prev)) cancels
    return O.wbfm(x[h:stop])[(start - h) // 8:]


@pytest.mark.parametrize("world", [2, 3])
def test_halo_settles_on_the_oracle(world):
    import oracle as O
    x = wbfm_input(N)
    full = O.wbfm(x)
    got = np.concatenate([_shard_oracle(x, r, world) for r in range(world)])
    assert len(got) == len(full)
    # The halo has settled (the residual is flat across each shard and does not
    # shrink with a longer halo); what remains is the f32 rounding of mixing from
    # another NCO phase, at the WBFM chain's rounding floor (~3e-6, the
    # discriminator amplifies last-bit differences): the end-to-end tolerance.
    report(f"oracle stream shards world={world} nrmse", nrmse(got, full), 1e-5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    x = wbfm_input(N)  # every rank holds the stream here; on GPUs a rank generates its slice only
    y = _shard_oracle(x, rank, world)
    gathered = [None] * world
    dist.all_gather_object(gathered, y.tolist())
    if rank == 0:
        q.put(gathered)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_two_ranks_rebuild_the_stream():
    import oracle as O
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got = np.concatenate([np.asarray(g, np.float32) for g in gathered])
    full = O.wbfm(wbfm_input(N))
    assert len(got) == len(full)
    report("gloo 2-rank stream shards nrmse", nrmse(got, full), 1e-5)
