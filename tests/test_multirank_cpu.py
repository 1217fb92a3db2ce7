"""N > 1 path of bench.py on CPU with gloo (world_size 2): replica sharding of the shifts and the
max-over-ranks timing reduction (the only collective; the data path has none)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    seeds = bench.shard_seeds(rank, world, 8)
    el = bench.max_over_ranks(1.0 + rank, "cpu")
    gathered = [None] * world
    dist.all_gather_object(gathered, seeds)
    q.put((rank, seeds, el, gathered))
    dist.destroy_process_group()


def test_two_rank_sharding_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    all_seeds = sorted(s for _, seeds, _, _ in res for s in seeds)
    assert all_seeds == list(range(1000, 1016))           # 64 at N=8; here 2 x 8, disjoint, complete
    assert all(el == 2.0 for _, _, el, _ in res)           # max over ranks
    assert res[0][3] == res[1][3]


def test_single_rank_helpers_without_process_group():
    import bench
    assert bench.shard_seeds(0, 1, 8) == list(range(1000, 1008))
    assert bench.max_over_ranks(3.5, "cpu") == 3.5


def _ysq_worker(rank, world, port, q):
    """C5 layout: each rank transforms its own outputs and forms its partial Y; one all-reduce."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastgaussianprocesses_amd.distributed import allreduce_sum_, output_shard
    from oracle.fgp_oracle import fftbr, ft_stable
    torch.manual_seed(5)
    y = torch.randn(7, 64, dtype=torch.float64)          # 7 outputs, n = 64 (same on every rank)
    a, b = output_shard(7, rank, world)
    yt = ft_stable(y[a:b], fftbr)
    ysq = (yt.abs() ** 2).sum(0)
    allreduce_sum_(ysq)
    q.put((rank, (a, b), ysq.numpy().copy()))   # (by value: a tensor would travel as a shared fd, lost at exit)
    dist.destroy_process_group()


def test_two_rank_multi_output_ysq_allreduce():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ysq_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1] for r in res] == [(0, 4), (4, 7)]
    from oracle.fgp_oracle import fftbr, ft_stable
    torch.manual_seed(5)
    y = torch.randn(7, 64, dtype=torch.float64)
    full = (ft_stable(y, fftbr).abs() ** 2).sum(0)
    r0, r1 = torch.from_numpy(res[0][2]), torch.from_numpy(res[1][2])
    assert torch.equal(r0, r1)                             # every rank holds the same Y
    assert torch.allclose(r0, full, rtol=1e-13, atol=0)


def test_output_shard_partition():
    from fastgaussianprocesses_amd.distributed import output_shard
    for total in (8, 9, 512, 513):
        for world in (1, 2, 3, 8):
            rng = [output_shard(total, r, world) for r in range(world)]
            assert rng[0][0] == 0 and rng[-1][1] == total
            assert all(rng[i][1] == rng[i + 1][0] for i in range(world - 1))
            assert max(b - a for a, b in rng) - min(b - a for a, b in rng) <= 1
