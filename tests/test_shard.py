"""Multi-GPU sharding path exercised on CPU with gloo, world_size 2/3.

The kernels need a GPU, so these tests check the data path around them: every image is
processed exactly once, slices are contiguous and ordered, the host gather reassembles
the batch bit-exactly, and bench.py's timing reduction takes the max over ranks.
"""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rpst.shard import gather_to_host, partition, shard_apply


@pytest.mark.parametrize("n,world", [(32, 1), (32, 2), (33, 2), (128, 8), (5, 8), (0, 3)])
def test_partition_covers_exactly_once(n, world):
    seen = []
    prev_end = 0
    for r in range(world):
        s, e = partition(n, world, r)
        assert s == prev_end and e >= s
        assert e - s in (n // world, n // world + 1)
        seen.extend(range(s, e))
        prev_end = e
    assert seen == list(range(n))


def test_partition_rejects_bad_rank():
    with pytest.raises(ValueError):
        partition(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(0)
        batch = torch.rand(n, 3, 4, 4, generator=g)  # every rank sees the same batch
        # per-image "stylisation": independent per image, so sharding must be exact
        local = shard_apply(lambda x: x * 2.0 + x.sum(dim=(1, 2, 3), keepdim=True), batch,
                            world, rank)
        full = gather_to_host(local)
        # bench.py's timing reduction: MAX over ranks
        t = torch.tensor([float(rank + 1)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if rank == 0:
            ref = batch * 2.0 + batch.sum(dim=(1, 2, 3), keepdim=True)
            q.put((torch.equal(full, ref), float(t.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 32), (2, 7), (3, 10)])
def test_gloo_shard_and_gather(world, n):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.spawn(_worker, args=(world, port, n, q), nprocs=world, join=True)
    ok, tmax = q.get(timeout=60)
    assert ok
    assert tmax == float(world)


def _grad_worker(rank, world, port, q):
    from rpst.shard import GradientAllReduce
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # data-parallel training: same weights, a different batch per rank; the averaged
        # gradient equals the gradient of the mean loss over the union of the batches
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 2))
        frozen = torch.nn.Parameter(torch.ones(3), requires_grad=False)
        xs = torch.rand(world, 4, 6, generator=torch.Generator().manual_seed(1))
        net(xs[rank]).pow(2).mean().backward()
        GradientAllReduce(list(net.parameters()) + [frozen])()
        if rank == 0:
            ref = copy.deepcopy(net)
            ref.zero_grad()
            torch.stack([ref(xs[r]).pow(2).mean() for r in range(world)]).mean().backward()
            ok = all(torch.allclose(a.grad, b.grad, rtol=1e-6, atol=1e-7)
                     for a, b in zip(net.parameters(), ref.parameters()))
            q.put(ok)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gradient_allreduce(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_grad_worker, args=(world, _free_port(), q), nprocs=world, join=True)
    assert q.get(timeout=60)
