"""Per-image batch sharding over the GPUs of one node.

Stylisation is independent per image (AdaIN statistics are per (n,c), WCT loops per
image (wct_rp.py:159), SANet bmm is batched per image (sanet.py:90,94)), so a batch is
split into contiguous per-GPU slices, every GPU runs the same kernels on its slice with
its own weight replica, and the outputs are gathered on the host. No collective ever
touches the data: RCCL/xGMI are unused by design.

Two launch styles:
  * one process per GPU (torch.distributed.run, bench.py): `partition(...)` gives each
    rank its slice; `gather_to_host` collects the CPU outputs on rank 0 over gloo
    (host memory, not RCCL);
  * one process driving N devices (`ShardedModel`): a host thread per device, each with
    its own stream, results concatenated on the host in batch order.
"""
from __future__ import annotations

import copy
import threading
from typing import Callable, List, Sequence, Tuple

import torch


def partition(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, end) slice of n items for `rank` of `world` (sizes differ by
    at most one; earlier ranks take the remainder)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, rem = divmod(n, world)
    start = rank * base + min(rank, rem)
    return start, start + base + (1 if rank < rem else 0)


def gather_to_host(local: torch.Tensor, group=None) -> torch.Tensor:
    """Collect every rank's CPU output slice on rank 0 (others get their own slice back).

    Uses the default process group, which must be gloo (host memory): RCCL is never
    used for data. Slices may differ in size by one image."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    local = local.detach().cpu().contiguous()
    sizes = [None] * world
    dist.all_gather_object(sizes, tuple(local.shape), group=group)
    if rank == 0:
        bufs = [torch.empty(s, dtype=local.dtype) for s in sizes]
        bufs[0] = local
        for r in range(1, world):
            dist.recv(bufs[r], src=r, group=group)
        return torch.cat(bufs, 0)
    dist.send(local, dst=0, group=group)
    return local


class ShardedModel:
    """Replicate a model over `devices` and stylise a batch split per image.

    `method` is the model method to call ("test" for AdaINRPNet / WCTRPNet / SAModel).
    Inputs may live on the host or any device; each shard is copied to its GPU, run on
    that GPU's current stream from its own host thread (ctypes releases the GIL during
    kernel launches), and the outputs are gathered on the host in batch order.
    """

    def __init__(self, model: torch.nn.Module, devices: Sequence[torch.device],
                 method: str = "test"):
        self.devices = [torch.device(d) for d in devices]
        self.method = method
        self.replicas = [copy.deepcopy(model).to(d) for d in self.devices]

    def __call__(self, content: torch.Tensor, style: torch.Tensor) -> torch.Tensor:
        assert content.shape == style.shape
        n = content.shape[0]
        world = len(self.devices)
        outs: List[torch.Tensor] = [None] * world
        errs: List[BaseException] = []

        def work(r: int):
            try:
                s, e = partition(n, world, r)
                if s == e:
                    outs[r] = content[:0].detach().cpu()
                    return
                dev = self.devices[r]
                with torch.cuda.device(dev):
                    c = content[s:e].to(dev, non_blocking=True)
                    st = style[s:e].to(dev, non_blocking=True)
                    y = getattr(self.replicas[r], self.method)(c, st)
                    outs[r] = y.to("cpu")
            except BaseException as ex:  # re-raised on the caller's thread
                errs.append(ex)

        threads = [threading.Thread(target=work, args=(r,)) for r in range(world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errs:
            raise errs[0]
        return torch.cat(outs, 0)


class GradientAllReduce:
    """Data-parallel training exchange (the one real collective of this package): after
    backward, every rank's parameter gradients are averaged over the process group.

    The RP encoder / decoder hold ~3 MB of gradients, so they travel as ONE flat buffer:
    one all-reduce per step (RCCL over xGMI with the "nccl" backend; gloo on CPU tests)
    instead of one launch per tensor. The buffer is allocated once and reused."""

    def __init__(self, params, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.flat = None

    def __call__(self) -> None:
        import torch.distributed as dist

        world = dist.get_world_size(self.group)
        grads = [p.grad for p in self.params]
        if any(g is None for g in grads):
            raise RuntimeError("GradientAllReduce: a parameter has no gradient (run backward first)")
        n = sum(g.numel() for g in grads)
        if self.flat is None or self.flat.numel() != n or self.flat.device != grads[0].device:
            self.flat = torch.empty(n, device=grads[0].device, dtype=grads[0].dtype)
        off = 0
        for g in grads:
            self.flat[off:off + g.numel()].copy_(g.reshape(-1))
            off += g.numel()
        dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group)
        self.flat.div_(world)
        off = 0
        for g in grads:
            g.copy_(self.flat[off:off + g.numel()].view_as(g))
            off += g.numel()


def shard_apply(fn: Callable[[torch.Tensor], torch.Tensor], x: torch.Tensor, world: int,
                rank: int) -> torch.Tensor:
    """Apply fn to this rank's contiguous slice of x (used by tests and bench)."""
    s, e = partition(x.shape[0], world, rank)
    return fn(x[s:e])
