"""Multi-GPU data parallelism for independent stereo pairs.

Pairs are independent (batch-vs-single EPE 1.1e-6), so a global batch is
split into contiguous per-rank shards and every rank runs its shard on its own GPU with
no data-path collective.  The only exchange is one ``all_gather`` of per-pair metric
vectors at the end (RCCL over xGMI with backend "nccl"; gloo in the CPU tests).
One process per GPU; rendezvous from the torchrun environment (RANK, LOCAL_RANK,
WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Tuple

import torch
import torch.distributed as dist


@dataclass
class Rank:
    rank: int = 0
    world: int = 1
    local_rank: int = 0

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def init_from_env(backend: str = "nccl") -> Rank:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return Rank()
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if backend == "nccl":
        torch.cuda.set_device(local)
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return Rank(rank, world, local)


def shard_range(global_batch: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous shard [start, stop) of rank; the first (global % world) ranks take one extra."""
    base, extra = divmod(global_batch, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_metrics(local: torch.Tensor, r: Rank) -> torch.Tensor:
    """all_gather per-pair metric rows [n_local, k] from every rank -> [n_global, k] on
    every rank (shards may be ragged: sizes are exchanged first)."""
    if r.world == 1:
        return local
    n = torch.tensor([local.shape[0]], device=local.device, dtype=torch.long)
    sizes = [torch.zeros_like(n) for _ in range(r.world)]
    dist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    pad = torch.zeros((mx,) + tuple(local.shape[1:]), device=local.device, dtype=local.dtype)
    pad[: local.shape[0]] = local
    bufs = [torch.zeros_like(pad) for _ in range(r.world)]
    dist.all_gather(bufs, pad)
    return torch.cat([b[: int(s.item())] for b, s in zip(bufs, sizes)], 0)


def gather_scalars(value: float, r: Rank, device) -> list:
    """all_gather of one float per rank -> [rank 0's, rank 1's, ...] on every rank (the per-rank
    timed-region lengths of bench.py: a slow rank shows as such, not only as the max)."""
    if r.world == 1:
        return [float(value)]
    t = torch.tensor([value], device=device, dtype=torch.float64)
    out = [torch.zeros_like(t) for _ in range(r.world)]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def max_over_ranks(value: float, r: Rank, device) -> float:
    if r.world == 1:
        return value
    t = torch.tensor([value], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def barrier(r: Rank) -> None:
    if r.world > 1:
        dist.barrier()
