"""Multi-rank sharding and metric gathering on CPU with the gloo backend (world size 2
and 3): the same code path bench.py uses with RCCL on the GPU box."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from stereoanywhere_amd import dist as D


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, gb, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    r = D.init_from_env("gloo")
    lo, hi = D.shard_range(gb, r.rank, r.world)
    local = torch.arange(lo, hi, dtype=torch.float64).unsqueeze(1).repeat(1, 3)
    allm = D.gather_metrics(local, r)
    mx = D.max_over_ranks(float(rank + 1), r, "cpu")
    D.barrier(r)
    q.put((rank, allm.tolist(), mx))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world,gb", [(2, 8), (3, 7), (2, 1)])
def test_shard_and_gather(world, gb):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, gb, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, allm, mx in res:
        assert [row[0] for row in allm] == list(range(gb))
        assert mx == world


def test_shard_range_covers_exactly():
    for gb in range(0, 20):
        for w in range(1, 9):
            spans = [D.shard_range(gb, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == gb
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1
