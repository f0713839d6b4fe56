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


class _TileMock(torch.nn.Module):
    """Deterministic per-tile 'model' (negated disparity, tile-size dependent like a real one)."""

    def __init__(self):
        super().__init__()
        self.p = torch.nn.Parameter(torch.zeros(1))

    def forward(self, l, r, ml, mr, iters=1, test_mode=True):
        H, W = l.shape[-2:]
        ramp = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W) / W
        return -(40 * l[:, :1] - 10 * r[:, 1:2] + ml * 3 + ramp + H / 100.0), None


def _tile_inputs():
    g = torch.Generator().manual_seed(5)
    return [torch.rand(1, c, 200, 330, generator=g) for c in (3, 3, 1, 1)]


def _eval_sample(i):
    """A deterministic guided_metrics dict per sample index (what run(...) returns)."""
    import numpy as np
    from stereoanywhere_amd import metrics
    rng = np.random.default_rng(100 + i)
    gt = (rng.random((1, 1, 16, 24)) * 30).astype(np.float32)
    occ = (rng.random(gt.shape) > 0.7).astype(np.float32) if i % 2 else np.zeros_like(gt)
    return metrics.guided_metrics(gt + rng.standard_normal(gt.shape).astype(np.float32) * (1 + i), gt,
                                  (rng.random(gt.shape) > 0.1).astype(np.float32), occ)


def _worker_harness(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from stereoanywhere_amd import harness, tiler
    r = D.init_from_env("gloo")
    # test.py / test_mapreduce_v2.py sample sharding + metric gather (5 samples, 2 tries)
    out = harness.evaluate(_eval_sample, 5, 2, r, "cpu")
    # TileWrapper(rank, world): tiles r, r+world, ...; partial maps summed by one all_reduce
    with torch.no_grad():
        st = tiler.TileWrapper(_TileMock(), tile_width=128, tile_height=96, overlap=32, rank=r.rank,
                               world=r.world)(*_tile_inputs(), iters=1, test_mode=True)
    q.put((rank, out, st.numpy()))
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_harness_and_tiles_sharded_equal_single_rank(world):
    """The multi-rank harness (sample shards, all_gather of metric rows) and the tile-sharded
    TileWrapper (all_reduce of the partial stitched / weight maps) give the single-rank
    results: the same aggregated metrics and the same stitched disparity."""
    import numpy as np
    from stereoanywhere_amd import harness, tiler
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_harness, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
    mean1, std1 = harness.evaluate(_eval_sample, 5, 2, D.Rank(), "cpu")
    mean, std = res[0][1]
    assert all(x[1] is None for x in res[1:])
    assert list(mean) == harness.METRIC_ORDER
    for k in harness.METRIC_ORDER:
        np.testing.assert_equal(mean[k], mean1[k])
        np.testing.assert_equal(std[k], std1[k])
    with torch.no_grad():
        st1 = tiler.TileWrapper(_TileMock(), tile_width=128, tile_height=96, overlap=32)(*_tile_inputs(), iters=1,
                                                                                          test_mode=True).numpy()
    for _, _, st in res:
        np.testing.assert_allclose(st, st1, rtol=1e-6, atol=1e-6)


_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, extra_env=None, timeout=240):
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["SA_DIST_BACKEND"] = "gloo"
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(_ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_its_own_ranks(world):
    """bench.py --gpus N outside torchrun starts N ranks itself (one child per GPU): every rank joins
    the process group and reports world == N (the --dry-run rendezvous, gloo on the CPU).  The line
    explains itself at N > 1: each rank's timed-region ms per step (stand-in
    steps: rank r sleeps 5 (r + 1) ms, so the last rank is the slowest), the metric all_gather's
    latency and size, and the cpu_baseline key (a tiny oracle sample in the dry run)."""
    import json
    res = _bench(["--gpus", str(world), "--dry-run", "--steps", "3"])
    assert res.returncode == 0, res.stderr
    line = json.loads([ln for ln in res.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == world
    assert line["ranks"] == list(range(world))
    assert line["worlds"] == [world]
    rt = line["rank_timing"]
    assert len(rt["per_rank_ms_per_step"]) == world and rt["slowest_rank"] == world - 1
    assert all(v >= 5.0 for v in rt["per_rank_ms_per_step"]) and rt["spread"] > 1.0
    assert rt["gather_ms"] > 0 and rt["gather_bytes"] == world * 2 * 8 and rt["backend"] == "gloo"
    cb = line["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1


def test_bench_world_size_mismatch_fails():
    """Under a torchrun environment whose WORLD_SIZE differs from --gpus, bench.py exits non-zero
    instead of reporting a line for the wrong GPU count."""
    res = _bench(["--gpus", "4", "--dry-run"], dict(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0",
                                                    MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port())))
    assert res.returncode != 0
    assert "WORLD_SIZE 2" in res.stderr


def test_bench_rank_dying_after_init_ends_the_launch():
    """a rank that dies after the rendezvous (here rank 1 exits right after
    init_process_group) leaves the others waiting in a collective; the launcher ends them and exits
    non-zero with the dead rank's code instead of hanging."""
    import time
    t0 = time.monotonic()
    res = _bench(["--gpus", "3", "--dry-run"], dict(SA_DRYRUN_FAIL_RANK="1"), timeout=180)
    assert res.returncode == 3, (res.returncode, res.stderr[-2000:])
    assert "rank exit codes" in res.stderr
    assert time.monotonic() - t0 < 120


def test_bench_failing_rank_fails_the_launch():
    """Ranks that fail (here: a process-group backend that does not exist, seen only by the children:
    the launcher itself joins no group) make the launcher exit non-zero."""
    res = _bench(["--gpus", "2", "--dry-run"], dict(SA_DIST_BACKEND="no_such_backend"))
    assert res.returncode != 0
    assert "rank exit codes" in res.stderr
