"""CPU: the N > 1 bench plumbing over gloo, world_size 2 (the GPU box runs it over RCCL).

bench.py runs one process per GPU; each rank commits and opens its own polynomial (no
data-path collective), and the job time is the max over ranks.  This exercises those helpers
with real torch.distributed processes rendezvousing on 127.0.0.1.
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      LOCAL_RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import bench
    r, lr, w = bench.dist_env()
    dist = bench.init_dist(w, lr, backend="gloo")
    try:
        bench.sync_barrier(dist)
        elapsed = bench.max_over_ranks(dist, 1.0 + r)  # rank 1 is the slow one
        seeds = [None] * w
        dist.all_gather_object(seeds, bench.replica_seed(r))
        bench.sync_barrier(dist)
        q.put((r, elapsed, seeds, bench.job_throughput(1 << 24, 10, w, elapsed)))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_bench_plumbing_world2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=100) for _ in range(2))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r, elapsed, seeds, thr in res:
        assert elapsed == 2.0                      # max over ranks
        assert len(set(seeds)) == 2                # independent replicas commit different data
        assert thr == (1 << 24) * 10 * 2 / 2.0     # whole-job units / slowest rank's time


def test_single_process_has_no_group():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.init_dist(1, 0) is None
    assert bench.max_over_ranks(None, 3.5) == 3.5
