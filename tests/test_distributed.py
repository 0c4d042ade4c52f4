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
        q.put((r, (r, elapsed, seeds, bench.job_throughput(1 << 24, 10, w, elapsed))))
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
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from conftest import collect_ranks
    res = sorted(collect_ranks(procs, q, 2, 100, "bench plumbing").values())
    for p in procs:
        assert p.exitcode == 0
    for r, elapsed, seeds, thr in res:
        assert elapsed == 2.0                      # max over ranks
        assert len(set(seeds)) == 2                # independent replicas commit different data
        assert thr == (1 << 24) * 10 * 2 / 2.0     # whole-job units / slowest rank's time


@pytest.mark.timeout(240)
def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` outside torch.distributed.run launches 2 ranks itself (before any torch
    import) and the rank-0 line reports the world they formed."""
    d = _spawn_plumbing({})
    assert d["n_gpus"] == 2 and d["world_formed"] == 2 and d["plumbing_only"] is True
    # a plain --gpus N spawn: rank k binds device k (LOCAL_RANK), and no rank carries a one-GPU
    # rehearsal variable -- what lets a SCALE record show N ranks on N distinct GPUs
    assert d["devices"] == [0, 1] and d["distinct_gpus"] == 2 and d["rehearsal"] is False
    assert [i["rank"] for i in d["ranks"]] == [0, 1]
    assert all(i["rehearsal_env"] == {} for i in d["ranks"])


def _spawn_plumbing(extra_env):
    import json
    import subprocess
    sys.path.insert(0, ROOT)
    import bench
    drop = ("RANK", "WORLD_SIZE", "LOCAL_RANK") + bench.REHEARSAL_VARS
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(extra_env)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--plumbing-only"], cwd=ROOT, env=env, capture_output=True, text=True, timeout=220)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


@pytest.mark.timeout(240)
def test_bench_rehearsal_is_reported():
    """the one-GPU rehearsal (every rank on GPU 0) is visible in the line, rank by rank"""
    d = _spawn_plumbing({"LCPC_BENCH_SHARE_GPU": "1", "LCPC_BENCH_BACKEND": "gloo"})
    assert d["devices"] == [0, 0] and d["distinct_gpus"] == 1 and d["rehearsal"] is True
    assert all(i["rehearsal_env"].get("LCPC_BENCH_SHARE_GPU") == "1" for i in d["ranks"])


def test_device_binding_is_local_rank(monkeypatch):
    sys.path.insert(0, ROOT)
    import bench
    for k in bench.REHEARSAL_VARS:
        monkeypatch.delenv(k, raising=False)
    assert bench.device_binding(3) == (3, {})
    monkeypatch.setenv("LCPC_BENCH_SHARE_GPU", "1")
    assert bench.device_binding(3) == (0, {"LCPC_BENCH_SHARE_GPU": "1"})


@pytest.mark.timeout(120)
def test_bench_rejects_world_mismatch():
    """under a launcher, --gpus must equal the world size it formed"""
    import subprocess
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--plumbing-only"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert r.returncode == 2 and "WORLD_SIZE=1" in r.stderr


def test_single_process_has_no_group():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.init_dist(1, 0) is None
    assert bench.max_over_ranks(None, 3.5) == 3.5
