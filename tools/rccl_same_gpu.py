#!/usr/bin/env python3
"""Run the native sharded protocol's RCCL multi-rank path with N ranks on ONE GPU.

RCCL refuses two ranks on one device ("Duplicate GPU detected": same host hash and bus id).  A
distinct NCCL_HOSTID per rank makes the ranks look like separate nodes, so RCCL connects them over
its socket transport on the loopback device, and liblcpc_mi's exchange groups (ncclGroupStart,
p2p_plan's ncclSend / ncclRecv on device buffers, ncclGroupEnd on the comm stream) run for real.

    python tools/rccl_same_gpu.py [--world 2] [--job rank|many] [--case ft127 | --fid F --n N] [--timeout 100]

Every rank is its own process under its own `timeout -k`, so a stuck rank cannot outlive the
call.  Prints one JSON line per rank (the checks of tests/test_gpu_shard_native.py) and exits
non-zero unless every check of every rank passed.
"""
import argparse
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(ROOT, "tests")


def worker(a):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(a.port), NCCL_IB_DISABLE="1",
                      NCCL_SOCKET_IFNAME="lo", NCCL_HOSTID=f"lcpc-rank-{a.rank}",
                      LCPC_SHARD_WATCHDOG_S=str(max(10, a.timeout - 20)))
    sys.path.insert(0, ROOT)
    sys.path.insert(0, TESTS)
    import torch.distributed as dist
    import lcpc_proof_of_storage_amd as L
    from conftest import _HipMem
    from lcpc_proof_of_storage_amd import shard
    import test_gpu_shard_native as T
    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    try:
        L.set_device(0)
        comm = shard.NativeComm.host(dist) if a.host else shard.NativeComm.rccl(dist)
        case = T.CASES[a.case] if a.n == 0 else (a.fid, a.n)
        dims = case[2] if len(case) > 2 else None
        if a.job == "rank":
            res = T._run_rank(L, _HipMem(), comm, case[0], case[1], 9, a.root, dims)
        else:
            res = T._run_many(L, _HipMem(), comm, case[0], case[1], a.polys, a.lag, dims)
        res = {k: (v if isinstance(v, list) else bool(v)) for k, v in res.items()}
        res["is_rccl"] = comm.is_rccl != a.host and comm.world == a.world
    except Exception as e:
        res = {"error": repr(e)}
    print(json.dumps({"rank": a.rank, "res": res}), flush=True)
    dist.destroy_process_group()
    return 0 if res and "error" not in res and all(v is True for v in res.values()) else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--job", choices=["rank", "many"], default="rank")
    ap.add_argument("--case", default="ft127")
    ap.add_argument("--fid", type=int, default=1, help="with --n: a Ligero polynomial of n coefficients instead of --case")
    ap.add_argument("--n", type=int, default=0, help="e.g. --n 16777216: cfg3 (512 rows, 9 leaf chunks, 8 ranks)")
    ap.add_argument("--root", type=int, default=0)
    ap.add_argument("--polys", type=int, default=6, help="--job many: polynomials")
    ap.add_argument("--host", action="store_true", help="host-staged gloo collectives instead of RCCL")
    ap.add_argument("--lag", type=int, default=2, help="--job many: schedule lag (0 = the driver's 2 + world)")
    ap.add_argument("--timeout", type=int, default=100)
    ap.add_argument("--rank", type=int, default=-1)
    ap.add_argument("--port", type=int, default=0)
    a = ap.parse_args()
    if a.rank >= 0:
        return worker(a)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [subprocess.Popen(["timeout", "-k", "5", str(a.timeout), sys.executable, os.path.abspath(__file__),
                               "--rank", str(r), "--port", str(port), "--world", str(a.world), "--job", a.job,
                               "--case", a.case, "--root", str(a.root), "--timeout", str(a.timeout),
                               "--fid", str(a.fid), "--n", str(a.n), "--polys", str(a.polys), "--lag", str(a.lag)]
                              + (["--host"] if a.host else []),
                              stdout=subprocess.PIPE, text=True) for r in range(a.world)]
    ok = True
    for p in procs:
        out, _ = p.communicate()
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        print(lines[-1] if lines else json.dumps({"rc": p.returncode, "res": None}))
        ok &= p.returncode == 0
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
