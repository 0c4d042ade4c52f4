"""GPU: a proof-of-storage request on ONE file whose rows are sharded over ranks
(lcpc_sharded_pos_request; networking/server.rs:652-737 over lcpc_online.rs:81-239, 454-484),
against the CPU oracle bit for bit: the commitment root and tree, u^T Enc(M) over the encoded
matrix at the client's point, and the client's columns (get_column_indicies_from_random_seed,
client.rs:443-456) with their Merkle paths.

Each rank packs only its own rows' bytes (7 per WriteableFt63 element, data_field.rs:38-46) on
the device, commits its rows (csrc/shard_native.cpp), and the request's partial sums and column
pieces are gathered at the root.  One rank (no exchanges), two / four ranks sharing the one
GPU with host-staged gloo collectives, and eight ranks on the one GPU through RCCL itself (a
distinct NCCL_HOSTID per rank: RCCL then connects the ranks over its socket transport instead of
refusing two ranks on one GPU) -- cfg5's N = 8 exchange pattern.
"""
import datetime
import hashlib
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))


def _request(L, hipmem, comm, n_bytes, seed=5, root=0, n_open=256):
    """one sharded PoS request; on `root` also the oracle's answers for the same file."""
    sys.path.insert(0, HERE)
    from lcpc_proof_of_storage_amd import pos as P
    from lcpc_proof_of_storage_amd import shard
    data = np.random.default_rng(seed).integers(0, 256, n_bytes, dtype=np.uint8)
    np_, nc, _ = P.get_aspect_ratio_default_from_file_len(n_bytes)
    n_el = -(-n_bytes // 7)
    n_rows = -(-n_el // np_)
    enc = L.LigeroEncoding.new_from_dims(L.FT63, np_, nc)
    r0, nr = shard.sharded_rows(L.FT63, n_rows, comm.world, comm.rank)
    # the whole file on the device (a server's resident file); this rank packs its rows only
    padded = np.zeros(-(-n_bytes // 8) * 8, np.uint8)
    padded[:n_bytes] = data
    d_bytes = hipmem.to_device(padded)
    d_rows = hipmem.to_device(np.zeros(max(nr * np_, 1), np.uint64))
    try:
        shard.pos_pack_shard(d_bytes, n_bytes, np_, r0, nr, d_rows)
        sc = shard.ShardedCommit(enc, comm, d_rows if nr else 0, n_rows)
        x = L.field_random(L.FT63, 1, 1337)
        left, _ = P.form_side_vectors_for_polynomial_evaluation_from_point(x, n_rows, nc)
        cols = P.get_column_indicies_from_random_seed(1337, n_open, nc)
        got = sc.pos_request(left, cols, root=root)
        res = {"tree_everywhere": len(sc.hashes) == 32 * (2 * nc - 1)}
        if comm.rank != root:
            res["nothing_elsewhere"] = got is None
            return res
        import oracle_ffi as O
        O.lib().of_set_threads(min(16, len(os.sched_getaffinity(0))))
        o_el = O.pos_bytes_to_field(data.tobytes())
        oc = O.Commit(O.Encoding.ligero(0, np_, nc), o_el)
        ev, opened = got
        m = oc.comm.reshape(n_rows, nc)
        res.update(
            root=sc.get_root() == oc.root(),
            hashes=hashlib.sha256(sc.hashes).digest() == hashlib.sha256(bytes(oc.hashes)).digest(),
            eval=np.array_equal(ev.reshape(-1), O.collapse(0, oc.comm, left.reshape(-1), n_rows, nc)),
            cols=all(np.array_equal(o.col.reshape(-1), m[:, c]) for c, o in zip(cols, opened)),
            paths=all(O.verify_path(bytes(oc.hashes)[32 * c:32 * c + 32], c, b"".join(o.path), oc.root())
                      for c, o in zip(cols, opened)),
        )
        return res
    finally:
        hipmem.free(d_bytes)
        hipmem.free(d_rows)


def test_sharded_pos_request_world1(gpu, hipmem):
    from lcpc_proof_of_storage_amd import shard
    res = _request(gpu, hipmem, shard.NativeComm.single(), 3 * (1 << 20) + 12345)
    assert all(res.values()), res


RCCL_SAME_GPU_ENV = {"NCCL_IB_DISABLE": "1", "NCCL_SOCKET_IFNAME": "lo", "LCPC_SHARD_WATCHDOG_S": "120"}


def _worker(rank, world, port, args, q, rccl=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if rccl:
        os.environ.update(RCCL_SAME_GPU_ENV, NCCL_HOSTID=f"lcpc-pos-rank-{rank}")
    sys.path.insert(0, ROOT)
    sys.path.insert(0, HERE)
    import torch.distributed as dist
    import lcpc_proof_of_storage_amd as L
    from conftest import _HipMem
    from lcpc_proof_of_storage_amd import shard
    from conftest import RENDEZVOUS_TIMEOUT_S
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=RENDEZVOUS_TIMEOUT_S))
    try:
        L.set_device(0)
        comm = shard.NativeComm.rccl(dist) if rccl else shard.NativeComm.host(dist)
        assert comm.is_rccl == rccl and comm.world == world
        q.put((rank, _request(L, _HipMem(), comm, *args)))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def _spawn(args, world, timeout=280, rccl=False):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, args, q, rccl)) for r in range(world)]
    for p in procs:
        p.start()
    from conftest import collect_ranks
    return collect_ranks(procs, q, world, timeout, "pos request")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,root", [(2, 0), (2, 1), (4, 3)])
def test_sharded_pos_request_64mib(gpu, world, root):
    res = _spawn((64 << 20, 7, root), world)
    for r in range(world):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("root", [0, 5])
def test_sharded_pos_request_64mib_world8_rccl_one_gpu(gpu, root):
    """cfg5's eight-rank exchanges (row shards cut at BLAKE3 chunk boundaries, chaining-value
    all-to-all, subtree all-gather, partial u^T Enc(M) and column-piece gathers) through RCCL,
    eight ranks on the one GPU: root, tree, u^T Enc(M), columns and paths against the oracle"""
    res = _spawn((64 << 20, 11, root), 8, rccl=True)
    bad = {r: res[r] for r in range(8) if "error" in res[r] or not all(res[r].values())}
    assert not bad, bad


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_sharded_pos_request_1gib_world2(gpu):
    res = _spawn((1 << 30, 2024, 0), 2, timeout=560)
    for r in (0, 1):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])
