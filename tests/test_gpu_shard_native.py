"""GPU: the native row-sharded protocol (csrc/shard_native.cpp through lcpc_comm / lcpc_sharded_*)
against the single-GPU commit / prove and the CPU oracle (every commit + prove case), bit for bit.

* one rank: RCCL with a 1-rank communicator (the RCCL code path: group calls, own-piece copies)
  and the no-exchange comm;
* two ranks sharing the one GPU, the collectives supplied over gloo (RCCL refuses two ranks on
  one GPU): commit (root, the whole Merkle tree on every rank), prove with the transcript on
  either rank, and the pipelined driver (lcpc_sharded_commit_prove_many) over several
  polynomials with the transcript rank rotating;
* cfg3 at BASELINE's full size (Ft127, 2^24, 512 x 32768 -> 65536) split over two ranks, against
  the oracle's commit and proof (tests/test_gpu_fullsize.py holds the unsharded cfg3 / cfg4 / cfg5).
"""
import datetime
import os
import socket
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = {"ft127": (1, 1 << 16), "ft63": (0, 3 * 4096 + 17), "ft255": (3, 20000), "ft127_ragged": (1, 5 * 2048 + 3),
         # Ft191's 24-byte elements: rank cuts only where a 1 KiB chunk starts on an element
         # (rows 84 + 128 k); 300 rows of 64 -> 128 give three such units
         "ft191": (2, 300 * 64 - 5, (64, 128)),
         # Brakedown (SdigCode3, seed 5): element-major shards, n_cols no power of two (the tree's
         # padded leaves are zero digests); 2^16 Ft127 has 48 rows of 1330 -> 2081
         "sdig_ft127": (1, 1 << 16, ("sdig", 5)), "sdig_ft63": (0, 3 * 4096 + 17, ("sdig", 5))}


def _encoding(L, fid, n, dims=None):
    if dims and dims[0] == "sdig":
        return L.SdigEncoding.new(fid, n, dims[1], 3)
    return L.LigeroEncoding.new_from_dims(fid, *dims) if dims else L.LigeroEncoding.new(fid, n)


def _oracle_encoding(O, fid, enc, dims=None):
    if dims and dims[0] == "sdig":
        return O.Encoding.sdig(fid, enc.n_per_row, seed=dims[1], code_id=3)
    return O.Encoding.ligero(fid, enc.n_per_row, enc.n_cols, enc.get_n_col_opens(), enc.get_n_degree_tests())


def _transcript(L, root, nco):
    tr = L.Transcript(b"test transcript")
    tr.append_message(b"polycommit", root)
    tr.append_message(b"ncols", nco.to_bytes(8, "big"))
    return tr


def _padded_rows(L, enc, coeffs):
    n_rows, n_per_row, _ = enc.get_dims(coeffs.shape[0])
    nl = L.limbs(enc.field)
    rows = np.zeros((n_rows * n_per_row, nl), np.uint64)
    rows[:coeffs.shape[0]] = coeffs
    return rows.reshape(n_rows, n_per_row * nl), n_rows


def _proof_fields(pf):
    return dict(p_eval=pf.p_eval.copy(), p_random=[x.copy() for x in pf.p_random_vec],
                cols=np.stack([c.col for c in pf.columns]), paths=[b"".join(c.path) for c in pf.columns])


def _same_proof(a, b):
    return (np.array_equal(a["p_eval"], b["p_eval"]) and len(a["p_random"]) == len(b["p_random"])
            and all(np.array_equal(x, y) for x, y in zip(a["p_random"], b["p_random"]))
            and np.array_equal(a["cols"], b["cols"]) and a["paths"] == b["paths"])


def _oracle_same(fid, enc, coeffs, outer, root, fields, dims=None):
    """the CPU oracle's commit + proof of the same polynomial (the reference's algorithm) against
    a sharded proof's fields"""
    sys.path.insert(0, HERE)
    import oracle_ffi as O
    nco, ndt = enc.get_n_col_opens(), enc.get_n_degree_tests()
    o_enc = _oracle_encoding(O, fid, enc, dims)
    oc = O.Commit(o_enc, coeffs.reshape(-1))
    op = oc.prove(o_enc, outer.reshape(-1), O.standard_transcript(nco, oc.root()))
    pr = np.concatenate([x.reshape(-1) for x in fields["p_random"]]) if ndt else np.zeros(0, np.uint64)
    return (oc.root() == root and np.array_equal(fields["p_eval"].reshape(-1), op.p_eval)
            and np.array_equal(pr, op.p_random) and np.array_equal(fields["cols"].reshape(-1), op.cols)
            and b"".join(fields["paths"]) == op.paths.tobytes())


def _run_rank(L, hipmem, comm, fid, n, seed=9, root_rank=0, dims=None):
    """commit + prove through the native sharded entry points; returns what rank-0 checks."""
    from lcpc_proof_of_storage_amd import shard
    enc = _encoding(L, fid, n, dims)
    coeffs = L.field_random(fid, n, seed)
    single = L.LcCommit.commit(coeffs, enc)
    outer = L.field_random(fid, single.get_n_rows(), seed + 1)
    nco = enc.get_n_col_opens()
    rows, n_rows = _padded_rows(L, enc, coeffs)
    r0, nr = shard.sharded_rows(fid, n_rows, comm.world, comm.rank)
    mine = np.ascontiguousarray(rows[r0:r0 + nr])
    d = hipmem.to_device(mine) if nr else 0
    try:
        sc = shard.ShardedCommit(enc, comm, d, n_rows)
        res = dict(root=sc.get_root() == single.get_root(), hashes=sc.hashes == single.hashes)
        tr = _transcript(L, sc.get_root(), nco) if comm.rank == root_rank else None
        spf = sc.prove(outer, tr, root=root_rank)
        if comm.rank == root_rank:
            pf = single.prove(outer, enc, _transcript(L, single.get_root(), nco))
            res["proof"] = _same_proof(_proof_fields(spf), _proof_fields(pf))
            res["oracle"] = _oracle_same(fid, enc, coeffs, outer, sc.get_root(), _proof_fields(spf), dims)
            # and the sharded proof verifies
            inner = L.field_random(fid, enc.n_per_row, seed + 2)
            ev = spf.verify(single.get_root(), outer, inner, enc, _transcript(L, single.get_root(), nco))
            ev2 = pf.verify(single.get_root(), outer, inner, enc, _transcript(L, single.get_root(), nco))
            res["verify"] = np.array_equal(ev, ev2)
        else:
            res["proof"] = spf is None
        del sc
    finally:
        if d:
            hipmem.free(d)
    return res


def _run_many(L, hipmem, comm, fid, n, n_polys=5, lag=0, dims=None):
    """the pipelined driver over n_polys polynomials (transcript rank i % world)."""
    from lcpc_proof_of_storage_amd import shard
    enc = _encoding(L, fid, n, dims)
    nco = enc.get_n_col_opens()
    polys = [L.field_random(fid, n, 100 + i) for i in range(n_polys)]
    singles = [L.LcCommit.commit(c, enc) for c in polys]
    n_rows = singles[0].get_n_rows()
    outer = L.field_random(fid, n_rows, 55)
    ptrs = []
    try:
        for c in polys:
            rows, _ = _padded_rows(L, enc, c)
            r0, nr = shard.sharded_rows(fid, n_rows, comm.world, comm.rank)
            ptrs.append(hipmem.to_device(np.ascontiguousarray(rows[r0:r0 + nr])))
        seen = []

        def make_tr(i, root):
            seen.append(i)
            return _transcript(L, root, nco)

        roots, proofs = shard.sharded_commit_prove_many(enc, comm, ptrs, n_rows, outer, make_tr, lag=lag)
        bad = [i for i, (r, s) in enumerate(zip(roots, singles)) if r != s.get_root()]
        res = dict(roots=not bad,
                   transcript_ranks=sorted(seen) == [i for i in range(n_polys) if i % comm.world == comm.rank])
        if bad:
            # which side is wrong: commit the polynomial again on one GPU
            again = [L.LcCommit.commit(polys[i], enc).get_root() for i in bad]
            res["bad_root_polys"] = [(i, a == roots[i], a == singles[i].get_root()) for i, a in zip(bad, again)]
            # (diagnostic) the single commitment's subtree roots at the ranks' block level
            G = comm.world
            np2 = len(singles[0].hashes) // 32 // 2 + 1
            for i in bad:
                h = singles[i].hashes
                off = 2 * np2 - 2 * G
                res.setdefault("want", []).append((i, roots[i][:4].hex(), singles[i].get_root()[:4].hex(),
                                                   [h[32 * (off + g):32 * (off + g) + 4].hex() for g in range(G)]))
        ok = True
        for i, (pf, s) in enumerate(zip(proofs, singles)):
            if i % comm.world != comm.rank:
                ok &= pf is None
                continue
            want = s.prove(outer, enc, _transcript(L, s.get_root(), nco))
            ok &= pf is not None and _same_proof(_proof_fields(pf), _proof_fields(want))
        res["proofs"] = bool(ok)
    finally:
        for p in ptrs:
            hipmem.free(p)
    return res


# ---------------------------------------------------------------- one rank
@pytest.mark.parametrize("kind", ["single", "rccl"])
@pytest.mark.parametrize("case", sorted(CASES))
def test_native_sharded_world1(gpu, hipmem, kind, case):
    import ctypes as C
    from lcpc_proof_of_storage_amd import shard
    if kind == "single":
        comm = shard.NativeComm.single()
    else:
        L = shard._lib()
        uid = (C.c_uint8 * 128)()
        from lcpc_proof_of_storage_amd import _native as N
        assert L.lcpc_comm_rccl_unique_id(uid) == 0, N.last_error()
        h = C.c_void_p()
        assert L.lcpc_comm_rccl_new(uid, 1, 0, C.byref(h)) == 0, N.last_error()
        comm = shard.NativeComm(h.value)
        assert comm.is_rccl
    res = _run_rank(gpu, hipmem, comm, *CASES[case][:2], dims=(CASES[case][2] if len(CASES[case]) > 2 else None))
    assert all(res.values()), res


def test_native_pipeline_world1(gpu, hipmem):
    from lcpc_proof_of_storage_amd import shard
    res = _run_many(gpu, hipmem, shard.NativeComm.single(), 1, 1 << 14, n_polys=6, lag=2)
    assert all(res.values()), res


def test_native_sharded_errors(gpu, hipmem):
    from lcpc_proof_of_storage_amd import shard
    comm = shard.NativeComm.single()
    sdig = gpu.SdigEncoding.new(1, 5000, 0)
    with pytest.raises(gpu.LcpcError):
        shard.ShardedCommit(sdig, comm, 0, 4)           # rows given, but no device pointer
    enc = gpu.LigeroEncoding.new(1, 1 << 12)
    with pytest.raises(gpu.LcpcError):
        shard.ShardedCommit(enc, comm, 0, 0)            # no rows


# ---------------------------------------------------------------- two ranks on the one GPU
# RCCL refuses two ranks on one GPU ("Duplicate GPU detected"): it compares (host hash, bus id).
# Giving every rank its own NCCL_HOSTID makes the ranks look like separate nodes, so RCCL connects
# them over its socket transport (loopback) and the multi-rank exchange path -- ncclGroupStart,
# the p2p_plan's ncclSend / ncclRecv on device buffers, ncclGroupEnd on the comm stream -- runs
# for real on the one GPU of this box.
RCCL_SAME_GPU_ENV = {"NCCL_IB_DISABLE": "1", "NCCL_SOCKET_IFNAME": "lo", "LCPC_SHARD_WATCHDOG_S": "90"}


def _worker(rank, world, port, job, args, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    rccl = job.endswith("_rccl")
    if rccl:
        os.environ.update(RCCL_SAME_GPU_ENV, NCCL_HOSTID=f"lcpc-test-rank-{rank}")
        job = job[:-len("_rccl")]
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
        hm = _HipMem()
        if job == "rank":
            q.put((rank, _run_rank(L, hm, comm, *args)))
        elif job == "many":
            q.put((rank, _run_many(L, hm, comm, *args)))
        else:
            q.put((rank, _full_size(L, hm, comm)))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, {"error": repr(e)}))
    finally:
        dist.destroy_process_group()


def _spawn(job, args, timeout=280, world=2):
    import torch.multiprocessing as mp
    from conftest import collect_ranks
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, job, args, q)) for r in range(world)]
    for p in procs:
        p.start()
    return collect_ranks(procs, q, world, timeout, job)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("root_rank", [0, 1])
@pytest.mark.parametrize("case", ["ft127", "ft63", "ft127_ragged", "ft191", "sdig_ft127", "sdig_ft63"])
def test_native_sharded_world2_one_gpu(gpu, case, root_rank):
    fid, n = CASES[case][:2]
    res = _spawn("rank", (fid, n, 9, root_rank, CASES[case][2] if len(CASES[case]) > 2 else None))
    for r in (0, 1):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("case,root_rank", [("ft127", 0), ("ft127_ragged", 1), ("ft63", 0), ("sdig_ft127", 1)])
def test_native_sharded_world2_rccl_one_gpu(gpu, case, root_rank):
    """two ranks through RCCL itself (device-side sends / receives), on the one GPU"""
    fid, n = CASES[case][:2]
    res = _spawn("rank_rccl", (fid, n, 9, root_rank, CASES[case][2] if len(CASES[case]) > 2 else None))
    for r in (0, 1):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.timeout(300)
def test_native_pipeline_world2_rccl_one_gpu(gpu):
    """the pipelined driver's tick groups (several polynomials' exchanges per ncclGroupStart /
    ncclGroupEnd) through RCCL, two ranks on the one GPU"""
    res = _spawn("many_rccl", (1, 1 << 14, 6, 2))
    for r in (0, 1):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.timeout(300)
def test_native_sharded_world4_rccl_one_gpu(gpu):
    res = _spawn("rank_rccl", (1, 1 << 22, 9, 3, None), world=4)
    for r in range(4):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.timeout(300)
def test_native_pipeline_world8_rccl_one_gpu(gpu):
    """the N = 8 exchange groups through RCCL: eight ranks on the one GPU, the pipelined driver on
    2^22 Ft127 (256 rows, 5 leaf chunks: three ranks own no rows), transcripts on ranks i % 8"""
    res = _spawn("many_rccl", (1, 1 << 22, 9, 0), world=8)
    bad = {r: res[r] for r in range(8) if "error" in res[r] or not all(res[r].values())}
    for r, v in bad.items():
        print("rank", r, v)
    assert not bad, bad


@pytest.mark.timeout(300)
def test_native_pipeline_world2_one_gpu(gpu):
    res = _spawn("many", (1, 1 << 14, 6, 2))
    for r in (0, 1):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.timeout(300)
def test_native_pipeline_sdig_world2_one_gpu(gpu):
    """the pipelined driver on Brakedown rows (element-major shards), two ranks"""
    res = _spawn("many", (1, 1 << 16, 5, 0, ("sdig", 5)))
    for r in (0, 1):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


def test_native_pipeline_sdig_world1(gpu, hipmem):
    from lcpc_proof_of_storage_amd import shard
    res = _run_many(gpu, hipmem, shard.NativeComm.single(), 1, 1 << 16, n_polys=4, dims=("sdig", 5))
    assert all(res.values()), res


# ---------------------------------------------------------------- four ranks on the one GPU
# (the rank count of a 4-GPU node; 2^22 splits its 5 BLAKE3 chunks 1/1/1/2, 2^16's single chunk
# leaves three ranks without rows, 2^20's three chunks leave one)
@pytest.mark.timeout(300)
@pytest.mark.parametrize("root_rank", [0, 3])
@pytest.mark.parametrize("fid,n,dims", [(1, 1 << 22, None), (1, 1 << 16, None), (0, 3 * 4096 + 17, None),
                                        (2, 300 * 64 - 5, (64, 128)), (1, 1 << 16, ("sdig", 5))])
def test_native_sharded_world4_one_gpu(gpu, fid, n, dims, root_rank):
    res = _spawn("rank", (fid, n, 9, root_rank, dims), world=4)
    for r in range(4):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.timeout(300)
def test_native_pipeline_world4_one_gpu(gpu):
    res = _spawn("many", (1, 1 << 20, 6, 2), world=4)
    for r in range(4):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


def _full_size(L, hipmem, comm):
    """cfg3 at 2^24 over two ranks: root, hashes and proof against the oracle."""
    sys.path.insert(0, HERE)
    import oracle_ffi as O
    from lcpc_proof_of_storage_amd import shard
    fid, n = L.FT127, 1 << 24
    enc = L.LigeroEncoding.new(fid, n)
    coeffs = O.random_coeffs(fid, n)
    rows, n_rows = _padded_rows(L, enc, coeffs.reshape(-1, 2))
    r0, nr = shard.sharded_rows(fid, n_rows, comm.world, comm.rank)
    d = hipmem.to_device(np.ascontiguousarray(rows[r0:r0 + nr]))
    nco = enc.get_n_col_opens()
    x = O.ChaCha(seed_u64=7).field_random(fid, 1)
    inner, outer = O.eval_tensors(fid, x, enc.n_per_row, n_rows)
    try:
        sc = shard.ShardedCommit(enc, comm, d, n_rows)
        root = sc.get_root()
        tr = _transcript(L, root, nco) if comm.rank == 0 else None
        spf = sc.prove(outer, tr, root=0)
        if comm.rank != 0:
            return {"proof_elsewhere": spf is None}
        O.lib().of_set_threads(min(16, len(os.sched_getaffinity(0))))
        o_enc = O.Encoding.ligero_new(fid, n)
        oc = O.Commit(o_enc, coeffs)
        op = oc.prove(o_enc, outer, O.standard_transcript(nco, oc.root()))
        cols = np.stack([c.col for c in spf.columns]).reshape(-1)
        return dict(root=root == oc.root(), hashes=sc.hashes == bytes(oc.hashes),
                    p_eval=np.array_equal(spf.p_eval.reshape(-1), op.p_eval),
                    p_random=np.array_equal(np.concatenate(spf.p_random_vec).reshape(-1), op.p_random),
                    cols=np.array_equal(cols, op.cols.reshape(-1)),
                    paths=b"".join(b"".join(c.path) for c in spf.columns) == op.paths.tobytes())
    finally:
        hipmem.free(d)


@pytest.mark.timeout(600)
def test_native_sharded_cfg3_full_size_world2(gpu):
    res = _spawn("full", (), timeout=560)
    for r in (0, 1):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])


@pytest.mark.slow
@pytest.mark.timeout(600)
def test_native_sharded_cfg3_full_size_world8_rccl_one_gpu(gpu):
    """cfg3 at the driver's N = 8 (512 rows: 62-66 rows and one or two leaf chunks per rank)
    through RCCL, the eight ranks on the one GPU: root, tree and proof against the oracle"""
    res = _spawn("full_rccl", (), timeout=560, world=8)
    for r in range(8):
        assert "error" not in res[r] and all(res[r].values()), (r, res[r])
