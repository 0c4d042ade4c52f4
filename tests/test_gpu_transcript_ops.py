"""prove / verify over a CALLER-owned transcript (lcpc_transcript_ops), on the GPU.

The reference's LcCommit::prove / LcEvalProof::verify mutate the caller's
`&mut merlin::Transcript` (lcpc-2d/src/lib.rs:319-326, 547-556, body :1034-1123 / :862-982), and
the caller keeps using it (proof-of-storage/src/tests.rs:223-233; one transcript over two
proofs, lcpc-2d/src/tests.rs:318-413).  Here the caller's transcript is the ORACLE's Merlin
restatement, driven through ctypes callbacks; the proof must be bit-identical to lcpc_prove with
the library's own transcript AND to the oracle's of_prove, and the caller's transcript must end in
the state both of those reach (the challenge_bytes(b"after") check).
"""
import ctypes as C

import numpy as np
import pytest

from test_transcript_ops import CountingOracleTranscript

pytestmark = pytest.mark.gpu


def rand_elems(oracle, fid, n, seed):
    return oracle.ChaCha(seed_u64=seed).field_random(fid, n)


def _prefix(tr, root, nco):
    tr.append_message(b"polycommit", root)
    tr.append_message(b"ncols", nco.to_bytes(8, "big"))
    return tr


def _same_proof(gp, op_or_gp, oracle=None):
    if oracle is None:  # two library proofs
        b = op_or_gp
        assert np.array_equal(gp.p_eval, b.p_eval)
        for x, y in zip(gp.p_random_vec, b.p_random_vec):
            assert np.array_equal(x, y)
        for x, y in zip(gp.columns, b.columns):
            assert np.array_equal(x.col, y.col) and x.path == y.path
        return
    op = op_or_gp
    assert np.array_equal(gp.p_eval.reshape(-1), op.p_eval)
    pr = np.concatenate([v.reshape(-1) for v in gp.p_random_vec]) if gp.n_degree_tests else np.zeros(0, np.uint64)
    assert np.array_equal(pr, op.p_random)
    o_cols = op.cols.reshape(gp.n_col_opens, -1)
    o_paths = op.paths.tobytes()
    for k, c in enumerate(gp.columns):
        assert np.array_equal(c.col.reshape(-1), o_cols[k])
        assert b"".join(c.path) == o_paths[k * 32 * op.path_len:(k + 1) * 32 * op.path_len]


@pytest.mark.parametrize("batched", [True, False])
@pytest.mark.parametrize("fid,n_per_row,n_cols,length,nco,ndt", [
    (1, 2048, 4096, 1 << 16, 309, 2),   # cfg1 shape
    (0, 100, 256, 3000, 128, 3),        # ragged last row
    (3, 256, 512, 1000, 40, 1),
    (4, 64, 128, 1000, 20, 2),          # big-endian repr
    (2, 512, 1024, 60 * 512 + 3, 64, 2),
    (1, 64, 128, 64 * 9, 16, 0),        # no degree tests (evaluation only)
])
def test_prove_verify_over_caller_transcript(gpu, oracle, fid, n_per_row, n_cols, length, nco, ndt, batched):
    coeffs = rand_elems(oracle, fid, length, 5)
    g_enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, ndt)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt)
    g = gpu.LcCommit.commit(coeffs, g_enc)
    o = oracle.Commit(o_enc, coeffs)
    root = g.get_root()
    assert root == o.root()
    x = rand_elems(oracle, fid, 1, 77)
    inner, outer = oracle.eval_tensors(fid, x, n_per_row, g.get_n_rows())
    # three provers: library transcript, caller (oracle) transcript through ops, the oracle itself
    own = _prefix(gpu.Transcript(b"test transcript"), root, nco)
    caller = _prefix(CountingOracleTranscript(oracle, batched=batched), root, nco)
    o_tr = oracle.standard_transcript(nco, root)
    gp_own = g.prove(outer, g_enc, own)
    gp_ops = g.prove(outer, g_enc, caller)  # any object with merlin's methods: CallerTranscript
    op = o.prove(o_enc, outer, o_tr)
    _same_proof(gp_ops, op, oracle)
    _same_proof(gp_ops, gp_own)
    after = own.challenge_bytes(b"after", 32)
    assert caller.challenge_bytes(b"after", 32) == after == o_tr.challenge_bytes(b"after", 32)
    # one challenge per degree test, one for the columns (+ "after"); absorptions batched per vector
    assert caller.calls["challenge_bytes"] == ndt + 2
    if batched:
        assert caller.calls["append_messages"] == ndt + 1
    # verify over a caller transcript: same evaluation, same end state as the oracle's verifier
    v_caller = _prefix(CountingOracleTranscript(oracle, batched=batched), root, nco)
    v_o = oracle.standard_transcript(nco, root)
    ev = gp_ops.verify(root, outer, inner, g_enc, v_caller)
    rc, o_ev = op.verify(root, outer, inner, o_enc, v_o)
    assert rc == 0 and np.array_equal(ev.reshape(-1), o_ev)
    assert v_caller.challenge_bytes(b"after", 32) == v_o.challenge_bytes(b"after", 32)


def test_one_caller_transcript_over_two_proofs(gpu, oracle):
    """lcpc-2d/src/tests.rs:318-413: the second proof continues the first one's transcript."""
    fid, n_per_row, n_cols, nco, ndt = 1, 256, 512, 32, 2
    enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, ndt)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt)
    caller = CountingOracleTranscript(oracle, label=b"two proofs")
    o_tr = oracle.Transcript(b"two proofs")
    for seed in (1, 2):
        coeffs = rand_elems(oracle, fid, 40 * n_per_row + seed, seed)
        g = gpu.LcCommit.commit(coeffs, enc)
        o = oracle.Commit(o_enc, coeffs)
        outer = rand_elems(oracle, fid, g.get_n_rows(), 10 + seed)
        for tr in (caller, o_tr):
            tr.append_message(b"polycommit", g.get_root())
        _same_proof(g.prove(outer, enc, caller), o.prove(o_enc, outer, o_tr), oracle)
    assert caller.challenge_bytes(b"after", 32) == o_tr.challenge_bytes(b"after", 32)


def test_sdig_prove_over_caller_transcript(gpu, oracle):
    """Brakedown (SdigCode3, seed 0) at a small n: same proof through ops as the oracle's."""
    fid, length = 1, 4096 * 4
    n_per_row = gpu.SdigEncoding.n_per_row_for(fid, length)
    g_enc = gpu.SdigEncoding.new(fid, length, 0)
    o_enc = oracle.Encoding.sdig(fid, n_per_row, seed=0, code_id=3)
    coeffs = rand_elems(oracle, fid, length, 9)
    g = gpu.LcCommit.commit(coeffs, g_enc)
    o = oracle.Commit(o_enc, coeffs)
    assert g.get_root() == o.root()
    outer = rand_elems(oracle, fid, g.get_n_rows(), 3)
    nco = g_enc.get_n_col_opens()
    caller = _prefix(CountingOracleTranscript(oracle), g.get_root(), nco)
    o_tr = oracle.standard_transcript(nco, o.root())
    _same_proof(g.prove(outer, g_enc, caller), o.prove(o_enc, outer, o_tr), oracle)
    assert caller.challenge_bytes(b"after", 32) == o_tr.challenge_bytes(b"after", 32)


def test_raw_prove_ops_entry_point(gpu, oracle):
    """lcpc_prove_ops / lcpc_verify_ops with a hand-built ops table (the C ABI a Rust shim binds)
    whose functions forward to a library transcript handle: same proof as lcpc_prove."""
    from lcpc_proof_of_storage_amd import _native as N
    lib = N.load()
    fid, n_per_row, n_cols, nco, ndt = 0, 512, 1024, 64, 3
    enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, ndt)
    coeffs = rand_elems(oracle, fid, 30 * n_per_row, 4)
    g = gpu.LcCommit.commit(coeffs, enc)
    root = g.get_root()
    outer = rand_elems(oracle, fid, g.get_n_rows(), 6)
    target = _prefix(gpu.Transcript(b"test transcript"), root, nco)
    th = target._h

    def am(ctx, lp, ln, mp, mn):
        lib.lcpc_transcript_append_message(th, lp, ln, mp, mn)
        return 0

    def ams(ctx, lp, ln, mp, ml, n):
        lib.lcpc_transcript_append_messages(th, lp, ln, mp, ml, n)
        return 0

    def ch(ctx, lp, ln, dp, n):
        lib.lcpc_transcript_challenge_bytes(th, lp, ln, dp, n)
        return 0

    cbs = (N.TR_APPEND_FN(am), N.TR_APPEND_MANY_FN(ams), N.TR_CHALLENGE_FN(ch))
    ops = N.TranscriptOps(None, *cbs)
    o = gpu.lcpc2d._elems(outer, fid)
    h = C.c_void_p()
    assert lib.lcpc_prove_ops(g._h, gpu.lcpc2d._p64(o), o.shape[0], enc._h, C.byref(ops), C.byref(h)) == 0
    via_ops = gpu.LcEvalProof(h.value)
    ref = _prefix(gpu.Transcript(b"test transcript"), root, nco)
    _same_proof(via_ops, g.prove(outer, enc, ref))
    assert target.challenge_bytes(b"after", 32) == ref.challenge_bytes(b"after", 32)
    # verify_ops on a fresh target
    target = _prefix(gpu.Transcript(b"test transcript"), root, nco)
    th = target._h
    inner = rand_elems(oracle, fid, n_per_row, 8)
    i = gpu.lcpc2d._elems(inner, fid)
    ev = np.zeros(1, np.uint64)
    rp = (C.c_uint8 * 32).from_buffer_copy(root)
    assert lib.lcpc_verify_ops(rp, gpu.lcpc2d._p64(o), o.shape[0], gpu.lcpc2d._p64(i), i.shape[0], via_ops._h,
                               enc._h, C.byref(ops), gpu.lcpc2d._p64(ev)) == 0
    want = via_ops.verify(root, outer, inner, enc, _prefix(gpu.Transcript(b"test transcript"), root, nco))
    assert np.array_equal(ev, want.reshape(-1))


def test_failing_caller_transcript_fails_prove_cleanly(gpu, oracle):
    """A callback that raises mid-proof: prove re-raises the caller's exception, and the library
    stays usable (the next proof on the same commitment is right)."""
    fid, n_per_row, n_cols, nco, ndt = 1, 256, 512, 32, 2
    enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, ndt)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt)
    coeffs = rand_elems(oracle, fid, 20 * n_per_row, 12)
    g = gpu.LcCommit.commit(coeffs, enc)
    outer = rand_elems(oracle, fid, g.get_n_rows(), 13)

    class DiesOnSecondChallenge(CountingOracleTranscript):
        def challenge_bytes(self, label, n):
            if self.calls["challenge_bytes"] == 1:
                raise KeyError("transcript revoked")
            return super().challenge_bytes(label, n)

    with pytest.raises(KeyError):
        g.prove(outer, enc, DiesOnSecondChallenge(oracle))
    caller = CountingOracleTranscript(oracle)
    o_tr = oracle.Transcript(b"test transcript")
    _same_proof(g.prove(outer, enc, caller), oracle.Commit(o_enc, coeffs).prove(o_enc, outer, o_tr), oracle)


def test_sharded_prove_over_caller_transcript(gpu, oracle, hipmem):
    """The row-sharded prove (lcpc_sharded_prove, one rank) with the caller's transcript on the
    root rank: the same proof and end state as the oracle's."""
    from lcpc_proof_of_storage_amd import shard
    fid, n_per_row, n_cols, nco, ndt = 1, 512, 1024, 48, 2
    enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, ndt)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt)
    n_rows = 24
    coeffs = rand_elems(oracle, fid, n_rows * n_per_row, 21)
    d = hipmem.to_device(coeffs)
    try:
        sc = shard.ShardedCommit(enc, shard.NativeComm.single(), d, n_rows)
        o = oracle.Commit(o_enc, coeffs)
        assert sc.get_root() == o.root()
        outer = rand_elems(oracle, fid, n_rows, 22)
        caller = _prefix(CountingOracleTranscript(oracle), sc.get_root(), nco)
        o_tr = oracle.standard_transcript(nco, o.root())
        pf = sc.prove(outer, caller, root=0)
        _same_proof(pf, o.prove(o_enc, outer, o_tr), oracle)
        assert caller.challenge_bytes(b"after", 32) == o_tr.challenge_bytes(b"after", 32)
        del sc
    finally:
        hipmem.free(d)


def test_pipelined_driver_over_caller_transcripts(gpu, oracle, hipmem):
    """lcpc_sharded_commit_prove_many (one rank): each polynomial's proof on the caller's own
    transcript -- the same proofs and end states as the oracle's."""
    from lcpc_proof_of_storage_amd import shard
    fid, n_per_row, n_cols, nco, ndt = 1, 256, 512, 24, 2
    enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, ndt)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt)
    n_rows = 16
    polys = [rand_elems(oracle, fid, n_rows * n_per_row, 31 + k) for k in range(3)]
    outer = rand_elems(oracle, fid, n_rows, 32)
    ds = [hipmem.to_device(p) for p in polys]
    made = {}
    try:
        def make_tr(i, root):
            made[i] = _prefix(CountingOracleTranscript(oracle), root, nco)
            return made[i]

        roots, proofs = shard.sharded_commit_prove_many(enc, shard.NativeComm.single(), ds, n_rows, outer, make_tr)
        for i, p in enumerate(polys):
            o = oracle.Commit(o_enc, p)
            assert roots[i] == o.root()
            o_tr = oracle.standard_transcript(nco, o.root())
            _same_proof(proofs[i], o.prove(o_enc, outer, o_tr), oracle)
            assert made[i].challenge_bytes(b"after", 32) == o_tr.challenge_bytes(b"after", 32)
    finally:
        for d in ds:
            hipmem.free(d)
