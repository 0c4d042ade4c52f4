"""GPU parity of the Brakedown / SDIG path (lcpc-brakedown-pc) against the oracle, bit for bit.

Encode (matgen + encode, lcpc-brakedown-pc/src/{matgen.rs:28-188, encode.rs:36-110}), commit
with the element-major codeword, prove / verify through lcpc-2d (lib.rs:651-1123) with the
SDIG encoding, and the golden Brakedown fixture.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def rand_elems(oracle, fid, n, seed):
    return oracle.ChaCha(seed_u64=seed).field_random(fid, n)


@pytest.mark.parametrize("fid", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("n_per_row,code,seed", [(21, 3, 0), (100, 3, 7), (1000, 3, 1), (4096, 3, 0),
                                                 (500, 1, 2), (500, 2, 3), (500, 4, 4), (500, 5, 5),
                                                 (500, 6, 6)])
def test_sdig_encode_matches_oracle(gpu, oracle, fid, n_per_row, code, seed):
    o = oracle.Encoding.sdig(fid, n_per_row, seed=seed, code_id=code)
    g = gpu.SdigEncoding.new_from_dims(fid, n_per_row, o.n_cols, seed, code)
    assert g.n_cols == o.n_cols and g.n_per_row == n_per_row
    nl = gpu.limbs(fid)
    row = np.zeros(o.n_cols * nl, np.uint64)
    row[:n_per_row * nl] = rand_elems(oracle, fid, n_per_row, seed + 100)
    want = o.encode(row)
    got = g.encode(row.copy())
    assert np.array_equal(got.reshape(-1), want)


def test_sdig_encode_rows_batched(gpu, oracle):
    fid, n_per_row = 1, 3000
    o = oracle.Encoding.sdig(fid, n_per_row, seed=9, code_id=3)
    g = gpu.SdigEncoding.new_from_dims(fid, n_per_row, o.n_cols, 9)
    nl = 2
    rows = np.zeros((5, o.n_cols, nl), np.uint64)
    for r in range(5):
        rows[r, :n_per_row] = rand_elems(oracle, fid, n_per_row, r).reshape(-1, nl)
    got = g.encode_rows(rows.copy())
    for r in range(5):
        assert np.array_equal(got[r].reshape(-1), o.encode(rows[r].reshape(-1)))


@pytest.mark.parametrize("fid", [0, 1, 3])
@pytest.mark.parametrize("n_valid_of", ["full", "ragged"])
def test_sdig_encode_rows_device_strided(gpu, oracle, hipmem, fid, n_valid_of):
    """lcpc_encode_rows_device on SDIG with separate, strided source and destination rows and a
    ragged message (n_valid < n_per_row: the rest of each message reads as zero).  The input
    transpose writes the message part of every destination row, the output transpose only the
    parity part; padding words past n_cols in a destination row stay untouched.  Also in place."""
    n_per_row, seed, R = 1500, 11, 37
    o = oracle.Encoding.sdig(fid, n_per_row, seed=seed, code_id=3)
    g = gpu.SdigEncoding.new_from_dims(fid, n_per_row, o.n_cols, seed)
    nl, nc = gpu.limbs(fid), o.n_cols
    nv = n_per_row if n_valid_of == "full" else n_per_row - 123
    ss, ds = n_per_row + 5, nc + 3
    src = np.zeros((R, ss, nl), np.uint64)
    for r in range(R):
        src[r, :nv] = rand_elems(oracle, fid, nv, seed + r).reshape(-1, nl)
    sentinel = np.uint64(0xA5A5A5A5A5A5A5A5)
    dst = np.full((R, ds, nl), sentinel, np.uint64)
    d_src, d_dst = hipmem.to_device(src), hipmem.to_device(dst)
    try:
        g.encode_rows_device(d_src, ss, nv, d_dst, ds, R)
        got = hipmem.to_host(d_dst, np.empty_like(dst))
    finally:
        hipmem.free(d_src)
        hipmem.free(d_dst)
    assert np.all(got[:, nc:] == sentinel)
    for r in range(R):
        row = np.zeros((nc, nl), np.uint64)
        row[:nv] = src[r, :nv]
        assert np.array_equal(got[r, :nc].reshape(-1), o.encode(row.reshape(-1))), r
    # in place: rows of n_cols whose message part holds the coefficients
    rows = np.zeros((R, nc, nl), np.uint64)
    rows[:, :n_per_row] = src[:, :n_per_row]
    d = hipmem.to_device(rows)
    try:
        g.encode_rows_device(d, nc, n_per_row, d, nc, R)
        got2 = hipmem.to_host(d, np.empty_like(rows))
    finally:
        hipmem.free(d)
    for r in range(R):
        assert np.array_equal(got2[r].reshape(-1), o.encode(rows[r].reshape(-1))), r
    # on a caller's stream (the scratch codeword is taken and fenced on that stream)
    import ctypes as C
    H = hipmem.L
    H.hipStreamCreate.argtypes = [C.POINTER(C.c_void_p)]
    H.hipStreamSynchronize.argtypes = [C.c_void_p]
    H.hipStreamDestroy.argtypes = [C.c_void_p]
    st = C.c_void_p()
    assert H.hipStreamCreate(C.byref(st)) == 0
    d_src, d_dst = hipmem.to_device(src), hipmem.to_device(dst)
    try:
        g.encode_rows_device(d_src, ss, nv, d_dst, ds, R, stream=st.value)
        assert H.hipStreamSynchronize(st) == 0
        got3 = hipmem.to_host(d_dst, np.empty_like(dst))
    finally:
        hipmem.free(d_src)
        hipmem.free(d_dst)
        H.hipStreamDestroy(st)
    assert np.array_equal(got3, got)


def test_sdig_dims_and_errors(gpu, oracle):
    L = oracle.lib()
    for code in range(1, 7):
        assert gpu.SdigEncoding.n_col_opens(code) == L.of_sdig_n_col_opens(code)
    for fid in [0, 1, 3]:
        for n in [1000, 1 << 16, 1 << 20, 1 << 24]:
            assert gpu.SdigEncoding.n_per_row_for(fid, n) == L.of_sdig_new_np(fid, 3, n)
    o = oracle.Encoding.sdig(1, 300, seed=0, code_id=3)
    with pytest.raises(gpu.LcpcError):
        gpu.SdigEncoding.new_from_dims(1, 300, o.n_cols + 1, 0)
    with pytest.raises(gpu.LcpcError):
        gpu.SdigEncoding.new_from_dims(1, 20, 64, 0)  # n_per_row must exceed baselen
    g = gpu.SdigEncoding.new_from_dims(1, 300, o.n_cols, 0)
    assert g.dims_ok(300, o.n_cols) and not g.dims_ok(300, o.n_cols - 1)
    assert g.get_n_col_opens() == o.n_col_opens and g.get_n_degree_tests() == o.n_degree_tests
    with pytest.raises(gpu.LcpcError):
        g.encode(np.zeros(2 * (o.n_cols - 1), np.uint64))


def _commit_both(gpu, oracle, fid, length, seed, code=3):
    L = oracle.lib()
    np_ = L.of_sdig_new_np(fid, code, length)
    o_enc = oracle.Encoding.sdig(fid, np_, seed=seed, code_id=code)
    g_enc = gpu.SdigEncoding.new(fid, length, seed, code)
    assert g_enc.n_per_row == np_ and g_enc.n_cols == o_enc.n_cols
    coeffs = rand_elems(oracle, fid, length, seed + 1)
    return coeffs, g_enc, o_enc, gpu.LcCommit.commit(coeffs, g_enc), oracle.Commit(o_enc, coeffs)


@pytest.mark.parametrize("fid,length,seed", [(1, 3000, 0), (0, 20000, 1), (1, 1 << 16, 0),
                                             (3, 5000, 2), (4, 4000, 3)])
def test_sdig_commit_matches_oracle(gpu, oracle, fid, length, seed):
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, fid, length, seed)
    assert g.get_n_rows() == o.n_rows and g.get_n_cols() == o.n_cols
    assert np.array_equal(g.coeffs.reshape(-1), o.coeffs)
    assert np.array_equal(g.comm.reshape(-1), o.comm)
    assert g.hashes == o.hashes
    assert g.get_root() == o.root()


@pytest.mark.parametrize("fid,length,seed", [(1, 10000, 4), (0, 1 << 14, 5), (3, 4097, 6)])
def test_sdig_commit_device_input(gpu, oracle, hipmem, fid, length, seed):
    # device input: the transpose writes the message part and the padded coefficient copy
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, fid, length, seed)
    d = hipmem.to_device(coeffs)
    try:
        gd = gpu.LcCommit.commit_device(d, length, g_enc)
        assert gd.get_root() == o.root()
        assert np.array_equal(gd.coeffs.reshape(-1), o.coeffs)
        assert np.array_equal(gd.comm.reshape(-1), o.comm)
        del gd
    finally:
        hipmem.free(d)


# (0, 3001) and (2, 2001) have an odd n_per_row (2569, 2001): the second p_random vector then
# starts 8 bytes off a 16-byte boundary, so the results come back through the 8-byte copy path
@pytest.mark.parametrize("fid,length,seed", [(1, 3000, 0), (0, 20000, 1), (3, 2500, 2), (0, 3001, 5),
                                             (2, 2001, 6)])
def test_sdig_prove_verify_matches_oracle(gpu, oracle, fid, length, seed):
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, fid, length, seed)
    root = g.get_root()
    x = oracle.ChaCha(seed_u64=seed + 7).field_random(fid, 1)
    inner, outer = oracle.eval_tensors(fid, x, g.get_n_per_row(), g.get_n_rows())
    nco = g_enc.get_n_col_opens()

    def tr_g():
        t = gpu.Transcript(b"test transcript")
        t.append_message(b"polycommit", root)
        t.append_message(b"ncols", nco.to_bytes(8, "big"))
        return t

    pf = g.prove(outer, g_enc, tr_g())
    opf = o.prove(o_enc, outer, oracle.standard_transcript(nco, root))
    assert np.array_equal(pf.p_eval.reshape(-1), opf.p_eval)
    assert np.array_equal(np.concatenate(pf.p_random_vec).reshape(-1), opf.p_random)
    cols = pf.columns
    assert np.array_equal(np.concatenate([c.col for c in cols]).reshape(-1), opf.cols)
    assert b"".join(b"".join(c.path) for c in cols) == opf.paths.tobytes()
    ev = pf.verify(root, outer, inner, g_enc, tr_g())
    rc, oev = opf.verify(root, outer, inner, o_enc, oracle.standard_transcript(nco, root))
    assert rc == 0 and np.array_equal(ev, oev)
    # a tampered opened column is rejected with the oracle's error
    bad = [gpu.LcColumn(c.col.copy(), list(c.path)) for c in cols]
    bad[3].col[0, 0] ^= 1
    pf_bad = gpu.LcEvalProof.from_parts(fid, pf.n_cols, pf.p_eval, pf.p_random_vec, bad)
    with pytest.raises(gpu.VerifierError) as e:
        pf_bad.verify(root, outer, inner, g_enc, tr_g())
    assert e.value.kind == "ColumnDegree"


def test_sdig_golden_fixture(gpu):
    import hashlib
    g = json.load(open(os.path.join(HERE, "golden", "golden.json")))["brakedown_ft127_4096_seed0"]
    enc = gpu.SdigEncoding.new_from_dims(g["field"], g["n_per_row"], g["n_cols"], g["seed"])
    nl = gpu.limbs(g["field"])
    row = np.zeros(g["n_cols"] * nl, np.uint64)
    row[:g["n_per_row"] * nl] = gpu.field_random(g["field"], g["n_per_row"], g["coeff_seed"]).reshape(-1)
    out = enc.encode(row)
    assert hashlib.sha256(out.tobytes()).hexdigest() == g["encoded_row_sha256"]
