"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit for bit.

Every test here runs the product library liblcpc_mi.so on the MI355X and compares with
oracle/ (the CPU restatement of the reference path).  Sizes are ones the oracle finishes in
seconds; full-size (2^24) behaviour is covered by size-independent properties in
test_gpu_properties.py.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIELDS = [0, 1, 2, 3, 4]  # Ft63, Ft127, Ft191, Ft255, Ft253_192


def rand_elems(oracle, fid, n, seed):
    return oracle.ChaCha(seed_u64=seed).field_random(fid, n)


@pytest.mark.parametrize("fid", FIELDS)
@pytest.mark.parametrize("log_n", [1, 2, 3, 5, 8, 11, 12, 13, 14, 15, 16])
def test_encode_matches_fffft(gpu, oracle, fid, log_n):
    """LcEncoding::encode (fft_io) on one row, zero-padded half (rho = 1/2)."""
    n = 1 << log_n
    np_ = n // 2
    nl = oracle.limbs(fid)
    enc = gpu.RsEncoding.new(fid, np_, n, 4, 1)
    row = np.zeros(n * nl, np.uint64)
    row[:np_ * nl] = rand_elems(oracle, fid, np_, 100 + log_n)
    want = oracle.fft_io(fid, row)
    got = row.copy()
    enc.encode(got)
    assert np.array_equal(got, want)


@pytest.mark.parametrize("fid", [0, 1])
@pytest.mark.parametrize("log_n", [13, 14, 15, 16])
def test_encode_full_rows(gpu, oracle, fid, log_n):
    """Full-length (no zero padding) batched rows."""
    n = 1 << log_n
    nl = oracle.limbs(fid)
    enc = gpu.RsEncoding.new(fid, 1, n, 4, 1)
    rows = rand_elems(oracle, fid, 3 * n, 7 + log_n).reshape(3, n * nl)
    got = enc.encode_rows(rows.copy()).reshape(3, n * nl)
    for r in range(3):
        assert np.array_equal(got[r], oracle.fft_io(fid, rows[r]))


def _words(v: int, nl: int):
    return [(v >> (64 * i)) & ((1 << 64) - 1) for i in range(nl)]


@pytest.mark.parametrize("fid", FIELDS)
@pytest.mark.parametrize("log_n", [13, 14, 16])  # (14: Ft127's cfg2 shape, 1024-thread radix-2^2 passes)
@pytest.mark.parametrize("pattern", ["max", "alternating", "max_zero_half", "max_halfz"])
def test_encode_extreme_values(gpu, oracle, fid, log_n, pattern):
    """Rows of the largest residue p - 1 (raw Montgomery words), alternating 0 / p - 1, and a
    full-length row whose second half is p - 1: every butterfly sum and difference of the
    passes' [0, 2p) residues then sits at its carry / borrow boundary."""
    n = 1 << log_n
    nl = oracle.limbs(fid)
    pm1 = oracle.modulus(fid) - 1
    w = np.array(_words(pm1, nl), np.uint64)
    if pattern == "max":
        row = np.tile(w, n)
    elif pattern == "alternating":
        row = np.zeros(n * nl, np.uint64)
        row.reshape(n, nl)[1::2] = w
    else:
        row = np.zeros(n * nl, np.uint64)
        half = slice(n // 2, None) if pattern == "max_zero_half" else slice(0, n // 2)
        row.reshape(n, nl)[half] = w
    if pattern == "max_halfz":  # rate-1/2 row: the upper half is known zero (pass A's first stage)
        enc = gpu.RsEncoding.new(fid, n // 2, n, 4, 1)
        got = row.copy()
        enc.encode(got)
    else:
        enc = gpu.RsEncoding.new(fid, 1, n, 4, 1)
        got = enc.encode_rows(row.reshape(1, -1).copy()).reshape(-1)
    assert np.array_equal(got, oracle.fft_io(fid, row))


def test_encode_errors(gpu):
    enc = gpu.RsEncoding.new(1, 8, 16, 4, 1)
    bad = np.zeros(12 * 2, np.uint64)
    with pytest.raises(gpu.FFTError) as e:
        enc.encode(bad)
    assert e.value.kind == "NotPowerOfTwo"
    with pytest.raises(gpu.FFTError) as e:
        enc.encode(np.zeros(32 * 2, np.uint64))
    assert e.value.kind == "WrongSizePrecomp"


def _commit_both(gpu, oracle, fid, n_per_row, n_cols, length, seed, nco=16, ndt=2):
    coeffs = rand_elems(oracle, fid, length, seed)
    g_enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, ndt)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, nco, ndt)
    g = gpu.LcCommit.commit(coeffs, g_enc)
    o = oracle.Commit(o_enc, coeffs)
    return coeffs, g_enc, o_enc, g, o


@pytest.mark.parametrize("fid,n_per_row,n_cols,length", [
    (1, 2048, 4096, 1 << 16),      # cfg1 shape
    (0, 100, 256, 3000),           # ragged: last row partial
    (1, 1, 2, 5),                  # smallest R-S code
    (0, 700, 1024, 700),           # one row
    (3, 512, 1024, 4096),
    (4, 300, 512, 2000),           # big-endian repr field
    (2, 300, 512, 2000),           # Ft191: 24-byte elements straddle BLAKE3 blocks and chunks
    (2, 2048, 4096, 100 * 2048 + 9),  # Ft191, 100 rows: a 2424-byte leaf message (3 chunks)
    (1, 8192, 16384, 128 * 8192),  # cfg2 shape: 128 x 8192 -> 16384
])
def test_commit_matches_oracle(gpu, oracle, fid, n_per_row, n_cols, length):
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, fid, n_per_row, n_cols, length, 11)
    assert g.get_n_rows() == o.n_rows and g.get_n_cols() == o.n_cols
    assert np.array_equal(g.comm.reshape(-1), o.comm)
    assert np.array_equal(g.coeffs.reshape(-1), o.coeffs)
    assert g.hashes == o.hashes
    assert g.get_root() == o.root()


@pytest.mark.parametrize("n_rows", [1000, 1100, 2040, 2100, 8180, 8300, 8400])
def test_leaf_merge_chunk_counts(gpu, oracle, n_rows):
    """Column leaves of 8, 9, 16, 17, 65 and 65 chunks (Ft63: 32 + 8 n_rows bytes): the chaining
    values fold in aligned groups of 8 chunks, then across groups (blake3.hip k_leaf_merge_groups,
    k_leaf_merge) -- whole groups, a ragged last group, a last group of one chunk, one group only."""
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, 0, 4, 8, 4 * n_rows, 5)
    assert g.get_n_rows() == n_rows
    assert g.hashes == o.hashes
    assert g.get_root() == o.root()


@pytest.mark.parametrize("fid", FIELDS)
@pytest.mark.parametrize("chunks", [1, 2, 3])
def test_column_major_leaves_by_chunk_count(gpu, oracle, fid, chunks):
    """Column-major leaves (lcpc_hash_field_columns: the SDIG commitments' and the PoS files'
    layout) of 1, 2 and 3 BLAKE3 chunks -- two-chunk messages (cfg4's 1184-byte leaves) are hashed
    whole by one wave (blake3.hip k_leaf_chunks_cm, fuse2) -- against the oracle's leaves of the
    same matrix (lcpc-2d/src/lib.rs:736-775)."""
    from lcpc_proof_of_storage_amd import pos
    wb = 8 * gpu.limbs(fid)
    n_rows = {1: (1024 - 32) // wb, 2: (2048 - 32) // wb - 1, 3: (2048 - 32) // wb + 3}[chunks]
    n_cols = 300
    m = rand_elems(oracle, fid, n_rows * n_cols, 31 + chunks).reshape(n_rows, n_cols, -1)
    want = oracle.hash_columns(fid, m.reshape(-1), n_rows, n_cols)
    cols = [np.ascontiguousarray(m[:, j, :]) for j in range(n_cols)]
    got = pos.hash_columns_to_digests(cols, fid)
    assert b"".join(got) == want


def test_commit_empty_and_oversized_inputs(gpu, oracle):
    """commit's shape asserts (lcpc-2d/src/lib.rs:659-661) are LcpcError here, not a panic: an
    empty polynomial has no rows ((n_rows - 1) underflows in the reference); a device commit of
    zero elements likewise.  Encoding dims that break dims_ok are refused at construction."""
    enc = gpu.RsEncoding.new(1, 8, 16, 4, 1)
    with pytest.raises(gpu.LcpcError):
        gpu.LcCommit.commit(np.zeros(0, np.uint64), enc)
    with pytest.raises(gpu.LcpcError):
        gpu.LcCommit.commit_device(0, 0, enc)
    with pytest.raises(gpu.LcpcError):
        gpu.RsEncoding.new(1, 8, 12, 4, 1)      # n_cols not a power of two
    with pytest.raises(gpu.LcpcError):
        gpu.RsEncoding.new(1, 16, 16, 4, 1)     # no redundancy (n_per_row == n_cols)
    # one element: a single row whose tail is zero-padded, as the reference pads
    c = gpu.LcCommit.commit(rand_elems(oracle, 1, 1, 3), enc)
    o = oracle.Commit(oracle.Encoding.ligero(1, 8, 16, 4, 1), rand_elems(oracle, 1, 1, 3))
    assert c.get_n_rows() == 1 and c.get_root() == o.root()


@pytest.mark.parametrize("fid,n_per_row,n_cols,length", [
    (1, 2048, 4096, 1 << 16),          # small-row kernel
    (0, 100, 256, 3000),               # ragged, small-row kernel
    (1, 1, 2, 5),
    (1, 8192, 16384, 128 * 8192),      # two-pass kernels, fused coefficient copy
    (1, 8192, 16384, 100 * 8192 + 77), # two-pass, ragged last row
    (0, 8192, 16384, 5000),            # two-pass, a single partial row (no full rows)
    (3, 2048, 8192, 3 * 2048 + 1),     # two-pass Ft255, rate 1/4
    (2, 8192, 16384, 50 * 8192 + 5),   # two-pass Ft191
])
def test_commit_device_matches_oracle(gpu, oracle, hipmem, fid, n_per_row, n_cols, length):
    """lcpc_commit_new_device: coefficients already in HBM (bench path); the commitment's own
    coefficient matrix is written by the first NTT pass."""
    coeffs = rand_elems(oracle, fid, length, 13)
    g_enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, 16, 2)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, 16, 2)
    d = hipmem.to_device(coeffs)
    try:
        g = gpu.LcCommit.commit_device(d, length, g_enc)
        o = oracle.Commit(o_enc, coeffs)
        assert np.array_equal(g.coeffs.reshape(-1), o.coeffs)
        assert np.array_equal(g.comm.reshape(-1), o.comm)
        assert g.hashes == o.hashes
        assert g.get_root() == o.root()
        # the caller's buffer is only read
        assert np.array_equal(hipmem.to_host(d, np.zeros_like(coeffs)), coeffs)
        # the device codeword holds the canonical values of the reference's comm
        from lcpc_proof_of_storage_amd import _native as N
        assert N.load().lcpc_commit_comm_canonical(g._h) == 1
        dev = hipmem.to_host(N.load().lcpc_commit_device_comm(g._h), np.zeros_like(o.comm))
        nl = oracle.limbs(fid)
        canon = np.zeros_like(o.comm)
        oracle.lib().of_to_canonical(fid, oracle.p64(o.comm), oracle.p64(canon), o.comm.size // nl)
        assert np.array_equal(dev, canon)
        del g
    finally:
        hipmem.free(d)


@pytest.mark.parametrize("fid,n_per_row,n_cols,length,nco,ndt", [
    (1, 2048, 4096, 1 << 16, 309, 2),
    (0, 100, 256, 3000, 128, 3),
    (3, 256, 512, 1000, 40, 1),
    (4, 64, 128, 1000, 20, 2),
    (2, 512, 1024, 60 * 512 + 3, 64, 2),  # Ft191
])
def test_prove_verify_matches_oracle(gpu, oracle, fid, n_per_row, n_cols, length, nco, ndt):
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, fid, n_per_row, n_cols, length, 5, nco, ndt)
    root = g.get_root()
    x = rand_elems(oracle, fid, 1, 77)
    inner, outer = oracle.eval_tensors(fid, x, n_per_row, g.get_n_rows())
    g_tr = gpu.Transcript(b"test transcript")
    g_tr.append_message(b"polycommit", root)
    g_tr.append_message(b"ncols", nco.to_bytes(8, "big"))
    o_tr = oracle.standard_transcript(nco, root)
    gp = g.prove(outer, g_enc, g_tr)
    op = o.prove(o_enc, outer, o_tr)
    assert np.array_equal(gp.p_eval.reshape(-1), op.p_eval)
    pr = np.concatenate([v.reshape(-1) for v in gp.p_random_vec]) if ndt else np.zeros(0, np.uint64)
    assert np.array_equal(pr, op.p_random)
    cols = gp.columns
    nl = oracle.limbs(fid)
    o_cols = op.cols.reshape(nco, -1)
    o_paths = op.paths.tobytes()
    for k, c in enumerate(cols):
        assert np.array_equal(c.col.reshape(-1), o_cols[k])
        assert b"".join(c.path) == o_paths[k * 32 * op.path_len:(k + 1) * 32 * op.path_len]
    # transcripts stay in lock step after the proof
    assert g_tr.challenge_bytes(b"after", 32) == o_tr.challenge_bytes(b"after", 32)
    # verify on the GPU and on the oracle; the evaluation equals p(x)
    v_tr = gpu.Transcript(b"test transcript")
    v_tr.append_message(b"polycommit", root)
    v_tr.append_message(b"ncols", nco.to_bytes(8, "big"))
    ev = gp.verify(root, outer, inner, g_enc, v_tr)
    rc, o_ev = op.verify(root, outer, inner, o_enc, oracle.standard_transcript(nco, root))
    assert rc == 0
    assert np.array_equal(ev.reshape(-1), o_ev)
    want = oracle.from_mont(fid, np.zeros(nl, np.uint64))[0]
    acc = 0
    p = oracle.modulus(fid)
    xs = oracle.from_mont(fid, x)[0]
    cs = oracle.from_mont(fid, coeffs)
    for c in reversed(cs):
        acc = (acc * xs + c) % p
    assert oracle.from_mont(fid, ev.reshape(-1))[0] == acc


def test_verify_rejects_tampering(gpu, oracle):
    fid, n_per_row, n_cols, nco = 1, 512, 1024, 64
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, fid, n_per_row, n_cols, 40 * 512, 9, nco, 2)
    root = g.get_root()
    x = rand_elems(oracle, fid, 1, 3)
    inner, outer = oracle.eval_tensors(fid, x, n_per_row, g.get_n_rows())

    def tr():
        t = gpu.Transcript(b"test transcript")
        t.append_message(b"polycommit", root)
        return t

    pf = g.prove(outer, g_enc, tr())
    pf.verify(root, outer, inner, g_enc, tr())
    cols = pf.columns

    def rebuilt(p_eval=None, p_random=None, columns=None):
        return gpu.LcEvalProof.from_parts(fid, n_cols, pf.p_eval if p_eval is None else p_eval,
                                          pf.p_random_vec if p_random is None else p_random,
                                          cols if columns is None else columns)

    # untouched rebuild verifies
    rebuilt().verify(root, outer, inner, g_enc, tr())
    # flip one opened value -> degree test fails first (ColumnDegree precedes ColumnEval/Path)
    bad_cols = [gpu.LcColumn(c.col.copy(), list(c.path)) for c in cols]
    bad_cols[3].col[5, 0] ^= 1
    with pytest.raises(gpu.VerifierError) as e:
        rebuilt(columns=bad_cols).verify(root, outer, inner, g_enc, tr())
    assert e.value.kind in ("ColumnDegree", "ColumnEval", "ColumnPath")
    # corrupt one Merkle path digest -> ColumnPath
    bad_cols = [gpu.LcColumn(c.col.copy(), list(c.path)) for c in cols]
    p0 = bytearray(bad_cols[0].path[2]); p0[0] ^= 0xff
    bad_cols[0].path[2] = bytes(p0)
    with pytest.raises(gpu.VerifierError) as e:
        rebuilt(columns=bad_cols).verify(root, outer, inner, g_enc, tr())
    assert e.value.kind == "ColumnPath"
    # wrong root -> ColumnPath
    with pytest.raises(gpu.VerifierError) as e:
        pf.verify(bytes(32), outer, inner, g_enc, tr())
    # wrong tensor sizes
    with pytest.raises(gpu.VerifierError) as e:
        pf.verify(root, outer[:-2], inner, g_enc, tr())
    assert e.value.kind == "OuterTensor"
    with pytest.raises(gpu.VerifierError) as e:
        pf.verify(root, outer, inner[:-2], g_enc, tr())
    assert e.value.kind == "InnerTensor"
    with pytest.raises(gpu.ProverError) as e:
        g.prove(outer[:-2], g_enc, tr())
    assert e.value.kind == "OuterTensor"


def test_open_column_and_free_functions(gpu, oracle):
    fid = 0
    coeffs, g_enc, o_enc, g, o = _commit_both(gpu, oracle, fid, 200, 512, 5000, 21)
    root = g.get_root()
    nl = oracle.limbs(fid)
    for col in [0, 1, 255, 511, 300]:
        c = g.open_column(col)
        assert gpu.verify_column_path(fid, c, col, root)
        assert not gpu.verify_column_path(fid, c, col ^ 1, root)
        ocol = np.zeros(o.n_rows * nl, np.uint64)
        opath = np.zeros(32 * 9, np.uint8)
        oracle.lib().of_open_column(o.ptr, col, oracle.p64(ocol), opath.ctypes.data_as(oracle.u8p))
        assert np.array_equal(c.col.reshape(-1), ocol)
        assert b"".join(c.path) == opath.tobytes()
    with pytest.raises(gpu.ProverError) as e:
        g.open_column(512)
    assert e.value.kind == "ColumnNumber"
    # collapse_columns / verify_column_value against the oracle
    t = rand_elems(oracle, fid, g.get_n_rows(), 4)
    got = gpu.collapse_columns(fid, g.coeffs, t, g.get_n_rows(), 200)
    want = np.zeros(200 * nl, np.uint64)
    oracle.lib().of_collapse_columns(fid, oracle.p64(o.coeffs), oracle.p64(t), oracle.p64(want),
                                     o.n_rows, 200)
    assert np.array_equal(got.reshape(-1), want)
    # merkle_tree / hash_columns
    leaves = o.hashes[:32 * 512]
    assert gpu.merkle_tree(leaves) == o.hashes[32 * 512:]
    assert gpu.hash_columns(fid, g.comm, o.n_rows, 512) == leaves
    comm = g.comm.reshape(o.n_rows, 512, nl)
    col7 = gpu.LcColumn(np.ascontiguousarray(comm[:, 7, :]), [])
    # linearity: sum_r t[r] * comm[r][j] == encode(collapse(coeffs, t))[j]
    row = np.zeros((512, nl), np.uint64)
    row[:200] = got
    g_enc.encode(row)
    assert gpu.verify_column_value(fid, col7, t, row[7])
    assert not gpu.verify_column_value(fid, col7, t, row[8])
