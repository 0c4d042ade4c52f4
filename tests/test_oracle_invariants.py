"""CPU: the reference's own invariant tests, ported onto the oracle.

The reference has no fixed-value tests; what it pins are relations, restated here with
seeded inputs instead of thread_rng:
  lcpc-2d/src/tests.rs:125-132     log2
  lcpc-2d/src/tests.rs:136-149     merkle tree == serial merkleization
  lcpc-2d/src/tests.rs:151-165     collapse_columns == serial row combination
  lcpc-2d/src/tests.rs:167-191     open_column paths verify
  lcpc-2d/src/tests.rs:193-234     commit encodes R-S evaluations (ifft_oi inverts encode)
  lcpc-2d/src/tests.rs:236-316     prove/verify round trip (+ rebuild from parts)
  lcpc-2d/src/tests.rs:318-413     two proofs on one transcript
  lcpc-ligero-pc/src/tests.rs:22-41  get_dims invariants
  lcpc-brakedown-pc/src/tests.rs:77-93  matgen + encode
plus the SURVEY.md §8 dims tables (derived values).
"""
import math
import struct

import numpy as np
import pytest

import pyref

FT63, FT127, FT255 = 0, 1, 3
N_COL_OPENS_2D_TEST = 128  # lcpc-2d/src/tests.rs:31


def _get_dims_2d(length, rho):
    """The lcpc-2d test module's LigeroEncoding::_get_dims (lcpc-2d/src/tests.rs:35-57)."""
    nc = 1 << max(0, math.ceil(math.log2(math.ceil(math.sqrt(length) / rho))))
    np_ = int(math.floor(nc * rho))
    nr = (length + np_ - 1) // np_
    return nr, np_, nc


def _random_coeffs_rho(rng, fid=FT63):
    """lcpc-2d/src/tests.rs:415-426 with a seeded generator."""
    lgl = 8 + int(rng.integers(0, 8))
    base = 1 << (lgl - 1)
    length = base + int(rng.integers(0, base))
    rho = float(rng.uniform(0.1, 0.9))
    return length, rho


def _enc_2d(oracle, fid, length, rho):
    nr, np_, nc = _get_dims_2d(length, rho)
    return oracle.Encoding.ligero(fid, np_, nc, N_COL_OPENS_2D_TEST, 2)


def _coeffs(oracle, fid, n, seed):
    return oracle.random_coeffs(fid, n, seed)


def _canon(oracle, fid, a):
    return oracle.from_mont(fid, a)


def test_log2(oracle):
    for idx in range(31):
        assert oracle.lib().of_log2(1 << idx) == idx
    # ceil semantics via next_power_of_two (lcpc-2d/src/lib.rs:857-859)
    assert oracle.lib().of_log2(1000) == 10
    assert oracle.lib().of_log2(1025) == 11


def test_merkle_tree_matches_serial(oracle):
    rng = np.random.default_rng(1)
    for n in [2, 4, 16, 64]:
        leaves = rng.integers(0, 256, size=32 * n, dtype=np.uint8)
        out = np.zeros(32 * (n - 1), np.uint8)
        oracle.lib().of_merkle_tree(leaves.ctypes.data_as(oracle.u8p), n, out.ctypes.data_as(oracle.u8p))
        level = [leaves[32 * i:32 * i + 32].tobytes() for i in range(n)]
        serial = []
        while len(level) > 1:
            level = [pyref.blake3(level[2 * i] + level[2 * i + 1]) for i in range(len(level) // 2)]
            serial += level
        assert out.tobytes() == b"".join(serial)


@pytest.mark.parametrize("fid", [FT63, FT127, FT255, 4])
def test_hash_columns_matches_spec(oracle, fid):
    f = pyref.Field(fid)
    n_rows, n_cols = 5, 8
    comm = _coeffs(oracle, fid, n_rows * n_cols, 11)
    out = np.zeros(32 * n_cols, np.uint8)
    oracle.lib().of_hash_columns(fid, oracle.p64(comm), n_rows, n_cols, out.ctypes.data_as(oracle.u8p))
    vals = _canon(oracle, fid, comm)
    for j in range(n_cols):
        msg = bytes(32) + b"".join(f.repr_bytes(vals[r * n_cols + j]) for r in range(n_rows))
        assert out[32 * j:32 * j + 32].tobytes() == pyref.blake3(msg), j


@pytest.mark.parametrize("fid", [FT63, FT127, FT255])
def test_collapse_columns_matches_serial(oracle, fid):
    f = pyref.Field(fid)
    rng = np.random.default_rng(fid)
    for n_rows, n_per_row in [(1, 7), (9, 16), (33, 5)]:
        coeffs = _coeffs(oracle, fid, n_rows * n_per_row, int(rng.integers(1, 1 << 30)))
        tensor = _coeffs(oracle, fid, n_rows, int(rng.integers(1, 1 << 30)))
        poly = np.zeros(n_per_row * f.nl, np.uint64)
        oracle.lib().of_collapse_columns(fid, oracle.p64(coeffs), oracle.p64(tensor), oracle.p64(poly),
                                         n_rows, n_per_row)
        c, t = _canon(oracle, fid, coeffs), _canon(oracle, fid, tensor)
        want = [sum(t[r] * c[r * n_per_row + j] for r in range(n_rows)) % f.p for j in range(n_per_row)]
        assert _canon(oracle, fid, poly) == want


def test_open_column_paths_verify(oracle):
    rng = np.random.default_rng(5)
    for _ in range(3):
        length, rho = _random_coeffs_rho(rng)
        enc = _enc_2d(oracle, FT63, length, rho)
        comm = oracle.Commit(enc, _coeffs(oracle, FT63, length, int(rng.integers(1, 1 << 30))))
        root = comm.root()
        path_len = int(math.log2(comm.n_cols))
        for col in [0, comm.n_cols - 1, int(rng.integers(0, comm.n_cols))]:
            colv = np.zeros(comm.n_rows, np.uint64)
            path = np.zeros(32 * path_len, np.uint8)
            assert oracle.lib().of_open_column(comm.ptr, col, oracle.p64(colv), path.ctypes.data_as(oracle.u8p)) == 0
            rp, keep = oracle.p8(root)
            assert oracle.lib().of_verify_column_path(FT63, oracle.p64(colv), comm.n_rows,
                                                      path.ctypes.data_as(oracle.u8p), path_len, col, rp) == 1
            # a flipped path byte must fail
            path[3] ^= 1
            assert oracle.lib().of_verify_column_path(FT63, oracle.p64(colv), comm.n_rows,
                                                      path.ctypes.data_as(oracle.u8p), path_len, col, rp) == 0
        # column number out of range is a ProverError::ColumnNumber
        colv = np.zeros(comm.n_rows, np.uint64)
        path = np.zeros(32 * path_len, np.uint8)
        assert oracle.lib().of_open_column(comm.ptr, comm.n_cols, oracle.p64(colv),
                                           path.ctypes.data_as(oracle.u8p)) != 0


def _eval_setup(oracle, fid, comm, seed):
    x = oracle.ChaCha(seed_u64=seed).field_random(fid, 1)
    inner, outer = oracle.eval_tensors(fid, x, comm.n_per_row, comm.n_rows)
    return x, inner, outer


def _poly_eval(oracle, fid, coeffs, x):
    f = pyref.Field(fid)
    xv = _canon(oracle, fid, x)[0]
    acc = 0
    for c in reversed(_canon(oracle, fid, coeffs)):
        acc = (acc * xv + c) % f.p
    return acc


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_commit_encodes_reed_solomon(oracle, seed):
    """lcpc-2d/src/tests.rs:193-234: eval_outer, eval_outer_fft, ifft_oi."""
    rng = np.random.default_rng(100 + seed)
    length, rho = _random_coeffs_rho(rng)
    enc = _enc_2d(oracle, FT63, length, rho)
    coeffs = _coeffs(oracle, FT63, length, seed + 9)
    comm = oracle.Commit(enc, coeffs)
    x, inner, outer = _eval_setup(oracle, FT63, comm, seed)
    eval1 = _poly_eval(oracle, FT63, comm.coeffs, x)
    f = pyref.Field(FT63)
    flat = np.zeros(comm.n_per_row, np.uint64)
    oracle.lib().of_collapse_columns(FT63, oracle.p64(comm.coeffs), oracle.p64(outer), oracle.p64(flat),
                                     comm.n_rows, comm.n_per_row)
    inn = _canon(oracle, FT63, inner)
    eval2 = sum(a * b for a, b in zip(_canon(oracle, FT63, flat), inn)) % f.p
    assert eval1 == eval2
    fft = np.zeros(comm.n_cols, np.uint64)
    oracle.lib().of_collapse_columns(FT63, oracle.p64(comm.comm), oracle.p64(outer), oracle.p64(fft),
                                     comm.n_rows, comm.n_cols)
    poly = _canon(oracle, FT63, oracle.ifft_oi(FT63, fft))
    assert all(v == 0 for v in poly[comm.n_per_row:])
    eval3 = sum(a * b for a, b in zip(poly, inn)) % f.p
    assert eval2 == eval3


def _rate_msg(rho):
    return struct.pack(">d", rho)


def _tr_2d(oracle, root, rho):
    tr = oracle.Transcript(b"test transcript")
    tr.append_message(b"polycommit", root)
    tr.append_message(b"rate", _rate_msg(rho))
    tr.append_message(b"ncols", N_COL_OPENS_2D_TEST.to_bytes(8, "big"))
    return tr


def _from_parts(oracle, pf):
    return oracle.Proof.from_parts(pf.fid, pf.n_cols, pf.n_per_row, pf.n_rows, pf.p_eval.copy(),
                                   pf.p_random.copy(), pf.cols.copy(), pf.paths.copy(),
                                   pf.n_degree_tests, pf.n_col_opens, pf.path_len)


@pytest.mark.parametrize("seed", [3, 4])
def test_end_to_end(oracle, seed):
    """lcpc-2d/src/tests.rs:236-316 (bincode round trip -> rebuild from parts)."""
    rng = np.random.default_rng(200 + seed)
    length, rho = _random_coeffs_rho(rng)
    enc = _enc_2d(oracle, FT63, length, rho)
    comm = oracle.Commit(enc, _coeffs(oracle, FT63, length, seed))
    root = comm.root()
    x, inner, outer = _eval_setup(oracle, FT63, comm, seed)
    eval1 = _poly_eval(oracle, FT63, comm.coeffs, x)
    pf = comm.prove(enc, outer, _tr_2d(oracle, root, rho))
    pf2 = _from_parts(oracle, pf)
    enc2 = oracle.Encoding.ligero(FT63, pf.n_per_row, pf.n_cols, N_COL_OPENS_2D_TEST, 2)
    for proof in (pf, pf2):
        rc, out = proof.verify(root, outer, inner, enc2, _tr_2d(oracle, root, rho))
        assert rc == 0
        assert _canon(oracle, FT63, out)[0] == eval1


def test_end_to_end_two_proofs(oracle):
    """lcpc-2d/src/tests.rs:318-413: transcript continuation across two proofs."""
    rng = np.random.default_rng(7)
    length, rho = _random_coeffs_rho(rng)
    enc = _enc_2d(oracle, FT63, length, rho)
    comm = oracle.Commit(enc, _coeffs(oracle, FT63, length, 77))
    root = comm.root()
    x, inner, outer = _eval_setup(oracle, FT63, comm, 77)
    eval1 = _poly_eval(oracle, FT63, comm.coeffs, x)

    def reprefix(tr):
        tr.append_message(b"polycommit", root)
        tr.append_message(b"rate", _rate_msg(rho))
        tr.append_message(b"ncols", N_COL_OPENS_2D_TEST.to_bytes(8, "big"))

    def challenge(tr):
        key = tr.challenge_bytes(b"ligero-pc//challenge", 32)
        return oracle.ChaCha(key).field_random(FT63, 1)

    tr1 = _tr_2d(oracle, root, rho)
    pf = comm.prove(enc, outer, tr1)
    ch_p = challenge(tr1)
    reprefix(tr1)
    pf2 = comm.prove(enc, outer, tr1)

    tr2 = _tr_2d(oracle, root, rho)
    enc2 = oracle.Encoding.ligero(FT63, pf.n_per_row, pf.n_cols, N_COL_OPENS_2D_TEST, 2)
    rc, out = pf.verify(root, outer, inner, enc2, tr2)
    assert rc == 0 and _canon(oracle, FT63, out)[0] == eval1
    assert np.array_equal(challenge(tr2), ch_p)
    reprefix(tr2)
    rc, out = pf2.verify(root, outer, inner, enc2, tr2)
    assert rc == 0 and _canon(oracle, FT63, out)[0] == eval1
    # the second proof opens different columns than the first
    assert not np.array_equal(pf.col_idx, pf2.col_idx)


def test_verify_error_codes(oracle):
    """VerifierError precedence (lcpc-2d/src/lib.rs:862-982): tensor lengths, then columns."""
    enc = oracle.Encoding.ligero_new(FT127, 1 << 12)
    comm = oracle.Commit(enc, _coeffs(oracle, FT127, 1 << 12, 3))
    root = comm.root()
    x, inner, outer = _eval_setup(oracle, FT127, comm, 3)
    tr = oracle.standard_transcript(enc.n_col_opens, root)
    pf = comm.prove(enc, outer, tr)
    rc, _ = pf.verify(root, outer, inner, enc, oracle.standard_transcript(enc.n_col_opens, root))
    assert rc == 0
    rc, _ = pf.verify(root, outer[:-2], inner, enc, oracle.standard_transcript(enc.n_col_opens, root))
    assert rc == 5  # OuterTensor
    rc, _ = pf.verify(root, outer, inner[:-2], enc, oracle.standard_transcript(enc.n_col_opens, root))
    assert rc == 6  # InnerTensor
    bad_root = bytes([root[0] ^ 1]) + root[1:]
    # same challenges, wrong root: degree and eval checks pass, the path check fails
    rc, _ = pf.verify(bad_root, outer, inner, enc, oracle.standard_transcript(enc.n_col_opens, root))
    assert rc == 2  # ColumnPath
    # a different transcript changes the degree-test tensors first
    rc, _ = pf.verify(bad_root, outer, inner, enc, oracle.standard_transcript(enc.n_col_opens, bad_root))
    assert rc == 4  # ColumnDegree
    # tamper an opened column value: degree test / eval checks fire before the path check
    pf2 = _from_parts(oracle, pf)
    cols = pf.cols.copy()
    cols[0] ^= 1
    pf3 = oracle.Proof.from_parts(pf.fid, pf.n_cols, pf.n_per_row, pf.n_rows, pf.p_eval.copy(),
                                  pf.p_random.copy(), cols, pf.paths.copy(), pf.n_degree_tests,
                                  pf.n_col_opens, pf.path_len)
    rc, _ = pf3.verify(root, outer, inner, enc, oracle.standard_transcript(enc.n_col_opens, root))
    assert rc == 4  # ColumnDegree
    rc, _ = pf2.verify(root, outer, inner, enc, oracle.standard_transcript(enc.n_col_opens, root))
    assert rc == 0


def test_ligero_get_dims_invariants(oracle):
    """lcpc-ligero-pc/src/tests.rs:22-41 (rho = 1/2, Ft63), seeded and thinned."""
    rng = np.random.default_rng(9)
    for _ in range(32):
        lgl = 8 + int(rng.integers(0, 8))
        base = 1 << (lgl - 1)
        for _ in range(32):
            length = base + int(rng.integers(0, base))
            nr, np_, nc = oracle.ligero_dims(FT63, length)
            assert nr * np_ >= length
            assert (nr - 1) * np_ < length
            assert np_ * 2 <= nc
            assert np_ < nc and nc & (nc - 1) == 0


@pytest.mark.parametrize("fid,log_len,rho,want,ndt", [
    (FT127, 16, (1, 2), (32, 2048, 4096), 2),
    (FT127, 20, (1, 2), (128, 8192, 16384), 2),
    (FT127, 24, (1, 2), (512, 32768, 65536), 2),
    (FT63, 24, (1, 2), (512, 32768, 65536), 3),
    (FT255, 24, (1, 2), (256, 65536, 131072), 1),
    (FT127, 24, (1, 4), (512, 32768, 131072), 2),
])
def test_survey_dims_table(oracle, fid, log_len, rho, want, ndt):
    """SURVEY.md §8 Ligero dims table (derived from lcpc-ligero-pc/src/lib.rs:61-112)."""
    assert oracle.ligero_dims(fid, 1 << log_len, rho) == want
    L = oracle.lib()
    assert L.of_n_degree_tests(128, want[2], L.of_field_num_bits(fid) - 1) == ndt


def test_ligero_col_opens(oracle):
    assert oracle.lib().of_ligero_n_col_opens(1, 2) == 309
    assert oracle.lib().of_ligero_n_col_opens(1, 4) == 189


def test_brakedown_dims_sdig3_ft127_2_24(oracle):
    """SdigCode3, Ft127, 2^24 -> 72 x 235173, 6 levels, 6593 opens, 4,077,302 nnz.

    SURVEY.md gives n_cols = 363568; that figure sums the postcodes' input widths.  The
    reference's codeword_length (lcpc-brakedown-pc/src/encode.rs:18-33) adds the postcodes'
    OUTPUT rows and the last postcode's column count (the R-S length), which totals
    ceil(n * r) = ceil(235173 * 1.521) = 357699.
    """
    L = oracle.lib()
    assert L.of_sdig_n_col_opens(3) == 6593
    n = 1 << 24
    np_ = L.of_sdig_new_np(FT127, 3, n)
    assert np_ == 235173
    assert (n + np_ - 1) // np_ == 72
    enc = oracle.Encoding.sdig(FT127, np_, seed=0, code_id=3)
    assert enc.n_cols == 357699 == -(-235173 * 1521 // 1000)
    assert L.of_sdig_levels(enc.ptr) == 6
    import ctypes as C
    nnz = 0
    shapes = {0: [], 1: []}
    for lvl in range(6):
        for which in (0, 1):
            r, c = C.c_size_t(), C.c_size_t()
            nnz += L.of_sdig_matrix(enc.ptr, lvl, which, C.byref(r), C.byref(c), None, None, None)
            shapes[which].append((c.value, r.value))
    assert nnz == 4077302
    assert shapes[0] == [(235173, 41861), (41861, 7452), (7452, 1327), (1327, 237), (237, 43), (43, 8)]
    assert shapes[1] == [(63671, 58855), (11335, 10475), (2019, 1864), (361, 331), (66, 58), (13, 10)]


@pytest.mark.parametrize("fid", [FT63, FT127])
def test_brakedown_encode_systematic_and_linear(oracle, fid):
    """lcpc-brakedown-pc/src/tests.rs:77-93 (matgen + encode), with the linear-code properties."""
    f = pyref.Field(fid)
    enc = oracle.Encoding.sdig(fid, 1000, seed=0, code_id=3)
    n = enc.n_cols
    a = np.zeros(n * f.nl, np.uint64)
    b = np.zeros(n * f.nl, np.uint64)
    a[:1000 * f.nl] = _coeffs(oracle, fid, 1000, 1)
    b[:1000 * f.nl] = _coeffs(oracle, fid, 1000, 2)
    ea, eb = enc.encode(a), enc.encode(b)
    assert np.array_equal(ea[:1000 * f.nl], a[:1000 * f.nl])  # systematic
    s = np.zeros_like(a)
    oracle.lib().of_add(fid, oracle.p64(a), oracle.p64(b), oracle.p64(s), n)
    es = enc.encode(s)
    s2 = np.zeros_like(a)
    oracle.lib().of_add(fid, oracle.p64(ea), oracle.p64(eb), oracle.p64(s2), n)
    assert np.array_equal(es, s2)  # linear


def test_brakedown_end_to_end(oracle):
    """lcpc-brakedown-pc/src/tests.rs:192-374 shape: commit/prove/verify with SdigCode3 seed 0."""
    length = 3000
    L = oracle.lib()
    np_ = L.of_sdig_new_np(FT127, 3, length)
    enc = oracle.Encoding.sdig(FT127, np_, seed=0, code_id=3)
    comm = oracle.Commit(enc, _coeffs(oracle, FT127, length, 5))
    root = comm.root()
    x, inner, outer = _eval_setup(oracle, FT127, comm, 5)
    tr = oracle.standard_transcript(enc.n_col_opens, root)
    pf = comm.prove(enc, outer, tr)
    rc, out = pf.verify(root, outer, inner, enc, oracle.standard_transcript(enc.n_col_opens, root))
    assert rc == 0
    assert _canon(oracle, FT127, out)[0] == _poly_eval(oracle, FT127, comm.coeffs, x)
