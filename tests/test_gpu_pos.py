"""GPU parity of the proof-of-storage producers (proof-of-storage/src) against the oracle."""
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
FT63 = 0
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def pos(gpu):
    from lcpc_proof_of_storage_amd import pos as P
    return P


def test_bytes_to_field_and_back(pos, oracle):
    rng = np.random.default_rng(1)
    for n in [1, 6, 7, 8, 55, 56, 57, 111, 112, 113, 999, 100003, 1 << 20]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        el = pos.convert_byte_vec_to_field_elements_vec(data)
        assert np.array_equal(el.reshape(-1), oracle.pos_bytes_to_field(data))
        assert pos.convert_field_elements_vec_to_byte_vec(el, n) == data


@pytest.mark.parametrize("off_in,off_out", [(0, 0), (8, 0), (0, 8)])
def test_bytes_to_field_device(gpu, oracle, hipmem, off_in, off_out):
    """lcpc_pos_bytes_to_field_device on 16-byte aligned buffers (the LDS-staged blocks of 2048
    elements plus a ragged tail) and on buffers only 8-byte aligned (the API's requirement: the
    per-thread path)."""
    import ctypes as C
    from lcpc_proof_of_storage_amd import _native as N
    rng = np.random.default_rng(2)
    n = 7 * 100000 + 3
    data = rng.integers(0, 256, n, dtype=np.uint8)
    d_in = hipmem.to_device(np.concatenate([np.zeros(off_in, np.uint8), data]))
    out = np.zeros((n + 6) // 7 + off_out // 8, np.uint64)
    d_out = hipmem.to_device(out)
    try:
        assert N.load().lcpc_pos_bytes_to_field_device(C.c_void_p(d_in + off_in), n, C.c_void_p(d_out + off_out),
                                                       None) == 0
        got = hipmem.to_host(d_out, out)[off_out // 8:]
        assert np.array_equal(got, oracle.pos_bytes_to_field(data.tobytes()))
    finally:
        hipmem.free(d_in)
        hipmem.free(d_out)


def test_default_dims_and_columns(pos, oracle):
    for n in [1, 5, 86, 1000, 4097, (1 << 30) // 8, 153391690]:
        assert pos.get_aspect_ratio_default_from_field_len(n) == oracle.pos_default_dims(n)
    assert pos.get_aspect_ratio_default_from_file_len(1 << 30) == (16384, 32768, 309)
    for seed, amount, mx in [(1337, 256, 32768), (1, 4, 10), (9, 10, 5)]:
        assert pos.get_column_indicies_from_random_seed(seed, amount, mx) == \
            oracle.pos_column_indices(seed, amount, mx)


@pytest.mark.parametrize("fid", [0, 1, 3])
def test_side_vectors(pos, oracle, fid):
    x = oracle.ChaCha(seed_u64=5).field_random(fid, 1)
    left, right = pos.form_side_vectors_for_polynomial_evaluation_from_point(x, 37, 64, fid)
    ol, orr = oracle.pos_side_vectors(fid, x, 37, 64)
    assert np.array_equal(left.reshape(-1), ol) and np.array_equal(right.reshape(-1), orr)


@pytest.mark.parametrize("fid", [0, 1, 3, 4])
@pytest.mark.parametrize("log_n", [0, 1, 2, 5, 11, 12, 13, 16])
def test_ifft_oi_matches_oracle(pos, oracle, fid, log_n):
    n = 1 << log_n
    rows = 3
    nl = oracle.limbs(fid)
    data = oracle.random_coeffs(fid, rows * n, 40 + log_n)
    got = pos.ifft_oi_rows(data.reshape(rows, n, nl), fid)
    for r in range(rows):
        want = oracle.ifft_oi(fid, data[r * n * nl:(r + 1) * n * nl])
        assert np.array_equal(got[r].reshape(-1), want)


def test_ifft_oi_errors(gpu, pos):
    with pytest.raises(gpu.FFTError):
        pos.ifft_oi_rows(np.zeros((1, 6, 1), np.uint64))


@pytest.mark.parametrize("np_,nc", [(4, 8), (8, 16), (1024, 2048), (8192, 32768)])
def test_eval_identity_and_parity(gpu, pos, oracle, np_, nc):
    """networking/tests.rs:374-466 on the GPU, and u^T Enc(M) bit-exact vs the oracle."""
    n = 32 if np_ <= 8 else np_ * 7 + 5
    coeffs = oracle.random_coeffs(FT63, n, 11)
    comm = pos.convert_file_data_to_commit(coeffs, pos.Commit(), pos.Specified(np_, nc))
    ocomm = oracle.Commit(oracle.Encoding.ligero(FT63, np_, nc), coeffs)
    assert comm.get_root() == ocomm.root()
    x = oracle.ChaCha(seed_u64=1337, rounds=8).field_random(FT63, 1)
    left, right = pos.form_side_vectors_for_polynomial_evaluation_from_point(x, comm.get_n_rows(), np_)
    r = pos.verifiable_polynomial_evaluation(comm, left)
    assert np.array_equal(r.reshape(-1), oracle.collapse(FT63, ocomm.comm, left, ocomm.n_rows, nc))
    dec = pos.decode_row(r)
    d = oracle.from_mont(FT63, dec.reshape(-1))
    assert all(v == 0 for v in d[np_:])
    p = 5102708120182849537
    got = sum(a * b for a, b in zip(d, oracle.from_mont(FT63, right.reshape(-1)))) % p
    xv = oracle.from_mont(FT63, x)[0]
    want = 0
    for c in reversed(oracle.from_mont(FT63, coeffs)):
        want = (want * xv + c) % p
    assert got == want


@pytest.mark.parametrize("n_bytes,dims", [
    (7 * 16384 * 20 + 12345, None),      # the default dims of the file length: the one-pass encode
    (7 * 16384 * 3, (16384, 32768)),      # whole rows, the one-pass encode
    (7 * 100 * 37 + 3, (100, 256)),       # other dims: packed, then the four-step encode; ragged row
    (13, (4, 8)),                         # two elements, one chunk per leaf (no merge)
    (7 * 1000 * 260 + 1, (1000, 2048)),   # many chunks per leaf, ragged last chunk
])
def test_commit_eval_fused(gpu, pos, oracle, hipmem, n_bytes, dims):
    """lcpc_pos_commit_eval_bytes_device (the request's commitment with u^T Enc(M) summed in the
    leaf pass) == lcpc_pos_commit_bytes_device + lcpc_pos_eval_encoded == the oracle"""
    rng = np.random.default_rng(n_bytes)
    data = rng.integers(0, 256, n_bytes, dtype=np.uint8)
    np_, nc = dims if dims else pos.get_aspect_ratio_default_from_file_len(n_bytes)[:2]
    enc = gpu.LigeroEncoding.new_from_dims(FT63, np_, nc)
    n_el = -(-n_bytes // 7)
    n_rows = -(-n_el // np_)
    x = oracle.ChaCha(seed_u64=1337, rounds=8).field_random(FT63, 1)
    left, _ = pos.form_side_vectors_for_polynomial_evaluation_from_point(x, n_rows, nc)
    d = hipmem.to_device(np.concatenate([data, np.zeros((-n_bytes) % 8 + 8, np.uint8)]))
    try:
        fc, fev = gpu.LcCommit.commit_pos_bytes_device_eval(d, n_bytes, enc, left)
        sc = gpu.LcCommit.commit_pos_bytes_device(d, n_bytes, enc)
    finally:
        hipmem.free(d)
    sev = pos.verifiable_polynomial_evaluation(sc, left)
    assert fc.get_root() == sc.get_root()
    assert np.array_equal(fev, sev)
    el = oracle.pos_bytes_to_field(data.tobytes())
    oc = oracle.Commit(oracle.Encoding.ligero(FT63, np_, nc), el)
    assert fc.get_root() == oc.root()
    assert np.array_equal(fev.reshape(-1), oracle.collapse(FT63, oc.comm, left, oc.n_rows, nc))


def test_commit_eval_fused_rejects(gpu, pos, hipmem):
    enc = gpu.LigeroEncoding.new_from_dims(FT63, 64, 128)
    d = hipmem.to_device(np.ones(7 * 64 * 3, np.uint8))
    try:
        with pytest.raises(gpu.LcpcError):  # left must have the commitment's n_rows (3) elements
            gpu.LcCommit.commit_pos_bytes_device_eval(d, 7 * 64 * 3, enc, np.zeros(4, np.uint64))
    finally:
        hipmem.free(d)


def test_request_types(gpu, pos, oracle):
    """CommitRequestType::{Leaves, ColumnsWithoutPath, ColumnsWithPath} (lcpc_online.rs:80-239)."""
    coeffs = oracle.random_coeffs(FT63, 5000, 3)
    np_, nc = 128, 256
    ocomm = oracle.Commit(oracle.Encoding.ligero(FT63, np_, nc), coeffs)
    cols = oracle.pos_column_indices(1337, 16, nc)
    leaves = pos.convert_file_data_to_commit(coeffs, pos.Leaves(cols), pos.Specified(np_, nc))
    hashes = ocomm.hashes
    assert leaves == [hashes[32 * c:32 * c + 32] for c in cols]
    got = pos.convert_file_data_to_commit(coeffs, pos.ColumnsWithoutPath(cols), pos.Specified(np_, nc))
    m = ocomm.comm.reshape(ocomm.n_rows, nc)
    for k, c in enumerate(cols):
        assert np.array_equal(got[k].reshape(-1), m[:, c])
    opened = pos.convert_file_data_to_commit(coeffs, pos.ColumnsWithPath(cols), pos.Specified(np_, nc))
    pos.client_online_verify_column_paths(ocomm.root(), cols, opened)
    with pytest.raises(pos.VerifierError):
        pos.client_online_verify_column_paths(ocomm.root(), cols[::-1], opened)
    comm = pos.convert_file_data_to_commit(coeffs, pos.Commit(), pos.Specified(np_, nc))
    for k, c in enumerate(cols):
        one = comm.open_column(c)
        assert np.array_equal(one.col, opened[k].col) and one.path == opened[k].path


def test_test_txt_golden(gpu, pos):
    g = json.load(open(os.path.join(HERE, "golden", "golden.json")))["pos_test_txt_square"]
    data = open(os.path.join(HERE, "golden", "pos_test.txt"), "rb").read()
    el = pos.convert_byte_vec_to_field_elements_vec(data)
    assert hashlib.sha256(el.tobytes()).hexdigest() == g["elems_sha256"]
    comm = pos.convert_file_data_to_commit(el, pos.Commit(), pos.Square())
    assert [comm.get_n_rows(), comm.get_n_per_row(), comm.get_n_cols()] == g["dims"]
    assert comm.get_root().hex() == g["root"]
    assert hashlib.sha256(comm.comm.tobytes()).hexdigest() == g["comm_sha256"]


def test_client_verification(gpu, pos, oracle):
    """The PoS client side (lcpc_online.rs:251-452): leaves recomputed locally (Leaves request),
    columns with and without paths, soundness counts, and each failure's error kind."""
    coeffs = oracle.random_coeffs(FT63, 7000, 4)
    np_, nc = 64, 128
    ocomm = oracle.Commit(oracle.Encoding.ligero(FT63, np_, nc), coeffs)
    root = ocomm.root()
    need = pos._get_POS_soundness_n_cols(np_, nc)
    cols = oracle.pos_column_indices(99, 20, nc)
    local = pos.convert_file_data_to_commit(coeffs, pos.Leaves(cols), pos.Specified(np_, nc))
    opened = pos.convert_file_data_to_commit(coeffs, pos.ColumnsWithPath(cols), pos.Specified(np_, nc))
    # hash_column_to_digest == the commitment's leaves
    assert pos.hash_columns_to_digests(opened) == [ocomm.hashes[32 * c:32 * c + 32] for c in cols]
    assert pos.hash_column_to_digest(opened[3]) == ocomm.hashes[32 * cols[3]:32 * cols[3] + 32]
    pos.client_verify_commitment(root, local, cols, opened, need)
    digests = [pos.hash_column_to_digest(c) for c in opened]
    pos.client_verify_commitment_without_full_columns(root, local, cols, digests, [c.path for c in opened], need)
    with pytest.raises(pos.VerifierError) as e:  # soundness count below the opened columns
        pos.client_verify_commitment(root, local, cols, opened, len(cols) - 1)
    assert e.value.kind == "NumColOpens"
    bad = [pos.LcColumn(c.col.copy(), c.path) for c in opened]
    bad[5].col[7, 0] ^= 1
    with pytest.raises(pos.VerifierError) as e:  # leaves differ from the local ones
        pos.client_verify_commitment(root, local, cols, bad, need)
    assert e.value.kind == "NumColOpens"
    bad_paths = [list(c.path) for c in opened]
    bad_paths[2][1] = bytes(32)
    with pytest.raises(pos.VerifierError) as e:
        pos.client_online_verify_column_paths_without_full_columns(root, cols, digests, bad_paths)
    assert e.value.kind == "ColumnEval"
    # the same check against the oracle's path verification
    for k, c in enumerate(cols):
        assert oracle.verify_path(digests[k], c, b"".join(opened[k].path), root)


def test_partial_and_full_polynomial_evaluation(gpu, pos, oracle):
    """verify_proper_partial_polynomial_evaluation / verifiable_full_polynomial_evaluation /
    left_multiply_unencoded_matrix_by_vector on a small file (lcpc_online.rs:454-566)."""
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, 7 * 64 * 40 - 11, dtype=np.uint8).tobytes()
    np_, nc = 64, 128
    el = oracle.pos_bytes_to_field(data)
    n_rows = -(-el.size // np_)
    comm = pos.convert_file_data_to_commit(el.reshape(-1, 1), pos.Commit(), pos.Specified(np_, nc))
    x = oracle.ChaCha(seed_u64=77).field_random(FT63, 1)
    # side vectors over the unencoded width: p(x) = <u^T M, right> with u = left
    left, right_np = pos.form_side_vectors_for_polynomial_evaluation_from_point(x, n_rows, np_)
    result = pos.verifiable_polynomial_evaluation(comm, left)            # u^T Enc(M), n_cols
    decoded = pos.left_multiply_unencoded_matrix_by_vector(data, np_, left)  # u^T M, n_per_row
    m = np.zeros(n_rows * np_, np.uint64)
    m[:el.size] = el
    assert np.array_equal(decoded.reshape(-1), oracle.collapse(FT63, m, left.reshape(-1), n_rows, np_))
    cols = sorted(oracle.pos_column_indices(5, 12, nc))
    opened = comm.open_columns(cols)
    pos.verify_proper_partial_polynomial_evaluation(left, result, cols, opened)
    tampered = result.copy().reshape(-1)
    tampered[cols[4]] ^= 1
    with pytest.raises(pos.VerifierError):
        pos.verify_proper_partial_polynomial_evaluation(left, tampered, cols, opened)
    # the full check: <u^T M, right> is p(x) for the file's polynomial, and Enc(u^T M) agrees
    # with the opened columns
    got = pos.verifiable_full_polynomial_evaluation(left, right_np, decoded, cols, opened, np_, nc)
    p = oracle.modulus(FT63)
    xv = oracle.from_mont(FT63, x)[0]
    want = 0
    for c in reversed(oracle.from_mont(FT63, m)):
        want = (want * xv + c) % p
    assert oracle.from_mont(FT63, got.reshape(-1))[0] == want
    bad = decoded.copy()
    bad[3, 0] = (int(bad[3, 0]) + 1) % p
    with pytest.raises(pos.VerifierError):
        pos.verifiable_full_polynomial_evaluation(left, right_np, bad, cols, opened, np_, nc)
    # server_retreive_columns (lcpc_online.rs:242-249) opens the same columns as the request path
    again = pos.server_retreive_columns(comm, cols)
    assert all(np.array_equal(a.col, b.col) and list(a.path) == list(b.path) for a, b in zip(again, opened))
    # the single-point wrapper (lcpc_online.rs:545-566) forms its side vectors over n_cols, as the
    # reference passes them, then runs the same check
    left_nc, right_nc = pos.form_side_vectors_for_polynomial_evaluation_from_point(x, n_rows, nc)
    dec_nc = pos.left_multiply_unencoded_matrix_by_vector(data, np_, left_nc)
    res_nc = pos.verifiable_polynomial_evaluation(comm, left_nc)
    pos.verify_proper_partial_polynomial_evaluation(left_nc, res_nc, cols, opened)
    got_w = pos.verify_full_polynomial_evaluation_wrapper_with_single_eval_point(x, dec_nc, n_rows, nc, cols,
                                                                                opened, np_)
    got_d = pos.verifiable_full_polynomial_evaluation(left_nc, right_nc, dec_nc, cols, opened, np_, nc)
    assert np.array_equal(got_w, got_d)
    bad_nc = dec_nc.copy()
    bad_nc[0, 0] = (int(bad_nc[0, 0]) + 1) % p
    with pytest.raises(pos.VerifierError):
        pos.verify_full_polynomial_evaluation_wrapper_with_single_eval_point(x, bad_nc, n_rows, nc, cols,
                                                                            opened, np_)
