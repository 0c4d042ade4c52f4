"""serde + bincode forms of LcRoot, LcColumn and LcCommit (lcpc-2d/src/lib.rs:193-283, 331-422,
424-514), the proof's already covered by tests/test_gpu_parity.py.  Ports the root / proof
round trip of lcpc-2d/src/tests.rs:255-313 (verify with the deserialized root and proof gives the
same evaluation), and checks a deserialized commitment (lcpc_commit_from_parts) proves exactly as
the one it was serialized from, for a Ligero and a Brakedown commitment."""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def L(gpu):
    from lcpc_proof_of_storage_amd import lcpc2d
    return lcpc2d


def _tr(gpu, root, nco):
    t = gpu.Transcript(b"test transcript")
    t.append_message(b"polycommit", root)
    t.append_message(b"ncols", nco.to_bytes(8, "big"))
    return t


def test_root_round_trip_and_verify(gpu, L, oracle):
    fid, n_per_row, n_cols = 0, 256, 512
    enc = L.LigeroEncoding.new_from_dims(fid, n_per_row, n_cols)
    coeffs = oracle.random_coeffs(fid, 40 * n_per_row, 11)
    comm = L.LcCommit.commit(coeffs, enc)
    root = L.LcRoot.new_from_root_digest(comm.get_root())
    enc_root = root.to_bincode()
    assert enc_root == struct.pack("<Q", 32) + comm.get_root()
    x = oracle.random_coeffs(fid, 1, 12)
    inner, outer = oracle.eval_tensors(fid, x, n_per_row, comm.get_n_rows())
    nco = enc.get_n_col_opens()
    pf = comm.prove(outer, enc, _tr(gpu, root.as_ref(), nco))
    encoded = pf.to_bincode()
    res = pf.verify(root.as_ref(), outer, inner, enc, _tr(gpu, root.as_ref(), nco))
    root2 = L.LcRoot.from_bincode(enc_root)
    pf2 = L.LcEvalProof.from_bincode(fid, encoded)
    enc3 = L.LigeroEncoding.new_from_dims(fid, pf2.get_n_per_row(), pf2.get_n_cols())
    res2 = pf2.verify(root2.as_ref(), outer, inner, enc3, _tr(gpu, root2.into_raw(), nco))
    assert np.array_equal(res, res2) and root2 == root
    for bad in (struct.pack("<Q", 31) + bytes(31), enc_root + b"\0", enc_root[:-1]):
        with pytest.raises(L.LcpcError):
            L.LcRoot.from_bincode(bad)


def test_column_round_trip(gpu, L, oracle):
    fid = 1
    enc = L.LigeroEncoding.new_from_dims(fid, 64, 128)
    comm = L.LcCommit.commit(oracle.random_coeffs(fid, 20 * 64, 13), enc)
    col = comm.open_column(77)
    b = col.to_bincode(fid)
    nl = L.limbs(fid)
    assert len(b) == 8 + comm.get_n_rows() * 8 * nl + 8 + 7 * 40
    back = L.LcColumn.from_bincode(fid, b)
    assert np.array_equal(back.col, col.col) and back.path == col.path
    assert L.verify_column_path(fid, back, 77, comm.get_root())
    with pytest.raises(L.LcpcError):
        L.LcColumn.from_bincode(fid, b[:-3])


def _check_commit_round_trip(gpu, L, oracle, fid, comm, enc, n_rows):
    data = comm.to_bincode()
    nl = L.limbs(fid)
    n_cols, n_per_row = comm.get_n_cols(), comm.get_n_per_row()
    n_hashes = len(comm.hashes) // 32
    assert len(data) == (8 + n_rows * n_cols * 8 * nl) + (8 + n_rows * n_per_row * 8 * nl) + 24 + 8 + n_hashes * 40
    back = L.LcCommit.from_bincode(fid, data)
    assert back.get_root() == comm.get_root()
    assert (back.get_n_rows(), back.get_n_cols(), back.get_n_per_row()) == (n_rows, n_cols, n_per_row)
    assert np.array_equal(back.comm, comm.comm) and np.array_equal(back.coeffs, comm.coeffs)
    assert back.hashes == comm.hashes
    assert back.to_bincode() == data
    back.check(enc)
    for c in (0, n_cols // 3, n_cols - 1):
        a, b = comm.open_column(c), back.open_column(c)
        assert np.array_equal(a.col, b.col) and a.path == b.path
    x = oracle.random_coeffs(fid, 1, 21)
    inner, outer = oracle.eval_tensors(fid, x, n_per_row, n_rows)
    nco = enc.get_n_col_opens()
    p1 = comm.prove(outer, enc, _tr(gpu, comm.get_root(), nco))
    p2 = back.prove(outer, enc, _tr(gpu, back.get_root(), nco))
    assert p1.to_bincode() == p2.to_bincode()
    p2.verify(back.get_root(), outer, inner, enc, _tr(gpu, back.get_root(), nco))


@pytest.mark.parametrize("fid,n_per_row,n_cols,rows", [(1, 512, 1024, 37), (0, 100, 256, 9), (3, 64, 128, 5)])
def test_commit_round_trip_ligero(gpu, L, oracle, fid, n_per_row, n_cols, rows):
    enc = L.LigeroEncoding.new_from_dims(fid, n_per_row, n_cols)
    comm = L.LcCommit.commit(oracle.random_coeffs(fid, rows * n_per_row - 3, 20), enc)
    _check_commit_round_trip(gpu, L, oracle, fid, comm, enc, rows)


def test_commit_round_trip_brakedown(gpu, L, oracle):
    fid, length = 1, 4096 * 6
    enc = L.SdigEncoding.new(fid, length, 0)
    comm = L.LcCommit.commit(oracle.random_coeffs(fid, length, 22), enc)
    _check_commit_round_trip(gpu, L, oracle, fid, comm, enc, comm.get_n_rows())


def test_commit_from_bincode_rejects(gpu, L, oracle):
    fid = 0
    enc = L.LigeroEncoding.new_from_dims(fid, 16, 32)
    data = L.LcCommit.commit(oracle.random_coeffs(fid, 100, 23), enc).to_bincode()
    with pytest.raises(L.LcpcError):
        L.LcCommit.from_bincode(fid, data[:-1])            # truncated
    with pytest.raises(L.LcpcError):
        L.LcCommit.from_bincode(fid, data + b"\0")         # trailing bytes
    # one hash too few: the count disagrees with 2 next_pow2(n_cols) - 1
    n_h = struct.unpack_from("<Q", data, len(data) - 63 * 40 - 8)[0]
    assert n_h == 63
    short = data[:len(data) - 63 * 40 - 8] + struct.pack("<Q", 62) + data[len(data) - 62 * 40:]
    with pytest.raises(L.LcpcError):
        L.LcCommit.from_bincode(fid, short)
