"""Multilinear constructors end to end on the GPU (ports of end_to_end_one_proof_ml,
lcpc-ligero-pc/src/tests.rs:265-315 and lcpc-brakedown-pc/src/tests.rs:239-289): new_ml(n_vars)
gives power-of-two dims covering exactly 2^n_vars monomials, and a proof over it verifies with an
encoding rebuilt from the proof's dims (new_from_dims), to the evaluation p(x) (checked by a
big-int Horner; the reference draws lgl and x from a thread RNG, here they are parameters)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
FT63 = 0


@pytest.fixture(scope="module")
def L(gpu):
    from lcpc_proof_of_storage_amd import lcpc2d
    return lcpc2d


def _end_to_end(gpu, L, oracle, comm, enc, enc2_of, coeffs, seed):
    root = comm.get_root()
    x = oracle.random_coeffs(FT63, 1, seed)
    inner, outer = oracle.eval_tensors(FT63, x, comm.get_n_per_row(), comm.get_n_rows())

    def tr():
        t = gpu.Transcript(b"test transcript")
        t.append_message(b"polycommit", root)
        t.append_message(b"ncols", enc.get_n_col_opens().to_bytes(8, "big"))
        return t

    pf = comm.prove(outer, enc, tr())
    ev = pf.verify(root, outer, inner, enc2_of(pf), tr())
    p = oracle.modulus(FT63)
    xv = oracle.from_mont(FT63, x)[0]
    want = 0
    for c in reversed(oracle.from_mont(FT63, coeffs)):
        want = (want * xv + c) % p
    assert oracle.from_mont(FT63, ev.reshape(-1))[0] == want


@pytest.mark.parametrize("lgl", [12, 15, 19])
def test_ligero_end_to_end_one_proof_ml(gpu, L, oracle, lgl):
    coeffs = oracle.random_coeffs(FT63, 1 << lgl, lgl)
    enc = L.LigeroEncoding.new_ml(FT63, lgl)
    comm = L.LcCommit.commit(coeffs, enc)
    n_rows, n_per_row = comm.get_n_rows(), comm.get_n_per_row()
    assert n_rows != 1
    assert n_rows & (n_rows - 1) == 0 and n_per_row & (n_per_row - 1) == 0 and n_rows * n_per_row == 1 << lgl
    _end_to_end(gpu, L, oracle, comm, enc,
                lambda pf: L.LigeroEncoding.new_from_dims(FT63, pf.get_n_per_row(), pf.get_n_cols()),
                coeffs, 100 + lgl)


@pytest.mark.parametrize("lgl", [5, 9, 14, 18])
def test_brakedown_end_to_end_one_proof_ml(gpu, L, oracle, lgl):
    coeffs = oracle.random_coeffs(FT63, 1 << lgl, lgl)
    enc = L.SdigEncoding.new_ml(FT63, lgl, 0)
    comm = L.LcCommit.commit(coeffs, enc)
    assert comm.get_n_rows() * comm.get_n_per_row() == 1 << lgl
    _end_to_end(gpu, L, oracle, comm, enc,
                lambda pf: L.SdigEncoding.new_from_dims(FT63, pf.get_n_per_row(), pf.get_n_cols(), 0),
                coeffs, 200 + lgl)
