"""GPU at BASELINE.json's full size (cfg3: Ft127, 2^24 coefficients, 512 x 32768 -> 65536).

* Bit-exactness against the oracle at the full size: the oracle (oracle/, 16 host threads)
  commits and proves the same polynomial in about a second, so root, hashes, p_random, p_eval,
  the opened columns and their paths are compared whole.
* Size-independent properties on top (lcpc-2d/src/tests.rs:193-234 and :136-191 restated):
  encode -> ifft_oi round trip on sampled rows, linearity of the encoding, leaves recomputed
  from opened columns, verify accepting the proof and rejecting a tampered one.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

LOG_LEN = 24


@pytest.fixture(scope="module")
def cfg3(gpu, oracle):
    oracle.lib().of_set_threads(min(16, len(os.sched_getaffinity(0))))
    fid, n = gpu.FT127, 1 << LOG_LEN
    coeffs = oracle.random_coeffs(fid, n)
    enc = gpu.LigeroEncoding.new(fid, n)
    comm = gpu.LcCommit.commit(coeffs, enc)
    o_enc = oracle.Encoding.ligero_new(fid, n)
    o_comm = oracle.Commit(o_enc, coeffs)
    return dict(fid=fid, n=n, coeffs=coeffs, enc=enc, comm=comm, o_enc=o_enc, o_comm=o_comm)


def _transcript(L, root, nco):
    tr = L.Transcript(b"test transcript")
    tr.append_message(b"polycommit", root)
    tr.append_message(b"ncols", nco.to_bytes(8, "big"))
    return tr


def test_cfg3_dims(cfg3):
    c = cfg3["comm"]
    assert (c.get_n_rows(), c.get_n_per_row(), c.get_n_cols()) == (512, 32768, 65536)
    assert cfg3["enc"].get_n_col_opens() == 309 and cfg3["enc"].get_n_degree_tests() == 2


def test_cfg3_commit_matches_oracle(cfg3):
    c, o = cfg3["comm"], cfg3["o_comm"]
    assert c.get_root() == o.root()
    assert c.hashes == bytes(o.hashes)
    assert np.array_equal(c.comm.reshape(-1), o.comm.reshape(-1))


def test_cfg3_prove_matches_oracle(gpu, oracle, cfg3):
    fid, c, o = cfg3["fid"], cfg3["comm"], cfg3["o_comm"]
    nco = cfg3["enc"].get_n_col_opens()
    x = oracle.ChaCha(seed_u64=7).field_random(fid, 1)
    inner, outer = oracle.eval_tensors(fid, x, c.get_n_per_row(), c.get_n_rows())
    pf = c.prove(outer, cfg3["enc"], _transcript(gpu, c.get_root(), nco))
    op = o.prove(cfg3["o_enc"], outer, oracle.standard_transcript(nco, o.root()))
    assert np.array_equal(pf.p_eval.reshape(-1), op.p_eval)
    assert all(np.array_equal(a.reshape(-1), b.reshape(-1))
               for a, b in zip(pf.p_random_vec, op.p_random.reshape(len(pf.p_random_vec), -1)))
    cols = np.stack([col.col for col in pf.columns]).reshape(-1)
    assert np.array_equal(cols, op.cols.reshape(-1))
    assert b"".join(b"".join(col.path) for col in pf.columns) == op.paths.tobytes()
    # verify accepts, and agrees with the oracle's evaluation
    ev = pf.verify(c.get_root(), outer, inner, cfg3["enc"], _transcript(gpu, c.get_root(), nco))
    rc, o_ev = op.verify(o.root(), outer, inner, cfg3["o_enc"], oracle.standard_transcript(nco, o.root()))
    assert rc == 0 and np.array_equal(ev.reshape(-1), o_ev)
    # a tampered root is rejected (ColumnPath)
    bad = bytes([c.get_root()[0] ^ 1]) + c.get_root()[1:]
    with pytest.raises(gpu.VerifierError):
        pf.verify(bad, outer, inner, cfg3["enc"], _transcript(gpu, bad, nco))


def test_cfg3_rows_decode_to_coefficients(oracle, cfg3):
    """encode -> ifft_oi round trip (lcpc-2d/src/tests.rs:222-234) on sampled rows."""
    fid, c = cfg3["fid"], cfg3["comm"]
    nr, npr, nc, nl = c.get_n_rows(), c.get_n_per_row(), c.get_n_cols(), oracle.limbs(fid)
    comm = c.comm.reshape(nr, nc * nl)
    coeffs = c.coeffs.reshape(nr, npr * nl)
    for r in [0, 1, 255, 300, nr - 1]:
        back = oracle.ifft_oi(fid, comm[r].copy())
        assert np.array_equal(back[:npr * nl], coeffs[r])
        assert not back[npr * nl:].any()


def test_cfg3_encoding_is_linear(gpu, oracle, cfg3):
    """Enc(a + b) = Enc(a) + Enc(b) column by column, at the full 512 x 65536 shape."""
    fid, n = cfg3["fid"], cfg3["n"]
    nl = oracle.limbs(fid)
    p = oracle.modulus(fid)
    a = cfg3["coeffs"]
    b = oracle.random_coeffs(fid, n, 99)
    ai = oracle.ints_from_limbs(a.reshape(-1, nl)[:4096], nl)
    bi = oracle.ints_from_limbs(b.reshape(-1, nl)[:4096], nl)
    s = oracle.limbs_from_ints([(x + y) % p for x, y in zip(ai, bi)], nl)
    ab = a.copy().reshape(-1, nl)
    ab[:4096] = s.reshape(-1, nl)          # a + b on the first 4096 coefficients, a elsewhere
    bb = np.zeros_like(ab)
    bb[:4096] = b.reshape(-1, nl)[:4096]   # b on the first 4096 coefficients, 0 elsewhere
    enc = cfg3["enc"]
    ca, cb, cab = cfg3["comm"], gpu.LcCommit.commit(bb.reshape(-1), enc), gpu.LcCommit.commit(ab.reshape(-1), enc)
    cols = [0, 1, 777, 32768, 65535]
    for j in cols:
        x = oracle.ints_from_limbs(ca.open_column(j).col.reshape(-1), nl)
        y = oracle.ints_from_limbs(cb.open_column(j).col.reshape(-1), nl)
        z = oracle.ints_from_limbs(cab.open_column(j).col.reshape(-1), nl)
        assert [(u + v) % p for u, v in zip(x, y)] == z


def test_cfg3_leaves_from_opened_columns(oracle, cfg3):
    """leaf_j = BLAKE3(32 zero bytes || repr(column j)) (lcpc-2d/src/lib.rs:736-775)."""
    fid, c = cfg3["fid"], cfg3["comm"]
    nl = oracle.limbs(fid)
    hashes = c.hashes
    for j in [0, 5, 4096, 65535]:
        col = c.open_column(j).col.reshape(-1, nl)
        canon = oracle.from_mont(fid, col)
        msg = bytes(32) + b"".join(int(v).to_bytes(16, "little") for v in canon)
        assert oracle.blake3(msg) == hashes[32 * j:32 * j + 32]
