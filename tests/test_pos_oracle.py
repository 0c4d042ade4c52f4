"""CPU: the proof-of-storage producers on the oracle, pinned by the reference's own tests.

  fields.rs:286-300                 bytes -> field elements -> bytes round trip
  lcpc_online.rs:588-601            decode_row (ifft_oi) inverts encode
  networking/tests.rs:374-466       u^T Enc(M) -> decode_row -> . right == p(x), tall and wide
  networking/server.rs:1139-1182    default dims (1 GiB -> 16384 / 32768, 9363 rows)
  networking/client.rs:443-456      column choice (ChaCha8 + choose_multiple), restated twice
The reference's committed fixture test_files/test.txt (598 B) is committed as
tests/golden/pos_test.txt (data, not source).
"""
import os

import numpy as np
import pytest

import pyref

FT63 = 0
HERE = os.path.dirname(os.path.abspath(__file__))


def test_bytes_round_trip(oracle):
    rng = np.random.default_rng(0)
    for n in [0, 1, 6, 7, 8, 55, 56, 57, 999]:
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        el = oracle.pos_bytes_to_field(data)
        assert len(el) == (n + 6) // 7
        assert all(int(v) < (1 << 56) for v in el)  # always valid raw limbs (< p)
        assert oracle.pos_field_to_bytes(el, n) == data
        # independent restatement: 7-byte LE chunks, zero padded
        padded = data + bytes(-n % 7)
        want = [int.from_bytes(padded[7 * i:7 * i + 7], "little") for i in range(len(padded) // 7)]
        assert [int(v) for v in el] == want


def test_default_dims(oracle):
    # a 1 GiB file, dims from file_len / 8 (WRITTEN_BYTES_WIDTH)
    assert oracle.pos_default_dims((1 << 30) // 8) == (16384, 32768, 309)
    n_elems = -(-(1 << 30) // 7)
    assert n_elems == 153391690 and -(-n_elems // 16384) == 9363
    assert oracle.pos_default_dims(86) == (16, 32, 32)  # test.txt, soundness capped at n_cols
    for n in [1, 2, 3, 4, 5, 17, 1000, 4096, 4097]:
        np_, nc, s = oracle.pos_default_dims(n)
        assert np_ & (np_ - 1) == 0 and nc == 1 << np_.bit_length() and s <= nc


def _choose_multiple_py(oracle, seed, amount, max_index):
    rng = oracle.ChaCha(seed_u64=seed, rounds=8)
    res = list(range(min(amount, max_index)))
    if len(res) == amount:
        for i in range(max_index - amount):
            k = rng.gen_range_u32(0, i + 1 + amount)
            if k < amount:
                res[k] = amount + i
    return res


@pytest.mark.parametrize("seed,amount,max_index", [(1337, 256, 32768), (1, 4, 10), (5, 10, 10),
                                                   (7, 20, 5), (0, 1, 1)])
def test_column_indices(oracle, seed, amount, max_index):
    got = oracle.pos_column_indices(seed, amount, max_index)
    assert got == _choose_multiple_py(oracle, seed, amount, max_index)
    assert len(got) == min(amount, max_index) and len(set(got)) == len(got)
    assert all(0 <= c < max_index for c in got)


def _commit_pos(oracle, elems, np_, nc):
    enc = oracle.Encoding.ligero(FT63, np_, nc)
    return enc, oracle.Commit(enc, elems)


@pytest.mark.parametrize("np_,nc", [(4, 8), (8, 16), (16, 64)])
def test_eval_identity(oracle, np_, nc):
    """networking/tests.rs:374-466: decode_row(u^T Enc(M)) . right == p(x)."""
    f = pyref.Field(FT63)
    coeffs = oracle.random_coeffs(FT63, 32, 11)
    enc, comm = _commit_pos(oracle, coeffs, np_, nc)
    x = oracle.ChaCha(seed_u64=1337, rounds=8).field_random(FT63, 1)
    left, right = oracle.pos_side_vectors(FT63, x, comm.n_rows, comm.n_per_row)
    r = oracle.collapse(FT63, comm.comm, left, comm.n_rows, comm.n_cols)
    dec = oracle.ifft_oi(FT63, r)
    d, rt = oracle.from_mont(FT63, dec), oracle.from_mont(FT63, right)
    assert all(v == 0 for v in d[comm.n_per_row:])
    got = sum(a * b for a, b in zip(d, rt)) % f.p
    xv = oracle.from_mont(FT63, x)[0]
    want = 0
    for c in reversed(oracle.from_mont(FT63, coeffs)):
        want = (want * xv + c) % f.p
    assert got == want


def test_decode_row_inverts_encode(oracle):
    """lcpc_online.rs:588-601: a one-row commitment decodes back to its coefficients."""
    row = oracle.random_coeffs(FT63, 16, 3)
    enc, comm = _commit_pos(oracle, row, 16, 256)
    dec = oracle.ifft_oi(FT63, comm.comm)
    assert np.array_equal(dec[:16], comm.coeffs)
    assert not dec[16:].any()


def test_test_txt_fixture_commit(oracle):
    data = open(os.path.join(HERE, "golden", "pos_test.txt"), "rb").read()
    assert len(data) == 598
    el = oracle.pos_bytes_to_field(data)
    np_, nc, _ = oracle.pos_default_dims(len(el))   # CommitDimensions::Square
    enc, comm = _commit_pos(oracle, el, np_, nc)
    assert (comm.n_rows, comm.n_per_row, comm.n_cols) == (6, 16, 32)
    import json
    g = json.load(open(os.path.join(HERE, "golden", "golden.json")))["pos_test_txt_square"]
    assert comm.root().hex() == g["root"]
