"""CPU tests of the PoS encoded-file layer (lcpc_proof_of_storage_amd/pos_files.py): the oracle
restatement of the writer / reader round trip on the reference's own test file, the size
helpers (port of lcpc_online/tests.rs:519-556 test_that_rate_aligns), the metadata JSON and the
MerkleTree byte format (merkle_tree.rs:61-86, port of its to_bytes_and_back test)."""
import io
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from lcpc_proof_of_storage_amd import pos_files as PF  # noqa: E402

TEST_TXT = os.path.join(HERE, "golden", "pos_test.txt")


def test_that_rate_aligns():
    rng = np.random.default_rng(1337)
    for k in range(2, 12):
        pre = 1 << k
        enc = 1 << pre.bit_length()  # (pre + 1).next_power_of_two()
        for n in rng.integers(1, 10000, 100):
            n = int(n)
            es = PF.get_encoded_file_size_from_rate(n, pre, enc)
            ds = PF.get_decoded_file_size_from_rate(es, pre, enc)
            unit = 7 * pre
            assert ds == -(-n // unit) * unit


def test_metadata_json_round_trip():
    m = PF.EncodedFileMetadata(16384, 32768, 9363, 18726, 1 << 30)
    s = m.to_json()
    # serde_json::to_string field order, compact separators, Ulid::default() string
    assert s == ('{"ulid":"00000000000000000000000000","pre_encoded_size":16384,"encoded_size":32768,'
                 '"rows_written":9363,"row_capacity":18726,"bytes_of_data":1073741824}')
    buf = io.BytesIO()
    m.write_to_file(buf)
    buf.seek(0)
    assert PF.EncodedFileMetadata.read_from_file(buf) == m


def test_merkle_tree_bytes_and_paths(oracle):
    w = 1 << 5
    rng = np.random.default_rng(3)
    leaves = b"".join(oracle.blake3(rng.integers(0, 256, 8, dtype=np.uint8).tobytes()) for _ in range(w))
    parents = np.zeros(32 * (w - 1), np.uint8)
    lp = np.frombuffer(leaves, np.uint8).copy()
    oracle.lib().of_merkle_tree(lp.ctypes.data_as(oracle.u8p), w, parents.ctypes.data_as(oracle.u8p))
    tree = PF.MerkleTree(np.frombuffer(leaves + parents.tobytes(), np.uint8))
    assert len(tree) == 2 * w - 1 and tree.width == w
    back = PF.MerkleTree.from_bytes(tree.to_bytes())
    assert back == tree and back.root() == tree.root()
    for idx in [0, 1, 17, w - 1]:
        path = tree.get_path(idx)
        assert len(path) == 5
        h, i = tree[idx], idx
        for sib in path:
            h = oracle.blake3(h + sib if i % 2 == 0 else sib + h)
            i >>= 1
        assert h == tree.root()
    assert tree.get_path(w) is None
    with pytest.raises(ValueError):
        PF.MerkleTree.from_bytes(bytes(32 * 3 + 32))  # 4 digests: not 2^k - 1
    with pytest.raises(ValueError):
        PF.MerkleTree.from_bytes(bytes(32 * 1))


@pytest.mark.parametrize("pre", [8, 16, 32])
def test_oracle_encode_then_decode_file(oracle, pre):
    """lcpc_online/tests.rs:29-149 on the oracle: sizes, capacity and the decode round trip."""
    data = open(TEST_TXT, "rb").read()
    enc = 1 << pre.bit_length()  # (pre + 1).next_power_of_two()
    img, tree, rows, cap = oracle.pos_encode_file(data, pre, enc)
    assert len(tree) == 32 * (2 * enc - 1)
    expected = PF.get_encoded_file_size_from_rate(len(data), pre, enc)
    assert len(img) in (expected, 2 * expected)
    assert len(img) == cap * enc * 8 and cap > rows
    assert oracle.pos_decode_rows(img, pre, enc, cap, rows)[:len(data)] == data


def test_oracle_file_tree_is_lcpc_commit_tree(oracle):
    """The .portree root is the lcpc-2d commitment root of the same encoded matrix."""
    data = open(TEST_TXT, "rb").read()
    img, tree, rows, cap = oracle.pos_encode_file(data, 16, 32)
    elems = oracle.pos_bytes_to_field(data)
    coeffs = np.zeros(rows * 16, np.uint64)
    coeffs[:len(elems)] = elems
    enc = oracle.Encoding.ligero(0, 16, 32, 1, 1)
    assert oracle.Commit(enc, coeffs).root() == tree[-32:]
