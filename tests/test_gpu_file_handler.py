"""GPU: the proof-of-storage FileHandler (pos_files.FileHandler over lcpc_pos_reencode_rows /
lcpc_pos_porenc_tree): ports of the reference's lcpc_online/tests.rs edit_file_is_correct
(:150-261), append_to_file_is_correct (:262-360) and reencode_rows_are_correct (:440-517), with
fewer random iterations.  On top of the reference's own checks (raw bytes, replaced bytes,
decode, verify_all_files_agree), every edited `.porenc` column and the tree are compared with
the oracle's fresh encode of the edited raw data (oracle_ffi.pos_encode_file), bit for bit.

The reference's 10000-byte fixture (test_files/10000_byte_file.bytes) is not in the
repository; 10000 bytes from numpy.random.default_rng stand in.  test.txt is the
reference's own (tests/golden/pos_test.txt).
"""
import os
import shutil

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TEST_TXT = os.path.join(HERE, "golden", "pos_test.txt")
WB = 8


@pytest.fixture(scope="module")
def PF(gpu):
    from lcpc_proof_of_storage_amd import pos_files
    return pos_files


def _read(p):
    with open(p, "rb") as f:
        return f.read()


def _bytes_10000(seed=1):
    return np.random.default_rng(seed).integers(0, 256, 10000, dtype=np.uint8).tobytes()


def _check_against_oracle(fh, oracle, contents):
    """the .porenc columns (first rows_written elements) and the tree equal a fresh encode"""
    pre, enc, rows = fh.get_dimensions()
    img, otree, orows, ocap = oracle.pos_encode_file(contents, pre, enc)
    assert orows == rows
    got = np.frombuffer(_read(fh.get_encoded_file_handle()), np.uint8).reshape(enc, -1)[:, :rows * WB]
    want = np.frombuffer(img, np.uint8).reshape(enc, -1)[:, :rows * WB]
    assert np.array_equal(got, want)
    assert fh.get_merkle_tree().to_bytes() == otree
    assert _read(fh.get_merkle_file_handle()) == otree


def _decode(PF, fh, tmp_path):
    m = fh.get_encoded_metadata()
    target = tmp_path / "decoded.bin"
    with open(fh.get_encoded_file_handle(), "rb") as f, open(target, "wb") as t:
        PF.EncodedFileReader.new_ligero(f, m.pre_encoded_size, m.encoded_size, m.rows_written,
                                        m.row_capacity).decode_to_target_file(t)
    return _read(target)


@pytest.mark.parametrize("pre", [2, 4, 8, 16, 32])
def test_edit_file_is_correct(PF, oracle, tmp_path, pre):
    rng = np.random.default_rng(pre)
    enc = 1 << pre.bit_length()              # (pre + 1).next_power_of_two()
    contents = bytearray(_bytes_10000())
    src = tmp_path / "edit_test.bin"
    src.write_bytes(bytes(contents))
    fh = PF.FileHandler.create_from_unencoded_file("01EDITTEST0000000000000000", str(src), pre, enc,
                                                   directory=str(tmp_path / "files"))
    fh.verify_all_files_agree()
    for i in range(12):
        new = rng.integers(0, 256, 1028, dtype=np.uint8).tobytes()
        start = int(rng.integers(0, len(contents) - 1028))
        old, tree = fh.edit_bytes(start, new)
        assert len(tree) == 2 * enc - 1
        assert old == bytes(contents[start:start + 1028])
        contents[start:start + 1028] = new
        assert _read(fh.get_raw_file_handle()) == bytes(contents)
        fh.verify_all_files_agree()
        if i % 4 == 0:
            assert _decode(PF, fh, tmp_path)[:len(contents)] == bytes(contents)
            _check_against_oracle(fh, oracle, bytes(contents))
    fh.delete_all_files()


@pytest.mark.parametrize("pre", [2, 4, 8, 16, 32])
def test_append_to_file_is_correct(PF, oracle, tmp_path, pre):
    rng = np.random.default_rng(100 + pre)
    enc = 1 << pre.bit_length()
    contents = bytearray(_read(TEST_TXT))
    src = tmp_path / "append_test.txt"
    shutil.copy(TEST_TXT, src)
    fh = PF.FileHandler.create_from_unencoded_file("01APPENDTEST00000000000000", str(src), pre, enc,
                                                   directory=str(tmp_path / "files"))
    fh.verify_all_files_agree()
    for i in range(24):
        new = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        tree = fh.append_bytes(new)
        assert len(tree) == 2 * enc - 1
        contents += new
        assert _read(fh.get_raw_file_handle()) == bytes(contents)
        if i % 6 == 0:
            assert _decode(PF, fh, tmp_path)[:len(contents)] == bytes(contents)
            fh.verify_all_files_agree()
            _check_against_oracle(fh, oracle, bytes(contents))
    m = fh.get_encoded_metadata()
    assert m.bytes_of_data == len(contents) and m.rows_written * pre * 7 >= len(contents)
    # the metadata on disk is what a later attach reads back
    again = PF.FileHandler.new_attach_to_existing_ulid(os.path.dirname(fh.get_raw_file_handle()),
                                                       "01APPENDTEST00000000000000")
    assert again.get_encoded_metadata() == m and again.get_merkle_tree() == fh.get_merkle_tree()
    fh.delete_all_files()


@pytest.mark.parametrize("pre", [8, 16, 32, 64])
def test_reencode_rows_are_correct(PF, tmp_path, pre):
    enc = 1 << pre.bit_length()
    src = tmp_path / "reencode_test.bin"
    src.write_bytes(_bytes_10000(7))
    fh = PF.FileHandler.create_from_unencoded_file("01REENCODETEST000000000000", str(src), pre, enc,
                                                   directory=str(tmp_path / "files"))
    fh.verify_all_files_agree()
    before = _read(fh.get_encoded_file_handle())
    expected_rows = -(-(-(-10000 // 7)) // pre)
    col = fh.read_full_columns([0])
    assert len(col[0].col) == expected_rows
    for row in range(expected_rows):
        fh.reencode_row(row)
    assert _read(fh.get_encoded_file_handle()) == before
    fh.verify_all_files_agree()
    fh.reencode_unencoded_file()
    assert _read(fh.get_encoded_file_handle()) == before
    fh.verify_all_files_agree()
    fh.delete_all_files()


def test_reshape_and_columns_verify(PF, oracle, tmp_path):
    """reshape (file_handler.rs:224-276) then verify_columns_are_correct's path checks (:362-438)."""
    data = _bytes_10000(3)
    src = tmp_path / "cols.bin"
    src.write_bytes(data)
    fh = PF.FileHandler.create_from_unencoded_file("01COLUMNSTEST0000000000000", str(src), 16, 32,
                                                   directory=str(tmp_path / "files"))
    fh.reshape(8, 16)
    fh.verify_all_files_agree()
    _check_against_oracle(fh, oracle, data)
    root = fh.get_commit_root()
    cols = fh.read_full_columns([0, 5, 15])
    for c, col in zip([0, 5, 15], cols):
        assert len(col.path) == 4
        h = oracle.blake3(bytes(32) + b"".join(int(v).to_bytes(8, "little") for v in col.col))
        for lvl, sib in enumerate(col.path):
            h = oracle.blake3(sib + h if (c >> lvl) & 1 else h + sib)
        assert h == root
    with pytest.raises(ValueError):
        fh.edit_bytes(len(data) - 10, b"x" * 11)
    fh.delete_all_files()


@pytest.mark.parametrize("chunks", [[0, 5, 7 * 4, 1], [7 * 4 * 3], [1] * 9])
def test_append_from_empty_and_on_row_boundaries(PF, oracle, tmp_path, chunks):
    """appends into an empty file, exactly up to row boundaries and byte by byte (the capacity
    starts at zero and doubles: EncodedFileReader::set_new_capacity layout)"""
    pre, enc = 4, 8
    src = tmp_path / "empty.bin"
    src.write_bytes(b"")
    fh = PF.FileHandler.create_from_unencoded_file("01EMPTYTEST000000000000000", str(src), pre, enc,
                                                   directory=str(tmp_path / "files"))
    contents = bytearray()
    rng = np.random.default_rng(len(chunks))
    for n in chunks:
        new = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        fh.append_bytes(new)
        contents += new
        assert _read(fh.get_raw_file_handle()) == bytes(contents)
        if contents:
            fh.verify_all_files_agree()
            _check_against_oracle(fh, oracle, bytes(contents))
    fh.delete_all_files()


def test_left_multiply_unencoded_matrix_by_vector(PF, oracle, tmp_path):
    """FileHandler::left_multiply_unencoded_matrix_by_vector (file_handler.rs:614-638): u^T M
    over the stored rows, against the oracle's row combination of the same elements (the
    reference's own returns an empty vector), and its size check."""
    data = _bytes_10000(5)
    src = tmp_path / "lm.bin"
    src.write_bytes(data)
    pre, enc = 16, 32
    fh = PF.FileHandler.create_from_unencoded_file("01LEFTMULTIPLY000000000000", str(src), pre, enc,
                                                   directory=str(tmp_path / "files"))
    rows = fh.get_dimensions()[2]
    left = oracle.random_coeffs(0, rows, 99)
    el = oracle.pos_bytes_to_field(data)
    m = np.zeros(rows * pre, np.uint64)
    m[:el.size] = el
    got = fh.left_multiply_unencoded_matrix_by_vector(left)
    assert np.array_equal(np.asarray(got).reshape(-1), oracle.collapse(0, m, left.reshape(-1), rows, pre))
    with pytest.raises(ValueError):
        fh.left_multiply_unencoded_matrix_by_vector(left[:-1])
    fh.delete_all_files()
