"""GPU parity of the PoS encoded-file layer (pos_files.py over lcpc_pos_writer_* /
lcpc_pos_porenc_tree / lcpc_pos_decode_porenc) against the oracle restatement
(oracle_ffi.pos_encode_file / pos_decode_rows): the .porenc bytes, the .portree bytes and the
decoded data must be identical.  Includes the ports of lcpc_online/tests.rs:29-149
(encode_then_decode_file) and the size/metadata assertions of :560-650."""
import io
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
TEST_TXT = os.path.join(HERE, "golden", "pos_test.txt")


@pytest.fixture(scope="module")
def PF(gpu):
    from lcpc_proof_of_storage_amd import pos_files
    return pos_files


def _read(path):
    with open(path, "rb") as f:
        return f.read()


@pytest.mark.parametrize("pre", [8, 16, 32])
def test_encode_then_decode_file(PF, oracle, tmp_path, pre):
    data = _read(TEST_TXT)
    enc = 1 << pre.bit_length()
    porenc, tree_p, meta_p = tmp_path / "t.porenc", tmp_path / "t.portree", tmp_path / "t.meta"
    with open(TEST_TXT, "rb") as src:
        meta, tree = PF.EncodedFileWriter.convert_unencoded_file(src, str(porenc), str(tree_p), str(meta_p),
                                                                 pre, enc)
    img, otree, rows, cap = oracle.pos_encode_file(data, pre, enc)
    assert _read(porenc) == img
    assert tree.to_bytes() == otree and _read(tree_p) == otree
    assert len(tree) == 2 * enc - 1
    with open(meta_p, "rb") as f:
        m2 = PF.EncodedFileMetadata.read_from_file(f)
    assert m2 == meta
    assert (meta.rows_written, meta.row_capacity, meta.bytes_of_data) == (rows, cap, len(data))
    assert meta.encoded_size == enc and meta.pre_encoded_size == pre
    assert os.path.getsize(porenc) == meta.row_capacity * enc * 8 and meta.row_capacity > meta.rows_written
    with open(porenc, "r+b") as f:
        rd = PF.EncodedFileReader.new_ligero(f, pre, enc, meta.rows_written, meta.row_capacity)
        out = io.BytesIO()
        rd.decode_to_target_file(out)
        assert out.getvalue()[:len(data)] == data
        assert out.getvalue() == oracle.pos_decode_rows(img, pre, enc, cap, rows)
        assert rd.process_file_to_merkle_tree() == tree
        a = np.frombuffer(img, "<u8").reshape(enc, cap)
        assert np.array_equal(rd.get_encoded_column_without_path(3), a[3, :rows])
        assert np.array_equal(rd.get_encoded_row(rows - 1), a[:, rows - 1])
        assert rd.get_unencoded_row_bytes(1) == data[7 * pre:14 * pre]


@pytest.mark.parametrize("n_bytes,pre,enc,batch", [
    (200_003, 64, 128, 128),       # several 1-chunk batches, ragged tail
    (7 * 64 * 700, 64, 128, 256),  # exact multiple of the row size, rows > batch
    (7 * 64 * 124, 64, 128, 128),  # rows end exactly on the first chunk boundary
    (99_999, 100, 256, 0),         # non-power-of-two row, automatic batch
    (5, 3, 4, 128),                # a single partial row
])
def test_streaming_writer_matches_oracle(PF, oracle, tmp_path, n_bytes, pre, enc, batch):
    rng = np.random.default_rng(n_bytes)
    data = rng.integers(0, 256, n_bytes, dtype=np.uint8).tobytes()
    img, otree, rows, cap = oracle.pos_encode_file(data, pre, enc)
    with open(tmp_path / "s.porenc", "w+b") as f:
        w = PF.EncodedFileWriter(pre, enc, n_bytes, f, batch_rows=batch)
        off = 0
        while off < n_bytes:  # ragged pushes, including empty ones and partial rows
            step = int(rng.integers(0, 7 * pre * 90))
            w.push_bytes(data[off:off + step])
            off += step
        meta, tree = w.finalize_to_merkle_tree()
    assert (meta.rows_written, meta.row_capacity, meta.bytes_of_data) == (rows, cap, n_bytes)
    assert _read(tmp_path / "s.porenc") == img
    assert tree.to_bytes() == otree


def test_finalize_variants(PF, oracle, tmp_path):
    data = np.random.default_rng(5).integers(0, 256, 30_000, dtype=np.uint8).tobytes()
    img, otree, rows, cap = oracle.pos_encode_file(data, 32, 64)
    leaves = [otree[32 * i:32 * i + 32] for i in range(64)]
    with open(tmp_path / "a", "w+b") as f:
        w = PF.EncodedFileWriter(32, 64, len(data), f)
        w.push_bytes(data)
        _, digests = w.finalize_to_column_digest()
    assert digests == leaves
    with open(tmp_path / "b", "w+b") as f:
        w = PF.EncodedFileWriter(32, 64, len(data), f)
        w.push_bytes(data)
        _, root = w.finalize_to_commit()
    assert root == otree[-32:]


def test_capacity_grows_like_the_reference(PF, oracle, tmp_path):
    """More bytes than announced: the capacity doubles when rows reach it (writer.rs:378-381),
    the file keeps the column-major layout of the final capacity."""
    data = np.random.default_rng(6).integers(0, 256, 50_000, dtype=np.uint8).tobytes()
    pre, enc = 16, 32
    with open(tmp_path / "g.porenc", "w+b") as f:
        w = PF.EncodedFileWriter(pre, enc, 3_000, f, batch_rows=128)  # capacity 2 * 27 rows
        for i in range(0, len(data), 4_000):
            w.push_bytes(data[i:i + 4_000])
        meta, tree = w.finalize_to_merkle_tree()
    rows = -(-(-(-len(data) // 7)) // pre)
    cap = 54
    while rows >= cap:
        cap *= 2
    assert (meta.rows_written, meta.row_capacity) == (rows, cap)
    img, otree, _, _ = oracle.pos_encode_file(data, pre, enc, cap)
    assert _read(tmp_path / "g.porenc") == img and tree.to_bytes() == otree
    with open(tmp_path / "g.porenc", "r+b") as f:  # the reader's re-layout keeps the tree
        rd = PF.EncodedFileReader(f, pre, enc, rows, cap)
        rd.set_new_capacity(cap * 2)
        assert rd.process_file_to_merkle_tree() == tree
        out = io.BytesIO()
        rd.decode_to_target_file(out)
        assert out.getvalue()[:len(data)] == data


def test_empty_file(PF, oracle, tmp_path):
    src = tmp_path / "empty"
    src.write_bytes(b"")
    with open(src, "rb") as f:
        meta, tree = PF.EncodedFileWriter.convert_unencoded_file(f, str(tmp_path / "e.porenc"), None, None, 8, 16)
    img, otree, rows, cap = oracle.pos_encode_file(b"", 8, 16)
    assert (meta.rows_written, meta.row_capacity) == (0, 0) and tree.to_bytes() == otree
    with open(tmp_path / "e.porenc", "r+b") as f:
        assert PF.EncodedFileReader(f, 8, 16, 0, 0).process_file_to_merkle_tree() == tree


def test_resize_to_target_file(PF, oracle, tmp_path):
    data = np.random.default_rng(7).integers(0, 256, 20_000, dtype=np.uint8).tobytes()
    src = tmp_path / "r.bin"
    src.write_bytes(data)
    with open(src, "rb") as f:
        meta, _ = PF.EncodedFileWriter.convert_unencoded_file(f, str(tmp_path / "r.porenc"), None, None, 16, 32)
    with open(tmp_path / "r.porenc", "r+b") as f, open(tmp_path / "r2.porenc", "w+b") as g:
        rd = PF.EncodedFileReader(f, 16, 32, meta.rows_written, meta.row_capacity)
        m2, t2 = rd.resize_to_target_file(g, 64, 128)
    # the reshaped file encodes the decoded (row-padded) data
    padded = data + bytes(meta.rows_written * 16 * 7 - len(data))
    img, otree, rows, cap = oracle.pos_encode_file(padded, 64, 128, m2.row_capacity)
    assert _read(tmp_path / "r2.porenc") == img and t2.to_bytes() == otree


def test_non_canonical_element_is_refused(PF, oracle, tmp_path):
    import lcpc_proof_of_storage_amd as L
    data = _read(TEST_TXT)
    with open(TEST_TXT, "rb") as f:
        meta, _ = PF.EncodedFileWriter.convert_unencoded_file(f, str(tmp_path / "x.porenc"), None, None, 8, 16)
    raw = bytearray(_read(tmp_path / "x.porenc"))
    raw[8 * 5:8 * 6] = (0x46d0760000000001 + 3).to_bytes(8, "little")  # >= p
    (tmp_path / "x.porenc").write_bytes(bytes(raw))
    with open(tmp_path / "x.porenc", "r+b") as f:
        rd = PF.EncodedFileReader(f, 8, 16, meta.rows_written, meta.row_capacity)
        with pytest.raises(L.LcpcError):
            rd.process_file_to_merkle_tree()
        with pytest.raises(L.LcpcError):
            rd.decode_to_target_file(io.BytesIO())


def test_default_dims_file_columns_verify(PF, oracle, tmp_path, gpu):
    """A 2 MiB file at the PoS default dims: file, tree, columns and their paths."""
    from lcpc_proof_of_storage_amd import pos as P
    data = np.random.default_rng(8).integers(0, 256, 2 << 20, dtype=np.uint8).tobytes()
    pre, enc, _ = P.get_aspect_ratio_default_from_file_len(len(data))
    src = tmp_path / "big.bin"
    src.write_bytes(data)
    with open(src, "rb") as f:
        meta, tree = PF.EncodedFileWriter.convert_unencoded_file(f, str(tmp_path / "big.porenc"), None, None,
                                                                 pre, enc)
    img, otree, rows, cap = oracle.pos_encode_file(data, pre, enc)
    assert _read(tmp_path / "big.porenc") == img and tree.to_bytes() == otree
    a = np.frombuffer(img, "<u8").reshape(enc, cap)
    with open(tmp_path / "big.porenc", "r+b") as f:
        rd = PF.EncodedFileReader(f, pre, enc, rows, cap)
        for c in oracle.pos_column_indices(42, 16, enc):
            col = rd.get_encoded_column_without_path(c)
            assert np.array_equal(col, a[c, :rows])
            h = oracle.blake3(bytes(32) + col.astype("<u8").tobytes())
            assert h == tree[c]
            i = c
            for sib in tree.get_path(c):
                h = oracle.blake3(h + sib if i % 2 == 0 else sib + h)
                i >>= 1
            assert h == tree.root()
