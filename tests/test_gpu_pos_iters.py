"""GPU parity of the streamed producers: FieldGeneratorIter (fields/field_generator_iter.rs) and
RowGeneratorIter (lcpc_online/row_generator_iter.rs) in pos.py / pos_files.py, against the
in-memory path and the oracle's commitment.  Ports of the reference's own tests:
  compare_iterator_to_normal            field_generator_iter.rs:57-80
  is_row_iterator_the_same_as_non_iter  row_generator_iter.rs:188-235
  are_specified_columns_correct         :237-284
  is_row_iterator_the_same_root         :286-329
  read_file_to_root_with_iterator       :331-364 (a synthetic 100000-byte file in place of
                                        test_files/100000_byte_file.bytes, which is not committed)
and the ColumnDigestAccumulator (column_digest_accumulator.rs) against the oracle's column hashes.
The reference fills its inputs from a thread RNG; here they are seeded."""
import io
import itertools

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
FT63 = 0


@pytest.fixture(scope="module")
def P(gpu):
    from lcpc_proof_of_storage_amd import lcpc2d, pos, pos_files
    return pos, pos_files, lcpc2d


def _bytes(n, seed):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def _commit(P, data, pre, enc):
    pos, _, _ = P
    return pos.convert_file_data_to_commit(pos.convert_byte_vec_to_field_elements_vec(data), pos.Commit(),
                                           pos.Specified(pre, enc))


def _rows(P, data, pre, enc, batch_rows=1024):
    pos, PF, _ = P
    return PF.RowGeneratorIter(pos.FieldGeneratorIter(iter(data)), pre, enc, batch_rows)


@pytest.mark.parametrize("n", [0, 1, 6, 7, 8, 999, 7 * 65536 + 3])
def test_field_iterator_is_the_same_as_the_vec(P, n):
    pos, _, _ = P
    data = _bytes(n, n)
    want = pos.convert_byte_vec_to_field_elements_vec(data).reshape(-1) if n else np.zeros(0, np.uint64)
    for src in (iter(data), data, (data[i:i + 1000] for i in range(0, n, 1000))):
        got = np.fromiter(pos.FieldGeneratorIter(src), np.uint64)
        assert np.array_equal(got, want)
    # part taken as elements, the rest as bytes: the same elements
    it = pos.FieldGeneratorIter(data)
    head = np.fromiter(itertools.islice(it, 5), np.uint64)
    rest = b"".join(it.byte_blocks())
    tail = pos.convert_byte_vec_to_field_elements_vec(rest).reshape(-1) if rest else np.zeros(0, np.uint64)
    assert np.array_equal(np.concatenate([head, tail]), want)


@pytest.mark.parametrize("n,pre,enc,batch", [(999, 4, 8, 1024), (999, 4, 8, 3), (60000, 64, 128, 7),
                                             (7 * 256 * 40 - 5, 256, 1024, 16)])
def test_row_iterator_is_the_same_as_non_iter(P, oracle, n, pre, enc, batch):
    data = _bytes(n, 3)
    comm = _commit(P, data, pre, enc)
    rows = list(_rows(P, data, pre, enc, batch))
    assert len(rows) == comm.get_n_rows()
    m = comm.comm.reshape(comm.get_n_rows(), enc)
    for r, row in enumerate(rows):
        assert np.array_equal(row, m[r])
    el = oracle.pos_bytes_to_field(data)
    coeffs = np.zeros(len(rows) * pre, np.uint64)
    coeffs[:el.size] = el
    ocomm = oracle.Commit(oracle.Encoding.ligero(FT63, pre, enc), coeffs)
    assert np.array_equal(np.stack(rows).reshape(-1), ocomm.comm.reshape(-1))


@pytest.mark.parametrize("n,pre,enc", [(999, 4, 8), (50000, 32, 64)])
def test_specified_columns_are_correct(P, oracle, n, pre, enc):
    data = _bytes(n, 4)
    digests = _rows(P, data, pre, enc).get_column_digests()
    el = oracle.pos_bytes_to_field(data)
    coeffs = np.zeros(-(-el.size // pre) * pre, np.uint64)
    coeffs[:el.size] = el
    ocomm = oracle.Commit(oracle.Encoding.ligero(FT63, pre, enc), coeffs)
    assert digests == [ocomm.hashes[32 * c:32 * c + 32] for c in range(enc)]
    idx = sorted(set(int(i) % enc for i in np.random.default_rng(5).integers(0, 1 << 30, 4)))
    partial = _rows(P, data, pre, enc).get_specified_column_digests(idx)
    assert partial == [digests[i] for i in idx]


@pytest.mark.parametrize("n,pre,enc,batch", [(999, 4, 8, 1024), (999, 4, 8, 5), (123457, 128, 256, 64)])
def test_row_iterator_is_the_same_root(P, n, pre, enc, batch):
    pos, PF, _ = P
    data = _bytes(n, 6)
    root = _commit(P, data, pre, enc).get_root()
    assert _rows(P, data, pre, enc, batch).convert_to_commit_root() == root
    # any element iterator (not a FieldGeneratorIter): encoded rows through the accumulator
    el = pos.convert_byte_vec_to_field_elements_vec(data).reshape(-1)
    assert PF.RowGeneratorIter(iter(el.tolist()), pre, enc, batch).convert_to_commit_root() == root


def test_read_file_to_root_with_iterator(P, tmp_path):
    pos, PF, _ = P
    data = _bytes(100000, 7)
    path = tmp_path / "100000_byte_file.bytes"
    path.write_bytes(data)
    reference = pos.convert_file_data_to_commit(pos.convert_byte_vec_to_field_elements_vec(data), pos.Commit(),
                                                pos.Square())
    with open(path, "rb") as f:
        reader = io.BufferedReader(f)
        field_iterator = pos.FieldGeneratorIter(iter(lambda: reader.read(4096), b""))
        streamed = PF.RowGeneratorIter.new_ligero(field_iterator, reference.get_n_per_row(),
                                                  reference.get_n_cols()).convert_to_commit_root()
    assert streamed == reference.get_root()


def test_partly_consumed_iterator(P):
    """The consuming methods cover the rows not yet yielded, as the reference's (which take self
    after any next() calls)."""
    pos, PF, _ = P
    pre, enc = 16, 32
    data = _bytes(7 * pre * 50 + 9, 8)
    el = pos.convert_byte_vec_to_field_elements_vec(data).reshape(-1)
    for taken, batch in [(3, 1024), (3, 2), (10, 4)]:
        it = _rows(P, data, pre, enc, batch)
        for _ in range(taken):
            next(it)
        rest = el[taken * pre:]
        want = pos.convert_file_data_to_commit(rest.reshape(-1, 1), pos.Commit(), pos.Specified(pre, enc))
        assert it.convert_to_commit_root() == want.get_root()
        assert list(it) == []


def test_get_full_columns(P, oracle):
    pos, PF, L = P
    pre, enc = 32, 64
    data = _bytes(20000, 9)
    comm = _commit(P, data, pre, enc)
    cols = [5, 63, 0, 17]
    got = _rows(P, data, pre, enc).get_full_columns(cols)
    # the reference pops the last column first: the result is in reverse order (:99-104)
    for c, col in zip(reversed(cols), got):
        want = comm.open_column(c)
        assert np.array_equal(col.col, want.col) and list(col.path) == list(want.path)
        assert L.verify_column_path(FT63, col, c, comm.get_root())


# ---------------------------------------------------------------- ColumnDigestAccumulator
@pytest.mark.parametrize("fid,n_rows,width,batch_rows,pushes", [
    (0, 1, 8, 0, [1]),
    (0, 124, 16, 0, [124]),              # exactly one chunk per column (Ft63: 124 rows)
    (0, 125, 16, 1, [1] * 125),          # two chunks, hashed as they complete
    (0, 1000, 64, 100, [7, 300, 1, 692]),
    (0, 2000, 32, 128, [2000]),
    (1, 300, 32, 50, [62, 63, 175]),     # Ft127: 62 rows in chunk 0
    (3, 97, 8, 16, [31, 66]),            # Ft255
    (4, 40, 4, 8, [40]),                 # Ft253_192 (big-endian repr)
])
def test_column_digest_accumulator(P, oracle, fid, n_rows, width, batch_rows, pushes):
    pos, PF, L = P
    nl = L.limbs(fid)
    m = oracle.random_coeffs(fid, n_rows * width, 17 + n_rows).reshape(n_rows, width * nl)
    want = oracle.hash_columns(fid, m, n_rows, width)
    acc = PF.ColumnDigestAccumulator(width, PF.ColumnsToCareAbout.All, fid, batch_rows)
    assert acc.get_width() == width
    r = 0
    for k in pushes:
        acc.update(m[r:r + k])
        r += k
    assert r == n_rows
    assert b"".join(acc.get_column_digests()) == want
    # finalize_to_merkle_tree: the lcpc-2d tree over the same leaves
    acc = PF.ColumnDigestAccumulator(width, PF.ColumnsToCareAbout.All, fid, batch_rows)
    for row in m:  # update one row at a time, as the reference does
        acc.update(row)
    tree = acc.finalize_to_merkle_tree()
    assert tree.to_bytes() == want + L.merkle_tree(want)


def test_column_digest_accumulator_commit_root_and_errors(P, oracle):
    pos, PF, L = P
    data = _bytes(50000, 10)
    comm = _commit(P, data, 64, 128)
    acc = PF.ColumnDigestAccumulator(128, batch_rows=10)
    for r in comm.comm.reshape(comm.get_n_rows(), 128):
        acc.update(r)
    assert acc.finalize_to_commit() == comm.get_root()
    # no rows: every digest is BLAKE3 of the 32 zero bytes alone
    assert PF.ColumnDigestAccumulator(4).get_column_digests() == [oracle.blake3(bytes(32))] * 4
    acc = PF.ColumnDigestAccumulator(8)
    with pytest.raises(ValueError):
        acc.update(np.zeros(7, np.uint64))            # ensure!(encoded_row.len() == width)
    with pytest.raises(NotImplementedError):
        PF.ColumnDigestAccumulator(8, PF.ColumnsToCareAbout.Only([1, 2]))
    acc = PF.ColumnDigestAccumulator(6)
    acc.update(np.arange(6, dtype=np.uint64))
    with pytest.raises(L.LcpcError):
        acc.finalize_to_merkle_tree()                  # MerkleTree::new: not a power of two
    with pytest.raises(L.LcpcError):
        PF.ColumnDigestAccumulator(8, field=2)         # Ft191 elements straddle chunks
