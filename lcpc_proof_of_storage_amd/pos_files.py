"""Proof-of-storage encoded files over liblcpc_mi.so: the `.porenc` / `.portree` / `.meta`
formats of the reference's proof-of-storage/src/lcpc_online (names kept):

  EncodedFileWriter     encoded_file_writer.rs:24-501  (new, push_bytes, finalize_*,
                        convert_unencoded_file, get_encoded_file_metadata)
  EncodedFileReader     encoded_file_reader.rs:20-381  (get_encoded_row,
                        get_encoded_column_without_path, get_unencoded_row[_bytes],
                        decode_to_target_file, process_file_to_merkle_tree, set_new_capacity,
                        resize_to_target_file, get_unencoded_file_len)
  EncodedFileMetadata   encoded_file_metadata.rs:6-27  (serde_json)
  MerkleTree            merkle_tree.rs:7-86             (digests = leaves || parents)
  read_tree / write_tree_to_file                         file_handler.rs:714-735
  get_encoded_file_size_from_rate / get_decoded_file_size_from_rate   reader.rs:384-407
  RowGeneratorIter      row_generator_iter.rs:8-165     (new_ligero, next, get_column_digests,
                        get_specified_column_digests, convert_to_commit_root, get_full_columns)
  ColumnDigestAccumulator, ColumnsToCareAbout   column_digest_accumulator.rs:9-118

Layout of a `.porenc` file (WriteableFt63): column c occupies row_capacity * 8 bytes starting at
byte c * row_capacity * 8; its first rows_written elements are the canonical little-endian repr
of the encoded matrix's column c, the rest zero.  The writer starts with row_capacity = 2 * rows
and doubles it when rows reach it.

Every byte of encoding, hashing and decoding runs on the GPU (liblcpc_mi.so); this module maps
the files and hands the library pointers into them.
"""
from __future__ import annotations

import ctypes as C
import itertools
import json
import mmap
import os
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np

from . import _native as N
from . import lcpc2d as L
from .lcpc2d import _raise

WRITTEN_BYTES_WIDTH = 8   # size_of::<WriteableFt63>() (data_field.rs:24)
DATA_BYTE_CAPACITY = 7    # CAPACITY / 8 (data_field.rs:22)
DIGEST_BYTES = 32
_NULL_ULID = "0" * 26     # Ulid::default() as serialized by the ulid crate's serde impl


def _u8(a: np.ndarray):
    return a.ctypes.data_as(N.u8p) if a.size else None


def _bytes_ptr(b) -> Tuple[Optional[C.POINTER(C.c_uint8)], object]:
    arr = np.frombuffer(b, dtype=np.uint8) if len(b) else np.zeros(0, np.uint8)
    return _u8(arr), arr


# ---------------------------------------------------------------- metadata / Merkle tree
@dataclass
class EncodedFileMetadata:
    """encoded_file_metadata.rs:6-13 (serde_json, field order kept)."""
    pre_encoded_size: int
    encoded_size: int
    rows_written: int
    row_capacity: int
    bytes_of_data: int
    ulid: str = _NULL_ULID

    def to_json(self) -> str:
        return json.dumps({"ulid": self.ulid, "pre_encoded_size": self.pre_encoded_size,
                           "encoded_size": self.encoded_size, "rows_written": self.rows_written,
                           "row_capacity": self.row_capacity, "bytes_of_data": self.bytes_of_data},
                          separators=(",", ":"))

    def write_to_file(self, writable) -> None:
        writable.write(self.to_json().encode())

    @classmethod
    def read_from_file(cls, readable) -> "EncodedFileMetadata":
        d = json.loads(readable.read())
        return cls(d["pre_encoded_size"], d["encoded_size"], d["rows_written"], d["row_capacity"],
                   d["bytes_of_data"], d.get("ulid", _NULL_ULID))


class MerkleTree:
    """merkle_tree.rs:7-86: 2 w - 1 digests, the w leaves then every parent level, root last."""

    def __init__(self, digests: np.ndarray):
        d = np.ascontiguousarray(digests, dtype=np.uint8).reshape(-1, DIGEST_BYTES)
        self.digests = d
        self.width = (d.shape[0] + 1) // 2

    @classmethod
    def new(cls, children_leaves) -> "MerkleTree":
        leaves = np.ascontiguousarray(np.frombuffer(bytes(children_leaves), np.uint8)
                                      if isinstance(children_leaves, (bytes, bytearray))
                                      else children_leaves, dtype=np.uint8).reshape(-1, DIGEST_BYTES)
        w = leaves.shape[0]
        if w < 2 or w & (w - 1):
            raise ValueError("Input needs to be a power of two, at least two.")
        d = np.zeros((2 * w - 1, DIGEST_BYTES), np.uint8)
        d[:w] = leaves
        _raise(N.load().lcpc_merkle_tree(_u8(d[:w]), w, _u8(d[w:])))
        return cls(d)

    def root(self) -> bytes:
        return self.digests[-1].tobytes()

    def get_path(self, index: int) -> Optional[List[bytes]]:
        if index >= self.width:
            return None
        path, base, level_len = [], 0, self.width
        while level_len > 1:
            path.append(self.digests[base + (index ^ 1)].tobytes())
            base += level_len
            level_len //= 2
            index >>= 1
        return path

    def __len__(self) -> int:
        return self.digests.shape[0]

    def __getitem__(self, i: int) -> bytes:
        return self.digests[i].tobytes()

    def __eq__(self, other) -> bool:
        return isinstance(other, MerkleTree) and np.array_equal(self.digests, other.digests)

    def to_bytes(self) -> bytes:
        return self.digests.tobytes()

    @classmethod
    def from_bytes(cls, data: bytes) -> "MerkleTree":
        n = len(data) // DIGEST_BYTES
        if (n + 1) & n:
            raise ValueError("input size must be a power of two")
        if n <= 2:
            raise ValueError("Merkle tree must be a non-trivial binary tree")
        return cls(np.frombuffer(data[:n * DIGEST_BYTES], np.uint8).copy())


def read_tree(tree_file) -> MerkleTree:
    tree_file.seek(0)
    return MerkleTree.from_bytes(tree_file.read())


def write_tree_to_file(tree_file, tree: MerkleTree) -> None:
    tree_file.write(tree.to_bytes())


def get_encoded_file_size_from_rate(decoded_file_size: int, pre_encoded_len: int, encoded_len: int) -> int:
    """reader.rs:384-395 (div_ceils first, in this order)."""
    return (-(-(-(-decoded_file_size // DATA_BYTE_CAPACITY)) // pre_encoded_len)
            * WRITTEN_BYTES_WIDTH * encoded_len)


def get_decoded_file_size_from_rate(encoded_file_size: int, pre_encoded_len: int, encoded_len: int) -> int:
    """reader.rs:397-407."""
    return (-(-(-(-encoded_file_size // encoded_len)) // WRITTEN_BYTES_WIDTH)
            * DATA_BYTE_CAPACITY * pre_encoded_len)


# ---------------------------------------------------------------- mapped file images
class _Image:
    """A read/write mmap of a `.porenc` file (zero-length files map to nothing)."""

    def __init__(self, f, size: int):
        self.f = f
        self.size = size
        f.truncate(size)
        f.flush()
        self.mm = mmap.mmap(f.fileno(), size) if size else None
        self.arr = np.frombuffer(self.mm, np.uint8) if size else np.zeros(0, np.uint8)

    def ptr(self):
        return _u8(self.arr)

    def close(self):
        if self.mm is not None:
            self.mm.flush()
            del self.arr
            self.mm.close()
            self.mm = None
            self.arr = np.zeros(0, np.uint8)

    def grow(self, old_rows: int, new_rows: int, n_cols: int) -> None:
        """EncodedFileReader::set_new_capacity (reader.rs:348-381): columns move back to
        front to their new stride, the space after each zeroed."""
        wb = WRITTEN_BYTES_WIDTH
        self.close()
        self.__init__(self.f, new_rows * n_cols * wb)
        a = self.arr
        old_len, new_len = old_rows * wb, new_rows * wb
        for c in range(n_cols - 1, 0, -1):
            a[c * new_len:c * new_len + old_len] = a[c * old_len:(c + 1) * old_len].copy()
            a[c * new_len + old_len:(c + 1) * new_len] = 0
        a[old_len:new_len] = 0


# ---------------------------------------------------------------- writer
class EncodedFileWriter:
    """EncodedFileWriter<WriteableFt63, Blake3, LigeroEncoding> (encoded_file_writer.rs)."""

    def __init__(self, num_pre_encoded_columns: int, num_encoded_columns: int,
                 original_file_size: int, target_file, batch_rows: int = 0):
        # new (:53-105): the assertions, then the file preallocated to 2 * rows
        if not (num_encoded_columns > 0 and num_encoded_columns & (num_encoded_columns - 1) == 0):
            raise ValueError("num_encoded_columns must be a power of two")
        if not num_pre_encoded_columns < num_encoded_columns:
            raise ValueError("num_pre_encoded_columns must be less than num_encoded_columns")
        if not num_pre_encoded_columns > 0:
            raise ValueError("num_pre_encoded_columns must be > 0")
        self.pre_encoded_size = num_pre_encoded_columns
        self.encoded_size = num_encoded_columns
        num_rows = -(-(-(-original_file_size // DATA_BYTE_CAPACITY)) // num_pre_encoded_columns)
        self.row_capacity = num_rows * 2
        self.bytes_received = 0
        self.rows_written = 0
        self._img = _Image(target_file, self.row_capacity * num_encoded_columns * WRITTEN_BYTES_WIDTH)
        h = N.vp()
        _raise(N.load().lcpc_pos_writer_new(num_pre_encoded_columns, num_encoded_columns,
                                            self._img.ptr(), self.row_capacity, batch_rows, C.byref(h)))
        self._h = h
        self._done = False

    def _rows_for(self, n_bytes: int) -> int:
        return -(-(-(-n_bytes // DATA_BYTE_CAPACITY)) // self.pre_encoded_size)

    def _ensure_capacity(self, rows: int) -> None:
        # the reference doubles the capacity whenever the rows written reach it (:378-381)
        new_cap = self.row_capacity
        while rows >= new_cap > 0:
            new_cap *= 2
        if rows > new_cap:  # zero-capacity files (empty original)
            new_cap = max(rows, 1) * 2
        if new_cap == self.row_capacity:
            return
        self._img.grow(self.row_capacity, new_cap, self.encoded_size)
        self.row_capacity = new_cap
        _raise(N.load().lcpc_pos_writer_set_target(self._h, self._img.ptr(), new_cap))

    def get_encoded_file_metadata(self) -> EncodedFileMetadata:
        return EncodedFileMetadata(self.pre_encoded_size, self.encoded_size, self.rows_written,
                                   self.row_capacity, self.bytes_received)

    def push_bytes(self, data: bytes) -> None:
        if self._done:
            raise RuntimeError("writer already finalized")
        self._ensure_capacity(self._rows_for(self.bytes_received + len(data)))
        p, keep = _bytes_ptr(data)
        _raise(N.load().lcpc_pos_writer_push_bytes(self._h, p, len(data)))
        self.bytes_received += len(data)

    def _finalize(self, want_digests: bool, want_tree: bool):
        if self._done:
            raise RuntimeError("writer already finalized")
        self._ensure_capacity(self._rows_for(self.bytes_received))
        w = self.encoded_size
        digests = np.zeros((w, DIGEST_BYTES), np.uint8) if want_digests else None
        tree = np.zeros((2 * w - 1, DIGEST_BYTES), np.uint8) if want_tree else None
        rows, nbytes = C.c_size_t(), C.c_size_t()
        try:
            _raise(N.load().lcpc_pos_writer_finalize(
                self._h, _u8(digests) if want_digests else None, _u8(tree) if want_tree else None,
                C.byref(rows), C.byref(nbytes)))
        finally:
            self._done = True
            N.load().lcpc_pos_writer_free(self._h)
            self._img.close()
        self.rows_written = rows.value
        return digests, tree

    def finalize_to_column_digest(self) -> Tuple[EncodedFileMetadata, List[bytes]]:
        d, _ = self._finalize(True, False)
        return self.get_encoded_file_metadata(), [r.tobytes() for r in d]

    def finalize_to_commit(self) -> Tuple[EncodedFileMetadata, bytes]:
        _, t = self._finalize(False, True)
        return self.get_encoded_file_metadata(), t[-1].tobytes()

    def finalize_to_merkle_tree(self) -> Tuple[EncodedFileMetadata, MerkleTree]:
        _, t = self._finalize(False, True)
        return self.get_encoded_file_metadata(), MerkleTree(t)

    def __del__(self):
        if getattr(self, "_done", True) is False:
            try:
                N.load().lcpc_pos_writer_free(self._h)
                self._img.close()
            except Exception:
                pass

    @staticmethod
    def convert_unencoded_file(unencoded_file, target_encoded_file: str,
                               target_digest_file: Optional[str], target_metadata_file: Optional[str],
                               num_pre_encoded_columns: int, num_encoded_columns: int
                               ) -> Tuple[EncodedFileMetadata, MerkleTree]:
        """encoded_file_writer.rs:134-231: the whole file in one pass of the GPU writer."""
        if num_pre_encoded_columns < 1:
            raise ValueError("Number of pre-encoded columns must be greater than 0")
        if num_encoded_columns < 2 or num_encoded_columns & (num_encoded_columns - 1):
            raise ValueError("Number of encoded columns must be a power of 2")
        if num_encoded_columns <= num_pre_encoded_columns:
            raise ValueError("Number of encoded columns must be greater than the number of columns")
        unencoded_file.seek(0, os.SEEK_END)
        total = unencoded_file.tell()
        unencoded_file.seek(0)
        num_rows = -(-(-(-total // DATA_BYTE_CAPACITY)) // num_pre_encoded_columns)
        cap = num_rows * 2
        with open(target_encoded_file, "w+b") as tf:
            img = _Image(tf, cap * num_encoded_columns * WRITTEN_BYTES_WIDTH)
            src = mmap.mmap(unencoded_file.fileno(), total, access=mmap.ACCESS_READ) if total else None
            try:
                data = np.frombuffer(src, np.uint8) if total else np.zeros(0, np.uint8)
                tree = np.zeros((2 * num_encoded_columns - 1, DIGEST_BYTES), np.uint8)
                rows = C.c_size_t()
                _raise(N.load().lcpc_pos_encode_file(_u8(data), total, num_pre_encoded_columns,
                                                     num_encoded_columns, cap, img.ptr(), _u8(tree),
                                                     C.byref(rows)))
                del data
            finally:
                if src is not None:
                    src.close()
                img.close()
        meta = EncodedFileMetadata(num_pre_encoded_columns, num_encoded_columns, rows.value, cap, total)
        mt = MerkleTree(tree)
        if target_metadata_file:
            with open(target_metadata_file, "wb") as f:
                meta.write_to_file(f)
        if target_digest_file:
            with open(target_digest_file, "wb") as f:
                write_tree_to_file(f, mt)
        return meta, mt


# ---------------------------------------------------------------- streamed rows
class ColumnsToCareAbout:
    """column_digest_accumulator.rs:9-15.  Only(indices) is kept as a type; the accumulator
    refuses it (see ColumnDigestAccumulator)."""
    All = "All"

    @dataclass
    class Only:
        indices: List[int]


class ColumnDigestAccumulator:
    """ColumnDigestAccumulator<Blake3, F> (column_digest_accumulator.rs:17-118) over the GPU
    accumulator (lcpc_column_digests_*): every column's digest is BLAKE3(32 zero bytes || repr of
    its elements), hashed in 1-KiB chunks as they complete, so memory stays one batch of rows.
    update takes one encoded row (num_encoded elements) or a (k, num_encoded) batch of them.

    ColumnsToCareAbout.Only raises NotImplementedError: the reference's update checks the row
    length against the number of tracked columns and then indexes the digests by column number
    (:63-84), so it only works where it equals All; no caller uses it."""

    def __init__(self, number_of_encoded_columns: int, columns_to_care_about=ColumnsToCareAbout.All,
                 field: int = 0, batch_rows: int = 0):
        if isinstance(columns_to_care_about, ColumnsToCareAbout.Only):
            raise NotImplementedError("ColumnsToCareAbout::Only (unusable in the reference; see the class doc)")
        self.field = field
        self._nl = L.limbs(field)
        h = N.vp()
        _raise(N.load().lcpc_column_digests_new(field, number_of_encoded_columns, batch_rows, C.byref(h)))
        self._h = h
        self._done = False

    def get_width(self) -> int:
        return N.load().lcpc_column_digests_width(self._h)

    def update(self, encoded_row) -> None:
        if self._done:
            raise RuntimeError("accumulator already finalized")
        a = np.ascontiguousarray(encoded_row, dtype=np.uint64)
        w = self.get_width()
        if a.size % (w * self._nl):
            raise ValueError("incorrect length of input")  # ensure! (:63-66)
        n = a.size // (w * self._nl)
        _raise(N.load().lcpc_column_digests_update(self._h, L._p64(a.reshape(-1)) if n else None, n))

    def _finalize(self, want_digests: bool, want_tree: bool):
        if self._done:
            raise RuntimeError("accumulator already finalized")
        w = self.get_width()
        digests = np.zeros((w, DIGEST_BYTES), np.uint8) if want_digests else None
        tree = np.zeros((2 * w - 1, DIGEST_BYTES), np.uint8) if want_tree else None
        try:
            _raise(N.load().lcpc_column_digests_finalize(self._h, _u8(digests) if want_digests else None,
                                                         _u8(tree) if want_tree else None))
        finally:
            self._done = True
            N.load().lcpc_column_digests_free(self._h)
        return digests, tree

    def get_column_digests(self) -> List[bytes]:
        d, _ = self._finalize(True, False)
        return [r.tobytes() for r in d]

    def finalize_to_commit(self) -> bytes:
        return self.finalize_to_merkle_tree().root()

    def finalize_to_merkle_tree(self) -> MerkleTree:
        _, t = self._finalize(False, True)
        return MerkleTree(t)

    def __del__(self):
        if getattr(self, "_done", True) is False:
            try:
                N.load().lcpc_column_digests_free(self._h)
            except Exception:
                pass


class RowGeneratorIter:
    """RowGeneratorIter<WriteableFt63, I, LigeroEncoding> (row_generator_iter.rs:8-165).

    Iterating yields the encoded rows (num_encoded elements each, uint64 raw limbs): every
    num_pre_encoded elements of `field_iterator` (the last row zero padded) Ligero-encoded, as
    `next` (:138-164) does row by row.  Here up to `batch_rows` rows are taken from the iterator at
    once and encoded in one GPU call (lcpc_encode_rows), then handed out one by one.

    The consuming methods work on the rows not yet yielded:
      get_column_digests / get_specified_column_digests / convert_to_commit_root (:29-77) stream
        them through a digest-only PoS writer (lcpc_pos_writer_new with no image), so memory stays
        one batch however long the input;
      get_full_columns (:79-107) commits to them and opens the columns.  Like the reference, it
        returns the columns in REVERSE order of `specified_columns` (it pops the last first,
        :99-104).
    From a FieldGeneratorIter (whole 7-byte data words) the data bytes go straight to the
    writer.  Any other element iterator streams its encoded rows through a
    ColumnDigestAccumulator, as the reference does (:33-40)."""

    def __init__(self, field_iterator, num_pre_encoded: int, num_encoded: int, batch_rows: int = 1024):
        if not (num_encoded > 0 and num_encoded & (num_encoded - 1) == 0) or not 0 < num_pre_encoded < num_encoded:
            raise ValueError("bad Ligero dimensions")
        self.field_iterator = field_iterator
        self.unencoded_len = num_pre_encoded
        self.encoded_len = num_encoded
        self.encoding = L.LigeroEncoding.new_from_dims(L.FT63, num_pre_encoded, num_encoded)
        self.batch_rows = max(1, batch_rows)
        self._elems = np.zeros(0, np.uint64)   # unencoded elements of the rows in _rows
        self._rows = np.zeros((0, num_encoded), np.uint64)
        self._next = 0

    @classmethod
    def new_ligero(cls, field_iterator, num_pre_encoded: int, num_encoded: int) -> "RowGeneratorIter":
        return cls(field_iterator, num_pre_encoded, num_encoded)

    def _take(self, n: int) -> np.ndarray:
        return np.fromiter(itertools.islice(self.field_iterator, n), dtype=np.uint64)

    def __iter__(self):
        return self

    def __next__(self) -> np.ndarray:
        if self._next == self._rows.shape[0]:
            pre, enc = self.unencoded_len, self.encoded_len
            el = self._take(self.batch_rows * pre)
            if el.size == 0:  # the empty case (:148-151)
                raise StopIteration
            n = -(-el.size // pre)
            flat = np.zeros(n * pre, np.uint64)
            flat[:el.size] = el
            m = np.zeros((n, enc), np.uint64)
            m[:, :pre] = flat.reshape(n, pre)
            self._rows = self.encoding.encode_rows(m).reshape(n, enc)
            self._elems = el
            self._next = 0
        row = self._rows[self._next].copy()
        self._next += 1
        return row

    def _rest_elements(self) -> np.ndarray:
        """The unencoded elements of every row not yet yielded (consumes the iterator)."""
        pre = self.unencoded_len
        head = self._elems[self._next * pre:]
        self._rows, self._elems, self._next = self._rows[:0], self._elems[:0], 0
        tail = np.fromiter(self.field_iterator, dtype=np.uint64)
        return np.concatenate([head, tail])

    def _rest_byte_blocks(self):
        """The rows not yet yielded as data bytes (FieldGeneratorIter inputs only)."""
        pre = self.unencoded_len
        head = self._elems[self._next * pre:]
        self._rows, self._elems, self._next = self._rows[:0], self._elems[:0], 0
        if head.size:
            yield head.astype("<u8").view(np.uint8).reshape(-1, 8)[:, :DATA_BYTE_CAPACITY].tobytes()
        yield from self.field_iterator.byte_blocks()

    def _digests_and_tree(self):
        from .pos import FieldGeneratorIter
        w = self.encoded_len
        digests = np.zeros((w, DIGEST_BYTES), np.uint8)
        tree = np.zeros((2 * w - 1, DIGEST_BYTES), np.uint8)
        if not isinstance(self.field_iterator, FieldGeneratorIter):
            acc = ColumnDigestAccumulator(w, ColumnsToCareAbout.All, L.FT63)
            batch = []
            for row in self:
                batch.append(row)
                if len(batch) == self.batch_rows:
                    acc.update(np.stack(batch))
                    batch = []
            if batch:
                acc.update(np.stack(batch))
            tree = acc.finalize_to_merkle_tree()
            return tree.digests[:w].copy(), tree.digests.copy()
        h = N.vp()
        _raise(N.load().lcpc_pos_writer_new(self.unencoded_len, w, None, 0, 0, C.byref(h)))
        try:
            for block in self._rest_byte_blocks():
                p, keep = _bytes_ptr(block)
                _raise(N.load().lcpc_pos_writer_push_bytes(h, p, len(block)))
            rows, nbytes = C.c_size_t(), C.c_size_t()
            _raise(N.load().lcpc_pos_writer_finalize(h, _u8(digests), _u8(tree), C.byref(rows), C.byref(nbytes)))
        finally:
            N.load().lcpc_pos_writer_free(h)
        return digests, tree

    def get_column_digests(self) -> List[bytes]:
        d, _ = self._digests_and_tree()
        return [r.tobytes() for r in d]

    def get_specified_column_digests(self, column_indices) -> List[bytes]:
        d = self.get_column_digests()
        return [d[i] for i in column_indices]

    def convert_to_commit_root(self) -> bytes:
        _, t = self._digests_and_tree()
        return t[-1].tobytes()

    def get_full_columns(self, specified_columns) -> List["L.LcColumn"]:
        el = self._rest_elements()
        comm = L.LcCommit.commit(el.reshape(-1, 1), self.encoding)
        return comm.open_columns(list(specified_columns))[::-1]


# ---------------------------------------------------------------- reader
class EncodedFileReader:
    """EncodedFileReader<WriteableFt63, Blake3, LigeroEncoding> (encoded_file_reader.rs)."""

    def __init__(self, file_to_read, pre_encoded_size: int, encoded_size: int, rows_written: int,
                 row_capacity: int):
        self.f = file_to_read
        self.pre_encoded_size = pre_encoded_size
        self.encoded_size = encoded_size
        self.rows_written = rows_written
        self.row_capacity = row_capacity

    @classmethod
    def new_ligero(cls, file_to_read, pre_encoded_size, encoded_size, rows_written, row_capacity):
        return cls(file_to_read, pre_encoded_size, encoded_size, rows_written, row_capacity)

    def _with_map(self, fn):
        """fn(u8 array over a read-only mmap of the file); no view of it may escape fn."""
        size = os.fstat(self.f.fileno()).st_size
        need = self.row_capacity * self.encoded_size * WRITTEN_BYTES_WIDTH
        if size < need:
            raise ValueError("encoded file shorter than row_capacity * encoded_size elements")
        if need == 0:
            return fn(np.zeros(0, np.uint8))
        mm = mmap.mmap(self.f.fileno(), need, access=mmap.ACCESS_READ)
        try:
            return fn(np.frombuffer(mm, np.uint8))
        finally:
            try:
                mm.close()
            except BufferError:  # an in-flight exception's traceback still holds the view
                pass

    def get_encoded_column_without_path(self, target_col: int) -> np.ndarray:
        """Canonical u64 values of the column's rows_written elements (reader.rs:317-326)."""
        wb = WRITTEN_BYTES_WIDTH
        self.f.seek(target_col * self.row_capacity * wb)
        raw = self.f.read(self.rows_written * wb)
        return np.frombuffer(raw, "<u8").copy()

    def get_encoded_row(self, target_row: int) -> np.ndarray:
        """Canonical u64 values of the row's encoded_size elements (reader.rs:214-253)."""
        return self._with_map(lambda a: a.view("<u8").reshape(self.encoded_size, self.row_capacity)
                              [:, target_row].copy())

    def get_unencoded_row_bytes(self, target_row: int) -> bytes:
        if not target_row < self.rows_written:
            raise IndexError("target row index is out of bounds")
        return self._decode(target_row, target_row + 1)

    def _decode(self, lo: int, hi: int) -> bytes:
        out = np.zeros((hi - lo) * self.pre_encoded_size * DATA_BYTE_CAPACITY, np.uint8)
        self._with_map(lambda a: _raise(N.load().lcpc_pos_decode_porenc(
            _u8(a), self.pre_encoded_size, self.encoded_size, self.row_capacity, lo, hi, _u8(out))))
        return out.tobytes()

    def get_unencoded_row(self, target_row: int) -> np.ndarray:
        """The row's pre_encoded_size elements, raw limbs (WriteableFt63 internal words)."""
        b = self.get_unencoded_row_bytes(target_row)
        return np.frombuffer(b"".join(b[i:i + 7] + b"\0" for i in range(0, len(b), 7)), "<u8").copy()

    def decode_to_target_file(self, target_file) -> None:
        """reader.rs:79-91: every written row's pre_encoded_size * 7 bytes, in order."""
        if self.rows_written:
            target_file.write(self._decode(0, self.rows_written))
        target_file.flush()

    def get_unencoded_file_len(self) -> int:
        return os.fstat(self.f.fileno()).st_size // (self.encoded_size // self.pre_encoded_size)

    def process_file_to_merkle_tree(self) -> MerkleTree:
        w = self.encoded_size
        tree = np.zeros((2 * w - 1, DIGEST_BYTES), np.uint8)
        self._with_map(lambda a: _raise(N.load().lcpc_pos_porenc_tree(
            _u8(a), w, self.rows_written, self.row_capacity, _u8(tree))))
        return MerkleTree(tree)

    def set_new_capacity(self, new_row_capacity: int) -> None:
        if new_row_capacity < self.rows_written:
            raise ValueError("Cannot set capacity to fewer than rows are written.")
        img = _Image.__new__(_Image)
        img.f, img.size = self.f, self.row_capacity * self.encoded_size * WRITTEN_BYTES_WIDTH
        img.mm = None
        img.arr = np.zeros(0, np.uint8)
        img.grow(self.row_capacity, new_row_capacity, self.encoded_size)
        img.close()
        self.row_capacity = new_row_capacity

    def resize_to_target_file(self, target_file, new_pre_encoded_size: int, new_encoded_size: int
                              ) -> Tuple[EncodedFileMetadata, MerkleTree]:
        """reader.rs:98-117: decode every row, push its bytes into a writer of the new shape."""
        w = EncodedFileWriter(new_pre_encoded_size, new_encoded_size, self.get_unencoded_file_len(),
                              target_file)
        if self.rows_written:
            w.push_bytes(self._decode(0, self.rows_written))
        return w.finalize_to_merkle_tree()


# ---------------------------------------------------------------- file handler
SERVER_FILE_FOLDER = "PoR_server_files"   # databases/constants.rs:1-5
UNENCODED_FILE_EXTENSION, ENCODED_FILE_EXTENSION = "porraw", "porenc"
MERKLE_FILE_EXTENSION, METADATA_FILE_EXTENSION = "portree", "meta"


def _location(directory: Optional[str], ulid: str, ext: str) -> str:
    """file_formatter.rs get_*_file_location_from_id: <dir>/<ulid>.<ext>, dir created on demand
    (the reference's dir is <cwd>/PoR_server_files)."""
    d = directory if directory is not None else os.path.join(os.getcwd(), SERVER_FILE_FOLDER)
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, f"{ulid}.{ext}")


class FileHandler:
    """FileHandler<Blake3, WriteableFt63, LigeroEncoding> (lcpc_online/file_handler.rs:29-712).

    The server-side owner of one stored file: the raw `.porraw` bytes, the column-major
    `.porenc` codeword, the `.portree` Merkle tree and the `.meta` JSON.  Edits and appends
    re-encode only the touched rows (lcpc_pos_reencode_rows: pack, NTT and transpose on the GPU,
    written into the mapped `.porenc`), then rebuild the tree from the file on the GPU
    (lcpc_pos_porenc_tree), as the reference's edit_bytes / append_bytes do.
    """

    def __init__(self, ulid: str, unencoded: str, encoded: str, merkle: str, metadata: str):
        # new_attach_to_existing_files (:73-143)
        with open(metadata, "rb") as f:
            m = EncodedFileMetadata.read_from_file(f)
        if m.ulid != ulid:
            raise ValueError("supplied metadata file ulid does not match!")
        self.file_ulid = ulid
        self.pre_encoded_size, self.encoded_size = m.pre_encoded_size, m.encoded_size
        self.rows_written, self.row_capacity = m.rows_written, m.row_capacity
        self.total_data_bytes = m.bytes_of_data
        self.unencoded_file_handle, self.encoded_file_handle = unencoded, encoded
        self.merkle_tree_file_handle, self.metadata_file_handle = merkle, metadata
        with open(merkle, "rb") as f:
            self.merkle_tree = MerkleTree.from_bytes(f.read())

    # -- construction
    @classmethod
    def new_attach_to_existing_ulid(cls, file_directory: str, ulid: str) -> "FileHandler":
        paths = [os.path.join(file_directory, f"{ulid}.{e}") for e in
                 (UNENCODED_FILE_EXTENSION, ENCODED_FILE_EXTENSION, MERKLE_FILE_EXTENSION, METADATA_FILE_EXTENSION)]
        for p, what in zip(paths, ("unencoded", "encoded", "merkle", "metadata")):
            if not os.path.isfile(p):
                raise FileNotFoundError(f"no {what} file found!")
        return cls(ulid, *paths)

    @classmethod
    def new_attach_to_existing_files(cls, ulid, unencoded, encoded, merkle, metadata) -> "FileHandler":
        return cls(ulid, unencoded, encoded, merkle, metadata)

    @classmethod
    def create_from_unencoded_file(cls, ulid: str, file_handle_if_not_already_ulid: Optional[str],
                                   pre_encoded_size: int, encoded_size: int,
                                   directory: Optional[str] = None) -> "FileHandler":
        """:145-199 -- the raw file is moved to <ulid>.porraw, then encoded (GPU writer)."""
        if encoded_size <= 0 or encoded_size & (encoded_size - 1):
            raise ValueError("encoded file size must be a power of two!")
        raw = _location(directory, ulid, UNENCODED_FILE_EXTENSION)
        enc = _location(directory, ulid, ENCODED_FILE_EXTENSION)
        tree = _location(directory, ulid, MERKLE_FILE_EXTENSION)
        meta = _location(directory, ulid, METADATA_FILE_EXTENSION)
        if file_handle_if_not_already_ulid is not None:
            os.rename(file_handle_if_not_already_ulid, raw)
        with open(raw, "r+b") as f:
            m, _ = EncodedFileWriter.convert_unencoded_file(f, enc, tree, meta, pre_encoded_size, encoded_size)
        m.ulid = ulid
        with open(meta, "wb") as f:
            m.write_to_file(f)
        return cls(ulid, raw, enc, tree, meta)

    # -- accessors
    def get_encoded_file_handle(self) -> str:
        return self.encoded_file_handle

    def get_raw_file_handle(self) -> str:
        return self.unencoded_file_handle

    def get_merkle_file_handle(self) -> str:
        return self.merkle_tree_file_handle

    def get_dimensions(self) -> Tuple[int, int, int]:
        return self.pre_encoded_size, self.encoded_size, self.rows_written

    def get_encoded_metadata(self) -> EncodedFileMetadata:
        return EncodedFileMetadata(self.pre_encoded_size, self.encoded_size, self.rows_written,
                                   self.row_capacity, self.total_data_bytes, self.file_ulid)

    def get_total_data_bytes(self) -> int:
        return self.total_data_bytes

    get_total_unencoded_bytes = get_total_data_bytes

    def get_merkle_tree(self) -> MerkleTree:
        return self.merkle_tree

    def get_commit_root(self) -> bytes:
        """LcRoot::new_from_root_digest(tree.root()) (:648-651)."""
        return self.merkle_tree.root()

    def _reader(self, f) -> EncodedFileReader:
        return EncodedFileReader.new_ligero(f, self.pre_encoded_size, self.encoded_size, self.rows_written,
                                            self.row_capacity)

    def _row_bytes(self) -> int:
        return self.pre_encoded_size * DATA_BYTE_CAPACITY

    # -- raw data
    def left_multiply_unencoded_matrix_by_vector(self, left_vector) -> np.ndarray:
        """file_handler.rs:614-638: u^T M over the stored file's unencoded rows (left_vector has
        rows_written elements).  The reference's result vector is never sized, so it returns an
        empty vector; this returns the sum it is written to accumulate (pos.py's function)."""
        from .pos import left_multiply_unencoded_matrix_by_vector
        left = np.asarray(left_vector, dtype=np.uint64).reshape(-1)
        if left.size != self.rows_written:
            raise ValueError(f"left_vector incorrect size, expected {self.rows_written} and received {left.size}")
        with open(self.unencoded_file_handle, "rb") as f:
            data = f.read(self.total_data_bytes)
        return left_multiply_unencoded_matrix_by_vector(data, self.pre_encoded_size, left)

    def get_unencoded_bytes(self, byte_start: int, byte_end: int) -> bytes:
        with open(self.unencoded_file_handle, "rb") as f:
            f.seek(byte_start)
            b = f.read(byte_end - byte_start)
        if len(b) != byte_end - byte_start:
            raise EOFError("failed to fill whole buffer")
        return b

    def get_unencoded_row(self, row_index: int) -> bytes:
        """:585-602"""
        if not row_index < self.rows_written:
            raise IndexError("row_index out of bounds")
        rb = self._row_bytes()
        return self.get_unencoded_bytes(row_index * rb, min((row_index + 1) * rb, self.total_data_bytes))

    # -- encoded data
    def get_encoded_row(self, row_index: int) -> np.ndarray:
        with open(self.encoded_file_handle, "rb") as f:
            return self._reader(f).get_encoded_row(row_index)

    def get_decoded_row(self, row_index: int) -> np.ndarray:
        """:368-373 (decode_row of the encoded row, first pre_encoded_size elements)."""
        with open(self.encoded_file_handle, "rb") as f:
            return self._reader(f).get_unencoded_row(row_index)

    def get_decoded_row_bytes(self, row_index: int) -> bytes:
        with open(self.encoded_file_handle, "rb") as f:
            return self._reader(f).get_unencoded_row_bytes(row_index)

    def read_only_digests(self, columns=None) -> List[bytes]:
        """:550-564 (columns None = ColumnsToCareAbout::All)."""
        cols = range(self.encoded_size) if columns is None else columns
        return [self.merkle_tree[c] for c in cols]

    def read_full_columns(self, columns=None):
        """:566-583: LcColumn(col = the column's canonical values, path = its Merkle path)."""
        from .lcpc2d import LcColumn
        cols = range(self.encoded_size) if columns is None else columns
        with open(self.encoded_file_handle, "rb") as f:
            r = self._reader(f)
            out = []
            for c in cols:
                if not 0 <= c < self.encoded_size:
                    raise IndexError("column index out of bounds")
                out.append(LcColumn(r.get_encoded_column_without_path(c), self.merkle_tree.get_path(c)))
        return out

    # -- re-encoding
    def _reencode_rows(self, row_lo: int, row_hi: int) -> None:
        """Rows [row_lo, row_hi) from the raw file into the .porenc (one batched GPU pass)."""
        if row_hi <= row_lo:
            return
        rb = self._row_bytes()
        data = self.get_unencoded_bytes(row_lo * rb, min(row_hi * rb, self.total_data_bytes))
        img_bytes = self.row_capacity * self.encoded_size * WRITTEN_BYTES_WIDTH
        with open(self.encoded_file_handle, "r+b") as f:
            if os.fstat(f.fileno()).st_size < img_bytes:
                raise ValueError("encoded file shorter than row_capacity * encoded_size elements")
            mm = mmap.mmap(f.fileno(), img_bytes)
            try:
                arr = np.frombuffer(mm, np.uint8)
                p, keep = _bytes_ptr(data)
                _raise(N.load().lcpc_pos_reencode_rows(p, len(data), self.pre_encoded_size, self.encoded_size,
                                                       row_lo, _u8(arr), self.row_capacity))
                del arr
                mm.flush()
            finally:
                mm.close()

    def reencode_row(self, row_index: int) -> None:
        """:380-402"""
        if not row_index < self.rows_written:
            raise IndexError("cannot reencode a row that is out of bounds")
        self._reencode_rows(row_index, row_index + 1)

    def reencode_unencoded_file(self) -> None:
        """:406-462 -- the whole raw file through the GPU writer again."""
        self.total_data_bytes = os.path.getsize(self.unencoded_file_handle)
        with open(self.unencoded_file_handle, "rb") as raw, open(self.encoded_file_handle, "w+b") as tf:
            w = EncodedFileWriter(self.pre_encoded_size, self.encoded_size, self.total_data_bytes, tf)
            if self.total_data_bytes:
                w.push_bytes(raw.read())
            m, tree = w.finalize_to_merkle_tree()
        self.write_tree(tree)
        self.pre_encoded_size, self.encoded_size = m.pre_encoded_size, m.encoded_size
        self.total_data_bytes, self.row_capacity, self.rows_written = m.bytes_of_data, m.row_capacity, m.rows_written
        self._write_metadata()
        self.merkle_tree = tree

    def edit_bytes(self, byte_start: int, unencoded_bytes_to_add: bytes) -> Tuple[bytes, MerkleTree]:
        """:279-333 -- returns the bytes that were replaced and the new tree."""
        if not os.path.isfile(self.unencoded_file_handle):
            raise FileNotFoundError("no unencoded file found!")
        n = len(unencoded_bytes_to_add)
        if byte_start + n > self.total_data_bytes:
            raise ValueError("can't edit more bytes than there are in the file!")
        with open(self.unencoded_file_handle, "r+b") as f:
            f.seek(byte_start)
            original = f.read(n)
            f.seek(byte_start)
            f.write(unencoded_bytes_to_add)
        rb = self._row_bytes()
        self._reencode_rows(byte_start // rb, -(-(byte_start + n) // rb))
        return original, self.recalculate_merkle_tree()

    def append_bytes(self, bytes_to_add: bytes) -> MerkleTree:
        """:335-366"""
        with open(self.unencoded_file_handle, "ab") as f:
            f.write(bytes_to_add)
        rb = self._row_bytes()
        start_row = self.total_data_bytes // rb
        end_row = -(-(self.total_data_bytes + len(bytes_to_add)) // rb)
        if end_row > self.row_capacity:
            with open(self.encoded_file_handle, "r+b") as f:
                self._reader(f).set_new_capacity(end_row * 2)
            self.row_capacity = end_row * 2
        self.total_data_bytes += len(bytes_to_add)
        self.rows_written = end_row
        self._reencode_rows(start_row, end_row)
        tree = self.recalculate_merkle_tree()
        self._write_metadata()
        return tree

    def reshape(self, new_pre_encoded_columns: int, new_encoded_columns: int
                ) -> Tuple[EncodedFileMetadata, MerkleTree]:
        """:224-276 (convert_unencoded_file with the new shape)."""
        with open(self.unencoded_file_handle, "r+b") as f:
            m, tree = EncodedFileWriter.convert_unencoded_file(
                f, self.encoded_file_handle, self.merkle_tree_file_handle, self.metadata_file_handle,
                new_pre_encoded_columns, new_encoded_columns)
        self.pre_encoded_size, self.encoded_size = new_pre_encoded_columns, new_encoded_columns
        self.rows_written, self.row_capacity = m.rows_written, m.row_capacity
        self.merkle_tree = tree
        self._write_metadata()  # keeps the ulid, which convert_unencoded_file's metadata lacks
        m.ulid = self.file_ulid
        return m, tree

    # -- tree and metadata
    def recalculate_merkle_tree(self) -> MerkleTree:
        """:474-481 (process_file_to_merkle_tree on the GPU)."""
        with open(self.encoded_file_handle, "rb") as f:
            tree = self._reader(f).process_file_to_merkle_tree()
        self.merkle_tree = tree
        self.write_tree(tree)
        return tree

    def write_tree(self, tree: MerkleTree) -> None:
        if len(tree) != self.encoded_size * 2 - 1:
            raise ValueError("this Merkle tree is the incorrect size")
        with open(self.merkle_tree_file_handle, "wb") as f:
            write_tree_to_file(f, tree)

    def _write_metadata(self) -> None:
        with open(self.metadata_file_handle, "wb") as f:
            self.get_encoded_metadata().write_to_file(f)

    def verify_all_files_agree(self) -> None:
        """:505-541: the tree from the .porenc, and the tree of a fresh encode of the raw file,
        must both equal the stored tree (and the raw file must hold total_data_bytes)."""
        if self.recalculate_tree_only() != self.merkle_tree:
            raise AssertionError("the encoded file's tree differs from the stored tree")
        n = os.path.getsize(self.unencoded_file_handle)
        if n != self.total_data_bytes:
            raise AssertionError("raw file length differs from the metadata")
        rows = -(-(-(-n // DATA_BYTE_CAPACITY)) // self.pre_encoded_size)
        img = np.zeros(max(rows, 1) * self.encoded_size * WRITTEN_BYTES_WIDTH, np.uint8)
        data = np.fromfile(self.unencoded_file_handle, np.uint8)
        tree = np.zeros((2 * self.encoded_size - 1, DIGEST_BYTES), np.uint8)
        out_rows = C.c_size_t()
        _raise(N.load().lcpc_pos_encode_file(_u8(data), n, self.pre_encoded_size, self.encoded_size, max(rows, 1),
                                             _u8(img), _u8(tree), C.byref(out_rows)))
        if MerkleTree(tree) != self.merkle_tree:
            raise AssertionError("the raw file's re-encoded tree differs from the stored tree")

    def recalculate_tree_only(self) -> MerkleTree:
        with open(self.encoded_file_handle, "rb") as f:
            return self._reader(f).process_file_to_merkle_tree()

    def delete_all_files(self) -> None:
        """:678-694"""
        for p in (self.unencoded_file_handle, self.encoded_file_handle, self.merkle_tree_file_handle,
                  self.metadata_file_handle):
            os.remove(p)
        d = os.path.dirname(self.unencoded_file_handle)
        if not os.listdir(d):
            os.rmdir(d)
