"""Host-resident inputs: the commit a drop-in caller actually makes.

The reference's commit reads the caller's coefficients from host memory (`coeffs_in: &[F]`,
lcpc-2d/src/lib.rs:651-682), and the proof-of-storage server re-commits a file it has just read
from disk on every proof request (networking/server.rs:670-679).  lcpc_commit_new /
lcpc_pos_commit_bytes move the input across PCIe in row blocks on a copy stream, encoding each
block as it lands; pageable memory takes the runtime's pageable path, page-locked memory is read
by the DMA engine directly.  Every case must give the oracle's commitment bit for bit, and the
same one as the device-resident entry points.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


class PinnedHost:
    """page-locked host buffers (hipHostMalloc) through the HIP runtime the library links"""

    def __init__(self):
        self.L = C.CDLL("libamdhip64.so.7")
        self.L.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
        self.L.hipHostFree.argtypes = [C.c_void_p]
        self.live = []

    def array(self, n, dtype):
        p = C.c_void_p()
        nbytes = max(n * np.dtype(dtype).itemsize, 16)
        assert self.L.hipHostMalloc(C.byref(p), nbytes, 0) == 0
        self.live.append(p.value)
        buf = (C.c_uint8 * nbytes).from_address(p.value)
        return np.frombuffer(buf, dtype=dtype, count=n)

    def free_all(self):
        for p in self.live:
            self.L.hipHostFree(p)
        self.live = []


@pytest.fixture
def pinned(gpu):
    h = PinnedHost()
    yield h
    h.free_all()


def rand_elems(oracle, fid, n, seed):
    return oracle.ChaCha(seed_u64=seed).field_random(fid, n)


@pytest.mark.parametrize("source", ["pageable", "pinned"])
@pytest.mark.parametrize("fid,n_per_row,n_cols,length", [
    (1, 2048, 4096, 1 << 16),            # cfg1 shape: one 8 MiB block holds every row
    (1, 8192, 16384, 128 * 8192),        # cfg2 shape: 16 MiB of rows -> two blocks
    (1, 8192, 16384, 100 * 8192 + 77),   # ragged last row in the last block
    (0, 32768, 65536, 70 * 32768 + 5),   # Ft63 rows of 256 KiB: 32-row blocks, ragged tail
    (1, 1 << 19, 1 << 20, 3 * (1 << 19) + 1),  # rows of 8 MiB: one row per block, 4 blocks
    (3, 2048, 8192, 3 * 2048 + 1),       # Ft255, rate 1/4
    (2, 512, 1024, 60 * 512 + 3),        # Ft191
])
def test_host_commit_matches_oracle_and_device(gpu, oracle, hipmem, pinned, source, fid, n_per_row, n_cols,
                                               length):
    from lcpc_proof_of_storage_amd import _native as N
    coeffs = rand_elems(oracle, fid, length, 41)
    if source == "pinned":
        host = pinned.array(coeffs.size, np.uint64)
        host[:] = coeffs
    else:
        host = coeffs.copy()
    enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, 16, 2)
    g = gpu.LcCommit.commit(host, enc)
    assert N.load().lcpc_last_upload_pinned() == (1 if source == "pinned" else 0)
    o = oracle.Commit(oracle.Encoding.ligero(fid, n_per_row, n_cols, 16, 2), coeffs)
    assert np.array_equal(g.coeffs.reshape(-1), o.coeffs)
    assert g.get_root() == o.root()
    if length <= (1 << 20):
        assert np.array_equal(g.comm.reshape(-1), o.comm)
    d = hipmem.to_device(coeffs)
    try:
        assert gpu.LcCommit.commit_device(d, length, enc).get_root() == g.get_root()
    finally:
        hipmem.free(d)
    assert np.array_equal(host.reshape(-1), coeffs)  # the caller's buffer is only read


def test_host_commit_sdig(gpu, oracle):
    """Brakedown from host memory (whole upload, then the element-major encode)."""
    fid, length = 1, 3 * 4096 + 11
    enc = gpu.SdigEncoding.new(fid, length, 0)
    coeffs = rand_elems(oracle, fid, length, 43)
    o_enc = oracle.Encoding.sdig(fid, gpu.SdigEncoding.n_per_row_for(fid, length), seed=0, code_id=3)
    assert gpu.LcCommit.commit(coeffs, enc).get_root() == oracle.Commit(o_enc, coeffs).root()


NP, NC = 1 << 14, 1 << 15  # the proof-of-storage default dims (one-pass fused kernel)


@pytest.mark.parametrize("source", ["pageable", "pinned"])
@pytest.mark.parametrize("dims,n_bytes,offset", [
    ((NP, NC), 7 * NP * 20, 0),              # 20 whole rows: one 8 MiB upload block (73 rows)
    ((NP, NC), 7 * NP * 150 + 12345, 0),     # three blocks, ragged last row
    ((NP, NC), 7 * NP * 80 + 3, 5),          # unaligned host image (offset into the buffer)
    ((NP, NC), 13, 0),                       # two elements, one row
    ((100, 256), 7 * 100 * 3 + 5, 0),        # other dims: uploaded, then packed and encoded
])
def test_host_pos_commit_bytes(gpu, oracle, hipmem, pinned, source, dims, n_bytes, offset):
    """lcpc_pos_commit_bytes (host file image) == DataField::from_byte_vec + LcCommit::commit
    (the oracle) == lcpc_pos_commit_bytes_device"""
    np_, nc = dims
    data = np.random.default_rng(n_bytes).integers(0, 256, n_bytes, dtype=np.uint8)
    data[-1] = 0xFF
    if source == "pinned":
        buf = pinned.array(n_bytes + offset, np.uint8)
    else:
        buf = np.empty(n_bytes + offset, np.uint8)
    buf[offset:] = data
    img = buf[offset:]
    enc = gpu.RsEncoding.new(0, np_, nc, 16, 2)
    g = gpu.LcCommit.commit_pos_bytes(img, enc)
    el = oracle.pos_bytes_to_field(data.tobytes())
    o = oracle.Commit(oracle.Encoding.ligero(0, np_, nc, 16, 2), el)
    assert g.get_root() == o.root()
    assert np.array_equal(g.coeffs.reshape(-1), o.coeffs)
    d = hipmem.to_device(np.concatenate([data, np.zeros((-n_bytes) % 8, np.uint8)]).view(np.uint64))
    try:
        assert gpu.LcCommit.commit_pos_bytes_device(d, n_bytes, enc).get_root() == g.get_root()
    finally:
        hipmem.free(d)


def test_host_pos_commit_bytes_rejects(gpu):
    enc127 = gpu.RsEncoding.new(1, 64, 128, 4, 1)
    with pytest.raises(gpu.LcpcError):
        gpu.LcCommit.commit_pos_bytes(b"\x01" * 64, enc127)  # not WriteableFt63
    enc = gpu.RsEncoding.new(0, 64, 128, 4, 1)
    with pytest.raises(gpu.LcpcError):
        gpu.LcCommit.commit_pos_bytes(b"", enc)


def test_host_commit_then_prove(gpu, oracle):
    """a host-input commitment proves like any other (cfg1 shape, oracle transcript lock step)"""
    fid, n_per_row, n_cols, nco = 1, 2048, 4096, 309
    coeffs = rand_elems(oracle, fid, 1 << 16, 47)
    enc = gpu.RsEncoding.new(fid, n_per_row, n_cols, nco, 2)
    o_enc = oracle.Encoding.ligero(fid, n_per_row, n_cols, nco, 2)
    g = gpu.LcCommit.commit(coeffs, enc)
    o = oracle.Commit(o_enc, coeffs)
    outer = rand_elems(oracle, fid, g.get_n_rows(), 48)
    tr = gpu.Transcript(b"test transcript")
    tr.append_message(b"polycommit", g.get_root())
    tr.append_message(b"ncols", nco.to_bytes(8, "big"))
    gp = g.prove(outer, enc, tr)
    op = o.prove(o_enc, outer, oracle.standard_transcript(nco, o.root()))
    assert np.array_equal(gp.p_eval.reshape(-1), op.p_eval)
    assert np.array_equal(np.stack([c.col for c in gp.columns]).reshape(-1), op.cols)
