"""Row-sharded Ligero commit / prove across GPUs (one process per GPU).

The product path is native: liblcpc_mi.so's lcpc_comm (RCCL over xGMI, or caller-supplied
collectives) and lcpc_sharded_* run the whole protocol in C++ on device buffers
(csrc/shard_native.cpp); this module's `NativeComm`, `ShardedCommit` and
`sharded_commit_prove_many` are thin drivers over those entry points.

The protocol (identical in both forms):

  commit  (lcpc-2d/src/lib.rs:651-815)
    1. rank g encodes rows [r_g, r_g+1) -- the cut points fall on BLAKE3 chunk boundaries of the
       leaf message (32 zero bytes || column), so rank g can compute the chaining values of its
       chunks [c_g, c_g+1) for every column by itself;
    2. all-to-all: rank g sends the chaining values of column block k to rank k
       ((chunks of g) x n_cols/G x 32 B -- 2-4 MiB at cfg3, not the 64 MiB codeword shard);
    3. rank k merges the chunks of its column block into leaves and builds that subtree;
    4. all-gather of the subtrees; every rank holds the whole tree (native form) or the G
       subtree roots and the top levels (RowShardedCommit below).
  prove   (lcpc-2d/src/lib.rs:1034-1123)
    the root rank owns the Merlin transcript; it broadcasts each degree-test tensor (the
    challenge vector, n_rows elements), every rank returns its partial row combination, the root
    folds them mod p and absorbs the result, and so on; the opened columns are assembled from
    every rank's rows and the Merkle paths from the tree.

`RowShardedCommit` is the same protocol written over a pluggable compute backend and
torch.distributed; the CPU tests run it with the CPU restatement as the backend (tests/test_shard.py):
the protocol the native form restates.  The proof is bit-identical to the single-GPU
LcCommit.prove either way.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np

LEAF_PREFIX = 32
CHUNK = 1024


# ---------------------------------------------------------------- partition
def chunk_partition(field_bytes: int, n_rows: int, world: int, n_chunks: Optional[int] = None):
    """[(chunk_lo, chunk_hi, row_lo, row_hi)] per rank; rows cut at chunk boundaries."""
    if n_chunks is None:
        n_chunks = -(-(LEAF_PREFIX + n_rows * field_bytes) // CHUNK)

    def first_row(c):
        if c <= 0:
            return 0
        if c >= n_chunks:
            return n_rows
        return min(n_rows, -(-(CHUNK * c - LEAF_PREFIX) // field_bytes))

    out = []
    for g in range(world):
        c_lo, c_hi = g * n_chunks // world, (g + 1) * n_chunks // world
        out.append((c_lo, c_hi, first_row(c_lo), first_row(c_hi)))
    return out


def _level_offset(n_leaves: int, level: int) -> int:
    """Offset of Merkle level `level` (>= 1) in merkle_tree's output [level1 | level2 | ...]."""
    return n_leaves - (n_leaves >> (level - 1))


# ---------------------------------------------------------------- collectives
class Comm:
    """torch.distributed on numpy buffers: gloo keeps them on the CPU, nccl (RCCL) stages them
    through the rank's GPU."""

    def __init__(self, dist=None, device: str = "cpu", group=None):
        self.dist = dist
        self.device = device
        self.group = group  # a process group of its own lets several commitments run concurrently
        self.rank = dist.get_rank(group) if dist else 0
        self.world = dist.get_world_size(group) if dist else 1

    def _t(self, a: np.ndarray):
        import torch
        return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1).copy()).to(self.device)

    def bcast(self, a: Optional[np.ndarray], shape, dtype, src: int = 0) -> np.ndarray:
        if self.world == 1:
            return a
        import torch
        nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        t = self._t(a) if self.rank == src else torch.zeros(nbytes, dtype=torch.uint8, device=self.device)
        self.dist.broadcast(t, src, group=self.group)
        return t.cpu().numpy().view(dtype).reshape(shape)

    def all_gather(self, a: np.ndarray) -> List[np.ndarray]:
        """Same-shaped arrays from every rank, in rank order."""
        if self.world == 1:
            return [a]
        t = self._t(a)
        outs = [t.clone() for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return [o.cpu().numpy().view(a.dtype).reshape(a.shape) for o in outs]

    def all_gather_v(self, a: np.ndarray) -> List[np.ndarray]:
        """Arrays whose first dimension differs per rank (padded to the max, then trimmed)."""
        if self.world == 1:
            return [a]
        lens = self.all_gather(np.array([a.shape[0]], np.int64))
        m = int(max(int(x[0]) for x in lens))
        pad = np.zeros((m,) + a.shape[1:], a.dtype)
        pad[:a.shape[0]] = a
        got = self.all_gather(pad)
        return [g[:int(n[0])] for g, n in zip(got, lens)]

    # -- device tensors (torch, on self.device): RCCL moves them in place; gloo stages via host
    @property
    def on_device(self) -> bool:
        return self.device != "cpu"

    def _nccl(self) -> bool:
        return self.dist is not None and self.dist.get_backend(self.group) == "nccl"

    def t_all_to_all(self, send, in_splits: Sequence[int], out_splits: Sequence[int]):
        """1-D byte tensors: send[sum(in_splits[:k]) ...] goes to rank k; returns the pieces
        received, concatenated in rank order."""
        if self.world == 1:
            return send
        import torch
        if self._nccl():
            out = torch.empty(int(sum(out_splits)), dtype=send.dtype, device=send.device)
            self.dist.all_to_all_single(out, send, list(map(int, out_splits)), list(map(int, in_splits)),
                                        group=self.group)
            return out
        h = send.cpu().numpy()
        offs = np.cumsum([0] + list(in_splits))
        got = self.all_to_all([h[offs[k]:offs[k + 1]] for k in range(self.world)])
        return torch.from_numpy(np.concatenate(got)).to(send.device)

    def t_all_gather(self, t):
        """Same-shaped device tensors from every rank, in rank order."""
        if self.world == 1:
            return [t]
        import torch
        if self._nccl():
            outs = [torch.empty_like(t) for _ in range(self.world)]
            self.dist.all_gather(outs, t.contiguous(), group=self.group)
            return outs
        return [torch.from_numpy(a.copy()).to(t.device) for a in self.all_gather(t.cpu().numpy())]

    def all_to_all(self, parts: Sequence[np.ndarray]) -> List[np.ndarray]:
        """parts[k] goes to rank k; returns what every rank sent here, in rank order.  Parts
        may differ in their first dimension across senders (not across receivers)."""
        if self.world == 1:
            return [parts[0]]
        recv = []
        for k in range(self.world):  # one all-gather per destination keeps it backend-neutral
            got = self.all_gather_v(parts[k])
            if k == self.rank:
                recv = got
        return recv


# ---------------------------------------------------------------- GPU backend
class GpuBackend:
    """The compute steps of a shard, through liblcpc_mi.so (the product path)."""

    def __init__(self, enc):
        from . import _native as N
        from .lcpc2d import limbs, log2
        self.N = N
        self.L = N.load()
        self.enc = enc
        self.field = enc.field
        self.limbs = limbs(enc.field)
        self.n_per_row, self.n_cols = enc.n_per_row, enc.n_cols
        self.n_col_opens = enc.get_n_col_opens()
        self.n_degree_tests = enc.get_n_degree_tests()
        self.path_len = log2(self.n_cols)

    def _raise(self, rc):
        from .lcpc2d import _raise
        _raise(rc)

    @staticmethod
    def _p64(a):
        return np.ascontiguousarray(a).ctypes.data_as(C.POINTER(C.c_uint64))

    def n_chunks(self, n_rows):
        return self.L.lcpc_leaf_n_chunks(self.field, n_rows)

    def shard_new(self, rows, row0: int, n_rows_total: int):
        """rows: host array of the shard's coefficient rows, or (device pointer, n_rows)."""
        h = C.c_void_p()
        if isinstance(rows, tuple):
            ptr, n = rows
            self._raise(self.L.lcpc_shard_new_device(self.enc._h, C.c_void_p(ptr) if n else None, row0, n,
                                                     n_rows_total, C.byref(h)))
            return (h.value, n)
        rows = np.ascontiguousarray(rows, dtype=np.uint64)
        n = rows.size // (self.limbs * self.n_per_row)
        self._raise(self.L.lcpc_shard_new(self.enc._h, self._p64(rows) if n else None, row0, n, n_rows_total,
                                          C.byref(h)))
        return (h.value, n)

    def shard_free(self, sh):
        self.L.lcpc_shard_free(sh[0])

    def chunk_cvs(self, sh, c_lo, c_hi) -> np.ndarray:
        out = np.zeros((max(c_hi - c_lo, 0), self.n_cols, 32), np.uint8)
        self._raise(self.L.lcpc_shard_chunk_cvs(sh[0], c_lo, c_hi, out.ctypes.data_as(self.N.u8p)))
        return out

    def leaves_from_cvs(self, cvs: np.ndarray) -> np.ndarray:
        cvs = np.ascontiguousarray(cvs, dtype=np.uint8)
        out = np.zeros((cvs.shape[1], 32), np.uint8)
        self._raise(self.L.lcpc_leaves_from_cvs(cvs.ctypes.data_as(self.N.u8p), cvs.shape[0], cvs.shape[1],
                                                out.ctypes.data_as(self.N.u8p)))
        return out

    def merkle(self, leaves: np.ndarray) -> np.ndarray:
        leaves = np.ascontiguousarray(leaves, dtype=np.uint8)
        n = leaves.shape[0]
        out = np.zeros((max(n - 1, 1), 32), np.uint8)
        if n > 1:
            self._raise(self.L.lcpc_merkle_tree(leaves.ctypes.data_as(self.N.u8p), n,
                                                out.ctypes.data_as(self.N.u8p)))
        return out[:n - 1]

    def collapse(self, sh, tensors: np.ndarray) -> np.ndarray:
        t = np.ascontiguousarray(tensors, dtype=np.uint64)
        nt = t.shape[0]
        out = np.zeros((nt, self.n_per_row, self.limbs), np.uint64)
        self._raise(self.L.lcpc_shard_collapse(sh[0], self._p64(t) if t.size else None, nt, self._p64(out)))
        return out

    def gather_columns(self, sh, idx: np.ndarray) -> np.ndarray:
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        out = np.zeros((len(idx), sh[1], self.limbs), np.uint64)
        if sh[1] and len(idx):
            self._raise(self.L.lcpc_shard_gather_columns(sh[0], self._p64(idx), len(idx), self._p64(out)))
        return out

    # -- device-resident forms (torch tensors in, the library writes through data_ptr())
    def chunk_cvs_dev(self, sh, c_lo, c_hi, device):
        import torch
        out = torch.empty((max(c_hi - c_lo, 0), self.n_cols, 32), dtype=torch.uint8, device=device)
        if c_hi > c_lo:
            _sync(out)
            self._raise(self.L.lcpc_shard_chunk_cvs_device(sh[0], c_lo, c_hi, C.c_void_p(out.data_ptr())))
        return out

    def leaves_tree_dev(self, cvs, n_chunks, n_cols):
        """cvs: [n_chunks][n_cols][32] device bytes (clobbered) -> leaves || levels || root."""
        import torch
        _sync(cvs)
        out = torch.empty((2 * n_cols - 1, 32), dtype=torch.uint8, device=cvs.device)
        _sync(out)
        self._raise(self.L.lcpc_leaves_tree_device(C.c_void_p(cvs.data_ptr()), n_chunks, n_cols,
                                                   C.c_void_p(out.data_ptr())))
        return out

    def collapse_dev(self, sh, tensors):
        import torch
        _sync(tensors)
        nt = tensors.shape[0]
        out = torch.empty((nt, self.n_per_row, self.limbs), dtype=torch.int64, device=tensors.device)
        self._raise(self.L.lcpc_shard_collapse_device(sh[0], C.c_void_p(tensors.data_ptr()), nt,
                                                      C.c_void_p(out.data_ptr())))
        return out

    def gather_columns_dev(self, sh, idx: np.ndarray, device):
        import torch
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        out = torch.zeros((len(idx), sh[1], self.limbs), dtype=torch.int64, device=device)
        if sh[1] and len(idx):
            _sync(out)
            self._raise(self.L.lcpc_shard_gather_columns_device(sh[0], self._p64(idx), len(idx),
                                                                C.c_void_p(out.data_ptr())))
        return out

    def field_sum_dev(self, vecs) -> np.ndarray:
        """vecs: [n_vecs][len][limbs] device tensor -> host sum mod p."""
        v = vecs.contiguous()
        _sync(v)
        out = np.zeros(v.shape[1:], np.uint64)
        self._raise(self.L.lcpc_field_sum_device(self.field, C.c_void_p(v.data_ptr()), v.shape[0], v.shape[1],
                                                 self._p64(out)))
        return out

    def field_sum(self, vecs: np.ndarray) -> np.ndarray:
        v = np.ascontiguousarray(vecs, dtype=np.uint64)
        out = np.zeros(v.shape[1:], np.uint64)
        self._raise(self.L.lcpc_field_sum(self.field, self._p64(v), v.shape[0], v.shape[1], self._p64(out)))
        return out

    def challenge_tensor(self, tr, n) -> np.ndarray:
        out = np.zeros((n, self.limbs), np.uint64)
        self._raise(self.L.lcpc_challenge_tensor(tr._h, self.field, n, self._p64(out)))
        return out

    def append_field_elems(self, tr, label: bytes, elems: np.ndarray):
        e = np.ascontiguousarray(elems, dtype=np.uint64)
        lab = (C.c_uint8 * len(label)).from_buffer_copy(label)
        self._raise(self.L.lcpc_transcript_append_field_elems(tr._h, C.cast(lab, self.N.u8p), len(label),
                                                              self.field, self._p64(e), e.size // self.limbs))

    def challenge_columns(self, tr, n) -> np.ndarray:
        out = np.zeros(n, np.uint64)
        self._raise(self.L.lcpc_challenge_columns(tr._h, self.n_cols, n, self._p64(out)))
        return out

    def proof_from_parts(self, p_eval, p_random, cols, paths):
        from .lcpc2d import LcEvalProof
        return LcEvalProof.from_arrays(self.field, self.n_cols, p_eval, list(p_random), cols, paths)


def _sync(t):
    """The library's streams are not torch's: let torch's work on t finish before it is read."""
    import torch
    torch.cuda.current_stream(t.device).synchronize()


LABEL_PR = b"$l//PR"
LABEL_PE = b"$l//PE"


# ---------------------------------------------------------------- the protocol
class RowShardedCommit:
    """One rank's share of a row-sharded commitment (see the module docstring)."""

    def __init__(self, backend, comm: Comm, n_rows: int, field_bytes: int):
        self.b, self.comm = backend, comm
        self.n_rows = n_rows
        G = comm.world
        self.n_chunks = backend.n_chunks(n_rows)
        self.part = chunk_partition(field_bytes, n_rows, G, self.n_chunks)
        self.c_lo, self.c_hi, self.r_lo, self.r_hi = self.part[comm.rank]
        np2 = backend.n_cols
        if np2 & (np2 - 1) or G & (G - 1) or np2 % G:
            raise ValueError("row shards need power-of-two n_cols and world size, world | n_cols")
        self.block = np2 // G
        self.sh = None

    # -- commit
    def commit(self, coeff_rows) -> bytes:
        """coeff_rows: this rank's rows [r_lo, r_hi) of the zero-padded coefficient matrix (host
        array, or (device pointer, n_rows) with the GPU backend)."""
        b, comm, G = self.b, self.comm, self.comm.world
        self.sh = b.shard_new(coeff_rows, self.r_lo, self.n_rows)
        if self.device_mode:
            return self._commit_dev()
        cvs = b.chunk_cvs(self.sh, self.c_lo, self.c_hi)                 # (my chunks, n_cols, 32)
        B = self.block
        recv = comm.all_to_all([cvs[:, k * B:(k + 1) * B] for k in range(G)])
        all_cvs = np.concatenate(recv, axis=0)                            # (n_chunks, B, 32)
        self.leaves = b.leaves_from_cvs(all_cvs)                          # my column block
        self.sub = b.merkle(self.leaves)                                  # B - 1 nodes
        sub_root = self.sub[-1] if B > 1 else self.leaves[0]
        self.roots = np.stack(comm.all_gather(sub_root))                  # (G, 32)
        self.top = b.merkle(self.roots)                                   # G - 1 nodes
        self.root = bytes(self.top[-1] if G > 1 else self.roots[0])
        return self.root

    @property
    def device_mode(self) -> bool:
        return self.comm.on_device and hasattr(self.b, "chunk_cvs_dev")

    def _commit_dev(self) -> bytes:
        """commit with the chaining values exchanged as device tensors (RCCL all-to-all)."""
        b, comm, G, B = self.b, self.comm, self.comm.world, self.block
        nch = self.c_hi - self.c_lo
        cvs = b.chunk_cvs_dev(self.sh, self.c_lo, self.c_hi, comm.device)        # [nch][n_cols][32]
        # column block k of every chunk goes to rank k: [k][chunk][B][32], contiguous per k
        send = cvs.view(nch, G, B, 32).transpose(0, 1).contiguous().view(-1)
        out_splits = [(p[1] - p[0]) * B * 32 for p in self.part]
        recv = comm.t_all_to_all(send, [nch * B * 32] * G, out_splits)           # [all chunks][B][32]
        tree = b.leaves_tree_dev(recv.view(self.n_chunks, B, 32), self.n_chunks, B)
        tree = tree.cpu().numpy()                                               # 2B - 1 digests
        self.leaves, self.sub = tree[:B], tree[B:]
        sub_root = tree[-1]
        self.roots = np.stack(comm.all_gather(sub_root))                         # (G, 32)
        self.top = b.merkle(self.roots)
        self.root = bytes(self.top[-1] if G > 1 else self.roots[0])
        return self.root

    @staticmethod
    def _tree_paths(tree: np.ndarray, width: int, idx: np.ndarray) -> np.ndarray:
        """Sibling digests of positions idx in a Merkle tree stored as leaves || level 1 || ...
        (width leaves): level l of the tree starts at 2 width - 2 (width >> l)."""
        lvls = width.bit_length() - 1
        idx = np.asarray(idx, dtype=np.int64).reshape(-1)
        if lvls == 0 or idx.size == 0:
            return np.zeros((idx.size, lvls, 32), np.uint8)
        lv = np.arange(lvls)
        base = 2 * width - 2 * (width >> lv)
        sib = (idx[:, None] >> lv[None, :]) ^ 1
        return tree[base[None, :] + sib]

    def _lower_paths(self, js: np.ndarray) -> np.ndarray:
        """Sibling digests of columns js (in my block) below the subtree root."""
        tree = np.concatenate([self.leaves, self.sub]) if len(self.sub) else self.leaves
        return self._tree_paths(tree, self.block, np.asarray(js, dtype=np.int64) - self.comm.rank * self.block)

    def _upper_paths(self, js: np.ndarray) -> np.ndarray:
        G = self.comm.world
        tree = np.concatenate([self.roots, self.top]) if G > 1 else self.roots
        return self._tree_paths(tree, G, np.asarray(js, dtype=np.int64) // self.block)

    # -- prove
    def prove(self, outer: np.ndarray, tr=None):
        """Every rank calls this; rank 0 passes the transcript and gets the LcEvalProof."""
        if self.device_mode:
            return self._prove_dev(outer, tr)
        b, comm = self.b, self.comm
        rank0 = comm.rank == 0
        nl = b.limbs
        n_rows, lo, hi = self.n_rows, self.r_lo, self.r_hi
        outer = np.ascontiguousarray(outer, dtype=np.uint64).reshape(n_rows, nl)
        ndt = b.n_degree_tests
        p_random = []
        p_eval = None
        for i in range(max(ndt, 1)):
            tens = []
            if i < ndt:
                t = b.challenge_tensor(tr, n_rows) if rank0 else None
                t = comm.bcast(t, (n_rows, nl), np.uint64)   # the challenge vector
                tens.append(t[lo:hi])
            if i == 0:
                tens.append(outer[lo:hi])                     # the evaluation tensor rides along
            parts = b.collapse(self.sh, np.stack(tens))        # (len(tens), n_per_row, limbs)
            allp = comm.all_gather(parts)
            if rank0:
                sums = [b.field_sum(np.stack([p[k] for p in allp])) for k in range(len(tens))]
                if i < ndt:
                    p_random.append(sums[0])
                    b.append_field_elems(tr, LABEL_PR, sums[0])
                if i == 0:
                    p_eval = sums[-1]
        if rank0:
            b.append_field_elems(tr, LABEL_PE, p_eval)
        nco = b.n_col_opens
        idx = b.challenge_columns(tr, nco) if rank0 else None
        idx = comm.bcast(idx, (nco,), np.uint64)
        cols = comm.all_gather_v(b.gather_columns(self.sh, idx).transpose(1, 0, 2).copy())
        lower = np.zeros((nco, self.block.bit_length() - 1, 32), np.uint8)
        own = (idx.astype(np.int64) // self.block) == comm.rank
        lower[own] = self._lower_paths(idx[own])
        lowers = comm.all_gather(lower)
        if not rank0:
            return None
        cols = np.concatenate(cols, axis=0).transpose(1, 0, 2)          # (nco, n_rows, limbs)
        owner = idx.astype(np.int64) // self.block
        low = np.stack(lowers)[owner, np.arange(nco)]                         # (nco, lower levels, 32)
        paths = np.concatenate([low, self._upper_paths(idx)], axis=1)
        return b.proof_from_parts(p_eval, p_random, np.ascontiguousarray(cols), paths)

    def _prove_dev(self, outer: np.ndarray, tr=None):
        """prove with the partial row combinations and opened column pieces as device tensors
        (RCCL all-gathers); rank 0 folds the partials on its GPU and runs the transcript."""
        import torch
        b, comm = self.b, self.comm
        dev = comm.device
        rank0 = comm.rank == 0
        nl = b.limbs
        n_rows, lo, hi = self.n_rows, self.r_lo, self.r_hi
        outer = np.ascontiguousarray(outer, dtype=np.uint64).reshape(n_rows, nl)
        ndt = b.n_degree_tests
        p_random = []
        p_eval = None
        for i in range(max(ndt, 1)):
            tens = []
            if i < ndt:
                t = b.challenge_tensor(tr, n_rows) if rank0 else None
                t = comm.bcast(t, (n_rows, nl), np.uint64)   # the challenge vector
                tens.append(t[lo:hi])
            if i == 0:
                tens.append(outer[lo:hi])                     # the evaluation tensor rides along
            dt = torch.from_numpy(np.ascontiguousarray(np.stack(tens)).view(np.int64)).to(dev)
            parts = b.collapse_dev(self.sh, dt)                # (len(tens), n_per_row, limbs)
            allp = torch.stack(comm.t_all_gather(parts))     # (G, len(tens), n_per_row, limbs)
            if rank0:
                sums = [b.field_sum_dev(allp[:, k]) for k in range(len(tens))]
                if i < ndt:
                    p_random.append(sums[0])
                    b.append_field_elems(tr, LABEL_PR, sums[0])
                if i == 0:
                    p_eval = sums[-1]
        if rank0:
            b.append_field_elems(tr, LABEL_PE, p_eval)
        nco = b.n_col_opens
        idx = b.challenge_columns(tr, nco) if rank0 else None
        idx = comm.bcast(idx, (nco,), np.uint64)
        rows = [p[3] - p[2] for p in self.part]
        mine = b.gather_columns_dev(self.sh, idx, dev)        # (nco, my rows, limbs)
        pad = torch.zeros((nco, max(rows), nl), dtype=torch.int64, device=dev)
        pad[:, :mine.shape[1]] = mine
        got = comm.t_all_gather(pad)
        lower = np.zeros((nco, self.block.bit_length() - 1, 32), np.uint8)
        own = (idx.astype(np.int64) // self.block) == comm.rank
        lower[own] = self._lower_paths(idx[own])
        lowers = comm.all_gather(lower)
        if not rank0:
            return None
        cols = torch.cat([g[:, :r] for g, r in zip(got, rows)], dim=1)        # (nco, n_rows, limbs)
        cols = cols.cpu().numpy().view(np.uint64)
        owner = idx.astype(np.int64) // self.block
        low = np.stack(lowers)[owner, np.arange(nco)]                         # (nco, lower levels, 32)
        paths = np.concatenate([low, self._upper_paths(idx)], axis=1)
        return b.proof_from_parts(p_eval, p_random, np.ascontiguousarray(cols), paths)

    def close(self):
        if self.sh is not None:
            self.b.shard_free(self.sh)
            self.sh = None


# ================================================================ native driver (the product path)
class NativeComm:
    """An lcpc_comm handle.

    * ``NativeComm.rccl(dist, group)``: RCCL over xGMI, one rank per GPU.  Rank 0 draws the
      unique id (lcpc_comm_rccl_unique_id) and sends it over `dist` (any backend).
    * ``NativeComm.host(dist, group)``: the collectives supplied from here over a CPU process
      group (gloo): device buffers are staged through the host.  For several ranks sharing one
      GPU (RCCL refuses duplicate GPUs) and for tests.
    * ``NativeComm.single()``: one rank, no exchanges.
    """

    def __init__(self, handle, keep=None):
        self._h = handle
        self._keep = keep  # ctypes callbacks must outlive the handle
        L = _lib()
        self.rank = L.lcpc_comm_rank(handle)
        self.world = L.lcpc_comm_nranks(handle)
        self.is_rccl = bool(L.lcpc_comm_is_rccl(handle))

    def __del__(self):
        try:
            _lib().lcpc_comm_free(self._h)
        except Exception:
            pass

    @classmethod
    def single(cls):
        from . import _native as N
        ops = N.CommOps()
        h = C.c_void_p()
        _check(_lib().lcpc_comm_from_ops(C.byref(ops), 1, 0, C.byref(h)))
        return cls(h.value, ops)

    @classmethod
    def rccl(cls, dist, group=None):
        import torch
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        uid = (C.c_uint8 * 128)()
        if rank == 0:
            _check(_lib().lcpc_comm_rccl_unique_id(uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group, device=torch.device("cpu") if dist.get_backend(group) == "gloo"
                                   else None)
        uid = (C.c_uint8 * 128).from_buffer_copy(obj[0])
        h = C.c_void_p()
        _check(_lib().lcpc_comm_rccl_new(uid, world, rank, C.byref(h)))
        return cls(h.value)

    @classmethod
    def host(cls, dist, group=None):
        from . import _native as N
        t = _HostTransport(dist, group)
        ops = N.CommOps(None, N.ALL_GATHER_FN(t.all_gather), N.ALL_TO_ALL_V_FN(t.all_to_all_v),
                        N.BROADCAST_FN(t.broadcast))
        h = C.c_void_p()
        _check(_lib().lcpc_comm_from_ops(C.byref(ops), t.world, t.rank, C.byref(h)))
        return cls(h.value, (ops, t))


class _HostTransport:
    """lcpc_comm_ops over a CPU torch.distributed group: device bytes -> host -> gloo -> device."""

    def __init__(self, dist, group=None):
        self.dist, self.group = dist, group
        self.rank, self.world = dist.get_rank(group), dist.get_world_size(group)
        self.hip = C.CDLL("libamdhip64.so.7")  # the runtime liblcpc_mi.so itself uses
        self.hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]

    def _d2h(self, ptr, n):
        import torch
        t = torch.empty(n, dtype=torch.uint8)
        if n and self.hip.hipMemcpy(t.data_ptr(), ptr, n, 2):
            raise RuntimeError("hipMemcpy D2H failed")
        return t

    def _h2d(self, ptr, t):
        n = t.numel()
        if n and self.hip.hipMemcpy(ptr, t.data_ptr(), n, 1):
            raise RuntimeError("hipMemcpy H2D failed")

    def all_gather(self, user, send, recv, nbytes):
        try:
            import torch
            src = self._d2h(send, nbytes)
            out = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
            self.dist.all_gather(out, src, group=self.group)
            self._h2d(recv, torch.cat(out))
            return 0
        except Exception:  # a C caller cannot take a Python exception
            return 1

    def all_to_all_v(self, user, send, sb, recv, rb):
        try:
            import torch
            sbl = [int(sb[k]) for k in range(self.world)]
            rbl = [int(rb[k]) for k in range(self.world)]
            src = self._d2h(send, sum(sbl))
            out = torch.empty(sum(rbl), dtype=torch.uint8)
            self.dist.all_to_all_single(out, src, rbl, sbl, group=self.group)
            self._h2d(recv, out)
            return 0
        except Exception:
            return 1

    def broadcast(self, user, buf, nbytes, root):
        try:
            if nbytes:
                t = self._d2h(buf, nbytes)
                src = self.dist.get_global_rank(self.group, root) if self.group is not None else root
                self.dist.broadcast(t, src, group=self.group)
                self._h2d(buf, t)
            return 0
        except Exception:
            return 1


def _lib():
    from . import _native as N
    return N.load()


def _check(rc):
    from .lcpc2d import _raise
    _raise(rc)


def sharded_rows(field: int, n_rows: int, world: int, rank: int):
    """(row0, n_shard_rows) of `rank` (lcpc_sharded_rows): cut on BLAKE3 chunk boundaries."""
    r0, n = C.c_size_t(), C.c_size_t()
    _check(_lib().lcpc_sharded_rows(field, n_rows, world, rank, C.byref(r0), C.byref(n)))
    return r0.value, n.value


class ShardedCommit:
    """lcpc_sharded_commit: this rank's share of a row-sharded commitment (collective)."""

    def __init__(self, enc, comm: NativeComm, d_rows: int, n_rows: int):
        h = C.c_void_p()
        _check(_lib().lcpc_sharded_commit_new_device(enc._h, C.c_void_p(d_rows) if d_rows else None, n_rows,
                                                     comm._h, C.byref(h)))
        self._h, self.enc, self.comm, self.n_rows = h.value, enc, comm, n_rows

    def __del__(self):
        try:
            _lib().lcpc_sharded_commit_free(self._h)
        except Exception:
            pass

    def get_root(self) -> bytes:
        out = (C.c_uint8 * 32)()
        _check(_lib().lcpc_sharded_commit_get_root(self._h, out))
        return bytes(out)

    @property
    def hashes(self) -> bytes:
        n = _lib().lcpc_sharded_commit_n_hashes(self._h)
        out = (C.c_uint8 * (32 * n))()
        _check(_lib().lcpc_sharded_commit_copy_hashes(self._h, out))
        return bytes(out)

    def prove(self, outer, tr=None, root: int = 0):
        """Collective; returns the LcEvalProof on rank `root` (which passes the transcript: the
        library's Transcript or the caller's own, as LcCommit.prove)."""
        from .lcpc2d import CallerTranscript, LcEvalProof, _elems, _transcript
        o = np.ascontiguousarray(_elems(outer, self.enc.field))
        h = C.c_void_p()
        tr = _transcript(tr) if tr is not None else None
        rc = _lib().lcpc_sharded_prove(self._h, o.ctypes.data_as(C.POINTER(C.c_uint64)), o.shape[0], self.enc._h,
                                       tr._h if tr is not None else None, root, C.byref(h))
        if isinstance(tr, CallerTranscript):
            tr.reraise(rc)
        _check(rc)
        return LcEvalProof(h.value) if h.value else None


    def pos_request(self, left, columns, root: int = 0):
        """Collective proof-of-storage request (lcpc_sharded_pos_request; networking/server.rs:652-737):
        on rank `root` returns (u^T Enc(M) as an (n_cols, limbs) array, [LcColumn] of the requested
        columns with their Merkle paths); None elsewhere."""
        from .lcpc2d import LcColumn, _elems, limbs, log2
        nl = limbs(self.enc.field)
        u = np.ascontiguousarray(_elems(left, self.enc.field))
        idx = np.ascontiguousarray(list(columns), dtype=np.uint64)
        n = len(idx)
        nc = self.enc.n_cols
        pl = log2(nc)
        mine = self.comm.rank == root
        ev = np.zeros((nc, nl), np.uint64) if mine else None
        cols = np.zeros((max(n, 1), self.n_rows, nl), np.uint64) if mine else None
        paths = (C.c_uint8 * max(32 * pl * n, 1))() if mine else None
        p64 = C.POINTER(C.c_uint64)
        _check(_lib().lcpc_sharded_pos_request(
            self._h, u.ctypes.data_as(p64), u.shape[0], idx.ctypes.data_as(p64) if n else None, n, root,
            ev.ctypes.data_as(p64) if mine else None, cols.ctypes.data_as(p64) if mine else None,
            C.cast(paths, C.POINTER(C.c_uint8)) if mine else None))
        if not mine:
            return None
        pb = bytes(paths)
        return ev, [LcColumn(cols[k].copy(), [pb[32 * (k * pl + i):32 * (k * pl + i + 1)] for i in range(pl)])
                    for k in range(n)]


def pos_pack_shard(d_bytes: int, n_bytes: int, n_per_row: int, row0: int, n_shard_rows: int, d_out: int,
                   stream=None):
    """This rank's rows of a proof-of-storage file on device: the file's bytes (device, d_bytes,
    n_bytes in all) of rows [row0, row0 + n_shard_rows) packed 7 per WriteableFt63 element
    (lcpc_pos_bytes_to_field_device; data_field.rs:38-46) into d_out, which must hold
    n_shard_rows * n_per_row zeroed elements (the last row's tail stays zero, as the file's
    zero padding does).  Row r starts at byte 7 n_per_row r, so each rank packs on its own."""
    lo = min(n_bytes, 7 * n_per_row * row0)
    hi = min(n_bytes, 7 * n_per_row * (row0 + n_shard_rows))
    if hi > lo:
        _check(_lib().lcpc_pos_bytes_to_field_device(C.c_void_p(d_bytes + lo), hi - lo, C.c_void_p(d_out),
                                                     C.c_void_p(stream) if stream else None))


def sharded_reserve(enc, comm: NativeComm, n_rows: int, n_polys: int, lag: int = 0):
    """lcpc_sharded_reserve: pre-populate the pools for sharded_commit_prove_many(n_polys, lag)."""
    _check(_lib().lcpc_sharded_reserve(enc._h, n_rows, comm._h, n_polys, lag))


def sharded_commit_prove_many(enc, comm: NativeComm, d_rows: Sequence[int], n_rows: int, outer, make_transcript,
                              lag: int = 0, keep_proofs: bool = True):
    """lcpc_sharded_commit_prove_many: pipelined commit + prove of len(d_rows) polynomials.

    make_transcript(i, root) -> the transcript for polynomial i (called on its root rank, i % world):
    the library's Transcript, or the caller's own transcript object (CallerTranscript: its proof's
    absorbs and squeezes go to it); returns (roots, proofs) with proofs[i] an LcEvalProof on the
    root rank of i, else None."""
    from . import _native as N
    from .lcpc2d import CallerTranscript, LcEvalProof, Transcript, _elems, _transcript
    L = _lib()
    n = len(d_rows)
    o = np.ascontiguousarray(_elems(outer, enc.field))
    rows = (C.c_void_p * max(n, 1))(*[C.c_void_p(p) for p in d_rows])
    proofs = (C.c_void_p * max(n, 1))()
    roots = (C.c_uint8 * max(32 * n, 1))()
    callers = []  # caller transcripts (their callbacks) live until the call returns

    def mk(user, i, root):
        tr = make_transcript(int(i), bytes(root[:32]))
        if isinstance(tr, Transcript):
            return L.lcpc_transcript_clone(tr._h)  # the library owns (and frees) the clone
        ct = _transcript(tr)
        callers.append(ct)
        # a second ops handle over the same callbacks: the library owns (and frees) it
        return L.lcpc_transcript_from_ops(C.byref(ct._ops))

    cb = N.MAKE_TRANSCRIPT_FN(mk)
    rc = L.lcpc_sharded_commit_prove_many(enc._h, rows, n, n_rows, o.ctypes.data_as(C.POINTER(C.c_uint64)),
                                          comm._h, cb, None, lag, proofs if keep_proofs else None, roots)
    for ct in callers:
        if isinstance(ct, CallerTranscript):
            ct.reraise(rc)
    _check(rc)
    rb = bytes(roots)
    return ([rb[32 * i:32 * i + 32] for i in range(n)],
            [LcEvalProof(proofs[i]) if proofs[i] else None for i in range(n)])
