"""Generate tests/golden/*.json from the oracle (test infrastructure).

    python tests/golden/gen_golden.py

The Rust reference cannot be built or run here, so these fixtures pin the
build's own oracle -- which is itself pinned by published KATs (tests/test_oracle_kats.py)
and by the reference's invariant tests (tests/test_oracle_invariants.py).  The GPU path is
then checked against them bit for bit (tests/test_golden.py).  Large arrays are stored as
SHA-256 digests of their little-endian u64 Montgomery limbs (the ff_derive in-memory layout).

Inputs follow SURVEY.md §8(d): coefficients = F::random draws from
ChaCha20Rng::seed_from_u64(0x1CDC2024); x = F::random from seed_from_u64(7); inner/outer
tensors as lcpc-ligero-pc/src/tests.rs:234-242; transcript prefix as :245-247.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_ffi as O  # noqa: E402

SEED = 0x1CDC2024


def sha(a) -> str:
    if isinstance(a, (bytes, bytearray)):
        return hashlib.sha256(a).hexdigest()
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


def ligero_case(fid, log_len, rho=(1, 2), length=None, x_seed=7):
    n = length if length is not None else 1 << log_len
    enc = O.Encoding.ligero_new(fid, n, rho)
    coeffs = O.random_coeffs(fid, n, SEED)
    comm = O.Commit(enc, coeffs)
    root = comm.root()
    x = O.ChaCha(seed_u64=x_seed).field_random(fid, 1)
    inner, outer = O.eval_tensors(fid, x, comm.n_per_row, comm.n_rows)
    pf = comm.prove(enc, outer, O.standard_transcript(enc.n_col_opens, root))
    rc, ev = pf.verify(root, outer, inner, enc, O.standard_transcript(enc.n_col_opens, root))
    assert rc == 0
    return {
        "field": fid, "len": n, "rho": list(rho), "coeff_seed": SEED, "x_seed": x_seed,
        "dims": [comm.n_rows, comm.n_per_row, comm.n_cols],
        "n_col_opens": enc.n_col_opens, "n_degree_tests": enc.n_degree_tests,
        "root": root.hex(),
        "comm_sha256": sha(comm.comm),
        "hashes_sha256": sha(comm.hashes),
        "p_eval_sha256": sha(pf.p_eval),
        "p_random_sha256": sha(pf.p_random),
        "cols_sha256": sha(pf.cols),
        "paths_sha256": sha(pf.paths.tobytes()),
        "col_idx": [int(v) for v in pf.col_idx],
        "eval": hex(O.from_mont(fid, ev)[0]),
    }


def encode_case(fid, log_len):
    n = 1 << log_len
    nr, np_, nc = O.ligero_dims(fid, n)
    enc = O.Encoding.ligero(fid, np_, nc)
    coeffs = O.random_coeffs(fid, n, SEED)
    comm = O.Commit(enc, coeffs)
    rows = comm.comm.reshape(nr, -1)
    return {
        "field": fid, "len": n, "dims": [nr, np_, nc], "coeff_seed": SEED,
        "rows_sha256": sha(rows),
        "row_sha256": {str(r): sha(rows[r]) for r in (0, nr // 2 - 1, nr - 1)},
    }


def brakedown_case(fid, n, seed):
    import ctypes as C
    enc = O.Encoding.sdig(fid, n, seed=seed, code_id=3)
    L = O.lib()
    nl = O.limbs(fid)
    mats = []
    for lvl in range(L.of_sdig_levels(enc.ptr)):
        for which in (0, 1):
            r, c = C.c_size_t(), C.c_size_t()
            nnz = L.of_sdig_matrix(enc.ptr, lvl, which, C.byref(r), C.byref(c), None, None, None)
            ptr = np.zeros(c.value + 1, np.uint64)
            idx = np.zeros(nnz, np.uint64)
            val = np.zeros(nnz * nl, np.uint64)
            szp = C.POINTER(C.c_size_t)
            L.of_sdig_matrix(enc.ptr, lvl, which, C.byref(r), C.byref(c), ptr.ctypes.data_as(szp),
                             idx.ctypes.data_as(szp), O.p64(val))
            mats.append({"level": lvl, "which": ["pre", "post"][which], "rows": r.value, "cols": c.value,
                         "nnz": nnz, "ptr_sha256": sha(ptr), "idx_sha256": sha(idx), "val_sha256": sha(val)})
    row = np.zeros(enc.n_cols * nl, np.uint64)
    row[:n * nl] = O.random_coeffs(fid, n, SEED)
    out = enc.encode(row)
    return {"field": fid, "n_per_row": n, "seed": seed, "code": "SdigCode3", "n_cols": enc.n_cols,
            "matrices": mats, "encoded_row_sha256": sha(out), "coeff_seed": SEED,
            "encoded_head": [hex(v) for v in O.from_mont(fid, out[:4 * nl])]}


def transcript_case():
    tr = O.Transcript(b"test protocol")
    tr.append_message(b"some label", b"some data")
    c1 = tr.challenge_bytes(b"challenge", 32)
    tr2 = O.Transcript(b"test transcript")
    tr2.append_message(b"polycommit", bytes(range(32)))
    tr2.append_message(b"ncols", (309).to_bytes(8, "big"))
    dt = tr2.challenge_bytes(b"$l//DT", 32)
    rng = O.ChaCha(dt)
    col = [rng.uniform(0, 65536) for _ in range(8)]
    return {"merlin_test_protocol": c1.hex(), "lcpc_prefix_DT": dt.hex(), "chacha_cols_65536": col,
            "seed_from_u64_7_u64": [O.ChaCha(seed_u64=7).next_u64() for _ in range(1)]}


def pos_case():
    """proof-of-storage: the reference's test_files/test.txt (committed as pos_test.txt) packed
    7 bytes per WriteableFt63 element and committed with CommitDimensions::Square."""
    data = open(os.path.join(HERE, "pos_test.txt"), "rb").read()
    el = O.pos_bytes_to_field(data)
    np_, nc, snd = O.pos_default_dims(len(el))
    enc = O.Encoding.ligero(0, np_, nc)
    comm = O.Commit(enc, el)
    x = O.ChaCha(seed_u64=1337, rounds=8).field_random(0, 1)
    left, right = O.pos_side_vectors(0, x, comm.n_rows, comm.n_per_row)
    r = O.collapse(0, comm.comm, left, comm.n_rows, comm.n_cols)
    return {"n_bytes": len(data), "elems_sha256": sha(el), "dims": [comm.n_rows, np_, nc],
            "soundness": snd, "root": comm.root().hex(), "comm_sha256": sha(comm.comm),
            "eval_x_seed_chacha8": 1337, "eval_encoded_sha256": sha(r),
            "columns_1337_8": O.pos_column_indices(1337, 8, nc)}


def main():
    out = {
        "cfg1_ft127_2_16": ligero_case(1, 16),
        "ft127_ragged_1000": ligero_case(1, 0, length=1000),
        "ft63_2_14": ligero_case(0, 14),
        "ft255_2_12": ligero_case(3, 12),
        "ft253_192_2_12": ligero_case(4, 12),
        "ft127_rho_1_4_2_14": ligero_case(1, 14, rho=(1, 4)),
        "cfg2_ft127_2_20_encode": encode_case(1, 20),
        "brakedown_ft127_4096_seed0": brakedown_case(1, 4096, 0),
        "transcript": transcript_case(),
        "pos_test_txt_square": pos_case(),
    }
    path = os.path.join(HERE, "golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main()
