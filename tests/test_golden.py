"""Golden fixtures (tests/golden/golden.json, made by tests/golden/gen_golden.py).

CPU: the oracle regenerates every fixture exactly (guards the checker itself).
GPU: the HIP path reproduces every Ligero / encode fixture bit for bit through the C ABI.
"""
import hashlib
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))

GOLDEN = json.load(open(os.path.join(HERE, "golden", "golden.json")))
LIGERO = [k for k, v in GOLDEN.items() if "root" in v and not k.startswith("pos_")]


def sha(a) -> str:
    if isinstance(a, (bytes, bytearray)):
        return hashlib.sha256(a).hexdigest()
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.uint64).tobytes()).hexdigest()


def test_oracle_reproduces_fixtures(oracle):
    import gen_golden as G
    for name, g in GOLDEN.items():
        if name.startswith("pos_"):
            got = G.pos_case()
        elif "root" in g:
            got = G.ligero_case(g["field"], 0, rho=tuple(g["rho"]), length=g["len"], x_seed=g["x_seed"])
        elif name.startswith("cfg2"):
            got = G.encode_case(g["field"], g["len"].bit_length() - 1)
        elif name.startswith("brakedown"):
            got = G.brakedown_case(g["field"], g["n_per_row"], g["seed"])
        else:
            got = G.transcript_case()
        assert got == g, name


def test_fixture_dims_match_survey():
    assert GOLDEN["cfg1_ft127_2_16"]["dims"] == [32, 2048, 4096]
    assert GOLDEN["cfg1_ft127_2_16"]["n_col_opens"] == 309
    assert GOLDEN["cfg2_ft127_2_20_encode"]["dims"] == [128, 8192, 16384]


@pytest.mark.gpu
@pytest.mark.parametrize("name", LIGERO)
def test_gpu_matches_golden(gpu, oracle, name):
    g = GOLDEN[name]
    fid, n = g["field"], g["len"]
    enc = gpu.LigeroEncoding.new(fid, n, tuple(g["rho"]))
    coeffs = gpu.field_random(fid, n, g["coeff_seed"])
    comm = gpu.LcCommit.commit(coeffs, enc)
    assert [comm.get_n_rows(), comm.get_n_per_row(), comm.get_n_cols()] == g["dims"]
    root = comm.get_root()
    assert root.hex() == g["root"]
    assert sha(comm.comm) == g["comm_sha256"]
    assert sha(comm.hashes) == g["hashes_sha256"]
    x = oracle.ChaCha(seed_u64=g["x_seed"]).field_random(fid, 1)
    inner, outer = oracle.eval_tensors(fid, x, g["dims"][1], g["dims"][0])
    tr = gpu.Transcript(b"test transcript")
    tr.append_message(b"polycommit", root)
    tr.append_message(b"ncols", g["n_col_opens"].to_bytes(8, "big"))
    pf = comm.prove(outer, enc, tr)
    assert sha(pf.p_eval) == g["p_eval_sha256"]
    assert sha(np.concatenate(pf.p_random_vec)) == g["p_random_sha256"]
    cols = pf.columns
    assert sha(np.concatenate([c.col for c in cols])) == g["cols_sha256"]
    assert sha(b"".join(b"".join(c.path) for c in cols)) == g["paths_sha256"]
    tr2 = gpu.Transcript(b"test transcript")
    tr2.append_message(b"polycommit", root)
    tr2.append_message(b"ncols", g["n_col_opens"].to_bytes(8, "big"))
    ev = pf.verify(root, outer, inner, enc, tr2)
    assert hex(oracle.from_mont(fid, ev)[0]) == g["eval"]


@pytest.mark.gpu
def test_gpu_matches_golden_encode_cfg2(gpu):
    g = GOLDEN["cfg2_ft127_2_20_encode"]
    nr, np_, nc = g["dims"]
    enc = gpu.LigeroEncoding.new_from_dims(g["field"], np_, nc)
    coeffs = gpu.field_random(g["field"], g["len"], g["coeff_seed"]).reshape(nr, np_, -1)
    rows = np.zeros((nr, nc, coeffs.shape[2]), np.uint64)
    rows[:, :np_] = coeffs
    out = enc.encode_rows(rows)
    assert sha(out) == g["rows_sha256"]
    for r, h in g["row_sha256"].items():
        assert sha(out[int(r)]) == h


@pytest.mark.gpu
def test_gpu_transcript_fixture(gpu):
    g = GOLDEN["transcript"]
    tr = gpu.Transcript(b"test protocol")
    tr.append_message(b"some label", b"some data")
    assert tr.challenge_bytes(b"challenge", 32).hex() == g["merlin_test_protocol"]
