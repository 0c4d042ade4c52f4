"""Child process of test_gpu_runtime_knobs.py: commit / prove / verify of a few small workloads
under whatever library knobs (LCPC_NO_MFMA, LCPC_STREAM_MODE, ...) this process was started with
(the library reads each once), printed as one JSON line {case: [root, sha256 of everything it returned]}."""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import lcpc_proof_of_storage_amd as L  # noqa: E402


def tr(root):
    t = L.Transcript(b"runtime knobs")
    t.append_message(b"polycommit", root)
    return t


def prove_verify(enc, coeffs, field, seed):
    c = L.LcCommit.commit(coeffs, enc)
    root = c.get_root()
    n_rows = c.get_n_rows()
    outer = L.field_random(field, n_rows, seed + 1)
    inner = L.field_random(field, enc.n_per_row, seed + 2)
    pf = c.prove(outer, enc, tr(root))
    ev = pf.verify(root, outer, inner, enc, tr(root))
    h = hashlib.sha256(root)
    h.update(c.comm.tobytes())
    h.update(pf.to_bincode())
    h.update(np.ascontiguousarray(ev).tobytes())
    return [root.hex(), h.hexdigest()]


def main():
    assert L.device_count() > 0, "no HIP device"
    L.set_device(0)
    out = {}
    for field in range(5):
        coeffs = L.field_random(field, (1 << 14) + 77, 11 + field)
        out[f"ligero_f{field}"] = prove_verify(L.LigeroEncoding.new(field, coeffs.shape[0]), coeffs, field, 20 + field)
    for field in (0, 1):
        coeffs = L.field_random(field, 1 << 14, 31 + field)
        out[f"sdig_f{field}"] = prove_verify(L.SdigEncoding.new(field, coeffs.shape[0], 5), coeffs, field, 40 + field)
    n_bytes = 7 * 16384 * 3 + 1001
    data = np.random.default_rng(n_bytes).integers(0, 256, n_bytes, dtype=np.uint8)
    c = L.LcCommit.commit_pos_bytes(data, L.RsEncoding.new(0, 16384, 32768, 16, 2))
    out["pos_bytes"] = [c.get_root().hex(), hashlib.sha256(c.get_root() + c.comm.tobytes() + c.coeffs.tobytes()).hexdigest()]
    # the sharded driver at one rank (lcpc_sharded_commit_prove_many), pipelined over 4 polynomials
    from conftest import _HipMem
    from lcpc_proof_of_storage_amd import shard
    hm = _HipMem()
    enc = L.RsEncoding.new(1, 256, 512, 24, 2)
    polys = [L.field_random(1, 64 * 256, 50 + k) for k in range(4)]
    ds = [hm.to_device(p) for p in polys]
    roots, proofs = shard.sharded_commit_prove_many(enc, shard.NativeComm.single(), ds, 64, L.field_random(1, 64, 60),
                                                    lambda i, root: tr(root))
    h = hashlib.sha256(b"".join(roots))
    for p in proofs:
        h.update(p.to_bincode())
    out["sharded_n1"] = [roots[0].hex(), h.hexdigest()]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
