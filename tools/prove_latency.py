#!/usr/bin/env python3
"""Latency of one cfg3 commit + prove, serial (no pipeline), with the library's host scopes.

    python tools/prove_latency.py [--reps 5] [--log-len 24]

Prints the wall time of commit_device and prove per rep and the library's per-scope averages
(prof_stats) so the host-side parts of one step (transcript, GPU waits) can be read apart.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--log-len", type=int, default=24)
    a = ap.parse_args()
    import torch
    import lcpc_proof_of_storage_amd as L
    L.set_device(0)
    fid, n = L.FT127, 1 << a.log_len
    enc = L.LigeroEncoding.new(fid, n)
    n_rows, n_per_row, n_cols = enc.get_dims(n)
    nco = enc.get_n_col_opens()
    coeffs = L.field_random(fid, n, 0x1CDC2024)
    outer = L.field_random(fid, n_rows, 7)
    d = torch.from_numpy(coeffs.view(np.int64)).to("cuda:0")
    torch.cuda.synchronize()
    for rep in range(a.reps + 2):
        if rep == 2:
            L.prof_reset()
            L.prof_enable(True)
        t0 = time.perf_counter()
        c = L.LcCommit.commit_device(d.data_ptr(), n, enc)
        root = c.get_root()
        t1 = time.perf_counter()
        tr = L.Transcript(b"test transcript")
        tr.append_message(b"polycommit", root)
        tr.append_message(b"ncols", nco.to_bytes(8, "big"))
        c.prove(outer, enc, tr)
        t2 = time.perf_counter()
        if rep >= 2:
            print(f"rep {rep - 2}: commit {1e3 * (t1 - t0):.3f} ms  prove {1e3 * (t2 - t1):.3f} ms", flush=True)
    L.prof_enable(False)
    for k, v in sorted(L.prof_stats().items()):
        print(f"  {k:28s} avg {v[0] / max(v[1], 1):8.4f} ms  x{v[1] / a.reps:.1f} per step")


if __name__ == "__main__":
    main()
