"""The per-row LcEncoding::encode drop-in path under concurrent callers.

INTEGRATION.md's level-1 binding routes every rayon worker's row through `lcpc_encode`
(lcpc-2d/src/lib.rs:677-682 encodes the rows of a commitment with `par_chunks_mut`; the PoS
writers call `encode` per row: encoded_file_writer.rs:300, row_generator_iter.rs:153).  This
times, at the cfg3 row size (Ft127, n_per_row 32768 -> 65536 columns, 1 MiB per encoded row):

* one caller, rows one at a time (`lcpc_encode`);
* T concurrent callers (host threads; ctypes drops the GIL inside the call), rows one at a time;
* the whole batch in one `lcpc_encode_rows` call;

host buffers in and out (PCIe-inclusive: this is the drop-in path, not the HBM-resident bench),
and checks that every path produces the same codewords.

    python tools/encode_rows_bench.py [--rows 512] [--threads 16] [--log-len 24]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=512)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--log-len", type=int, default=24)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    import lcpc_proof_of_storage_amd as L
    L.set_device(0)
    fid = L.FT127
    enc = L.LigeroEncoding.new(fid, 1 << args.log_len)
    _, n_per_row, n_cols = enc.get_dims(1 << args.log_len)
    nl = L.limbs(fid)
    rows = np.zeros((args.rows, n_cols, nl), np.uint64)
    rows[:, :n_per_row] = L.field_random(fid, args.rows * n_per_row, 11).reshape(args.rows, n_per_row, nl)
    row_bytes = n_cols * nl * 8

    def fresh():
        return [r.copy() for r in rows]  # (a row view is contiguous: encode would write into rows)

    # reference result: one batched call
    want = enc.encode_rows(rows.copy())

    def one_at_a_time(bufs, idx):
        for i in idx:
            bufs[i] = enc.encode(bufs[i])

    res = {"field": "Ft127", "n_per_row": n_per_row, "n_cols": n_cols, "rows": args.rows,
           "row_bytes": row_bytes}
    # warm-up (pinned slots, pools) on every thread count used
    one_at_a_time(fresh(), range(min(4, args.rows)))

    # 1 caller
    best = 1e30
    for _ in range(args.reps):
        bufs = fresh()
        t0 = time.perf_counter()
        one_at_a_time(bufs, range(args.rows))
        best = min(best, time.perf_counter() - t0)
    ok1 = all(np.array_equal(b, w) for b, w in zip(bufs, want))
    res["serial"] = {"s": best, "rows_per_s": args.rows / best, "us_per_row": 1e6 * best / args.rows,
                     "gb_per_s_h2d_d2h": 2 * args.rows * row_bytes / best / 1e9, "equal": ok1}

    # T callers
    best = 1e30
    for _ in range(args.reps):
        bufs = fresh()
        parts = [range(t, args.rows, args.threads) for t in range(args.threads)]
        th = [threading.Thread(target=one_at_a_time, args=(bufs, p)) for p in parts]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        best = min(best, time.perf_counter() - t0)
    okT = all(np.array_equal(b, w) for b, w in zip(bufs, want))
    res["concurrent"] = {"threads": args.threads, "s": best, "rows_per_s": args.rows / best,
                         "us_per_row": 1e6 * best / args.rows,
                         "gb_per_s_h2d_d2h": 2 * args.rows * row_bytes / best / 1e9, "equal": okT}

    # one batched call
    best = 1e30
    for _ in range(args.reps):
        b = rows.copy()
        t0 = time.perf_counter()
        out = enc.encode_rows(b)
        best = min(best, time.perf_counter() - t0)
    res["batched"] = {"s": best, "rows_per_s": args.rows / best, "us_per_row": 1e6 * best / args.rows,
                      "gb_per_s_h2d_d2h": 2 * args.rows * row_bytes / best / 1e9,
                      "equal": bool(np.array_equal(out, want))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
