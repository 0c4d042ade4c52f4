"""Host-inclusive timing of the PoS file path (not the bench.py metric): a file image in host
memory -> lcpc_pos_encode_file -> .porenc image in host memory (+ tree), then the reader's
lcpc_pos_porenc_tree and lcpc_pos_decode_porenc over the whole image.  Prints one JSON line."""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lcpc_proof_of_storage_amd as L  # noqa: E402
from lcpc_proof_of_storage_amd import _native as N, pos as P  # noqa: E402


def u8(a):
    return a.ctypes.data_as(N.u8p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=1 << 30)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    L.set_device(0)
    lib = N.load()
    n = args.bytes
    data = np.random.default_rng(1).integers(0, 256, n, dtype=np.uint8)
    pre, enc, _ = P.get_aspect_ratio_default_from_file_len(n)
    rows = -(-(-(-n // 7)) // pre)
    cap = 2 * rows
    img = np.zeros(cap * enc * 8, np.uint8)
    img[::4096] = 0  # fault the pages in once (a warm page cache / mmap)
    tree = np.zeros((2 * enc - 1) * 32, np.uint8)
    out = np.zeros(rows * pre * 7, np.uint8)
    got = C.c_size_t()
    res = {"bytes": n, "pre": pre, "enc": enc, "rows": rows}
    for name, fn in [
        ("encode_file", lambda: lib.lcpc_pos_encode_file(u8(data), n, pre, enc, cap, u8(img), u8(tree), C.byref(got))),
        ("porenc_tree", lambda: lib.lcpc_pos_porenc_tree(u8(img), enc, rows, cap, u8(tree))),
        ("decode_file", lambda: lib.lcpc_pos_decode_porenc(u8(img), pre, enc, cap, 0, rows, u8(out))),
    ]:
        ts = []
        for _ in range(args.reps + 1):
            t = time.perf_counter()
            rc = fn()
            ts.append(time.perf_counter() - t)
            if rc:
                raise RuntimeError(f"{name}: {rc} {N.last_error()}")
        best = min(ts[1:])
        res[name + "_s"] = round(best, 4)
        res[name + "_GBps_of_data"] = round(n / best / 1e9, 3)
    res["decode_roundtrip_ok"] = bool(np.array_equal(out[:n], data))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
