#!/usr/bin/env python3
"""HBM traffic of the Brakedown encode per level (review item: where the 7.5x counted traffic goes).

    python tools/pmc_sdig_levels.py RUN_DIR [--json OUT]

RUN_DIR holds the two rocprofv3 PMC passes of `bench.py --code sdig-encode --pipeline 1`
(pmc_fetch/, pmc_write/: FETCH_SIZE, WRITE_SIZE in KiB per dispatch).  The last complete encode
(k_transpose, 12 SpMM launches + k_reed_solomon in sdig.hip's order pre0..pre5, R-S, post5..post0,
k_transpose back) is split level by level; FETCH_SIZE is doubled (MI355X_MICROARCH.md's gfx950
correction for 16-B-per-lane coalesced reads: a SpMM lane loads one 16-B element of a 1152-B run).

Each level's gather model (the bytes its access pattern must move): every nonzero gathers its
input's R-row run (R x 16 B), reads its 16-B value and 4-B index, and every output row writes
R x 16 B.  Per-level nonzeros come from the oracle's matrix generation (seed 0, SdigCode3).
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = ["pre0", "pre1", "pre2", "pre3", "pre4", "pre5", "reed_solomon",
         "post5", "post4", "post3", "post2", "post1", "post0"]


def dispatches(path):
    """[(dispatch id, kernel name, bytes)] in dispatch order"""
    rows = {}
    for r in csv.DictReader(open(path)):
        d = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        v = float(r["Counter_Value"]) * 1024.0
        if d in rows:
            rows[d] = (rows[d][0], rows[d][1] + v)
        else:
            rows[d] = (r["Kernel_Name"], v)
    return [(d, k, v) for d, (k, v) in sorted(rows.items())]


def last_encode(ds):
    idx = [i for i, (_, k, _) in enumerate(ds) if "k_transpose" in k]
    for i in reversed(idx):
        seq = [x for x in ds[i + 1:] if "k_spmm" in x[1] or "k_reed_solomon" in x[1]][:13]
        if len(seq) == 13:
            back = next((x for x in ds[i + 1:] if "k_transpose" in x[1] and x[0] > seq[-1][0]), None)
            return ds[i], seq, back
    sys.exit("no complete encode among the dispatches")


def oracle_levels(n_per_row=235173, fid=1):
    """(nnz, outputs) per entry of NAMES from the oracle's SdigCode3 matrices (seed 0): rows =
    outputs, cols = inputs; the Reed-Solomon level writes post5's input count from pre5's outputs"""
    import ctypes as C
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_ffi as O
    L = O.lib()
    e = O.Encoding.sdig(fid, n_per_row, seed=0, code_id=3)
    dims = {}
    for which, tag in ((0, "pre"), (1, "post")):
        for lvl in range(L.of_sdig_levels(e.ptr)):
            r, c = C.c_size_t(), C.c_size_t()
            nz = L.of_sdig_matrix(e.ptr, lvl, which, C.byref(r), C.byref(c), None, None, None)
            dims[f"{tag}{lvl}"] = (nz, r.value, c.value)
    nnz, outs = [], []
    for name in NAMES:
        if name == "reed_solomon":
            outs.append(dims["post5"][2])
            continue
        nz, rows, _ = dims[name]
        nnz.append(nz)
        outs.append(rows)
    return nnz, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("--json", default=None)
    ap.add_argument("--rows", type=int, default=72, help="R: rows of the commitment (72 at cfg4)")
    ap.add_argument("--nnz", default=None, help="JSON list of the 12 SpMM levels' nonzeros in NAMES order "
                                                "(without R-S); default: from the oracle")
    ap.add_argument("--outs", default=None, help="JSON list of the 13 levels' output counts")
    a = ap.parse_args()
    f = dispatches(glob.glob(os.path.join(a.run_dir, "pmc_fetch", "*counter_collection.csv"))[0])
    w = dispatches(glob.glob(os.path.join(a.run_dir, "pmc_write", "*counter_collection.csv"))[0])
    tf, sf, bf = last_encode(f)
    tw, sw, bw = last_encode(w)
    if a.nnz and a.outs:
        nnz, outs = json.loads(a.nnz), json.loads(a.outs)
    else:
        nnz, outs = oracle_levels()
    R, B = a.rows, 16
    rows = []
    tot_c = tot_m = 0.0
    for i, name in enumerate(NAMES):
        rd, wr = 2.0 * sf[i][2], sw[i][2]
        r = {"level": name, "read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr, "kernel": sf[i][1][:40]}
        if nnz is not None and outs is not None:
            k = i if i < 6 else i - 1
            model = (0 if name == "reed_solomon" else nnz[k] * (R * B + B + 4)) + outs[i] * R * B
            r["model_bytes"] = model
            r["counted_over_model"] = (rd + wr) / model if model else None
            tot_m += model
        tot_c += rd + wr
        rows.append(r)
    for t, tw_, name in ((tf, tw, "transpose_in"), (bf, bw, "transpose_back")):
        if t is not None and tw_ is not None:
            rows.append({"level": name, "read_bytes": 2.0 * t[2], "write_bytes": tw_[2],
                         "hbm_bytes": 2.0 * t[2] + tw_[2]})
    for r in rows:
        extra = (f"  model {r['model_bytes'] / 1e9:7.3f} GB  x{r['counted_over_model']:.2f}"
                 if r.get("model_bytes") else "")
        print(f"{r['level']:16s} read {r['read_bytes'] / 1e9:7.3f} GB  write {r['write_bytes'] / 1e9:7.3f} GB{extra}")
    print(f"levels total {tot_c / 1e9:.3f} GB" + (f", model {tot_m / 1e9:.3f} GB" if tot_m else ""))
    if a.json:
        json.dump({"levels": rows, "levels_total_bytes": tot_c, "levels_model_bytes": tot_m or None,
                   "source": a.run_dir}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
