#!/usr/bin/env python3
"""HBM traffic of the encode kernels from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE).

    python tools/pmc_traffic.py gpurun_out/<tag> profiles/pmc_traffic[_<code>].json [--len N --field F --code C]

bench.py reads every profiles/pmc_traffic*.json and uses the one whose (len, field, code)
matches its workload.

Counter units are KiB.  Per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950
FETCH_SIZE reports half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores.  Both NTT passes load and
store 16 B per lane for Ft127 (fe_load / fe_store of 4 x u32).
"""
import argparse
import collections
import csv
import glob
import json
import os

KERNELS = {"ntt_pass_a": "k_pass_a", "ntt_pass_b": "k_pass_b", "leaf_chunks": "k_leaf_chunks",
           "collapse_partial": "k_collapse_partial", "collapse_mfma": "k_collapse_mfma",
           # Brakedown (--code sdig): the transpose into element-major form, the SpMM levels
           # (matrix-core or VALU kernel) and the Reed-Solomon base
           "transpose": "k_transpose", "spmm": "k_spmm", "reed_solomon": "k_reed_solomon",
           "pos_pack7": "k_pack7", "ntt_row1": "k_row_ntt15"}
SDIG_ENCODE = ("transpose", "spmm", "reed_solomon")


def per_kernel(path):
    """mean bytes per launch and launch count per kernel; also the total bytes per kernel"""
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        for short, pat in KERNELS.items():
            if pat in row["Kernel_Name"]:
                acc[short].append(float(row["Counter_Value"]) * 1024.0)
                break
    return ({k: sum(v) / len(v) for k, v in acc.items()}, {k: len(v) for k, v in acc.items()},
            {k: sum(v) for k, v in acc.items()})


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("run_dir")
    ap.add_argument("out")
    ap.add_argument("--len", type=int, default=1 << 24)
    ap.add_argument("--field", default="Ft127")
    ap.add_argument("--code", default="ligero", help="bench.py --code of the profiled run")
    a = ap.parse_args()
    fpath = glob.glob(os.path.join(a.run_dir, "pmc_fetch", "*counter_collection.csv"))[0]
    wpath = glob.glob(os.path.join(a.run_dir, "pmc_write", "*counter_collection.csv"))[0]
    fetch, nf, ftot = per_kernel(fpath)
    write, nw, wtot = per_kernel(wpath)
    kern = {}
    for k in fetch:
        rd = 2.0 * fetch[k]
        wr = write.get(k, 0.0)
        kern[k] = {"fetch_bytes_raw": fetch[k], "read_bytes_corrected": rd, "write_bytes": wr,
                   "hbm_bytes": rd + wr, "launches": nf[k]}
    # per step (one commitment), not per launch: total over the run / the launches of a kernel that
    # runs once per step.  A PoS step encodes the file's ragged last row with a one-row NTT of its
    # own, so its NTT kernels launch twice per step and a per-launch mean would halve the figure.
    if a.code == "sdig":
        # one encode = one transpose + every SpMM level + the R-S base
        n_enc = nf["transpose"]
        enc = sum(2.0 * ftot.get(k, 0.0) + wtot.get(k, 0.0) for k in SDIG_ENCODE) / n_enc
    elif a.code.startswith("sdig-encode"):
        # LcEncoding::encode of row-major device rows: transpose in, the levels, transpose back
        n_enc = nf["transpose"] // 2
        enc = sum(2.0 * ftot.get(k, 0.0) + wtot.get(k, 0.0) for k in SDIG_ENCODE) / n_enc
    elif a.code == "encode":
        # the R-S encode alone: one pass-A + pass-B pair per step
        n_enc = nf["ntt_pass_a"]
        enc = sum(2.0 * ftot.get(k, 0.0) + wtot.get(k, 0.0) for k in ("ntt_pass_a", "ntt_pass_b")) / n_enc
    else:
        # (pos-row1: the one-pass Ft63 row kernel, whose 8-byte loads arrive as 128-byte runs; the
        # x2 read correction is checked by its read figure against the input's size)
        n_enc = nf["pos_pack7"] if a.code == "pos" else nf["leaf_chunks"]
        enc = sum(2.0 * ftot.get(k, 0.0) + wtot.get(k, 0.0) for k in ("ntt_pass_a", "ntt_pass_b", "ntt_row1")) / n_enc
    for k in kern:
        kern[k]["hbm_bytes_per_step"] = (2.0 * ftot[k] + wtot.get(k, 0.0)) / n_enc
    out = {
        "config_len": a.len, "field": a.field, "code": a.code,
        "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes "
                  "(bench.py --pipeline 1); FETCH_SIZE x2 (gfx950 wide-read correction), KiB -> B",
        "ntt_encode_bytes_per_launch": enc,  # (per step: every encode launch of one commitment)
        "steps": n_enc,
        "kernels": kern,
        "source": os.path.relpath(a.run_dir),
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps({k: round(v["hbm_bytes"] / 2**20, 1) for k, v in kern.items()}), "MiB;",
          "encode", round(enc / 2**20, 1), "MiB")


if __name__ == "__main__":
    main()
