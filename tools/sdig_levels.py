#!/usr/bin/env python3
"""Per-level times of the last Brakedown encode in a rocprofv3 kernel trace (bench.py --code sdig).

    python tools/sdig_levels.py gpurun_out/<tag>/prof/run_kernel_trace.csv

The encode of one commitment is a transpose, 5 precode SpMMs, the last precode, Reed-Solomon and
6 postcode SpMMs (sdig.hip encode_rows_slice); the last such run of launches in the trace is
printed level by level, with the leaf hashing that follows it.
"""
import csv
import sys

NAMES = ["pre0", "pre1", "pre2", "pre3", "pre4", "pre5 (to scratch)", "reed_solomon",
         "post5", "post4", "post3", "post2", "post1", "post0"]


def main():
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Grid_Size", ""))
                for r in csv.DictReader(open(sys.argv[1])))
    # index of the last k_transpose followed by 13 SpMM / R-S launches
    starts = [i for i, e in enumerate(ev) if "k_transpose" in e[2]]
    for i in reversed(starts):
        seq = [e for e in ev[i + 1:] if "k_spmm" in e[2] or "k_reed_solomon" in e[2]][:13]
        if len(seq) == 13:
            break
    else:
        sys.exit("no complete encode in the trace")
    t = ev[i]
    print(f"{'transpose':22s}{(t[1] - t[0]) / 1e3:9.1f} us")
    tot = 0.0
    for name, e in zip(NAMES, seq):
        us = (e[1] - e[0]) / 1e3
        tot += us
        print(f"{name:22s}{us:9.1f} us  grid {e[3]:>9s}  {e[2][:48]}")
    print(f"# SpMM + R-S total {tot:.1f} us")
    leaf = [e for e in ev if e[0] > seq[-1][1] and ("k_leaf" in e[2])][:2]
    for e in leaf:
        print(f"{e[2][:40]:40s}{(e[1] - e[0]) / 1e3:9.1f} us")


if __name__ == "__main__":
    main()
