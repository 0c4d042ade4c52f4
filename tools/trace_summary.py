#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of bench.py (tools/gpu_check.sh) per kernel.

    python tools/trace_summary.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--last R]

Prints, per kernel, the launch count and average duration over all launches and over the last
R launches -- bench.py's roofline steps run serially at the end of the process, so the last R
encode launches are the ones its HIP-event roofline figure is taken on -- plus the GPU busy
fraction of the trace span (union of kernel intervals).
"""
import argparse
import collections
import csv
import json

SHORT = ["k_row_ntt15", "k_spmm", "k_transpose", "k_pass_a", "k_pass_b", "k_leaf_chunks", "k_leaf_merge", "k_merkle", "k_collapse_partial", "k_collapse_mfma", "k_tensor_digits",
         "k_collapse_fold", "k_convert", "k_gather_cols", "k_gather_paths", "k_ntt_small", "k_copy_words",
         "copyBuffer", "fillBuffer", "k_tw_table", "k_column_checks", "k_path_checks", "k_dot"]


def short(name):
    for k in SHORT:
        if k in name:
            return k
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    ev = []
    for r in csv.DictReader(open(a.trace)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    ev.sort()
    per = collections.defaultdict(list)
    for s, e, k in ev:
        per[k].append((e - s) / 1e6)
    out = {}
    for k, d in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        last = d[-a.last:]
        out[k] = {"launches": len(d), "avg_ms": sum(d) / len(d), "last_avg_ms": sum(last) / len(last)}
        print(f"{k:22s} n={len(d):5d} avg={out[k]['avg_ms']:8.4f} ms  last{a.last}={out[k]['last_avg_ms']:8.4f} ms")
    busy, cs, ce = 0, None, None
    for s, e, _ in ev:
        if ce is None or s > ce:
            if ce is not None:
                busy += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    busy += ce - cs
    span = ev[-1][1] - ev[0][0]
    print(f"busy {busy / 1e6:.2f} ms of span {span / 1e6:.2f} ms")
    if a.json:
        json.dump({"kernels": out, "busy_ms": busy / 1e6, "span_ms": span / 1e6}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
