#!/usr/bin/env python3
"""Where a K-step replicas run of bench.py goes ("the K = 20 bound").

    python tools/timeline_k20.py TIMELINE.json [--trace run_kernel_trace.csv] [--json OUT]

TIMELINE.json is `bench.py --timeline` (per step: admission gate, commit start / end = the root
on the host, prove end; seconds from the start of the timed region).  With the rocprofv3 kernel
trace of the same run (its timeline JSON carries t0_monotonic_ns, the clock rocprofv3 stamps
kernels with), the GPU side is split into commit kernels (encode, leaves, Merkle) and prove
kernels (row combinations, conversions, gathers, copies) inside the timed region, and the bound

    T_bound = (all commit kernels back to back) + (the last proof's serial tail after its root)

is set against the measured run: the gap is what admission order could still recover.
"""
import argparse
import csv
import json

COMMIT = ("k_pass_a", "k_pass_b", "k_row_ntt15", "k_ntt_small", "k_leaf", "k_merkle")


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("timeline")
    ap.add_argument("--trace", default=None)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    tl = json.load(open(a.timeline))
    steps = tl["steps"]
    el = tl["elapsed"] * 1e3
    roots = sorted(1e3 * s[3] for s in steps)
    proves = sorted(1e3 * s[4] for s in steps)
    last = max(steps, key=lambda s: s[3])
    out = {
        "elapsed_ms": el, "steps": len(steps),
        "first_root_ms": roots[0], "last_root_ms": roots[-1],
        "last_prove_end_ms": proves[-1],
        "tail_after_last_root_ms": el - roots[-1],
        "last_step_prove_ms": 1e3 * (last[4] - last[3]),
        "root_intervals_ms": [round(b - a_, 3) for a_, b in zip(roots, roots[1:])],
        "commit_ms": sorted(round(1e3 * (s[3] - s[2]), 3) for s in steps),
        "prove_ms": sorted(round(1e3 * (s[4] - s[3]), 3) for s in steps),
    }
    if a.trace and "t0_monotonic_ns" in tl:
        t0 = tl["t0_monotonic_ns"]
        t1 = t0 + int(tl["elapsed"] * 1e9)
        com, prv = [], []
        per = {}
        for r in csv.DictReader(open(a.trace)):
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if e < t0 or s > t1:
                continue
            s, e = max(s, t0), min(e, t1)
            name = r["Kernel_Name"]
            (com if any(k in name for k in COMMIT) else prv).append((s, e))
            key = next((k for k in COMMIT if k in name), name.split("(")[0].split("<")[0][-40:])
            per[key] = per.get(key, 0) + (e - s)
        out["gpu_busy_ms"] = union(com + prv) / 1e6
        out["commit_kernels_busy_ms"] = union(com) / 1e6
        out["prove_kernels_busy_ms"] = union(prv) / 1e6
        out["kernel_time_ms"] = {k: round(v / 1e6, 3) for k, v in sorted(per.items(), key=lambda kv: -kv[1])}
        # last commit kernel's end (the GPU side of the last root) and the GPU-idle time after it
        last_commit_end = max(e for _, e in com) if com else t0
        out["last_commit_kernel_end_ms"] = (last_commit_end - t0) / 1e6
        out["bound_ms"] = out["commit_kernels_busy_ms"] + out["last_step_prove_ms"]
        out["gap_to_bound_ms"] = el - out["bound_ms"]
    for k, v in out.items():
        if not isinstance(v, (list, dict)):
            print(f"{k:28s} {v:.3f}" if isinstance(v, float) else f"{k:28s} {v}")
    if "kernel_time_ms" in out:
        print("kernel time in the timed region (ms):", out["kernel_time_ms"])
    print("root intervals (ms):", out["root_intervals_ms"])
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
