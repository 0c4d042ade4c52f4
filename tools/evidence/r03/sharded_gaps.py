"""GPU idle time inside the sharded driver's timed region, from a rocprofv3 kernel trace.

Usage: python tools/evidence/r03/sharded_gaps.py <kernel_trace.csv> <warmup> <steps>

bench.py --mode sharded runs `warmup` polynomials, then the timed `steps`, then serial roofline
commits; the timed region is taken from the first k_pass_a of polynomial `warmup` to the last kernel
that ends before the first serial pass A.  Prints the busy fraction, each polynomial's encode
window, and the longest idle gaps with the kernel that ended before and started after each one.
"""
import csv
import sys


def short(name):
    for k in ("k_pass_a", "k_pass_b", "k_leaf_chunks", "k_leaf_merge", "k_merkle", "k_collapse_mfma",
              "k_collapse_fold", "k_tensor_digits", "k_gather_cols", "k_gather_paths", "k_copy", "k_d2h", "k_h2d"):
        if k in name:
            return k
    return name.split("(")[0][-40:]


def main():
    path, warm, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    pa = [r for r in rows if r[2] == "k_pass_a"]
    t_begin = pa[warm][0]
    t_stop = pa[warm + steps][0] if len(pa) > warm + steps else rows[-1][1] + 1
    ks = [r for r in rows if t_begin <= r[0] < t_stop]
    t_end = max(r[1] for r in ks)
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    last_name = None
    for s, e, n in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append((s - cur_e, (cur_e - t_begin) / 1e6, last_name, n))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
        last_name = n
    busy += cur_e - cur_s
    span = t_end - t_begin
    print(f"timed region {span / 1e6:.2f} ms, GPU busy {busy / 1e6:.2f} ms ({busy / span:.2f}), "
          f"{len(ks)} kernels")
    tot = {}
    for s, e, n in ks:
        tot[n] = tot.get(n, 0) + (e - s)
    for n, v in sorted(tot.items(), key=lambda x: -x[1]):
        print(f"  {n:20s} {v / 1e6:7.2f} ms (sum of durations)")
    enc = [r for r in ks if r[2] == "k_pass_a"]
    print("encode starts (ms):", " ".join(f"{(r[0] - t_begin) / 1e6:.2f}" for r in enc))
    pb = [r for r in ks if r[2] == "k_pass_b"]
    print("pass B ends (ms):  ", " ".join(f"{(r[1] - t_begin) / 1e6:.2f}" for r in pb))
    gaps.sort(reverse=True)
    print(f"idle gaps: {len(gaps)}, total {sum(g[0] for g in gaps) / 1e6:.2f} ms; longest:")
    for g, at, a, b in gaps[:25]:
        print(f"  {g / 1e3:8.1f} us at {at:7.2f} ms  after {a} before {b}")


if __name__ == "__main__":
    main()


def drain(path, warm, steps, host_csv):
    """Chronological host phases (LCPC_PROF_TIMELINE) and GPU idle gaps from 2 ms before the last
    pass B to the end of the timed region."""
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])))
    rows.sort()
    pa = [r for r in rows if r[2] == "k_pass_a"]
    t_begin = pa[warm][0]
    t_stop = pa[warm + steps][0] if len(pa) > warm + steps else rows[-1][1] + 1
    ks = [r for r in rows if t_begin <= r[0] < t_stop]
    last_b = max(r[1] for r in ks if r[2] == "k_pass_b")
    lo = (last_b - t_begin) / 1e6 - 2.0
    ev = []
    cur_e = None
    for s, e, n in ks:
        if cur_e is not None and s - cur_e > 50_000 and (cur_e - t_begin) / 1e6 >= lo:
            ev.append(((cur_e - t_begin) / 1e6, (s - t_begin) / 1e6, "GPU idle", f"before {n}"))
        cur_e = e if cur_e is None else max(cur_e, e)
    with open(host_csv) as f:
        for line in f:
            name, a, b, tid = line.strip().split(",")
            a, b = float(a) - t_begin / 1e6, float(b) - t_begin / 1e6
            if b >= lo and a <= (cur_e - t_begin) / 1e6 and name != "tick_total" and b - a >= 0.01:
                ev.append((a, b, name, f"thread {tid}"))
    for a, b, n, w in sorted(ev):
        print(f"  {a:8.3f} {b:8.3f} {b - a:7.3f}  {n:24s} {w}")


if __name__ == "__main__" and len(sys.argv) > 4:
    drain(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4])
