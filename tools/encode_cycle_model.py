#!/usr/bin/env python3
"""The Ligero encode's issue-floor model (round 6): is the cfg3 encode at the floor of its own
instruction stream?

Inputs (all measured on MI355X, committed under profiles/):
  * per-class issue cost: tools/microbench/issue_cost.hip at 4 waves/SIMD (pass A and pass B's
    occupancy: 97 VGPRs + AGPRs, 38 KiB LDS per 256-thread block) -- wall time per wave-instruction
    per SIMD, so the DVFS clock the VALU-dense loop runs at is inside the figure;
  * per-class static instruction counts of k_pass_a / k_pass_b<Ft127, 8, 3, 8>
    (tools/isa_attribution.py -> profiles/r06_encode_isa_attribution.txt, after the carry-free mads; r05 before);
  * the passes' dynamic VALU count per wave (SQ_INSTS_VALU / SQ_WAVES, tools/pmc_ntt.sh);
  * the passes' isolated durations (rocprofv3 kernel trace, fastest launch = a serial one).

Model: time = (waves / 1024 SIMDs) x sum_class(static count x cost) x (dynamic / static VALU).

    python tools/encode_cycle_model.py ISSUE_COST.json PMC_DIR TRACE_STATS.csv [OUT.txt [OUT.json]]

OUT.json (profiles/issue_floor_encode.json) is what bench.py quotes in roofline_valu.issue_floor.
"""
import collections
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# attribution classes -> the issue_cost class that prices them
PRICE = {
    "mad_u64_u32": "v_mad_u64_u32",
    "addc/subb (carry)": "v_addc_co_u32 (independent SGPR carries)",
    "add/sub_co (carry out)": "v_add_co_u32 (SGPR carry out)",
    "cndmask (select)": "v_cmp_gt_u32 + v_cndmask_b32 (vcc just written)",  # vcc written by VALU, as in the passes
    "mov": "v_mov_b32",
    "lshl_add_u64 / 64-bit": "v_add_co_u32 (SGPR carry out)",
    "shift/logic/bfe": "v_add_u32 (reference: full-rate)",
    "add/sub u32 (no carry)": "v_add_u32 (reference: full-rate)",
    "cmp": "v_cmp_gt_u32 + v_cndmask_b32 (vcc just written)",
    "mul/mad other": "v_mad_u64_u32",
}


def issue_costs(path, k=4):
    d = json.load(open(path))
    out = {}
    for r in d["rows"]:
        if r["waves_per_simd"] != k:
            continue
        n_instr = 16384 * 8 * (2 if r["class"].startswith(("v_add_u32 + s_nop", "carry chain", "v_cmp_gt", "mad_u64 (carry")) else 1)
        out[r["class"]] = r["kernel_ms"] * 1e6 / (n_instr * k)  # ns per wave-instruction per SIMD
    return out


def attribution(path=os.path.join(ROOT, "profiles", "r06_encode_isa_attribution.txt")):
    passes, cur = {}, None
    for line in open(path):
        m = re.match(r"^(k_pass_[ab])<.*VALU (\d+), s_nop (\d+)", line)
        if m:
            cur = m.group(1)
            passes[cur] = {"valu": int(m.group(2)), "s_nop": int(m.group(3)), "classes": {}}
            continue
        m = re.match(r"^\s{3}(\S.*?)\s{2,}(\d+)\s+\(", line)
        if cur and m:
            passes[cur]["classes"][m.group(1).strip()] = int(m.group(2))
    return passes


def pmc(pmc_dir):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(pmc_dir, "p*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = "k_pass_a" if "k_pass_a" in r["Kernel_Name"] else "k_pass_b" if "k_pass_b" in r["Kernel_Name"] else None
            if k:
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def durations(stats_csv):
    out = {}
    for r in csv.DictReader(open(stats_csv)):
        for k in ("k_pass_a", "k_pass_b"):
            if k in r["Name"] and "Ft127" in r["Name"]:
                out[k] = float(r["MinNs"]) / 1e6
    return out


def main():
    cost = issue_costs(sys.argv[1])
    att = attribution()
    ctr = pmc(sys.argv[2])
    dur = durations(sys.argv[3])
    out = open(sys.argv[4], "w") if len(sys.argv) > 4 else sys.stdout
    print("# cfg3 encode (Ft127, 512 x 65536, 65536 waves per pass) against its VALU issue floor", file=out)
    print("# issue cost per wave-instruction per SIMD at 4 waves/SIMD (ns, wall time: tools/microbench/issue_cost.hip)",
          file=out)
    for c in sorted(set(PRICE.values())):
        print(f"#   {c:52s} {cost[c]:.3f} ns", file=out)
    print(f"#   s_nop 0 beside VALU work (pair - add alone): "
          f"{2 * cost['v_add_u32 + s_nop 0 (pair)'] - cost['v_add_u32 (reference: full-rate)']:.3f} ns", file=out)
    res = {}
    for k in ("k_pass_a", "k_pass_b"):
        a, c = att[k], ctr[k]
        per_wave = sum(n * cost[PRICE[cls]] for cls, n in a["classes"].items())
        waves = c["SQ_WAVES"]
        dyn = c["SQ_INSTS_VALU"] / waves if waves else a["valu"]
        scale = dyn / a["valu"]
        model_ms = (65536 / 1024) * per_wave * scale * 1e-6
        clock = (c["GRBM_GUI_ACTIVE"] / 8 / (waves / 65536)) / (dur[k] * 1e-3) / 1e9 if dur.get(k) else None
        res[k] = model_ms
        print(f"{k}: static VALU {a['valu']}/wave, dynamic {dyn:.0f}/wave (x{scale:.3f}); issue time per wave "
              f"{per_wave * scale:.0f} ns -> {model_ms:.3f} ms for 64 waves/SIMD; measured {dur.get(k, float('nan')):.3f} ms "
              f"(fastest launch) -> model / measured = {model_ms / dur[k]:.2f}", file=out)
        wc = c["SQ_WAVE_CYCLES"]
        print(f"    wave cycles: issuing {c['SQ_ACTIVE_INST_ANY'] / wc:.2f}, issue-stalled {c['SQ_WAIT_INST_ANY'] / wc:.2f}, "
              f"parked (waitcnt / barrier) {c['SQ_WAIT_ANY'] / wc:.2f}; LDS bank-conflict cycles / LDS instr "
              f"{c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_INSTS_LDS'], 1):.1f}"
              + (f"; in-kernel clock {clock:.2f} GHz (GRBM_GUI_ACTIVE / 8 over the traced time)" if clock else ""),
              file=out)
    tot_model = sum(res.values())
    tot_meas = sum(dur.values())
    print(f"encode: model {tot_model:.3f} ms, measured {tot_meas:.3f} ms: the passes run at "
          f"{tot_model / tot_meas:.0%} of their VALU issue floor", file=out)
    if len(sys.argv) > 5:
        json.dump({"config_len": 1 << 24, "field": "Ft127", "code": "ligero",
                   "model_ms": {k: round(v, 4) for k, v in res.items()},
                   "measured_ms": {k: round(v, 4) for k, v in dur.items()},
                   "frac_of_issue_floor": round(tot_model / tot_meas, 3),
                   "source": "tools/encode_cycle_model.py: per-class issue cost at 4 waves/SIMD "
                             "(tools/microbench/issue_cost.hip) x the passes' instruction counts x their dynamic VALU "
                             "count (SQ_INSTS_VALU), against the fastest traced launch; profiles/r06_encode_cycle_model.txt"},
                  open(sys.argv[5], "w"), indent=1)


if __name__ == "__main__":
    main()
