#!/usr/bin/env python3
"""Issue-level summary of one kernel from tools/pmc_ntt.sh's rocprofv3 --pmc passes: where its
wave-cycles go (issuing / issue-stalled / parked on waitcnt or barriers), its dynamic VALU and LDS
instructions per wave, LDS bank conflicts, and the in-kernel clock.

    python tools/pmc_kernel_summary.py PMC_DIR KERNEL_SUBSTRING [OUT.txt]

PMC_DIR holds one directory (or CSV) per pass: p1 .. p5 with *counter_collection.csv inside.
Counters are summed over every dispatch of the kernel; per-wave figures divide by SQ_WAVES.
"""
import collections
import csv
import glob
import os
import sys


def main():
    d, sub = sys.argv[1], sys.argv[2]
    out = open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout
    files = glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True) + \
        glob.glob(os.path.join(d, "p*.csv"))
    agg = collections.defaultdict(float)
    durs = {}
    name = None
    for f in files:
        for r in csv.DictReader(open(f)):
            if sub not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"]
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                durs[(f, r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    if not name:
        sys.exit(f"no dispatch of a kernel matching {sub!r} in {d}")
    waves = agg["SQ_WAVES"]
    wc = agg["SQ_WAVE_CYCLES"]
    print(f"# {name}", file=out)
    print(f"# {len(files)} counter passes, SQ_WAVES {waves:.0f}", file=out)
    print(f"wave-cycles: issuing {agg['SQ_ACTIVE_INST_ANY'] / wc:.2f}, issue-stalled {agg['SQ_WAIT_INST_ANY'] / wc:.2f}, "
          f"parked on waitcnt / barriers {agg['SQ_WAIT_ANY'] / wc:.2f}", file=out)
    print(f"per wave: VALU {agg['SQ_INSTS_VALU'] / waves:.0f}, SALU {agg['SQ_INSTS_SALU'] / waves:.0f}, "
          f"LDS {agg['SQ_INSTS_LDS'] / waves:.0f}, VMEM rd {agg['SQ_INSTS_VMEM_RD'] / waves:.0f} / "
          f"wr {agg['SQ_INSTS_VMEM_WR'] / waves:.0f}", file=out)
    print(f"LDS bank-conflict cycles per LDS instruction {agg['SQ_LDS_BANK_CONFLICT'] / max(agg['SQ_INSTS_LDS'], 1):.2f}; "
          f"issue-stalled on LDS {agg['SQ_WAIT_INST_LDS'] / wc:.2f} of wave-cycles", file=out)
    if durs:
        t = sum(durs.values())
        print(f"in-kernel clock {agg['GRBM_GUI_ACTIVE'] / 8 / t / 1e9:.2f} GHz (GRBM_GUI_ACTIVE / 8 XCDs over "
              f"{len(durs)} dispatches, {t / len(durs) * 1e3:.3f} ms each)", file=out)


if __name__ == "__main__":
    main()
