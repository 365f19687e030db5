#!/usr/bin/env python3
"""Per-wave SQ counters of the flat-round launches by pending count NP, from
rocprofv3 --pmc passes (counter_collection.csv files, any number):

    python3 tools/sq_counters.py OUT/pass1/run_counter_collection.csv ...

Prints, per k_flat NP (-1 = every-round store, m - 1 = the storing round)
and k_parts: instructions per wave (VALU, SALU, SMEM, VMEM), the wave's
cycles split into active / waiting on memory / issue-stalled, VGPR and
SGPR counts.  Passes without SQ_WAVES (e.g. TCP / TA counters) print their
per-dispatch values instead."""
import collections
import csv
import json
import re
import sys


def key(name):
    if "k_parts<" in name or "k_parts_seg<" in name:
        return "k_parts"
    m = re.search(r"k_flat<([^>]*)>", name)
    if not m:
        return None
    a = [x.strip() for x in m.group(1).split(",")]
    return f"k_flat {a[0]} NT={a[3]} R={a[4]} NP={a[11 if len(a) > 11 and a[8].strip() == "256" else 8]}"


def main(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    regs = {}
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = key(r["Kernel_Name"])
            if k is None:
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
            regs[k] = (r["VGPR_Count"], r["SGPR_Count"])
    out = {}
    for k in sorted(acc):
        c = acc[k]
        per = {n: v / max(1, len(disp[(k, n)])) for n, v in c.items()}  # per dispatch
        waves = per.get("SQ_WAVES")
        row = {"vgpr_sgpr": regs[k], "per_dispatch": per}
        if waves:
            row["per_wave"] = {n: round(v / waves, 1) for n, v in per.items() if n != "SQ_WAVES"}
        out[k] = row
        pw = row.get("per_wave") or {n: round(v, 1) for n, v in per.items()}
        print(f"{k:40s} v/s {regs[k]}  " + "  ".join(f"{n.replace('SQ_', '')}={v}"
                                                    for n, v in sorted(pw.items())))
    return out


if __name__ == "__main__":
    res = main([a for a in sys.argv[1:] if not a.startswith("--json=")])
    for a in sys.argv[1:]:
        if a.startswith("--json="):
            json.dump(res, open(a[7:], "w"), indent=1)
