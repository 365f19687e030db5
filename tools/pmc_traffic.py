#!/usr/bin/env python3
"""Per-launch HBM traffic of the hot kernels from rocprofv3 PMC passes.

    python tools/pmc_traffic.py --workload hilbert8192_f64 --n 8192 \
        --fetch gpurun_out/X/pmc_fetch/run_counter_collection.csv \
        --write gpurun_out/X/pmc_write/run_counter_collection.csv \
        --trace gpurun_out/X/prof/run_kernel_trace.csv \
        --out profiles/r01_hilbert8192_pmc.json

FETCH_SIZE and WRITE_SIZE come from separate passes (they do not fit one
pass on gfx950) and are reported in KiB.  Per MI355X_MICROARCH.md §HBM,
FETCH_SIZE reads exactly half the bytes of a wide (16 B/lane) coalesced
streaming read on gfx950, so the read side is doubled; WRITE_SIZE is exact
for 16 B/lane streaming stores.  Launches that did no work (device-gated
rounds after convergence) are dropped (< 10 % of the median traffic).
The kernel trace gives the per-launch duration of the same command.
Deferred-write launches of k_flat (template argument NP >= 0) are reported
as k_flat_np<NP> against their own algorithmic bytes (N^2 b read-only), or
k_flat_np<NP>_store (2 N^2 b) for the launches whose WRITE_SIZE shows they
stored the block (one instance serves both); k_flat is the every-round
transform.  Launches are matched across the three runs by dispatch order.
"""
import argparse
import collections
import csv
import json
import statistics


def flat_np(name):
    """k_flat's NP template argument: -1 = the every-round transform, else
    the pending rounds a deferred-write launch re-applies (the 9th template
    argument since round 6; the 12th, after BLK = 256 as the 9th, in
    earlier rounds' traces)."""
    args = name.split("(")[0].split("<", 1)[1].rsplit(">", 1)[0].split(",")
    i = 11 if len(args) > 11 and args[8].strip() == "256" else 8   # old: BLK = 256 there
    return int(args[i]) if len(args) > i else -1


def short(name):
    base = name.split("(")[0].replace("void ", "")
    k = base.split("<")[0].split("::")[-1]
    if k == "k_flat" and flat_np(name) >= 0:   # deferred writes (st_device.h FlatPending)
        k = f"k_flat_np{flat_np(name)}"
    return k


def load_seq(path, value):
    """Per kernel instance, its launches in dispatch order."""
    out = collections.defaultdict(list)
    rows = list(csv.DictReader(open(path)))
    key = "Dispatch_Id" if rows and "Dispatch_Id" in rows[0] else None
    if key:
        rows.sort(key=lambda r: int(r[key]))
    for r in rows:
        out[r["Kernel_Name"].split("(")[0]].append(value(r))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", required=True)
    ap.add_argument("--n", type=int, required=True)
    ap.add_argument("--elem", type=int, default=8)
    ap.add_argument("--dtype", default="double", help="template element type to keep")
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--trace")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    nb = 1.0 * a.n * a.n * a.elem
    # deferred writes: m rounds per store (st_defer_rounds); a storing
    # launch moves 2 N^2 b, the others read N^2 b
    m = 6  # st_defer_rounds (round 2: every block)
    fetch = load_seq(a.fetch, lambda r: float(r["Counter_Value"]))
    write = load_seq(a.write, lambda r: float(r["Counter_Value"]))
    trace = load_seq(a.trace, lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                     * 1e-6) if a.trace else {}
    algo = {"k_round": 2.0 * nb, "k_flat": 2.0 * nb, "k_mfree": nb, "k_fused": nb,
            "k_flat_sum": nb}   # k_flat_sum: K0 in the flat form (round 6)
    for npend in range(m):
        algo[f"k_flat_np{npend}"] = nb
        algo[f"k_flat_np{npend}_store"] = 2.0 * nb
    # one deferred instance serves a read-only round and a storing one
    # (the storing round of a group, a final flush): the i-th launch of an
    # instance is the same launch in the three runs of the command, and it
    # stored the matrix if its WRITE_SIZE is at least half the block
    groups = collections.defaultdict(lambda: ([], [], []))
    for full, f in fetch.items():
        kname = short(full)
        if f"<{a.dtype}," not in full or (kname not in algo):
            continue
        w = write.get(full, [])
        d = trace.get(full, [])
        if len(d) != len(f):
            # a trace of another command length: its launches stored where
            # they took well over the instance's median (a storing round
            # moves twice the bytes)
            med_d = statistics.median(d) if d else 0.0
            d_ro = [x for x in d if x <= 1.5 * med_d]
            d_st = [x for x in d if x > 1.5 * med_d]
            d = None
        for i, fv in enumerate(f):
            wv = w[i] if i < len(w) else 0.0
            label = kname
            if kname.startswith("k_flat_np") and wv * 1024.0 >= 0.5 * nb:
                label += "_store"
            g = groups[(label, full)]
            g[0].append(fv)
            g[1].append(wv)
            if d is not None:
                g[2].append(d[i])
            elif not g[2]:
                g[2].extend(d_st if label.endswith("_store") and kname != "k_flat" else d_ro)
    entries = []
    for (kname, full), (f, w, d) in sorted(groups.items()):
        med = statistics.median(f)
        keep = [i for i, x in enumerate(f) if x >= 0.1 * med]
        f_kb = statistics.median([f[i] for i in keep])
        w_kb = statistics.median([w[i] for i in keep])
        hbm = (2.0 * f_kb + w_kb) * 1024.0
        e = {"kernel": kname, "instance": full, "launches": len(f), "launches_used": len(keep),
             "fetch_size_kib": f_kb, "write_size_kib": w_kb,
             "hbm_bytes_per_launch": hbm, "correction": "FETCH_SIZE x2 (gfx950 wide-stream read)",
             "algorithmic_bytes": algo[kname], "traffic_over_algorithmic": hbm / algo[kname]}
        dk = [d[i] for i in keep if i < len(d)] if len(d) == len(f) else \
            [x for x in d if x >= 0.1 * statistics.median(d)] if d else []
        if dk:
            e["trace_ms_avg"] = sum(dk) / len(dk)
            e["trace_launches"] = len(d)
            e["achieved_gbs_from_trace"] = algo[kname] / (e["trace_ms_avg"] * 1e-3) / 1e9
        entries.append(e)
    fused = [e for e in entries if e["kernel"] in ("k_round", "k_flat")]
    doc = {"workload": a.workload, "n": a.n, "entries": entries,
           "fused_bytes_per_launch": fused[0]["hbm_bytes_per_launch"] if fused else None}
    json.dump(doc, open(a.out, "w"), indent=1)
    for e in entries:
        print(f'{e["kernel"]:>17}: {e["hbm_bytes_per_launch"] / 1e9:8.3f} GB/launch '
              f'(algorithmic {e["algorithmic_bytes"] / 1e9:.3f}, x{e["traffic_over_algorithmic"]:.4f})'
              + (f', trace {e["trace_ms_avg"]:.4f} ms' if "trace_ms_avg" in e else ""))


if __name__ == "__main__":
    main()
