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
as k_flat_np<NP> against their own algorithmic bytes (N^2 b read-only,
2 N^2 b for the storing launch); k_flat is the every-round transform.
"""
import argparse
import collections
import csv
import json
import statistics


def flat_np(name):
    """k_flat's NP template argument (the 12th): -1 = the every-round
    transform, else the pending rounds a deferred-write launch re-applies."""
    args = name.split("(")[0].split("<", 1)[1].rsplit(">", 1)[0].split(",")
    return int(args[11]) if len(args) > 11 else -1


def flat_stores(name, m):
    """Whether a deferred k_flat instance stores the matrix: the launch with
    m - 1 pending rounds.  (A final flush after a partial group also stores,
    with fewer pending rounds and the same instance as a read-only round;
    the profiled runs end on whole store cycles, so they have none.)"""
    args = [x.strip() for x in name.split("(")[0].split("<", 1)[1].rsplit(">", 1)[0].split(",")]
    # a 4-row launch with no pending round only ever stores (the flush after
    # a partial group; the read-only NP = 0 rounds take 2 rows)
    return flat_np(name) == m - 1 or (flat_np(name) == 0 and args[4] == "4")


def short(name, m=3):
    base = name.split("(")[0].replace("void ", "")
    k = base.split("<")[0].split("::")[-1]
    if k == "k_flat" and flat_np(name) >= 0:   # deferred writes (st_device.h FlatPending)
        k = f"k_flat_np{flat_np(name)}" + ("_store" if flat_stores(name, m) else "")
    return k


def load_pmc(path, m):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        out[(short(r["Kernel_Name"], m), r["Kernel_Name"].split("(")[0])].append(
            float(r["Counter_Value"]))
    return out


def load_trace(path, m):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6  # ms
        out[(short(r["Kernel_Name"], m), r["Kernel_Name"].split("(")[0])].append(dur)
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
    fetch, write = load_pmc(a.fetch, m), load_pmc(a.write, m)
    trace = load_trace(a.trace, m) if a.trace else {}
    algo = {"k_round": 2.0 * nb, "k_flat": 2.0 * nb, "k_mfree": nb, "k_fused": nb}
    for npend in range(m):
        algo[f"k_flat_np{npend}"] = nb
        algo[f"k_flat_np{npend}_store"] = 2.0 * nb
    entries = []
    for key in sorted(fetch):
        kname, full = key
        if kname not in algo or f"<{a.dtype}," not in full:
            continue
        f = fetch[key]
        w = write.get(key, [])
        med = statistics.median(f)
        keep = [i for i, x in enumerate(f) if x >= 0.1 * med]
        f_kb = statistics.median([f[i] for i in keep])
        w_kb = statistics.median([w[i] for i in keep if i < len(w)]) if w else 0.0
        hbm = (2.0 * f_kb + w_kb) * 1024.0
        e = {"kernel": kname, "instance": full, "launches": len(f), "launches_used": len(keep),
             "fetch_size_kib": f_kb, "write_size_kib": w_kb,
             "hbm_bytes_per_launch": hbm, "correction": "FETCH_SIZE x2 (gfx950 wide-stream read)",
             "algorithmic_bytes": algo[kname], "traffic_over_algorithmic": hbm / algo[kname]}
        if key in trace:
            d = trace[key]
            dm = statistics.median(d)
            dk = [x for x in d if x >= 0.1 * dm]
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
