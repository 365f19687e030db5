#!/usr/bin/env python3
"""The deferred-write flat round (the solve loops' form for blocks of >= 144
MiB) over whole store cycles, for rocprofv3 kernel traces and PMC passes,
with HIP-event timing of the same launches.

    rocprofv3 --kernel-trace --stats -d OUT -o run -- \\
        python3 tools/defer_profile.py --kind random --n 32768 --events OUT/events.json
    python3 tools/defer_profile.py --kind random --n 32768 \\
        --trace OUT/run_kernel_trace.csv --events OUT/events.json --json OUT/cycle.json

Run mode: ShardedSimilarityTransform at P = 1 (the same st_round_flat_
deferred launches as DeviceSolver's solve loop) runs 2 warm-up cycles, then
--cycles store cycles of m rounds (bench.py timed_deferred: the first round
after a store ... the storing round, no flush), timed with HIP events; the
per-round figure goes to --events.  Summary mode reads the kernel trace:
k_flat launches by their last template argument NP (the pending rounds a
launch re-applies; NP = m - 1 also stores; -1 = stores every round) and the
k_parts launch that follows each, and writes per-NP averages and their sum
over one cycle per round (`cycle_ms_per_round`) next to the events' figure
(--json: profiles/rNN_defer_cycle_<workload>.json, read by bench.py).
"""
import argparse
import csv
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


# RELOAD_NOTE: the A/B modes regenerate A_0 before every pass.  A rank
# block timed alone (--rank-block) holds the other ranks' row sums at 1.0,
# so its off-block columns shrink by 1/s_r every round (Hilbert 5824 x 11648:
# below 1e-300 after ~800 rounds, zeros after ~1300), and on blocks the
# memory-side cache assists, zero-valued lines stream faster (8192^2 fp64:
# the identity 0.1411 ms per round against 0.1533 for Hilbert or random
# data, profiles/r03_data_dependence.log): passes over thousands of rounds
# would drift.  Round 3's earlier A/B files (r03_everyab_*, r03_ntab*_*,
# r03_capsab*_*) ran without the reload; their rank-block passes are
# interleaved, so the comparisons hold, but late passes saw decayed data.


def rounds_per_store(n, elem, f64):
    # st_defer_rounds: 6 on every block (round 2; round 1 took 3 or 4)
    return 6


def set_caps(spec, dtype, n, elem, nrows=None):
    """--caps a,b,c,d,e,f,g: workgroups per CU of the deferred launches
    (slots 0..4 = read-only rounds by pending count, 6 = the storing round;
    0 = uncapped) for this block's dtype and launch form (st_set_defer_caps)."""
    from eigen_value_amd import _lib
    L = _lib.load()
    nt = 1 if (nrows or n) * n * elem >= (2 << 30) else 0
    for slot, c in enumerate(int(x) for x in spec.split(",")):
        if slot == 5:
            continue
        _lib.check(L.st_set_defer_caps(1 if dtype == "f64" else 0, nt, slot, c), "caps")


def set_ntload(mask, n, elem, nrows=None):
    """--ntload-ab: the non-temporal-load mask of the deferred launches on
    cached fp64 blocks (st_set_defer_ntload; bit NP 0..4 = read-only round
    with NP pending, bit 6 = storing round) for this block's size class."""
    from eigen_value_amd import _lib
    L = _lib.load()
    cls = L.st_defer_ntload_class(nrows or n, n, 1 if elem == 8 else 0)
    _lib.check(L.st_set_defer_ntload(cls, int(mask, 0)), "ntload")


def set_every(policy, n, elem, nrows=None):
    """--every-ab: the cache policy of the every-round flat launch
    (st_set_every_cache: 0 the form's own, 1 / 2 / 3 turn the loads' /
    stores' / both policies over, cached <-> non-temporal) for this block's
    size class; "P:T" also sets the piece tile (st_set_every_tile: 1 =
    row-major, t = tiles of t row groups, 0 = the library's table)."""
    from eigen_value_amd import _lib
    L = _lib.load()
    cls = L.st_every_cache_class(nrows or n, n, 1 if elem == 8 else 0)
    # "P", "P:T" or "P:T:C" (T: st_set_every_tile, C: st_set_every_caps)
    pol, tile, cap = (policy.split(":") + ["", ""])[:3]
    old_pol = _lib.check(L.st_set_every_cache(cls, int(pol, 0)), "every_cache")
    old_tile = _lib.check(L.st_set_every_tile(cls, int(tile or "0", 0)), "every_tile")
    old_cap = _lib.check(L.st_set_every_caps(cls, int(cap or "0", 0)), "every_caps")
    return f"{old_pol}:{old_tile}:{old_cap}"


def run_mfree_ab(args):
    """--mfree-ab 's;s;...': the matrix-free round (k_mfree) under each
    launch shape (st_set_mfree_shape), --steps rounds per pass from a fresh
    A_0, interleaved over --passes repeats; prints and returns the medians."""
    import torch
    import bench
    from eigen_value_amd import _lib, sharded
    L = _lib.load()
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    rb = (args.rank_block, 0) if args.rank_block else None
    sh = sharded.ShardedSimilarityTransform(args.n, dt, rank_block=rb, matrix_free=True)
    sh.load(args.kind, seed=0)
    specs = args.mfree_ab.split(";")
    res = {sp: [] for sp in specs}
    _lib.check(L.st_set_mfree_shape(int(specs[0])), "mfree_shape")
    bench.timed_rounds(sh, args.steps, 10, torch, None, 1)             # warm-up
    for _ in range(args.passes):
        for sp in specs:
            _lib.check(L.st_set_mfree_shape(int(sp)), "mfree_shape")
            res[sp].append(bench.timed_rounds(sh, args.steps, 4, torch, None, 1)[1])
    out = {"workload": f"{args.kind}{args.n}_{args.dtype}" + (
               f" rank 0 of {args.rank_block}" if args.rank_block else ""),
           "form": "matrix-free round (k_mfree)",
           "steps": args.steps, "passes": args.passes, "ms_per_round": {}}
    for sp in specs:
        v = sorted(res[sp])
        out["ms_per_round"][sp] = {"median": v[len(v) // 2], "min": v[0], "max": v[-1]}
        print(f"{out['workload']} mfree-shape {sp:4s} median {v[len(v) // 2]:.5f} ms/round "
              f"(min {v[0]:.5f}, max {v[-1]:.5f})", flush=True)
    L.st_set_mfree_shape(0)
    sh.close()
    return out


def run_every_ab(args):
    """--every-ab 'p;p;...': the every-round flat round (bench.py's timed
    step) under each cache policy, --steps rounds per pass, interleaved over
    --passes repeats; prints and returns the median ms per round of each."""
    import torch
    import bench
    from eigen_value_amd import sharded
    elem = 8 if args.dtype == "f64" else 4
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    rb = (args.rank_block, 0) if args.rank_block else None
    sh = sharded.ShardedSimilarityTransform(args.n, dt, rank_block=rb)
    sh.load(args.kind, seed=0)
    specs = args.every_ab.split(";")
    res = {sp: [] for sp in specs}
    shipped = set_every(specs[0], args.n, elem, sh.part.nrows)
    bench.timed_rounds(sh, args.steps, 10, torch, None, 1)             # warm-up
    for _ in range(args.passes):
        for sp in specs:
            set_every(sp, args.n, elem, sh.part.nrows)
            sh.load(args.kind, seed=0)        # fresh A_0 per pass (see RELOAD_NOTE)
            res[sp].append(bench.timed_rounds(sh, args.steps, 4, torch, None, 1)[1])
    out = {"workload": f"{args.kind}{args.n}_{args.dtype}" + (
               f" rank 0 of {args.rank_block}" if args.rank_block else ""),
           "form": "every-round flat round (k_flat + k_parts)",
           "steps": args.steps, "passes": args.passes, "ms_per_round": {}}
    for sp in specs:
        v = sorted(res[sp])
        out["ms_per_round"][sp] = {"median": v[len(v) // 2], "min": v[0], "max": v[-1]}
        print(f"{out['workload']} every-cache {sp:6s} median {v[len(v) // 2]:.5f} ms/round "
              f"(min {v[0]:.5f}, max {v[-1]:.5f})", flush=True)
    set_every(shipped, args.n, elem, sh.part.nrows)           # the library's own again
    sh.close()
    return out


def set_defer_cache(mask, n, elem, nrows=None):
    """--defer-cache-ab: the deferred rounds' cache-policy flips for this
    block's dtype and size class (st_set_defer_cache: bit NP 0..4 = read-only
    round with NP pending, bit 6 = storing round's loads, bit 7 its stores)."""
    from eigen_value_amd import _lib
    L = _lib.load()
    d = 1 if elem == 8 else 0
    cls = L.st_every_cache_class(nrows or n, n, d)
    _lib.check(L.st_set_defer_cache(d, cls, int(mask, 0)), "defer_cache")


def run_caps_ab(args):
    """--caps-ab 'spec;spec;...' (st_set_defer_caps) or --ntload-ab
    'mask;mask;...' (st_set_defer_ntload): the same store cycles under each
    spec, interleaved over --passes repeats so that clock drift hits every
    spec alike; prints and returns the median ms per round of each spec."""
    import torch
    import bench
    from eigen_value_amd import sharded
    elem = 8 if args.dtype == "f64" else 4
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    rb = (args.rank_block, 0) if args.rank_block else None
    sh = sharded.ShardedSimilarityTransform(args.n, dt, rank_block=rb)
    assert sh.deferred_writes
    sh.load(args.kind, seed=0)
    if args.ntload_ab:
        what, specs = "ntload", args.ntload_ab.split(";")

        def apply(sp):
            set_ntload(sp, args.n, elem, sh.part.nrows)
    elif args.defer_cache_ab:
        what, specs = "defer-cache", args.defer_cache_ab.split(";")

        def apply(sp):
            set_defer_cache(sp, args.n, elem, sh.part.nrows)
    else:
        what, specs = "caps", args.caps_ab.split(";")

        def apply(sp):
            set_caps(sp, args.dtype, args.n, elem, sh.part.nrows)
    res = {sp: [] for sp in specs}
    apply(specs[0])
    bench.timed_deferred(sh, args.cycles, 2, torch, None, 1)          # warm-up
    for _ in range(args.passes):
        for sp in specs:
            apply(sp)
            sh.load(args.kind, seed=0)        # fresh A_0 per pass (see RELOAD_NOTE)
            res[sp].append(bench.timed_deferred(sh, args.cycles, 1, torch, None, 1)[1])
    out = {"workload": f"{args.kind}{args.n}_{args.dtype}" + (
               f" rank 0 of {args.rank_block}" if args.rank_block else ""),
           "cycles": args.cycles, "passes": args.passes, "ms_per_round": {}}
    for sp in specs:
        v = sorted(res[sp])
        out["ms_per_round"][sp] = {"median": v[len(v) // 2], "min": v[0], "max": v[-1]}
        print(f"{out['workload']} {what} {sp:24s} median {v[len(v) // 2]:.5f} ms/round "
              f"(min {v[0]:.5f}, max {v[-1]:.5f})", flush=True)
    sh.close()
    return out


def run(args):
    import torch
    import bench
    from eigen_value_amd import sharded
    if args.caps:
        set_caps(args.caps, args.dtype, args.n, 8 if args.dtype == "f64" else 4)
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    rb = (args.rank_block, 0) if args.rank_block else None
    sh = sharded.ShardedSimilarityTransform(args.n, dt, rank_block=rb)
    assert sh.deferred_writes, "block below the flat-round size: no deferred writes"
    sh.load(args.kind, seed=0)
    el, ev_ms, m = bench.timed_deferred(sh, args.cycles, 2, torch, None, 1)
    out = {"workload": f"{args.kind}{args.n}_{args.dtype}" + (
               f" rank 0 of {args.rank_block}" if args.rank_block else ""),
           "m": m, "cycles": args.cycles,
           "event_ms_per_round": ev_ms, "host_ms_per_round": el / (args.cycles * m) * 1e3,
           "caps": args.caps}
    if args.passes > 1:   # more passes over the same cycles (the first warmed up above)
        more = [bench.timed_deferred(sh, args.cycles, 0, torch, None, 1)[1]
                for _ in range(args.passes - 1)]
        out["event_ms_per_round_passes"] = [ev_ms] + more
        out["event_ms_per_round"] = sorted(out["event_ms_per_round_passes"])[len(more) // 2 + 0]
    print(json.dumps(out), flush=True)
    if args.events:
        json.dump(out, open(args.events, "w"), indent=1)
    sh.close()


def np_of(name):
    """k_flat's last template argument: -1 = stores every round, else the
    number of pending rounds it re-applies (its position in the group)."""
    m = re.search(r"k_flat<([^>]*)>", name)
    args = m.group(1).split(",")
    # before round 6 the 9th argument was BLK (256) and NP the 12th
    return int(args[11 if len(args) > 11 and args[8].strip() == "256" else 8])


def summarise(path, n, elem, m, workload, events=None, launches=None, block_rows=None):
    """Per-NP averages of a kernel trace.  `launches`: also write the
    deferred launches themselves (kernel, NP, start, duration; one row per
    launch, in trace order) to this CSV - the trimmed trace that a committed
    summary cites, so its averages can be re-derived from tracked files."""
    rows = list(csv.DictReader(open(path)))
    if rows and "Start_Timestamp" in rows[0]:
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    elif rows:
        # a committed trimmed trace (--launches) re-summarised
        rows = [{"Kernel_Name": r["kernel_name"], "Start_Timestamp": r["start_ns"],
                 "End_Timestamp": str(int(r["start_ns"]) + int(r["duration_ns"]))}
                for r in csv.DictReader(open(path))]
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        launches = None
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6  # noqa: E731
    flat, parts, last = {}, {}, None
    kept = []
    for r in rows:
        name = r["Kernel_Name"]
        if "k_flat<" in name:
            last = np_of(name)
            flat.setdefault(last, []).append(dur(r))
            kept.append(("k_flat", last, r))
        elif ("k_parts<" in name or "k_parts_seg<" in name) and last is not None:
            parts.setdefault(last, []).append(dur(r))
            kept.append(("k_parts", last, r))
            last = None
    if launches:
        t0 = int(kept[0][2]["Start_Timestamp"]) if kept else 0
        with open(launches, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "np", "start_ns", "duration_ns", "kernel_name"])
            for kind, pos, r in kept:
                w.writerow([kind, pos, int(r["Start_Timestamp"]) - t0,
                            int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                            r["Kernel_Name"][:160]])
    nb = (block_rows or n) * n * elem     # a rank block (--rank-block): its rows
    avg = lambda x: sum(x) / len(x)  # noqa: E731
    # the steady state: the first store cycles of a trace run cold (the
    # first storing launch 3.17 ms against 2.82 later at 32768^2 fp64), which
    # the averages keep and the medians do not
    med = lambda x: sorted(x)[len(x) // 2]  # noqa: E731
    out = {"workload": workload, "m": m,
           "trace": os.path.basename(launches) if launches else path,
           "k_flat": {}, "k_parts": {}}
    for pos in sorted(flat):
        t = avg(flat[pos])
        b = 2 * nb if pos in (-1, m - 1) else nb
        tm = med(flat[pos])
        out["k_flat"][str(pos)] = {"launches": len(flat[pos]), "avg_ms": round(t, 5),
                                   "median_ms": round(tm, 5),
                                   "bytes": b, "GBs": round(b / (t * 1e-3) / 1e9, 1),
                                   "GBs_median": round(b / (tm * 1e-3) / 1e9, 1)}
        if pos in parts:
            out["k_parts"][str(pos)] = round(avg(parts[pos]), 5)
        print(f"k_flat NP={pos}: {len(flat[pos])} launches, avg {t:.4f} ms "
              f"({b / (t * 1e-3) / 1e9:.0f} GB/s)" + (
                  f", k_parts {avg(parts[pos]):.4f} ms" if pos in parts else ""))
    if all(p in flat and p in parts for p in range(m)):
        cyc = sum(avg(flat[p]) + avg(parts[p]) for p in range(m)) / m
        out["cycle_ms_per_round"] = round(cyc, 5)
        by = (m + 1.0) / m * nb
        out["cycle_GBs"] = round(by / (cyc * 1e-3) / 1e9, 1)
        cm = sum(med(flat[p]) + med(parts[p]) for p in range(m)) / m
        out["cycle_ms_per_round_median"] = round(cm, 5)
        out["cycle_GBs_median"] = round(by / (cm * 1e-3) / 1e9, 1)
        print(f"steady state (medians): {cm:.4f} ms per round")
        print(f"one store cycle: {cyc:.4f} ms per round ({out['cycle_GBs']:.0f} GB/s on "
              f"(m+1)/m N^2 b)")
    if events:
        ev = json.load(open(events))
        out["event_ms_per_round"] = round(ev["event_ms_per_round"], 5)
        if "cycle_ms_per_round" in out:
            out["events_over_rocprof"] = round(ev["event_ms_per_round"]
                                               / out["cycle_ms_per_round"], 4)
            print(f"HIP events: {ev['event_ms_per_round']:.4f} ms per round "
                  f"(x{out['events_over_rocprof']:.4f} the rocprof cycle sum)")
    return out


def leg_blocks(leg_out, kind):
    """(workload, m, cycles, warm, HIP-event passes, bytes per round) of
    every deferred block in a `bench.py --leg ...` stdout file."""
    LEG_TAG = "@@LEG "
    leg = None
    for ln in open(leg_out):
        if ln.startswith(LEG_TAG):
            leg = json.loads(ln[len(LEG_TAG):])
    assert leg is not None, f"no {LEG_TAG.strip()} line in {leg_out}"
    blocks = []
    if "deferred_writes" in leg:
        for name, d in leg["deferred_writes"].items():
            wl = name.split()[-1]
            blocks.append((wl, d["stores_every"], d["cycles"], 2, d["ms_per_iteration_passes"],
                           d["bytes_per_round"]))
    for key in ("weak_rank_blocks", "rank_blocks"):
        for P, d in leg.get(key, {}).items():
            if not P.startswith("P") or "deferred_writes" not in d:
                continue
            dw = d["deferred_writes"]
            m = dw["stores_every"]
            blocks.append((f"{kind}{d['cols']}_p{P[1:]}_f64", m, dw["cycles"], 1,
                           dw["ms_per_iteration_passes"],
                           (m + 1.0) / m * d["rows"] * d["cols"] * 8))
    return blocks


def summarise_bench_leg(trace, leg_out, kind, plain_out=None):
    """--bench-leg: a rocprofv3 kernel trace of bench.py's own deferred
    leg (`bench.py --leg deferred|weak_rank_blocks|rank_blocks`), summarised
    the way the leg times it with HIP events: every pass
    starts at its k_recip (deferred_start, after a fresh load), runs `warm`
    store cycles and then the timed `cycles` x m rounds; per pass the
    k_flat + k_parts kernel time of the timed rounds / rounds, per block the
    median of its 3 passes beside the leg's own HIP-event passes.
    plain_out: the same leg run WITHOUT the profiler on the same box; its
    HIP-event medians give the trace's own slowdown (kernel tracing adds a
    completion signal and timestamps to every dispatch: ~2 % on rounds of
    0.1 ms, nothing on rounds of 1 ms and more)."""
    blocks = leg_blocks(leg_out, kind)
    plain = {b[0]: b[4] for b in leg_blocks(plain_out, kind)} if plain_out else {}
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6  # noqa: E731
    segs, cur, flat = [], None, None
    for r in rows:
        name = r["Kernel_Name"]
        if "k_recip<" in name:
            cur = []
            segs.append(cur)
            flat = None
        elif cur is not None and "k_flat<" in name and np_of(name) >= 0:
            flat = dur(r)
        elif cur is not None and flat is not None and ("k_parts<" in name
                                                       or "k_parts_seg<" in name):
            cur.append(flat + dur(r))
            flat = None
    segs = [x for x in segs if x]
    out = {"source": "bench.py leg under rocprofv3 --kernel-trace", "trace": trace,
           "leg_out": leg_out, "blocks": []}
    i = 0
    med = lambda x: sorted(x)[len(x) // 2]  # noqa: E731
    for wl, m, cycles, warm, ev_passes, by in blocks:
        passes = []
        for _ in range(3):
            while i < len(segs) and len(segs[i]) < (warm + cycles) * m:
                i += 1            # not a timed pass (e.g. the leg's bitwise check)
            assert i < len(segs), f"{wl}: trace ends before its 3 passes"
            t = segs[i][warm * m:(warm + cycles) * m]
            passes.append(sum(t) / len(t))
            i += 1
        rp = med(passes)
        ev = med(ev_passes)
        b = {"workload": wl, "m": m, "cycles": cycles, "warm_cycles": warm,
             "rocprof_ms_per_round_passes": [round(x, 5) for x in passes],
             "rocprof_ms_per_round": round(rp, 5),
             "rocprof_GBs": round(by / (rp * 1e-3) / 1e9, 1),
             "rocprof_frac": round(by / (rp * 1e-3) / 1e9 / 8000.0, 4),
             "event_ms_per_round_passes": ev_passes, "event_ms_per_round": ev,
             "events_over_rocprof": round(ev / rp, 4), "bytes_per_round": by}
        if wl in plain:
            pe = med(plain[wl])
            b["event_ms_per_round_untraced"] = pe
            b["event_ms_per_round_untraced_passes"] = plain[wl]
            b["trace_slowdown"] = round(ev / pe, 4)
        out["blocks"].append(b)
        print(f"{wl}: rocprof {rp:.5f} ms per round (passes "
              f"{', '.join(f'{x:.5f}' for x in passes)}), HIP events {ev:.5f} "
              f"(x{ev / rp:.4f}), {b['rocprof_frac']:.4f} of 8 TB/s")
    return out


def summarise_pmc(fetch, write, n, elem, m, rows=None):
    """HBM bytes per deferred k_flat launch by pending count: 2*FETCH_SIZE
    (the gfx950 wide-read correction, MI355X_MICROARCH.md §HBM) + WRITE_SIZE,
    KiB counters, from separate passes."""
    def per_pos(path):
        out = {}
        for r in csv.DictReader(open(path)):
            if "k_flat<" in r["Kernel_Name"] and np_of(r["Kernel_Name"]) >= 0:
                out.setdefault(np_of(r["Kernel_Name"]), []).append(
                    float(r["Counter_Value"]) * 1024.0)
        return out

    f, w = per_pos(fetch), per_pos(write)
    nb = (rows or n) * n * elem
    res = {}
    for pos in sorted(f):
        if pos in w:
            rd, wr = 2 * sum(f[pos]) / len(f[pos]), sum(w[pos]) / len(w[pos])
            alg = (2 if pos == m - 1 else 1) * nb
            res[str(pos)] = {"read": rd, "write": wr, "algorithmic": alg,
                             "ratio": round((rd + wr) / alg, 4)}
            print(f"deferred k_flat, {pos} pending: read {rd / 1e9:.3f} GB, "
                  f"write {wr / 1e9:.3f} GB per launch; algorithmic {alg / 1e9:.3f} GB "
                  f"(x{(rd + wr) / alg:.4f})")
    return res


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=32768)
    p.add_argument("--kind", default="random", choices=["hilbert", "random", "identity"])
    p.add_argument("--cycles", type=int, default=8)
    p.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    p.add_argument("--events", help="run mode: write the HIP-event figure here; summary "
                                    "mode: read it")
    p.add_argument("--trace", help="summarise a rocprofv3 kernel trace instead of running")
    p.add_argument("--json", help="summary mode: write the summary here")
    p.add_argument("--launches", help="summary mode: write the per-launch rows (trimmed "
                                      "trace) here; the summary cites this file")
    p.add_argument("--fetch", help="with --write: summarise FETCH_SIZE / WRITE_SIZE passes")
    p.add_argument("--caps", help="run mode: workgroups per CU of the deferred launches, "
                                  "slots 0..6 comma-separated (st_set_defer_caps)")
    p.add_argument("--passes", type=int, default=1, help="run mode: timed passes (median)")
    p.add_argument("--caps-ab", help="A/B of caps specs separated by ';' (interleaved passes)")
    p.add_argument("--ntload-ab", help="A/B of non-temporal-load masks (cached fp64 blocks) "
                                       "separated by ';', e.g. '0;0x1;0x41'")
    p.add_argument("--defer-cache-ab", help="A/B of deferred cache-policy masks "
                   "(st_set_defer_cache, any dtype / size class) separated by ';'")
    p.add_argument("--mfree-ab", help="A/B of matrix-free launch shapes (st_set_mfree_shape: "
                   "0 table, 1 / 2 cached 2 / 4 rows, 3 non-temporal 4 rows) separated by ';'")
    p.add_argument("--every-ab", help="A/B of every-round cache policies (st_set_every_cache: "
                   "0 the form's, 1 / 2 / 3 loads / stores / both turned over) separated by ';'")
    p.add_argument("--steps", type=int, default=100, help="with --every-ab: rounds per pass")
    p.add_argument("--ab-json", help="with --caps-ab / --every-ab: write the medians here")
    p.add_argument("--rank-block", type=int, default=0,
                   help="rank 0's block of a P-way row partition (no exchange)")
    p.add_argument("--write")
    p.add_argument("--bench-leg", help="with --trace: the stdout of the profiled "
                   "`bench.py --leg ...` run; summarise its timed deferred passes")
    p.add_argument("--bench-leg-plain", help="with --bench-leg: the stdout of the same leg "
                   "run without the profiler (the trace's own slowdown)")
    a = p.parse_args()
    elem = 8 if a.dtype == "f64" else 4
    m = rounds_per_store(a.n, elem, a.dtype == "f64")
    wl = f"{a.kind}{a.n}_{a.dtype}"
    rows = -(-a.n // a.rank_block) if a.rank_block else a.n
    if a.rank_block:
        wl = f"{a.kind}{a.n}_p{a.rank_block}_{a.dtype}"
    if a.caps_ab or a.ntload_ab or a.every_ab or a.defer_cache_ab or a.mfree_ab:
        r = (run_mfree_ab(a) if a.mfree_ab else
             run_every_ab(a) if a.every_ab else run_caps_ab(a))
        if a.ab_json:
            json.dump(r, open(a.ab_json, "w"), indent=1)
    elif a.trace and a.bench_leg:
        res = summarise_bench_leg(a.trace, a.bench_leg, a.kind, a.bench_leg_plain)
        if a.json:
            json.dump(res, open(a.json, "w"), indent=1)
    elif a.trace or a.fetch:
        res = {}
        if a.trace:
            res = summarise(a.trace, a.n, elem, m, wl, a.events, a.launches, rows)
        if a.fetch and a.write:
            res["pmc"] = summarise_pmc(a.fetch, a.write, a.n, elem, m, rows)
        if a.json:
            json.dump(res, open(a.json, "w"), indent=1)
    else:
        run(a)
