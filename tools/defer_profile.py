#!/usr/bin/env python3
"""Fixed-round device solves with and without deferred writes, for
rocprofv3 kernel traces and PMC passes of the deferred flat round.

    rocprofv3 --kernel-trace --stats -d OUT -o run -- python3 tools/defer_profile.py
    python3 tools/defer_profile.py --trace OUT/run_kernel_trace.csv   # summarise

One solve of --rounds rounds (eps = 0) per mode on an --n x --n random
matrix (fp64 by default), so the trace holds the deferred k_flat launches
(last template argument NP = 0, 1, 2: the pending rounds each re-applies;
NP = 2 also stores) next to the every-round ones (NP = -1).
"""
import argparse
import csv
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def run(args):
    import torch
    from eigen_value_amd import device as dev
    dt = torch.float64 if args.dtype == "f64" else torch.float32
    a0 = dev.generate("random", args.n, dt, seed=0, device="cuda:0")
    solver = dev.DeviceSolver("cuda:0")
    out = {}
    for every in (False, True):
        a = a0.clone()
        lam, v, it, st = solver.solve(a, inplace=True, eps=0.0, max_itr=args.rounds,
                                      write_every_round=every)
        torch.cuda.synchronize()
        out[every] = (lam, v.cpu(), a)
        print(f"write_every_round={every}: {it} rounds, lambda={lam!r}, "
              f"loop {st['loop_ms']:.3f} ms", flush=True)
    same = out[False][0] == out[True][0] and torch.equal(out[False][1], out[True][1]) \
        and torch.equal(out[False][2], out[True][2])
    print(f"bitwise equal (lambda, v, final matrix): {same}", flush=True)
    solver.close()


def np_of(name):
    """k_flat's last template argument: -1 = stores every round, else the
    number of pending rounds it re-applies (its position in the group)."""
    import re
    m = re.search(r"k_flat<([^>]*)>", name)
    return int(m.group(1).split(",")[11])


def summarise(path, n, elem, m=3):
    rows = [r for r in csv.DictReader(open(path)) if "k_flat<" in r["Kernel_Name"]]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    nb = n * n * elem
    every = [dur(r) for r in rows if np_of(r["Kernel_Name"]) < 0]
    if every:
        t = sum(every) / len(every)
        print(f"every-round k_flat: {len(every)} launches, avg {t:.4f} ms "
              f"({2 * nb / (t * 1e-3) / 1e9:.0f} GB/s on 2 N^2 b)")
    for pos in range(m):
        g = [dur(r) for r in rows if np_of(r["Kernel_Name"]) == pos]
        if g:
            t = sum(g) / len(g)
            b = (2 if pos == m - 1 else 1) * nb
            print(f"deferred k_flat, {pos} pending ({'read + write' if pos == m - 1 else 'read only'}):"
                  f" {len(g)} launches, avg {t:.4f} ms ({b / (t * 1e-3) / 1e9:.0f} GB/s)")


def summarise_pmc(fetch, write, n, elem, m=3):
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
    nb = n * n * elem
    for pos in sorted(f):
        if pos in w:
            rd, wr = 2 * sum(f[pos]) / len(f[pos]), sum(w[pos]) / len(w[pos])
            alg = (2 if pos == m - 1 else 1) * nb
            print(f"deferred k_flat, {pos} pending: read {rd / 1e9:.3f} GB, "
                  f"write {wr / 1e9:.3f} GB per launch; algorithmic {alg / 1e9:.3f} GB "
                  f"(x{(rd + wr) / alg:.4f})")


if __name__ == "__main__":
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=32768)
    p.add_argument("--rounds", type=int, default=30)
    p.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    p.add_argument("--trace", help="summarise a rocprofv3 kernel trace instead of running")
    p.add_argument("--fetch", help="with --write: summarise FETCH_SIZE / WRITE_SIZE passes")
    p.add_argument("--write")
    a = p.parse_args()
    elem = 8 if a.dtype == "f64" else 4
    # rounds per store (st_defer_rounds): 4 on blocks of >= 2 GiB, else 3 fp64 / 4 fp32
    m = 4 if a.n * a.n * elem >= 2 << 30 else (3 if a.dtype == "f64" else 4)
    if a.trace or a.fetch:
        if a.trace:
            summarise(a.trace, a.n, elem, m)
        if a.fetch and a.write:
            summarise_pmc(a.fetch, a.write, a.n, elem, m)
    else:
        run(a)
