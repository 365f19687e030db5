#!/usr/bin/env python3
"""Rounds per host flag check (st_options.batch) of the solve loop, timed on
whole Hilbert solves at the sizes where a round is a few microseconds.

The loop enqueues `batch` rounds, then one state mirror, and waits on the
PREVIOUS batch's flag while this one runs (st_solve.hip): the launches queued
past the stopping round run as gated no-ops of a few microseconds each, so
the batch trades host round trips against wasted launches.  Median of
--reps solves per (N, dtype, batch), batches interleaved; `loop_ms` is the
library's own loop time (st_stats), H2D excluded.

    python3 tools/batch_probe.py --n 512 1024 2048 4096 --batch 1 2 3 4 6 8 12 16
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, nargs="+", default=[512, 1024, 2048, 4096])
    p.add_argument("--batch", type=int, nargs="+", default=[1, 2, 3, 4, 6, 8, 12, 16])
    p.add_argument("--dtype", nargs="+", default=["f32", "f64"])
    p.add_argument("--reps", type=int, default=15)
    p.add_argument("--json")
    a = p.parse_args()
    import torch
    from eigen_value_amd import device as dev
    solver = dev.DeviceSolver(torch.device("cuda", 0))
    out = {}
    for dt in a.dtype:
        tdt = torch.float64 if dt == "f64" else torch.float32
        for n in a.n:
            mat = dev.generate("hilbert", n, tdt, device="cuda:0")
            res = {b: [] for b in a.batch}
            iters = {}
            for b in a.batch:                      # warm-up
                solver.solve(mat, batch=b)
            for _ in range(a.reps):
                for b in a.batch:
                    lam, v, it, st = solver.solve(mat, batch=b)
                    res[b].append(st["loop_ms"])
                    iters[b] = (it, lam)
            assert len({x for x in iters.values()}) == 1, iters   # the batch moves no result
            row = {}
            for b in a.batch:
                xs = sorted(res[b])
                row[str(b)] = xs[len(xs) // 2]
            out[f"hilbert{n}_{dt}"] = {"iter_count": iters[a.batch[0]][0], "loop_ms": row}
            print(f"hilbert{n}_{dt} iters {iters[a.batch[0]][0]}: " +
                  "  ".join(f"b{b} {row[str(b)]:.4f}" for b in a.batch), flush=True)
    solver.close()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
