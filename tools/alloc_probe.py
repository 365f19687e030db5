#!/usr/bin/env python3
"""Does the every-round flat round's time at 32768^2 fp64 depend on where
the 8 GiB block lands?  Allocates the block REPS times (keeping the
previous ones alive, so each lands on other physical memory), generates
the same matrix into it and times 20 rounds with HIP events.

    python3 tools/alloc_probe.py [--n 32768] [--reps 6] [--dtype f64]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--dtype", default="f64")
    ap.add_argument("--keep", type=int, default=1, help="keep previous blocks alive")
    ap.add_argument("--pre", default="", help="comma-separated sizes to generate and free "
                                               "first (torch.cuda.empty_cache after each)")
    a = ap.parse_args()
    import torch
    from eigen_value_amd import device as dev
    dt = torch.float64 if a.dtype == "f64" else torch.float32
    for m in [int(x) for x in a.pre.split(",") if x]:
        t = dev.generate("random", m, dt, seed=0, device="cuda")
        torch.cuda.synchronize()
        del t
        torch.cuda.empty_cache()
    n, K = a.n, 20
    held = []
    s = 1.0 + 1e-6 * torch.rand(n, dtype=dt, device="cuda")
    s_next = torch.empty(n, dtype=dt, device="cuda")
    v = torch.ones(n, dtype=dt, device="cuda")
    part = dev.flat_scratch(n, n, dt, "cuda")
    for r in range(a.reps):
        m = dev.generate("random", n, dt, seed=0, device="cuda")
        state = dev.new_state("cuda")
        for k in range(3):
            dev.flat_round(m, s, s_next, part, v, state, eps=0.0, k=k, max_itr=2 ** 31)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for k in range(3, 3 + K):
            dev.flat_round(m, s, s_next, part, v, state, eps=0.0, k=k, max_itr=2 ** 31)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / K
        print(json.dumps({"rep": r, "ptr": hex(m.data_ptr()), "ms": round(ms, 4),
                          "GBs": round(2 * n * n * m.element_size() / ms / 1e6, 1)}), flush=True)
        if a.keep:
            held.append(m)
        del m


if __name__ == "__main__":
    main()
