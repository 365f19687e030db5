#!/usr/bin/env python3
"""Why the bench's configs[1] rounds run slower than the same rounds in a
fresh process (round 6: HIP events 0.1593 ms per round inside bench.py,
0.1534 in tools/sync_probe.py on the same box).  One process, one 8192^2
fp64 block: a pass of the bench's timed schedule (load, start, W = 5
warm-up rounds, K = 20 rounds between two events; median of 3) first
fresh, then after each step bench.py's main() runs before its timed
region, in that order, and once more at the end.

    python3 tools/prefix_probe.py [--json OUT]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
BIG = 2 ** 31


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    torch.cuda.set_device(0)
    sh = ShardedSimilarityTransform(8192, torch.float64)
    out = []

    def one_pass(tag):
        rows = []
        for _ in range(a.reps):
            sh.load("hilbert")
            sh.start()
            sh.rounds(5, 0.0, BIG)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ev[0].record()
            sh.rounds(20, 0.0, BIG)
            ev[1].record()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            rows.append((ev[0].elapsed_time(ev[1]) / 20, el * 1e3 / 20))
        rows.sort()
        r = {"step": tag, "event_ms_per_round": [round(x[0], 5) for x in rows],
             "host_ms_per_round": [round(x[1], 5) for x in rows]}
        out.append(r)
        print(json.dumps(r), flush=True)

    one_pass("fresh")
    one_pass("fresh again")
    sh.load("hilbert")
    sh.solve(eps=1e-3, max_itr=1000, batch=1)
    torch.cuda.synchronize()
    one_pass("after solve eps=1e-3 (deferred writes)")
    a0 = sh.load("hilbert")
    lam, v, _, _ = sh.solve(eps=1e-3, max_itr=1000, batch=1)
    a0 = sh.load("hilbert")
    bench.cw_bound(torch, a0, v, lam)
    torch.cuda.synchronize()
    one_pass("after cw_bound (torch.mv on the block)")
    sh.solve(eps=1e-6, max_itr=1000, batch=1)
    torch.cuda.synchronize()
    one_pass("after solve eps=1e-6")
    sh.load("hilbert", mat=None)
    el, ev = bench.timed_rounds(sh, 20, 5, torch, None, 1, clocks_key="probe")
    r = {"step": "bench.timed_rounds", "event_ms_per_round": [round(ev, 5)],
         "host_ms_per_round": [round(el * 1e3 / 20, 5)]}
    out.append(r)
    print(json.dumps(r), flush=True)
    one_pass("after bench.timed_rounds")
    time.sleep(2.0)
    one_pass("after 2 s idle")
    sh.close()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
