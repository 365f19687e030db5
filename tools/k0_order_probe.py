#!/usr/bin/env python3
"""K0's walk order on cacheable blocks (st_set_k0_reverse, tuning build):
after a generator writes A_0 front to back, the memory-side cache holds the
block's tail.  A K0 that walks from the end starts on those lines and leaves
the block's start cached for round 0, which walks front to back.  Per block
and order (interleaved passes, median): HIP-event ms of K0, of rounds 0 and
1 right after it (the flat round, st_round_flat), and host ms of the whole
reference-semantics solve (eps 1e-3, the deferred loop) from a fresh A_0.

    EIGEN_VALUE_LIB=eigen_value_amd/lib/libsimilarity_transform_tuning.so \\
        python3 tools/k0_order_probe.py [--passes 7] [--json OUT]
"""
import argparse
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=7)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    from eigen_value_amd import _lib, device as dev
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    L = _lib.load()
    if not hasattr(L, "st_set_k0_reverse"):
        raise SystemExit("needs the tuning build (EIGEN_VALUE_LIB=...tuning.so)")
    torch.cuda.set_device(0)
    out = {}
    for kind, n, dt in (("hilbert", 8192, torch.float64), ("hilbert", 8192, torch.float32),
                        ("random", 6144, torch.float64), ("random", 12288, torch.float32),
                        ("random", 14336, torch.float64)):
        key = f"{kind}{n}_{'f64' if dt == torch.float64 else 'f32'}"
        m = dev.generate(kind, n, dt, device="cuda:0")
        s0 = torch.empty(n, dtype=dt, device="cuda:0")
        s1, s2 = torch.empty_like(s0), torch.empty_like(s0)
        v = torch.ones_like(s0)
        part = dev.flat_scratch(n, n, dt, "cuda:0")
        res = {0: {"k0": [], "r0": [], "r1": []}, 1: {"k0": [], "r0": [], "r1": []}}
        sums = {}
        for _ in range(a.passes):
            for mode in (0, 1):
                L.st_set_k0_reverse(mode)
                dev.generate(kind, n, dt, device="cuda:0", out=m)
                v.fill_(1.0)
                st = dev.new_state("cuda:0")
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                torch.cuda.synchronize()
                ev[0].record()
                dev.rowsum_flat(m, s0, part)
                ev[1].record()
                dev.flat_round(m, s0, s1, part, v, st, eps=0.0, k=0)
                ev[2].record()
                dev.flat_round(m, s1, s2, part, v, st, eps=0.0, k=1)
                ev[3].record()
                torch.cuda.synchronize()
                for j, nm in enumerate(("k0", "r0", "r1")):
                    res[mode][nm].append(ev[j].elapsed_time(ev[j + 1]))
                sums[mode] = s0.clone()
        same = bool(torch.equal(sums[0], sums[1]))
        del m, part
        torch.cuda.empty_cache()
        # the whole solve (K0 + the deferred loop) from a fresh A_0
        sh = ShardedSimilarityTransform(n, dt)
        solve = {0: [], 1: []}
        its = {}
        for _ in range(a.passes):
            for mode in (0, 1):
                L.st_set_k0_reverse(mode)
                sh.load(kind)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                lam, _, it, _ = sh.solve(eps=1e-3, max_itr=1000, batch=1)
                torch.cuda.synchronize()
                solve[mode].append((time.perf_counter() - t0) * 1e3)
                its[mode] = (it, lam)
        sh.close()
        torch.cuda.empty_cache()
        L.st_set_k0_reverse(-1)
        med = {mode: {nm: round(statistics.median(x), 5) for nm, x in r.items()}
               for mode, r in res.items()}
        for mode in (0, 1):
            med[mode]["solve_ms"] = round(statistics.median(solve[mode]), 4)
        out[key] = {"forward": med[0], "reversed": med[1], "sums_identical": same,
                    "solve_same": its[0] == its[1], "iter_count": its[0][0]}
        print(key, json.dumps(out[key]), flush=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
