#!/usr/bin/env python3
"""The matrix-free round in its flat form (st_mfree_round_flat: k_flat<MF>
+ k_mparts) against the grid-stride k_mfree (st_mfree_round), on the same
block: agreement of λ, the row sums and v after K launches (fp64 1e-12,
fp32 1e-5 relative; the two sum each row in another association), and the
time per launch by HIP events (median of 5 passes of 20 launches).

    python3 tools/mfree_flat_probe.py [N[xC][:f32] ...]
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def run(nr, n, dt, K=12):
    import torch
    from eigen_value_amd import device as dev
    d = torch.device("cuda", 0)
    a = dev.generate("random", n, dt, nrows=nr, seed=0, device=d)
    part = dev.flat_scratch(nr, n, dt, d)

    def fresh():
        s = [torch.ones(n, dtype=dt, device=d) for _ in range(2)]
        dev.rowsum(a, out=s[0][:nr])
        v = [torch.ones(n, dtype=dt, device=d) for _ in range(2)]
        return s, v, dev.new_state(d)

    def launches(flat, s, v, st, k0, cnt):
        for k in range(k0, k0 + cnt):
            sp, sn = s[(k - 1) & 1], s[k & 1]
            vp, vc = v[(k - 1) & 1], v[k & 1]
            if flat:
                dev.mfree_round_flat(a, sp, sn[:nr], vp, vc, part, st, eps=0.0, k=k,
                                     max_itr=1 << 30)
            else:
                dev.mfree_round(a, sp, sn[:nr], vp, vc, st, eps=0.0, k=k, max_itr=1 << 30)

    res = {}
    for flat in (False, True):
        s, v, st = fresh()
        launches(flat, s, v, st, 1, K)
        torch.cuda.synchronize()
        res[flat] = (s[K & 1][:nr].clone(), v[K & 1].clone(), dev.read_state(st))
    rel_s = ((res[True][0] - res[False][0]).abs() / res[False][0].abs()).max().item()
    rel_v = ((res[True][1] - res[False][1]).abs() / res[False][1].abs()).max().item()
    lam = (res[True][2]["eigen_val"], res[False][2]["eigen_val"])
    times = {}
    for flat in (False, True):
        s, v, st = fresh()
        launches(flat, s, v, st, 1, 4)
        per = []
        for p in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            launches(flat, s, v, st, 5 + p * 20, 20)
            e1.record()
            torch.cuda.synchronize()
            per.append(e0.elapsed_time(e1) / 20)
        times["flat" if flat else "k_mfree"] = sorted(per)[2]
    b = nr * n * (8 if dt == torch.float64 else 4)
    out = {"block": f"{nr}x{n}", "dtype": str(dt).split(".")[-1], "bytes": b,
           "ms": {k: round(v, 5) for k, v in times.items()},
           "GBs": {k: round(b / (v * 1e-3) / 1e9, 1) for k, v in times.items()},
           "frac_of_8TBs": {k: round(b / (v * 1e-3) / 8e12, 4) for k, v in times.items()},
           "max_rel_diff_s": rel_s, "max_rel_diff_v": rel_v,
           "lambda": lam, "rounds": K}
    tol = 1e-12 if dt == torch.float64 else 1e-5
    out["agree"] = rel_s <= tol and rel_v <= tol and abs(lam[0] - lam[1]) <= tol * abs(lam[1])
    print(json.dumps(out), flush=True)
    return out


def main():
    import torch
    specs = sys.argv[1:] or ["8192", "12288", "16384", "32768", "8192:f32", "32768:f32"]
    outs = []
    for sp in specs:
        size, _, dts = sp.partition(":")
        nr, _, n = size.partition("x")
        nr, n = int(nr), int(n or nr)
        outs.append(run(nr, n, torch.float32 if dts == "f32" else torch.float64))
    if not all(o["agree"] for o in outs):
        sys.exit(1)


if __name__ == "__main__":
    main()
