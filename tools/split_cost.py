#!/usr/bin/env python3
"""Per-round cost of splitting a round in two for the overlapped exchange,
on one GPU with no communication: the unsplit round (flat or one-launch
k_round, as the library picks) against the same block as local + remote
halves (st_round_split_flat when the flat round pays, else
st_round_split).  Block shapes are the rank-0 row blocks of the weak-scaled
bench sizes (n = 8192*sqrt(P)), f64, with the local columns = own rows."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from eigen_value_amd import device as dev
    import bench
    out = []
    K = int(os.environ.get("K", "200"))
    for p in (1, 2, 4, 8):
        n = bench.scaled_n(8192, p)
        rows = (n + p - 1) // p
        a = dev.generate("random", n, torch.float64, nrows=rows, seed=1, device="cuda")
        # scales within 1e-6 of 1: A stays finite over hundreds of rounds
        s = 1.0 + 1e-6 * torch.rand(n, dtype=torch.float64, device="cuda")
        s_next = torch.empty(rows, dtype=torch.float64, device="cuda")
        v = torch.ones(n, dtype=torch.float64, device="cuda")
        flat = dev.flat_round_pays(rows, n, torch.float64)
        col0, col1 = 0, rows

        def unsplit(k, state, part):
            if flat:
                dev.flat_round(a, s, s_next, part, v, state, eps=0.0, k=k, max_itr=2**31)
            else:
                dev.fused_round(a, s, s_next, v, state, eps=0.0, k=k, max_itr=2**31)

        def split(k, state, part):
            fn = dev.split_flat_round if flat else dev.split_round
            fn(a, s, None, part, None, state, span=dev.SPAN_LOCAL, col0=col0, col1=col1,
               eps=0.0, k=k, max_itr=2**31)
            fn(a, s, s_next, part, v, state, span=dev.SPAN_REMOTE, col0=col0, col1=col1,
               eps=0.0, k=k, max_itr=2**31)

        parts = {
            "unsplit": dev.flat_scratch(rows, n, torch.float64, "cuda") if flat else None,
            "split": (dev.split_flat_scratch(rows, n, col0, col1, torch.float64, "cuda") if flat
                      else torch.empty(rows, dtype=torch.float64, device="cuda")),
        }
        res = {"p": p, "n": n, "rows": rows, "flat": flat,
               "block_gib": rows * n * 8 / 2**30}
        for rep in range(2):
            for name, fn in (("unsplit", unsplit), ("split", split)):
                state = dev.new_state("cuda")
                for k in range(10):
                    fn(k, state, parts[name])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for k in range(10, 10 + K):
                    fn(k, state, parts[name])
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / K
                res[f"{name}_ms"] = min(ms, res.get(f"{name}_ms", 1e9))
        for name in ("unsplit", "split"):
            res[f"{name}_gbs"] = 2 * rows * n * 8 / res[f"{name}_ms"] / 1e6
        res["split_cost_us"] = (res["split_ms"] - res["unsplit_ms"]) * 1e3
        print(json.dumps(res), flush=True)
        out.append(res)
        del a
        torch.cuda.empty_cache()
    return out


if __name__ == "__main__":
    main()
