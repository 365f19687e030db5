#!/usr/bin/env python3
"""K0 (the initial row-sum pass, s_0 = A_0 1; similarity_transform.cpp:40)
in both launch forms on the same matrix: the grid-stride k_fused
(st_rowsum) and the flat form (st_rowsum_flat: k_flat_sum + k_parts), timed
with HIP events on the launch stream, priced against N^2 b bytes at 8 TB/s,
and the two sums compared.  Run under rocprofv3 --kernel-trace --stats for
the per-kernel averages.

    python3 tools/k0_probe.py [--reps 20]
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    from eigen_value_amd import device as dev
    torch.cuda.set_device(0)
    out = {}
    for kind, n, dt in (("hilbert", 8192, torch.float64), ("random", 32768, torch.float64),
                        ("random", 32768, torch.float32)):
        m = dev.generate(kind, n, dt, device="cuda:0")
        s1 = torch.empty(n, dtype=dt, device="cuda:0")
        s2 = torch.empty_like(s1)
        part = dev.flat_scratch(n, n, dt, "cuda:0")
        by = n * n * m.element_size()
        res = {}
        for name, fn in (("k_fused", lambda: dev.rowsum(m, out=s1)),
                         ("flat", lambda: dev.rowsum_flat(m, s2, part))):
            for _ in range(3):
                fn()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            ev[0].record()
            for _ in range(a.reps):
                fn()
            ev[1].record()
            torch.cuda.synchronize()
            ms = ev[0].elapsed_time(ev[1]) / a.reps
            res[name] = {"ms": round(ms, 5), "frac": round(by / (ms * 1e-3) / 8e12, 4)}
        rel = ((s1 - s2).abs() / s1.abs()).max().item()
        res["max_rel_diff"] = rel
        key = f"{kind}{n}_{'f64' if dt == torch.float64 else 'f32'}"
        out[key] = res
        print(key, json.dumps(res), flush=True)
        del m, part
        torch.cuda.empty_cache()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
