#!/usr/bin/env python3
"""The flat round's second launch in its two forms (st_set_parts_form,
tuning build): k_parts_lane (a row per lane) against k_parts_seg (rows of
16 / 32 lanes), on the bench's every-round step - interleaved passes of
K rounds from a fresh A_0, HIP events on the launch stream, median - for
configs[1] (Hilbert 8192^2 fp64, 8 partials per row) and configs[4]
(random 32768^2 fp32).  Run under rocprofv3 --kernel-trace --stats for the
per-kernel averages.

    EIGEN_VALUE_LIB=eigen_value_amd/lib/libsimilarity_transform_tuning.so \\
        python3 tools/parts_form_probe.py [--passes 9] [--json OUT]
"""
import argparse
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=9)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    import bench
    from eigen_value_amd import _lib
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    L = _lib.load()
    if not hasattr(L, "st_set_parts_form"):
        raise SystemExit("needs the tuning build (EIGEN_VALUE_LIB=...tuning.so)")
    torch.cuda.set_device(0)
    out = {}
    for kind, n, dt in (("hilbert", 8192, torch.float64), ("random", 32768, torch.float32)):
        key = f"{kind}{n}_{'f64' if dt == torch.float64 else 'f32'}"
        sh = ShardedSimilarityTransform(n, dt)
        res = {0: [], 1: []}
        saved = L.st_set_parts_form(1)
        sh.load(kind)
        bench.timed_rounds(sh, a.steps, 5, torch, None, 1)            # warm-up
        for _ in range(a.passes):
            for form in (0, 1):
                L.st_set_parts_form(form)
                sh.load(kind)
                res[form].append(bench.timed_rounds(sh, a.steps, 5, torch, None, 1)[1])
        L.st_set_parts_form(saved)
        sh.close()
        torch.cuda.empty_cache()
        out[key] = {("lane" if f == 0 else "seg"): {"median": round(statistics.median(v), 5),
                                                    "min": round(min(v), 5),
                                                    "max": round(max(v), 5)}
                    for f, v in res.items()}
        print(key, json.dumps(out[key]), flush=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
