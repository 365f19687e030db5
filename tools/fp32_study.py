#!/usr/bin/env python3
"""BASELINE.json configs[4]: 32768x32768 fp32 on one MI355X — packed (float4)
loads, ms/iteration, and a tolerance study against fp64 on the same input.

For k = 0..K-1 rounds of the reference iteration (eps = 0, so every round
runs) on the seeded random matrix in fp32 and in fp64, records λ_k, the
largest adjacent row-sum difference max|s_i - s_{i+1}| (cyclic; the stop
test passes when it is < EPS = 1e-3) and, at the end, the eigenvector
difference.  SURVEY.md §0.4: at N >= 16384 the fp32 row sums (≈ N/2) have
an ulp above EPS, so the reference's fp32 stop test can never pass; the
study shows where the fp32 iteration plateaus.  torch is used only to read
the vectors (the checker side); every round runs the HIP kernels.

    python tools/fp32_study.py [--n 32768] [--rounds 12] [--out file.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--timed", type=int, default=20)
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from eigen_value_amd.sharded import ShardedSimilarityTransform

    n = a.n
    res = {"n": n, "seed": 0, "rounds": []}
    traj = {}
    vecs = {}
    for dt, name in ((torch.float64, "f64"), (torch.float32, "f32")):
        sh = ShardedSimilarityTransform(n, dt)
        sh.load("random", seed=0)
        sh.start()
        lam, dmax = [], []
        for k in range(a.rounds):
            s = sh.s[sh.cur][:n].double()
            lam.append(float(s[0]))
            dmax.append(float((s - torch.roll(s, -1)).abs().max()))
            sh.round(0.0, 2**31)
        torch.cuda.synchronize()
        traj[name] = (lam, dmax)
        vecs[name] = sh.eigen_vector().double().clone()
        # timing: fixed rounds, both forms
        for mf in (False, True):
            t = ShardedSimilarityTransform(n, dt, matrix_free=mf)
            t.load("random", seed=0)
            t.start()
            for _ in range(3):
                t.round(0.0, 2**31)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.timed):
                t.round(0.0, 2**31)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / a.timed * 1e3
            b = 4 if name == "f32" else 8
            by = (1 if mf else 2) * n * n * b
            res[f"{name}_{'matrix_free' if mf else 'transform'}"] = {
                "ms_per_iteration": round(ms, 4), "gbs": round(by / (ms * 1e-3) / 1e9, 1)}
            del t
            torch.cuda.empty_cache()
        # reference-semantics solve: does fp32 ever stop at EPS = 1e-3?
        sh.load("random", seed=0)
        t0 = time.perf_counter()
        lam_s, _, it_s, rounds_s = sh.solve(eps=1e-3, max_itr=1000, batch=16)
        res[f"{name}_solve"] = {"iter_count": it_s, "rounds_evaluated": rounds_s,
                                "eigen_val": lam_s,
                                "seconds": round(time.perf_counter() - t0, 3)}
        del sh
        torch.cuda.empty_cache()
    for k in range(a.rounds):
        l64, d64 = traj["f64"][0][k], traj["f64"][1][k]
        l32, d32 = traj["f32"][0][k], traj["f32"][1][k]
        res["rounds"].append({"k": k, "lambda_f64": l64, "lambda_f32": l32,
                              "lambda_rel_diff": abs(l32 - l64) / l64,
                              "max_adjacent_diff_f64": d64, "max_adjacent_diff_f32": d32,
                              "f64_would_stop": d64 < 1e-3, "f32_would_stop": d32 < 1e-3})
    res["eigen_vec_max_abs_diff_after_rounds"] = float((vecs["f32"] - vecs["f64"]).abs().max())
    res["fp32_ulp_at_row_sum"] = float(torch.finfo(torch.float32).eps * 2 ** (n.bit_length() - 2))
    line = json.dumps(res)
    print(line)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
