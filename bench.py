#!/usr/bin/env python3
"""Benchmark of the similarity-transform round (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n N0]
                    [--kind hilbert|random] [--dtype f64|f32] [--no-cpu]
                    [--no-north-star]

One *step* = one round of the hot path on the HBM-resident matrix: the
single fused launch (max / eigenvector update / stop test of s_k, then
A_{k+1} = D^-1 A_k D in place and its row sums) that moves 2*N^2*b bytes
(read A_k, write A_{k+1}), plus, for N > 1 GPUs, the all-gather of the
row-sum vector.  The stop
tolerance is set to 0 inside the timed region so that every one of the K
rounds does the full work (after convergence the reference would stop;
a fixed round count is how SURVEY.md §8d prices ms/iteration).

Workload (config.workload): BASELINE.json configs[1], 8192x8192 Hilbert
fp64 on one GPU.  For N GPUs the row-block sharded path runs with
per-GPU bytes held constant (weak scaling): n = 8192*sqrt(N) rounded to a
multiple of 64*N, rows split in contiguous blocks, one RCCL all-gather per
round.  `--strong` keeps n fixed instead (configs[3]:
`--n 65536 --kind random --strong` on 8 GPUs).  `value` = algorithmic bytes of all ranks / max-over-ranks time
(GB/s); `ms_per_step` = ms/iteration.

Extra objects on the JSON line: `roofline` (fused kernel, HIP events on
the launch stream), `cpu_baseline` (the CPU oracle's 3-pass schedule on
the host cores, rank 0 at N=1), `solve` (the reference-semantics solve to
convergence: rounds, λ), `matrix_free` (the read-only form of the same
iteration, SURVEY.md §8f item 1, priced against its own N^2*b bytes),
`north_star` (32768x32768 random fp64, 1 GPU, both forms),
`deferred_writes` (the library's solve loop, which stores the matrix every
m-th round — 4 on blocks of >= 2 GiB, else 3 fp64 / 4 fp32 (st_defer_rounds) —
with bit-identical results, against storing every
round; priced against its own (m+1)/m*N^2*b bytes) and, under
`reference_headline`, `config0_hilbert128_gpu` (configs[0]'s 128^2 Hilbert
solved on the GPU in one workgroup launch).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
MALL_BYTES = 256 << 20  # memory-side (Infinity) cache
# fp64 Hilbert 8192, reference semantics (cyclic, EPS=1e-3): 17 rounds,
# λ = 2.5999921826283514 (CPU oracle; README.md:76 publishes 17 rounds)
HILBERT8192_F64 = (17, 2.5999921826283514)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--n", type=int, default=8192, help="matrix size at N=1 GPU")
    p.add_argument("--kind", default="hilbert", choices=["hilbert", "random"])
    p.add_argument("--dtype", default="f64", choices=["f64", "f32"])
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-north-star", action="store_true")
    p.add_argument("--no-headline", action="store_true",
                   help="skip the fp32 whole-solve comparison with the published numbers")
    p.add_argument("--cpu-seconds", type=float, default=15.0,
                   help="CPU baseline sample length (rounds are calibrated to it)")
    p.add_argument("--strong", action="store_true",
                   help="keep n fixed for every N (strong scaling; e.g. configs[3]: "
                        "--n 65536 --kind random --strong)")
    p.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                   help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI)")
    p.add_argument("--overlap", action="store_true",
                   help="N > 1: time the overlapped exchange (split round, all-gather on a "
                        "second stream) as the headline instead of an extra leg")
    p.add_argument("--no-overlap-leg", action="store_true",
                   help="N > 1: skip the extra overlapped-exchange leg")
    p.add_argument("--one-gpu", action="store_true",
                   help="rehearsal: every rank on cuda:0 (use with --backend gloo)")
    return p.parse_args()


def scaled_n(n1: int, world: int) -> int:
    if world == 1:
        return n1
    q = 64 * world
    return int(round(n1 * math.sqrt(world) / q)) * q


def true_lambda(n, dtype, seed):
    """Committed CPU Perron root (tests/golden/large_pins.json) or None."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden",
                        "large_pins.json")
    try:
        for c in json.load(open(path))["cases"]:
            if (c["n"], c["dtype"], c["seed"]) == (n, dtype, seed):
                return c["lambda"]
    except (OSError, ValueError, KeyError):
        pass
    return None


def load_traffic(workload: str, kernel: str = "k_round"):
    """Per-launch HBM bytes of a hot kernel from the committed rocprofv3 PMC
    passes of this workload (profiles/*_pmc.json, tools/pmc_traffic.py;
    FETCH_SIZE and WRITE_SIZE from separate passes, FETCH_SIZE doubled per
    the gfx950 correction).  The latest round's file wins."""
    import glob
    best = None
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("workload") != workload:
            continue
        for e in d.get("entries", []):
            if e.get("kernel") == kernel:
                best = (e["hbm_bytes_per_launch"], os.path.relpath(f, HERE))
    return best


def cw_bound(torch, a0, v, lam):
    """Bound on |λ - λ_true| / λ from the Collatz–Wielandt bracket of a
    positive matrix: λ_true lies in [min, max] of (A0 v)_i / v_i."""
    q = torch.mv(a0, v.to(a0.dtype)) / v.to(a0.dtype)
    lo, hi = q.min().item(), q.max().item()
    return max(abs(lam - lo), abs(lam - hi)) / abs(lam)


def timed_rounds(sh, steps, warmup, torch, dist, world):
    """Warmup + K timed rounds; returns (elapsed_s_max, kernel_ms_avg).

    The kernel's average launch duration comes from HIP events recorded on
    the launch stream (torch's current stream, which the C-ABI launches on).
    At N = 1 the timed region holds nothing but the round launches, so two
    events bracket it (per-launch events would add ~7 us of event work to
    every 175 us round).  With N > 1 the all-gathers sit between launches:
    the timed region runs without events, and a separate pass after it
    brackets each launch with its own pair for the kernel average."""
    sh.start()
    for _ in range(warmup):
        sh.round(0.0, 2**31)
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if world == 1:
        ev[0][0].record()
    for k in range(steps):
        sh.round(0.0, 2**31)
    if world == 1:
        ev[0][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if world == 1:
        fused = ev[0][0].elapsed_time(ev[0][1]) / steps
    else:  # kernel-only average, outside the timed region
        n_ev = min(steps, 50)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(n_ev)]
        for k in range(n_ev):
            sh.round(0.0, 2**31, events=ev[k])
        torch.cuda.synchronize()
        fused = sum(a.elapsed_time(b) for a, b in ev) / n_ev
        t = torch.tensor([el, fused], dtype=torch.float64,
                         device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el, fused = float(t[0]), float(t[1])
    return el, fused


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    from eigen_value_amd import sharded
    from eigen_value_amd import _lib
    from eigen_value_amd import device as dev

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dev_index = 0 if args.one_gpu else local
    torch.cuda.set_device(dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")
    _lib.load()   # fail loudly before anything else if the HIP library is missing

    dt = torch.float64 if args.dtype == "f64" else torch.float32
    b = 8 if args.dtype == "f64" else 4
    n = args.n if args.strong else scaled_n(args.n, world)
    workload = f"{args.kind}{n}_{args.dtype}"
    sh = sharded.ShardedSimilarityTransform(n, dt, overlap=args.overlap)
    p = sh.part

    # ---- reference-semantics solve to convergence (EPS = 1e-3) ----------
    sh.load(args.kind)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # batch=1: the host checks the stop flag after every round, as the
    # reference does (similarity_transform.cpp:45-50); no gated launches
    lam, v, iters, rounds = sh.solve(eps=1e-3, max_itr=1000, batch=1)
    torch.cuda.synchronize()
    solve_ms = (time.perf_counter() - t0) * 1e3
    solve = {"eps": 1e-3, "iter_count": iters, "rounds_evaluated": rounds,
             "eigen_val": lam, "ms": round(solve_ms, 3)}
    if args.kind == "hilbert" and n == 8192 and args.dtype == "f64":
        solve["check"] = {"iter_count_expected": HILBERT8192_F64[0],
                          "eigen_val_rel_err_vs_oracle":
                              abs(lam - HILBERT8192_F64[1]) / HILBERT8192_F64[1]}
    if world == 1:
        # accuracy against the TRUE eigenvalue: Collatz–Wielandt bracket of the
        # positive input, min (A0 v)_i / v_i <= λ_true <= max (A0 v)_i / v_i
        # (torch.mv as the checker); and the same solve at eps = 1e-6
        a0 = sh.load(args.kind)
        solve["rel_err_bound_vs_true"] = cw_bound(torch, a0, v, lam)
        lam6, v6, it6, _ = sh.solve(eps=1e-6, max_itr=1000, batch=1)
        a0 = sh.load(args.kind)
        solve["eps_1e-6"] = {"iter_count": it6, "eigen_val": lam6,
                             "rel_err_bound_vs_true": cw_bound(torch, a0, v6, lam6)}
        del a0

    # ---- timed rounds ----------------------------------------------------
    sh.load(args.kind, mat=None)
    el, fused_ms = timed_rounds(sh, args.steps, args.warmup, torch, dist, world)
    bytes_round_total = 2.0 * n * n * b
    bytes_round_local = 2.0 * p.nrows * n * b
    value = bytes_round_total * args.steps / el / 1e9
    achieved = bytes_round_local / (fused_ms * 1e-3) / 1e9
    flat_pays = dev.flat_round_pays(p.nrows, n, dt)
    flat = (not args.overlap) and flat_pays
    traffic = load_traffic(workload, "k_flat" if flat else "k_round")
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None if traffic is None else traffic[0],
                "kernel": (("flat split: k_flat local + k_flat remote + k_parts" if flat_pays
                            else "k_round_split local + remote") + " (overlapped exchange)"
                           if args.overlap
                           else "flat round: k_flat + k_parts" if flat
                           else "k_round (fused stats + scale + row-sum)"),
                "fused_ms_avg": round(fused_ms, 5),
                "bytes_per_launch": bytes_round_local,
                "timing": ("HIP events bracketing the K timed rounds on the launch stream"
                           + ("; a round is k_flat + k_parts: compare with the sum of their "
                              "rocprof averages (profiles/*_kernel_stats.csv)" if flat else "")
                           if world == 1 else
                           "HIP events around every launch of a 50-round pass after the timed region"),
                "traffic_source": None if traffic is None else traffic[1]}
    if bytes_round_local / 2 <= 2 * MALL_BYTES:
        roofline["note"] = ("matrix partly resident in the 256 MB memory-side cache: an "
                            "effective rate, not an HBM-roofline claim (see north_star)")

    # ---- N > 1: the same rounds with the exchange overlapped --------------
    # (split launch: local columns while the all-gather runs on a second
    # stream, sharded.py overlap=True); reported beside the headline
    overlap_leg = None
    if world > 1 and not args.overlap and not args.no_overlap_leg:
        ov = sharded.ShardedSimilarityTransform(n, dt, overlap=True)
        ov.load(args.kind)
        lam_ov, _, it_ov, _ = ov.solve(eps=1e-3, max_itr=1000, batch=1)
        ov.load(args.kind)
        el_ov, k_ov = timed_rounds(ov, args.steps, args.warmup, torch, dist, world)
        overlap_leg = {"ms_per_iteration": round(el_ov / args.steps * 1e3, 5),
                       "value": round(bytes_round_total * args.steps / el_ov / 1e9, 2),
                       "round_ms_avg": round(k_ov, 5),
                       "solve_iter_count": it_ov,
                       "eigen_val_rel_diff": abs(lam_ov - lam) / abs(lam)}
        ov.close()
        del ov

    # ---- the matrix-free form on the same workload (N^2*b per round) -----
    mf = sharded.ShardedSimilarityTransform(n, dt, matrix_free=True)
    mf.load(args.kind)
    lam_mf, _, it_mf, _ = mf.solve(eps=1e-3, max_itr=1000, batch=1)
    el_mf, k_mf = timed_rounds(mf, args.steps, args.warmup, torch, dist, world)
    by_mf_local = 1.0 * p.nrows * n * b
    tr_mf = load_traffic(workload, "k_mfree")
    matrix_free = {"ms_per_iteration": round(el_mf / args.steps * 1e3, 5),
                   "traffic": None if tr_mf is None else tr_mf[0],
                   "value": round(1.0 * n * n * b * args.steps / el_mf / 1e9, 2),
                   "kernel_ms_avg": round(k_mf, 5),
                   "achieved": round(by_mf_local / (k_mf * 1e-3) / 1e9, 1),
                   "frac": round(by_mf_local / (k_mf * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "bytes_per_round": 1.0 * n * n * b, "solve_iter_count": it_mf,
                   "eigen_val": lam_mf}
    mf.close()
    del mf

    out = {"metric": "ms/iteration + achieved HBM GB/s (% roofline), N×N Hilbert fp64",
           "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(el / args.steps * 1e3, 5),
           "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
           "vs_baseline": None,
           "dtype": args.dtype, "data": f"synthetic ({args.kind}, generated in HBM)",
           "config": {"workload": workload, "n": n, "rows_per_gpu": p.chunk,
                      "bytes_per_round": bytes_round_total, "parallelism": f"rowblock{world}",
                      "baseline_config": ("configs[1]: 8192x8192 Hilbert fp64, 1xMI355X"
                                          if (world == 1 and n == 8192) else
                                          f"row-block sharding over {world} GPU(s), "
                                          + ("strong" if args.strong else "weak") + "-scaled")},
           "roofline": roofline, "solve": solve, "matrix_free": matrix_free}
    if args.overlap:
        out["config"]["exchange"] = "overlapped (split round, all-gather on a second stream)"
    if overlap_leg is not None:
        out["exchange_overlap"] = overlap_leg
    sh.close()
    del sh
    torch.cuda.empty_cache()

    # ---- north-star size: 32768^2 random fp64 on one GPU ---------------
    if world == 1 and not args.no_north_star:
        ns = sharded.ShardedSimilarityTransform(32768, torch.float64)
        ns.load("random", seed=0)
        lam_ns, _, it_ns, _ = ns.solve(eps=1e-3, max_itr=1000, batch=1)
        ns.load("random", seed=0)
        el_ns, fused_ns = timed_rounds(ns, 50, 3, torch, dist, 1)
        by = 2.0 * 32768 * 32768 * 8
        ach = by / (fused_ns * 1e-3) / 1e9
        flat_ns = dev.flat_round_pays(32768, 32768, torch.float64)
        tr = load_traffic("random32768_f64", "k_flat" if flat_ns else "k_round")
        out["north_star"] = {"workload": "random32768_f64",
                             "kernel": ("flat round: k_flat + k_parts (round time)"
                                        if flat_ns else "k_round"),
                             "ms_per_iteration": round(el_ns / 50 * 1e3, 4),
                             "fused_ms_avg": round(fused_ns, 4), "achieved": round(ach, 1),
                             "frac": round(ach / HBM_PEAK_GBS, 4), "target_frac": 0.70,
                             "traffic": None if tr is None else tr[0],
                             "solve_iter_count": it_ns, "eigen_val": lam_ns}
        pin = true_lambda(32768, "f64", 0)
        if pin is not None:  # CPU Perron root of the same matrix (tests/golden)
            out["north_star"]["eigen_val_rel_err_vs_true"] = abs(lam_ns - pin) / pin
        del ns
        torch.cuda.empty_cache()
        # the matrix-free form on the same 32768^2 input (N^2*b per round)
        mf = sharded.ShardedSimilarityTransform(32768, torch.float64, matrix_free=True)
        mf.load("random", seed=0)
        lam_mf, _, it_mf, _ = mf.solve(eps=1e-3, max_itr=1000, batch=1)
        el_mf, k_mf = timed_rounds(mf, 50, 3, torch, dist, 1)
        by_mf = 1.0 * 32768 * 32768 * 8
        tr_mf = load_traffic("random32768_f64", "k_mfree")
        out["north_star"]["matrix_free"] = {
            "traffic": None if tr_mf is None else tr_mf[0],
            "ms_per_iteration": round(el_mf / 50 * 1e3, 4), "kernel_ms_avg": round(k_mf, 4),
            "achieved": round(by_mf / (k_mf * 1e-3) / 1e9, 1),
            "frac": round(by_mf / (k_mf * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "bytes_per_round": by_mf, "solve_iter_count": it_mf,
            "eigen_val_rel_diff_vs_transform": abs(lam_mf - lam_ns) / lam_ns}
        del mf
        torch.cuda.empty_cache()

    # ---- deferred writes: the library's solve loop (flat round, >= 144 MiB)
    # stores A every m-th round (st_defer_rounds) and re-applies the pending
    # scalings in registers, bit-identical to storing every round.  Per-round time from
    # the host clock of whole solves of 10 and 40 fixed rounds (eps = 0), the
    # difference over 30 rounds; the same with ST_FLAG_WRITE_EVERY_ROUND.
    if world == 1 and not args.no_north_star:
        solver = dev.DeviceSolver(torch.device("cuda", dev_index))
        deferred = {}
        for name, kind, nn, ddt in (("configs[1] " + workload, args.kind, n, dt),
                                    ("north_star random32768_f64", "random", 32768,
                                     torch.float64),
                                    ("configs[4] random32768_f32", "random", 32768,
                                     torch.float32)):
            a0 = dev.generate(kind, nn, ddt, seed=0, device=torch.device("cuda", dev_index))
            if not dev.flat_round_pays(nn, nn, a0.dtype):
                continue
            bpe = a0.element_size()
            per, res = {}, {}
            for every in (False, True):
                t = {}
                for kk in (10, 40):
                    best = float("inf")
                    for _ in range(3):
                        a = a0.clone()
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        r = solver.solve(a, inplace=True, eps=0.0, max_itr=kk,
                                         write_every_round=every)
                        best = min(best, time.perf_counter() - t0)
                        if kk == 10:
                            res[every] = (r[0], r[1].clone(), a.clone() if nn <= 8192 else None)
                        del a
                    t[kk] = best
                per[every] = (t[40] - t[10]) / 30 * 1e3
            same = (res[False][0] == res[True][0] and torch.equal(res[False][1], res[True][1])
                    and (res[False][2] is None or torch.equal(res[False][2], res[True][2])))
            every_m = dev.defer_rounds(nn, nn, a0.dtype)
            by = (every_m + 1.0) / every_m * nn * nn * bpe
            deferred[name] = {
                "stores_every": every_m, "ms_per_iteration": round(per[False], 4),
                "ms_per_iteration_write_every_round": round(per[True], 4),
                "speedup": round(per[True] / per[False], 3),
                "bytes_per_round": by, "achieved": round(by / (per[False] * 1e-3) / 1e9, 1),
                "frac": round(by / (per[False] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                "bitwise_equal_to_write_every_round": bool(same)}
            del a0, res
            torch.cuda.empty_cache()
        solver.close()
        out["deferred_writes"] = deferred

    # ---- the reference's own headline, apples to apples ----------------
    # README.md:66-158 of the reference publishes whole solves of the fp32
    # 8192x8192 Hilbert matrix through its C++ entry (host matrix in, H2D
    # inside the timed region); the fastest published device is a Xeon
    # Platinum 8358 at 126 ms (17 rounds).  Same call shape here: the
    # drop-in max_eigen_value on a host fp32 Hilbert matrix.
    if world == 1 and rank == 0 and not args.no_headline:
        from eigen_value_amd.similarity_transform import EigenValue
        idx = np.arange(8192, dtype=np.int64)
        h32 = np.float32(1.0) / (idx[:, None] + idx[None, :] + 1).astype(np.float32)  # utils.cpp:150
        with EigenValue() as e:
            e.similarity_transform(h32)                      # warm the context
            runs = [e.similarity_transform_ex(h32) for _ in range(3)]
        lam32, _, ts32, it32, st32 = min(runs, key=lambda r: r[4]["h2d_ms"] + r[4]["loop_ms"])
        out["reference_headline"] = {
            "workload": "hilbert8192_f32 whole solve via max_eigen_value (host matrix)",
            "ms": round(st32["h2d_ms"] + st32["loop_ms"], 3), "h2d_ms": round(st32["h2d_ms"], 3),
            "loop_ms": round(st32["loop_ms"], 3), "iter_count": it32,
            "published_ms": {"Xeon Platinum 8358": 126, "i9-10920X": 510, "Xeon Gold 6128": 339,
                             "Xeon E5-2686 v4": 3759, "Iris Xe MAX": 2509, "UHD P630": 8259},
            "speedup_vs_fastest_published": round(126.0 / (st32["h2d_ms"] + st32["loop_ms"]), 1)}
        # configs[0]'s size (128x128 Hilbert) on the GPU through the same
        # drop-in call: the whole solve is ONE workgroup launch
        # (k_solve_small); the per-round launch loop beside it
        c0 = {}
        with EigenValue() as e:
            for name, dt in (("f32", np.float32), ("f64", np.float64)):
                h = (dt(1.0) / (np.arange(128)[:, None] + np.arange(128)[None, :] + 1)
                     .astype(dt))
                e.similarity_transform(h)                    # warm
                one = min((e.similarity_transform_ex(h) for _ in range(5)),
                          key=lambda r: r[4]["loop_ms"])
                loop = min((e.similarity_transform_ex(h, round_loop=True) for _ in range(5)),
                           key=lambda r: r[4]["loop_ms"])
                c0[name] = {"iter_count": one[3], "eigen_val": float(one[0]),
                            "loop_ms_single_launch": round(one[4]["loop_ms"], 4),
                            "loop_ms_round_launches": round(loop[4]["loop_ms"], 4)}
        out["reference_headline"]["config0_hilbert128_gpu"] = c0

    # ---- CPU baseline (rank 0, N = 1) ------------------------------------
    if world == 1 and rank == 0 and not args.no_cpu:
        from oracle import oracle as orc
        threads = min(16, len(os.sched_getaffinity(0)))
        npdt = np.float64 if args.dtype == "f64" else np.float32
        mat = orc.hilbert(n, npdt) if args.kind == "hilbert" else orc.random_matrix(n, 0, npdt)
        # bounded sample: calibrate on 3 rounds, then ~--cpu-seconds of rounds
        cal = orc.similarity_transform(mat, orc.SEM_SYCL, eps=0.0, max_itr=3, nthreads=threads)
        est = max(cal.loop_ms / 3, 1e-3)
        rounds_cpu = int(min(5000, max(3, args.cpu_seconds * 1e3 / est)))
        r = orc.similarity_transform(mat, orc.SEM_SYCL, eps=0.0, max_itr=rounds_cpu,
                                     nthreads=threads)
        # every round = row-sum pass + stats + transform pass (the last round's
        # transform is skipped, as in the reference loop); priced with the same
        # 2*N^2*b accounting as `value`
        per_round_ms = r.loop_ms / rounds_cpu
        solve_cpu = orc.similarity_transform(mat, orc.SEM_SYCL, nthreads=threads)
        out["cpu_baseline"] = {"value": round(bytes_round_total / (per_round_ms * 1e-3) / 1e9, 3),
                               "unit": "GB/s", "ms_per_iteration": round(per_round_ms, 3),
                               "cores": threads, "kind": "port",
                               "sample": f"{workload}: {rounds_cpu} rounds (eps=0, "
                                         f"{r.loop_ms / 1e3:.1f} s) of the reference's 3-pass "
                                         "schedule (oracle/st_oracle.c, gcc -O3, OpenMP over rows)",
                               "solve_ms": round(solve_cpu.loop_ms, 2),
                               "solve_iter_count": solve_cpu.iter_count}
        out["speedup_vs_cpu"] = round(out["ms_per_step"] and per_round_ms / out["ms_per_step"], 1)
        # configs[0]: 128x128 Hilbert on the CPU path:
        # the C restatement on one core (fp64 / fp32, the SYCL loop), a numpy
        # restatement of main.py's loop, eigenvalues against eigvalsh
        h64 = orc.hilbert(128)
        true128 = float(np.max(np.linalg.eigvalsh(h64)))
        c64 = orc.similarity_transform(h64, orc.SEM_SYCL, nthreads=1)
        c32 = orc.similarity_transform(orc.hilbert(128, np.float32), orc.SEM_SYCL, nthreads=1)
        t0 = time.perf_counter()
        a, v, itr = h64.copy(), np.ones(128), 0
        for itr in range(1000):          # main.py:30-47, elementwise (no O(N^3) matmul)
            s_ = a.sum(axis=1)
            v = v * (s_ / s_.max())
            if np.all(np.abs(np.diff(s_)) < 1e-3):
                break
            a = (a / s_[:, None]) * s_[None, :]
        np_ms = (time.perf_counter() - t0) * 1e3
        out["cpu_baseline"]["config1_hilbert128"] = {
            "c_1core_f64": {"ms": round(c64.loop_ms, 4), "iter_count": c64.iter_count,
                            "rel_err_vs_eigvalsh": abs(c64.eigen_val - true128) / true128},
            "c_1core_f32": {"ms": round(c32.loop_ms, 4), "iter_count": c32.iter_count},
            "numpy_mainpy_semantics": {"ms": round(np_ms, 3), "iter_count": itr + 1,
                                       "eigen_val": float(s_[0])}}

    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
