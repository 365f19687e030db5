#!/usr/bin/env python3
"""Extended parity sweep on the GPU against the CPU oracle (the test suite's
test_fuzz_vs_oracle, widened): seeded random cases over size (including the
flat round's deferred-write sizes from 144 MiB and ragged, odd and
non-16-byte widths), dtype, semantics, form (transform with deferred writes,
transform storing every round, matrix-free), batch, eps and input kind,
through the drop-in host path and the device-resident solver.  Every case
must reproduce the oracle's iteration count; λ and v are held to the test
suite's tolerances (fp64 1e-10, fp32 2e-5 / 5e-4) and the worst errors are
recorded.  Both sides run traced (tests/stop_parity.py): a case is excused
from the count check only when its two solves' own row sums put a round's
max |Δs| on opposite sides of eps (listed under `straddles` with the margin
and the measured row-sum deviation that explains it); every case's
row-sum deviation in ulps is recorded.  Test infrastructure: the oracle is
the checker.

    python3 tools/fuzz_parity.py --cases 300 --json OUT.json
    python3 tools/fuzz_parity.py --profile wrapper --cases 200 --json OUT.json

`--profile wrapper`: only the reference's own wrapper-test shape
(wrapper/python/test.py:3-18) - fp32 random matrices through the drop-in
max_eigen_value at its EPS = 1e-3f and MAX_ITR = 1000, SYCL semantics, the
default (deferred-write) form - at N log-uniform over 200 .. 8192, so that
the fp32 flat path (N >= 6145) is in it too.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, "tests"))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cases", type=int, default=300)
    p.add_argument("--seed", type=int, default=20261017)
    p.add_argument("--json", default=None)
    p.add_argument("--profile", choices=["mixed", "wrapper"], default="mixed")
    a = p.parse_args()
    import numpy as np
    import torch
    from eigen_value_amd import device as dev
    from eigen_value_amd.similarity_transform import EigenValue
    from oracle import oracle as orc
    import stop_parity as sp
    torch.cuda.set_device(0)
    rng = np.random.default_rng(a.seed)
    small = [1, 2, 3, 5, 7, 16, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 1000, 1023,
             1024, 1025, 2047, 2049, 2051, 3001]
    flat = [4352, 4353, 4480, 5000, 5121, 6144]           # >= 144 MiB fp64: the flat round
    worst = {"f64": {"lam": 0.0, "v": 0.0}, "f32": {"lam": 0.0, "v": 0.0}}
    out = {"seed": a.seed, "profile": a.profile, "cases": [], "straddles": [], "dev_ulps_max": {"f64": 0.0, "f32": 0.0},
           "dev_ulps_max_transform": {"f64": 0.0, "f32": 0.0},
           "rule": "tests/stop_parity.py: traced row sums on both sides; a count may differ "
                   "only in a round whose max|ds| straddles eps between the two solves"}
    solver = dev.DeviceSolver("cuda:0")
    t0 = time.time()
    with EigenValue() as ev:
        for case in range(a.cases):
            if a.profile == "wrapper":
                n = int(round(np.exp(rng.uniform(np.log(200), np.log(8192)))))
                dt, sem, form, batch, eps = np.float32, 0, "deferred", 0, 1e-3
                kind, path, max_itr = "random", "dropin", orc.MAX_ITR
            else:
                big = rng.random() < 0.25
                n = int(rng.choice(flat if big else small))
                dt = np.float64 if (big or rng.random() < 0.6) else np.float32
                sem = int(rng.integers(0, 2))
                form = str(rng.choice(["deferred", "every", "mfree"]))
                batch = int(rng.choice([0, 1, 2, 5, 8]))
                eps = float(rng.choice([1e-3, 1e-6, 1e-2]))
                kind = "hilbert" if rng.random() < 0.5 else "random"
                path = "device" if rng.random() < 0.5 else "dropin"
                max_itr = 60 if big else 200
            mat = orc.hilbert(n, dt) if kind == "hilbert" else orc.random_matrix(n, case, dt)
            if path == "dropin":
                lam, v, _, itr, _ = ev.similarity_transform_ex(
                    mat, eps=eps, semantics=sem, matrix_free=form == "mfree", batch=batch,
                    max_itr=max_itr, write_every_round=form == "every", trace_sums=True)
                sums = ev.last_round_sums()
            else:
                t = torch.from_numpy(mat).to("cuda:0")
                lam, v, itr, _ = solver.solve(t, eps=eps, semantics=sem,
                                              matrix_free=form == "mfree", batch=batch,
                                              max_itr=max_itr,
                                              write_every_round=form == "every",
                                              trace_sums=True)
                sums = solver.last_round_sums()
                v = v.cpu().numpy()
                del t
            ref = orc.similarity_transform(mat, sem, eps=dt(eps), max_itr=max_itr,
                                           nthreads=16, trace=True)
            key = "f64" if dt == np.float64 else "f32"
            cmp = sp.compare(sums, ref.row_sums, dt(eps), sem == 0, max_itr,
                             matrix_free=form == "mfree")
            out["dev_ulps_max"][key] = max(out["dev_ulps_max"][key], cmp["max_dev_ulps"])
            if form != "mfree":
                out["dev_ulps_max_transform"][key] = max(out["dev_ulps_max_transform"][key],
                                                         cmp["max_dev_ulps"])
            try:
                must_match = sp.assert_stop_parity(cmp, case)
                trace_ok = True
            except AssertionError as e:
                must_match, trace_ok = True, False
                print(f"TRACE CHECK FAILED {e}", flush=True)
            if not must_match:
                out["straddles"].append({"case": case, "n": n, "dtype": key, "sem": sem,
                                         "eps": eps, "kind": kind, "form": form,
                                         "iters": int(itr), "iters_oracle": int(ref.iter_count),
                                         **cmp["straddle"]})
                print(f"STRADDLE {out['straddles'][-1]}", flush=True)
                continue
            el = abs(float(lam) - float(ref.eigen_val)) / max(abs(float(ref.eigen_val)), 1e-300)
            evv = float(np.max(np.abs(np.asarray(v, dtype=np.float64) - ref.eigen_vec)))
            tol_l, tol_v = (1e-10, 1e-10) if key == "f64" else (2e-5, 5e-4)
            ok = trace_ok and itr == ref.iter_count and el <= tol_l and evv <= tol_v
            worst[key]["lam"] = max(worst[key]["lam"], el)
            worst[key]["v"] = max(worst[key]["v"], evv)
            rec = {"case": case, "n": n, "dtype": key, "sem": sem, "form": form, "batch": batch,
                   "eps": eps, "kind": kind, "path": path, "iters": int(itr),
                   "iters_oracle": int(ref.iter_count), "lam_rel_err": el, "v_max_err": evv,
                   "dev_ulps_max": cmp["max_dev_ulps"], "ok": bool(ok)}
            out["cases"].append(rec)
            print(json.dumps(rec), flush=True)
            if not ok:
                print(f"MISMATCH {rec}", flush=True)
    solver.close()
    out["worst"] = worst
    out["n_cases"] = len(out["cases"])
    out["n_ok"] = sum(c["ok"] for c in out["cases"])
    out["seconds"] = round(time.time() - t0, 1)
    out["straddles_by_eps"] = {str(e): sum(1 for c in out["straddles"] if c["eps"] == e)
                               for e in (1e-3, 1e-6, 1e-2)}
    # the fp32 random cases the reference's own shape covers (N >= 200,
    # wrapper/python/test.py), per eps
    out["f32_random_n200_checked"] = {
        str(e): sum(1 for c in out["cases"] if c["dtype"] == "f32" and c["kind"] == "random"
                    and c["n"] >= 200 and c["eps"] == e) for e in (1e-3, 1e-6, 1e-2)}
    print(f"{out['n_ok']} / {out['n_cases']} cases match the oracle "
          f"({len(out['straddles'])} straddling stops excused); worst {worst}; "
          f"row-sum deviation {out['dev_ulps_max']} ulps; fp32 random N>=200 checked "
          f"{out['f32_random_n200_checked']}", flush=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=0)
    return 0 if out["n_ok"] == out["n_cases"] else 1


if __name__ == "__main__":
    sys.exit(main())
