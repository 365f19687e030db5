"""The CPU oracle's reference-semantics solves of the BASELINE full-size
random inputs, committed as golden outputs (parity at the
full sizes against the oracle, not only through properties).

    python tests/golden/make_large_oracle.py        # ~2 min on 8 cores

Each case runs oracle.similarity_transform_gen (oracle/st_oracle.c
orc_similarity_transform_gen_*): the SYCL loop of similarity_transform.cpp:
39-53 with the cyclic stop of :413-421 and the count of :54, on the seeded
splitmix64 matrix, regenerated in row blocks every round so that 65536^2
fp64 (32 GiB, configs[3]) never has to fit the host; it is bit-identical to
the plain oracle loop (tests/test_oracle.py::test_generated_solve_bit_
identical).  Cases:

* configs[2] 32768^2 fp64, EPS = 1e-3: to convergence;
* configs[4] 32768^2 fp32: 8 fixed rounds (at the reference's EPS = 1e-3f the
  fp32 iteration never stops at this size), so max_itr = 8;
* configs[3] 65536^2 fp64, EPS = 1e-3: to convergence.

Writes tests/golden/large_oracle.json (iteration counts, λ, eigenvector
summaries) and large_oracle_v.npz (the eigenvectors).
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import oracle  # noqa: E402

CASES = [  # (name, n, dtype, eps, max_itr)
    ("random32768_f64", 32768, np.float64, 1e-3, 64),
    ("random32768_f32_8rounds", 32768, np.float32, 1e-3, 8),
    ("random65536_f64", 65536, np.float64, 1e-3, 64),
]


def main():
    res = {"_comment": __doc__.strip().splitlines()[0],
           "semantics": "SYCL (cyclic stop, A*((1/s_r)*s_c), iter_count = break index)",
           "seed": 0, "kind": "random", "cases": {}}
    vecs = {}
    for name, n, dt, eps, max_itr in CASES:
        t0 = time.time()
        r = oracle.similarity_transform_gen("random", n, 0, dt, oracle.SEM_SYCL,
                                            eps=dt(eps), max_itr=max_itr, chunk_rows=1024)
        v = r.eigen_vec
        res["cases"][name] = {
            "n": n, "dtype": "f64" if dt == np.float64 else "f32", "eps": eps,
            "max_itr": max_itr, "iter_count": r.iter_count,
            "rounds_evaluated": r.rounds_evaluated, "eigen_val": float(r.eigen_val),
            "v_sum": float(np.sum(v, dtype=np.float64)), "v_min": float(v.min()),
            "v_max": float(v.max())}
        vecs[name] = v
        print(name, res["cases"][name], f"{time.time() - t0:.1f}s", flush=True)
    json.dump(res, open(os.path.join(HERE, "large_oracle.json"), "w"), indent=1)
    np.savez_compressed(os.path.join(HERE, "large_oracle_v.npz"), **vecs)
    print("wrote large_oracle.json, large_oracle_v.npz")


if __name__ == "__main__":
    main()
