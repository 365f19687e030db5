"""True Perron roots of the BASELINE full-size random matrices, computed on
the CPU and committed as scalars (SURVEY.md §8c "Large-N numpy reference":
np.linalg.eigvals is infeasible at these sizes).

    python tests/golden/make_large_pins.py        # ~10 min on 8 cores

For each (n, dtype, seed) the matrix is regenerated bit-identically by the
oracle's C generator (oracle/st_oracle.c orc_random_*, the same splitmix64
bits as the HIP generator), in row chunks, and a plain fp64 power iteration
runs until the Collatz–Wielandt bracket
    min_i (A x)_i / x_i  <=  lambda_true  <=  max_i (A x)_i / x_i
(valid for any positive x and positive A) is tighter than 1e-13 relative.
The fp32 matrix (configs[4]) is the fp32 generator's values, iterated in
fp64.  Writes tests/golden/large_pins.json.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

from oracle import oracle  # noqa: E402

CHUNK_BYTES = 1 << 30


def gen_rows(n, dtype, seed, row0, nrows, out):
    fn = getattr(oracle.lib(), "orc_random_f64" if dtype == "f64" else "orc_random_f32")
    fn(out.ctypes.data_as(ctypes.c_void_p), nrows, n, row0, seed)


def matvec(n, dtype, seed, x, cache):
    """A @ x in fp64, A regenerated per chunk unless it fits the cache."""
    npdt = np.float64 if dtype == "f64" else np.float32
    if cache is not None:  # fp64 values of the matrix
        return cache @ x
    rows = max(1, CHUNK_BYTES // (n * np.dtype(npdt).itemsize))
    y = np.empty(n, np.float64)
    buf = np.empty((rows, n), npdt)
    for r0 in range(0, n, rows):
        nr = min(rows, n - r0)
        gen_rows(n, dtype, seed, r0, nr, buf[:nr])
        blk = buf[:nr] if dtype == "f64" else buf[:nr].astype(np.float64)
        y[r0:r0 + nr] = blk @ x
    return y


def perron(n, dtype, seed, keep_bytes=16 << 30):
    t0 = time.time()
    npdt = np.float64 if dtype == "f64" else np.float32
    cache = None
    if n * n * 8 <= keep_bytes:
        gen = np.empty((n, n), npdt)
        gen_rows(n, dtype, seed, 0, n, gen)
        cache = gen if dtype == "f64" else gen.astype(np.float64)
        del gen
    x = np.ones(n, np.float64)
    hist = []
    for it in range(1, 40):
        y = matvec(n, dtype, seed, x, cache)
        q = y / x
        lo, hi = float(q.min()), float(q.max())
        hist.append((it, lo, hi))
        print(f"  n={n} {dtype} it={it} lo={lo!r} hi={hi!r} rel={(hi - lo) / hi:.3e} "
              f"({time.time() - t0:.0f}s)", flush=True)
        x = y / np.max(y)
        if (hi - lo) / hi < 1e-13:
            break
    del cache
    return {"n": n, "dtype": dtype, "seed": seed, "kind": "random",
            "lambda": 0.5 * (lo + hi), "cw_lo": lo, "cw_hi": hi,
            "cw_rel_width": (hi - lo) / hi, "power_iterations": it,
            "v_min_over_max": float(np.min(x)),
            "method": "fp64 power iteration from ones, Collatz-Wielandt bracket"}


def main():
    out = os.path.join(HERE, "large_pins.json")
    cases = [(32768, "f64", 0), (32768, "f32", 0), (65536, "f64", 0)]
    res = {"_comment": __doc__.strip().splitlines()[0], "cases": []}
    for n, dt, seed in cases:
        res["cases"].append(perron(n, dt, seed))
        json.dump(res, open(out, "w"), indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
