"""Generate golden vectors by running the reference's own sequential
implementation (/root/reference/main.py, fp64 numpy) on seeded inputs.

Run in the build container only (the reference does not exist on the GPU
box):  python tests/golden/make_golden.py

Writes tests/golden/mainpy_golden.json (index + scalars) and
tests/golden/mainpy_golden.npz (eigenvectors).  Inputs are NOT stored: they
are regenerated bit-identically from (kind, n, seed) by oracle.hilbert /
oracle.random_matrix, except the literal 3x3 known-answer matrix
(main.py:53, tests/test.cpp:84-94).
"""
import importlib.util
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.dont_write_bytecode = True  # never write a .pyc into /root/reference

from oracle import oracle  # noqa: E402

REF_MAIN = "/root/reference/main.py"


def load_reference_main():
    spec = importlib.util.spec_from_file_location("reference_main", REF_MAIN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)   # __main__ guard (main.py:50) skips the sweep
    return mod


def cases():
    yield "kat3", "literal", 3, 0, np.array([[1, 1, 2], [2, 1, 3], [2, 3, 5]])
    for n in (1, 2, 8, 32, 64, 100, 128, 256, 333, 512, 1024, 2048):
        yield f"hilbert{n}", "hilbert", n, 0, oracle.hilbert(n, np.float64)
    for n, seed in ((4, 1), (16, 0), (64, 0), (127, 3), (256, 0), (513, 7), (1024, 0), (1024, 1)):
        yield f"random{n}_s{seed}", "random", n, seed, oracle.random_matrix(n, seed, np.float64)


def main():
    ref = load_reference_main()
    index, vecs = {}, {}
    for name, kind, n, seed, mat in cases():
        t0 = time.time()
        val, vec, itr = ref.max_eigen_value_and_vector(mat)
        dt = time.time() - t0
        true_max = float(np.max(np.linalg.eigvals(mat.astype(np.float64)).real))
        index[name] = dict(kind=kind, n=n, seed=seed, eigen_val=float(val),
                           eigen_val_hex=float(val).hex(), itr=int(itr),
                           numpy_max_eig=true_max, ref_seconds=round(dt, 3))
        vecs[name] = np.asarray(vec, dtype=np.float64)
        print(f"{name:>16}  λ={float(val)!r:<22} itr={itr:<3} "
              f"rel(np)={abs(val - true_max) / true_max:.2e}  {dt:.2f}s", flush=True)
    meta = dict(generator="tests/golden/make_golden.py",
                reference="/root/reference/main.py:30-47 (max_eigen_value_and_vector)",
                numpy=np.__version__, cases=index)
    with open(os.path.join(HERE, "mainpy_golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    np.savez_compressed(os.path.join(HERE, "mainpy_golden.npz"), **vecs)


if __name__ == "__main__":
    main()
