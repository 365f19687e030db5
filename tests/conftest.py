"""Shared pytest setup.

Markers: ``gpu`` — needs an MI355X (run with ``-m gpu`` on the GPU box);
everything else runs on CPU (oracle vs golden vectors, host logic, C-ABI
exports, gloo world_size-2 sharding).
"""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X)")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    here = os.path.join(REPO, "tests", "golden")
    meta = json.load(open(os.path.join(here, "mainpy_golden.json")))
    vecs = np.load(os.path.join(here, "mainpy_golden.npz"))
    pins = json.load(open(os.path.join(here, "reference_pins.json")))
    return meta["cases"], {k: vecs[k] for k in vecs.files}, pins


def golden_input(case, orc):
    import numpy as np
    if case["kind"] == "literal":
        return np.array([[1, 1, 2], [2, 1, 3], [2, 3, 5]], dtype=np.float64)
    if case["kind"] == "hilbert":
        return orc.hilbert(case["n"], np.float64)
    return orc.random_matrix(case["n"], case["seed"], np.float64)


def large_pin(n, dtype, seed=0):
    """True Perron root of a full-size seeded random matrix
    (tests/golden/large_pins.json, make_large_pins.py)."""
    import json
    doc = json.load(open(os.path.join(REPO, "tests", "golden", "large_pins.json")))
    for c in doc["cases"]:
        if (c["n"], c["dtype"], c["seed"]) == (n, dtype, seed):
            return c
    raise KeyError((n, dtype, seed))


def large_oracle(name):
    """The oracle's reference-semantics solve of a full-size seeded random
    input (tests/golden/large_oracle.json + large_oracle_v.npz,
    make_large_oracle.py): (case dict, eigenvector)."""
    import json

    import numpy as np
    here = os.path.join(REPO, "tests", "golden")
    doc = json.load(open(os.path.join(here, "large_oracle.json")))
    with np.load(os.path.join(here, "large_oracle_v.npz")) as z:
        return doc["cases"][name], z[name]


def host_threads() -> int:
    """CPUs the oracle may use on this host: the affinity mask bounded by the
    cgroup quota and OMP_NUM_THREADS (bench.host_info)."""
    import bench
    return bench.host_info()["threads"]
