"""Per-round stop-decision parity between a device solve and the oracle.

TEST INFRASTRUCTURE (imported by tests/ and tools/fuzz_parity.py only).

The reference stops at the first round k whose row sums satisfy
|s_k[i] - s_k[i+1]| < EPS for every inspected pair (cyclic in
similarity_transform.cpp:413-421, open in main.py:25-27).  The GPU and the
oracle sum rows in different orders (wave trees vs numpy's pairwise order),
so their s_k differ by a few ulps of the row sums, and a round whose
max |Δs| lies that close to EPS can stop on one side and not on the other.
That is a legitimate fp rounding difference only when the two solves' OWN
row sums put max |Δs| on opposite sides of EPS, so the check works from
both traces (the library's ST_FLAG_TRACE_SUMS and the oracle's
``trace=True``), never from a window around EPS:

* each solve's stop round must be the first round whose traced s_k passes
  the stop test, computed here in the solve's dtype exactly as the kernels
  and ``orc_stop`` do (self-consistency of the traces);
* per round k, the row sums must agree to ``DEV_ULPS + k`` ulps of
  max s_k: each round's matrix is built from the previous round's sums,
  so the two solves' rounding differences compound - slowly.  Measured
  over 3300 cases (``profiles/r06_fuzz_parity_*.json``): at most 8 ulps in
  fp64 and 12 in fp32 within the first 20 rounds; over 200 non-converging
  fp32 rounds the transform forms drift by up to ~0.2 ulp per round and
  the matrix-free form, which evaluates s_k = (A_0 x) ⊘ x - a different
  rounding path from the transform the oracle runs - by up to ~0.6;
* if no round straddles EPS, the two solves stop in the same round (the
  iteration counts are equal); otherwise the first straddling round is
  reported with its margin |max|Δs|_oracle - EPS|, which the measured row
  sum deviation bounds (margin <= max|Δs|_gpu - max|Δs|_oracle| <= 2 dev).
"""
from __future__ import annotations

from typing import Optional

import numpy as np

# row sums of the device and the oracle agree within DEV_ULPS + k ulps of
# round k's largest row sum (stated bound; the sweeps record the measured
# deviations)
DEV_ULPS = 16


def max_dsum(s: np.ndarray, cyclic: bool):
    """max |s[i] - s[i+1]| over the pairs the stop test inspects, in s's dtype."""
    if s.size < 2:
        return s.dtype.type(0) if not cyclic else s.dtype.type(abs(s[0] - s[0]))
    d = np.abs(s[:-1] - s[1:])
    m = d.max()
    if cyclic:
        m = max(m, np.abs(s[-1] - s[0]))
    return s.dtype.type(m)


def stops(s: np.ndarray, eps, cyclic: bool) -> bool:
    """The stop test in the dtype (!(|d| < eps) fails, as orc_stop / the kernels)."""
    e = s.dtype.type(eps)
    if s.size < 2 and not cyclic:
        return True
    return bool(max_dsum(s, cyclic) < e)


def first_stop(sums: np.ndarray, eps, cyclic: bool) -> Optional[int]:
    for k in range(sums.shape[0]):
        if stops(sums[k], eps, cyclic):
            return k
    return None


def compare(gpu_sums: np.ndarray, orc_sums: np.ndarray, eps, cyclic: bool,
            max_itr: int, matrix_free: bool = False) -> dict:
    """Check two traces (shape (rounds, n), one row per evaluated round) and
    return a summary:
      consistent  both traces stop where their solves stopped
      straddle    None, or {round, dmax_gpu, dmax_oracle, margin, dev} of the
                  first round whose decisions differ
      same_stop   the solves stopped in the same round (=> equal counts)
      dev_ulps    per compared round, max |s_gpu - s_oracle| / ulp(max s)
      dev_excess  rounds k whose deviation exceeds DEV_ULPS + k ulps
    A solve that ran out of rounds evaluated max_itr rounds and stopped in
    none of them."""
    out = {"rounds_gpu": int(gpu_sums.shape[0]), "rounds_oracle": int(orc_sums.shape[0])}
    ok = True
    for name, tr in (("gpu", gpu_sums), ("oracle", orc_sums)):
        k = first_stop(tr, eps, cyclic)
        r = tr.shape[0]
        # a converged solve stops in its last evaluated round; an exhausted
        # one evaluated max_itr rounds and passed none
        ok &= (k == r - 1) if k is not None else (r == max_itr)
    out["consistent"] = bool(ok)
    rounds = min(gpu_sums.shape[0], orc_sums.shape[0])
    dev_ulps, straddle = [], None
    for k in range(rounds):
        g, o = gpu_sums[k], orc_sums[k]
        ulp = float(np.spacing(np.abs(o).max().astype(o.dtype)))
        dev = float(np.max(np.abs(g.astype(np.float64) - o.astype(np.float64))))
        dev_ulps.append(dev / ulp if ulp > 0 else 0.0)
        if straddle is None and stops(g, eps, cyclic) != stops(o, eps, cyclic):
            dg, do = float(max_dsum(g, cyclic)), float(max_dsum(o, cyclic))
            straddle = {"round": k, "dmax_gpu": dg, "dmax_oracle": do,
                        "margin": abs(do - float(o.dtype.type(eps))), "dev": dev}
    out["dev_ulps"] = [round(x, 2) for x in dev_ulps]
    out["dev_excess"] = [k for k, x in enumerate(dev_ulps) if x > DEV_ULPS + k]
    out["matrix_free"] = bool(matrix_free)
    out["max_dev_ulps"] = round(max(dev_ulps), 2) if dev_ulps else 0.0
    out["straddle"] = straddle
    out["same_stop"] = gpu_sums.shape[0] == orc_sums.shape[0]
    return out


def assert_stop_parity(cmp: dict, tag=None) -> bool:
    """Assert what ``compare`` found is legitimate; returns True when the
    counts must agree (no straddle), False for a reported straddle."""
    assert cmp["consistent"], ("trace does not stop where its solve stopped", tag, cmp)
    assert not cmp["dev_excess"], ("row sums deviate", tag, cmp)
    st = cmp["straddle"]
    if st is None:
        assert cmp["same_stop"], ("no straddling round, yet different stop rounds", tag, cmp)
        return True
    # the margin the flip needed is covered by the measured deviation
    # (plus the rounding of the two |Δs| subtractions)
    slack = 4.0 * float(np.spacing(np.float32(max(st["dmax_oracle"], 1e-30))))
    assert st["margin"] <= 2.0 * st["dev"] + slack, ("unexplained straddle", tag, cmp)
    return False
