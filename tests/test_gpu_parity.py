"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Tolerances (stated here):
  * generators, the D^-1 A D element update: BIT-exact;
  * fp64 solves vs the oracle with the same semantics: iteration count equal,
    λ relative <= 1e-10, eigenvector max-abs <= 1e-10 (summation order
    differs: tree on the GPU, numpy pairwise in the oracle);
  * fp64 ST_SEM_MAINPY solves vs the reference's main.py golden vectors:
    iteration count equal, λ relative <= 1e-12, eigenvector max-abs <= 1e-12;
  * fp32: iteration counts equal to the reference's published counts
    (README.md:70-76), λ relative <= 1e-5.
"""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no HIP device", allow_module_level=True)

import eigen_value_amd as ev  # noqa: E402
from eigen_value_amd import _lib  # noqa: E402
from eigen_value_amd import device as dev  # noqa: E402
from conftest import golden_input, large_pin  # noqa: E402

DEV = "cuda:0"
TD = {np.float64: torch.float64, np.float32: torch.float32}


@pytest.fixture(scope="module")
def eigen():
    e = ev.EigenValue()
    yield e
    e.close()


@pytest.fixture(scope="module")
def solver():
    s = dev.DeviceSolver(DEV)
    yield s
    s.close()


def to_np(t):
    torch.cuda.synchronize()
    return t.cpu().numpy()


# ---------------------------------------------------------------------------
# generators
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("n,nrows,row0", [(1, 1, 0), (7, 7, 0), (130, 17, 33), (1000, 3, 997)])
def test_generators_bitexact(orc, dt, n, nrows, row0):
    h = dev.generate("hilbert", n, TD[dt], nrows=nrows, row0=row0, device=DEV)
    assert np.array_equal(to_np(h), orc.hilbert(n, dt, nrows=nrows, row0=row0))
    r = dev.generate("random", n, TD[dt], nrows=nrows, row0=row0, seed=42, device=DEV)
    assert np.array_equal(to_np(r), orc.random_matrix(n, 42, dt, nrows=nrows, row0=row0))
    i = dev.generate("identity", n, TD[dt], nrows=nrows, row0=row0, device=DEV)
    assert np.array_equal(to_np(i), np.eye(n, dtype=dt)[row0:row0 + nrows])


# ---------------------------------------------------------------------------
# per-kernel pins: tests/test.cpp:22-73
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_kernel_unit_pins(dt):
    n = 1024
    eye = dev.generate("identity", n, TD[dt], device=DEV)
    assert np.all(to_np(dev.rowsum(eye)) == 1.0)                 # test.cpp:22-30
    s = torch.arange(1, n + 1, dtype=TD[dt], device=DEV)
    v = torch.ones(n, dtype=TD[dt], device=DEV)
    state = dev.new_state(DEV)
    dev.epilogue(s, v, state, eps=1e-3, max_itr=1000)
    st = dev.read_state(state)
    assert st["max"] == n                                          # test.cpp:32-41
    assert np.max(np.abs(to_np(s) / n - to_np(v))) == 0.0         # test.cpp:43-54
    assert st["stop"] == 0 and st["done"] == 0 and st["round"] == 1
    ok = torch.full((n,), float(np.float32(1) + np.float32(1e-4)), dtype=TD[dt], device=DEV)
    dev.reset_state(state)
    dev.epilogue(ok, None, state, eps=1e-3)
    assert dev.read_state(state)["stop"] == 1                      # test.cpp:56-64
    fail = (torch.arange(n, dtype=TD[dt], device=DEV) + 1) * float(np.float32(1e-4))
    dev.reset_state(state)
    dev.epilogue(fail, None, state, eps=1e-3)
    assert dev.read_state(state)["stop"] == 0                      # test.cpp:66-73 (cyclic)
    dev.reset_state(state)
    dev.epilogue(fail, None, state, eps=1e-3, semantics=_lib.ST_SEM_MAINPY)
    assert dev.read_state(state)["stop"] == 1                      # main.py:25-27


# ---------------------------------------------------------------------------
# row sums and the fused round body
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("nrows,ncols", [(1, 1), (5, 3), (37, 1001), (2051, 256), (4100, 515), (64, 8192)])
def test_rowsum_vs_oracle(orc, dt, nrows, ncols):
    a = orc.random_matrix(ncols, 7, dt, nrows=nrows)
    got = to_np(dev.rowsum(torch.from_numpy(a).to(DEV)))
    ref = orc.rowsum(a)
    tol = 1e-13 if dt == np.float64 else 2e-6
    assert np.max(np.abs(got - ref) / np.abs(ref)) <= tol


@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("nrows,ncols", [(1, 1), (5, 3), (37, 1001), (2051, 256), (333, 8200),
                                         (1031, 4099), (64, 12288)])
def test_rowsum_flat_vs_oracle(orc, dt, nrows, ncols):
    """K0 in the flat form (st_rowsum_flat: k_flat_sum + k_parts), the solve
    loops' initial row sums wherever the flat round pays, at any shape -
    ragged pieces, odd row counts, columns no multiple of the vector width
    (similarity_transform.cpp:40, the first sum_across_rows): against the
    oracle to rounding, and bit for bit the flat round's own sums of the
    same matrix (a round with unit scales leaves A unchanged: x·((1/1)·1) =
    x), and partition-independent: any row block's sums equal the same rows'
    sums in the whole block."""
    a = orc.random_matrix(ncols, 11, dt, nrows=nrows)
    ta = torch.from_numpy(a).to(DEV)
    part = dev.flat_scratch(nrows, ncols, TD[dt], DEV)
    got = torch.empty(nrows, dtype=TD[dt], device=DEV)
    dev.rowsum_flat(ta, got, part)
    got = to_np(got)
    ref = orc.rowsum(a)
    tol = 1e-13 if dt == np.float64 else 2e-6
    assert np.max(np.abs(got - ref) / np.abs(ref)) <= tol
    # the flat round's sums, unit scales (a row block inside the s vector)
    if nrows <= ncols:
        ones = torch.ones(ncols, dtype=TD[dt], device=DEV)
        s_next = torch.empty(nrows, dtype=TD[dt], device=DEV)
        v = torch.ones(ncols, dtype=TD[dt], device=DEV)
        dev.flat_round(ta, ones, s_next, part, v, dev.new_state(DEV), eps=0.0, k=0)
        assert np.array_equal(to_np(ta), a)
        assert np.array_equal(to_np(s_next), got)
    # a row block of the same columns
    r0, r1 = nrows // 3, nrows // 3 + max(1, nrows // 2)
    sub = torch.from_numpy(np.ascontiguousarray(a[r0:r1])).to(DEV)
    got_sub = torch.empty(r1 - r0, dtype=TD[dt], device=DEV)
    dev.rowsum_flat(sub, got_sub, dev.flat_scratch(r1 - r0, ncols, TD[dt], DEV))
    assert np.array_equal(to_np(got_sub), got[r0:r1])


@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("sem", [_lib.ST_SEM_SYCL, _lib.ST_SEM_MAINPY])
@pytest.mark.parametrize("nrows,ncols,row0", [(3, 3, 0), (64, 257, 100), (2050, 4096, 1000), (4099, 4100, 1)])
def test_fused_step_vs_oracle(orc, dt, sem, nrows, ncols, row0):
    n_full = max(ncols, row0 + nrows)
    a = orc.random_matrix(ncols, 3, dt, nrows=nrows)
    s_full = (orc.random_matrix(n_full, 9, dt, nrows=1)[0] + dt(0.5)).astype(dt)
    ta = torch.from_numpy(a).to(DEV)
    ts = torch.from_numpy(s_full).to(DEV)
    s_next = torch.empty(nrows, dtype=TD[dt], device=DEV)
    dev.scale_rowsum(ta, ts, s_next, row0=row0, semantics=sem)
    got = to_np(ta)
    ref = orc.compute_next(a, s_full, row0=row0, order=0 if sem == _lib.ST_SEM_SYCL else 1)
    assert np.array_equal(got, ref)                    # element update is bit-exact
    ref_s = orc.rowsum(ref)
    tol = 1e-13 if dt == np.float64 else 2e-6
    assert np.max(np.abs(to_np(s_next) - ref_s) / np.abs(ref_s)) <= tol


@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("sem", [_lib.ST_SEM_SYCL, _lib.ST_SEM_MAINPY])
@pytest.mark.parametrize("nrows,ncols,row0", [(1, 1, 0), (3, 3, 0), (7, 257, 100), (1025, 2048, 1000),
                                              (2049, 3000, 0), (1500, 1500, 0)])
def test_round_kernel_vs_oracle(orc, dt, sem, nrows, ncols, row0):
    """st_round_*: stats of s_k, v update of the local rows, transform, s_{k+1}."""
    n_full = max(ncols, row0 + nrows)
    a = orc.random_matrix(ncols, 3, dt, nrows=nrows)
    s_full = (orc.random_matrix(n_full, 9, dt, nrows=1)[0] + dt(0.5)).astype(dt)[:ncols]
    s_full = np.ascontiguousarray(s_full)
    v0 = orc.random_matrix(n_full, 5, dt, nrows=1)[0]
    ta, ts, tv = (torch.from_numpy(x).to(DEV) for x in (a, s_full, v0))
    s_next = torch.empty(nrows, dtype=TD[dt], device=DEV)
    state = dev.new_state(DEV)
    if row0 + nrows > ncols:
        pytest.skip("row block must lie inside the s vector")
    dev.fused_round(ta, ts, s_next, tv, state, row0=row0, eps=1e-3, k=0, semantics=sem)
    order = 0 if sem == _lib.ST_SEM_SYCL else 1
    ref = orc.compute_next(a, s_full, row0=row0, order=order)
    assert np.array_equal(to_np(ta), ref)
    ref_s = orc.rowsum(ref)
    tol = 1e-13 if dt == np.float64 else 2e-6
    assert np.max(np.abs(to_np(s_next) - ref_s) / np.abs(ref_s)) <= tol
    m = orc.find_max(s_full)
    vref = v0.copy()
    vref[row0:row0 + nrows] = orc.compute_eigen_vector(s_full[row0:row0 + nrows], m,
                                                       v0[row0:row0 + nrows])
    assert np.array_equal(to_np(tv), vref)                 # untouched outside the block
    st = dev.read_state(state)
    assert st["max"] == m and st["eigen_val"] == s_full[0] and st["round"] == 0
    assert st["stop"] == int(orc.stop(s_full, eps=dt(1e-3), cyclic=sem == _lib.ST_SEM_SYCL))


@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("sem", [_lib.ST_SEM_SYCL, _lib.ST_SEM_MAINPY])
@pytest.mark.parametrize("nrows,ncols,row0", [(1, 1, 0), (3, 3, 0), (7, 257, 100), (1025, 2048, 1000),
                                              (2049, 3000, 0), (1500, 1501, 0),
                                              # fp64: >= 384 MiB, the every-round launch's
                                              # tiles of 8 rows, a ragged last tile
                                              (6203, 8192, 0)])
def test_flat_round_vs_round(orc, dt, sem, nrows, ncols, row0):
    """st_round_flat_* (k_stats + k_flat + k_parts) against st_round_* and the
    oracle: A_{k+1} and v bit for bit, the state identical, s_{k+1} to
    rounding (pieces summed apart)."""
    if row0 + nrows > ncols:
        pytest.skip("row block must lie inside the s vector")
    a = orc.random_matrix(ncols, 3, dt, nrows=nrows)
    s_full = np.ascontiguousarray((orc.random_matrix(ncols, 9, dt, nrows=1)[0]
                                   + dt(0.5)).astype(dt))
    v0 = orc.random_matrix(ncols, 5, dt, nrows=1)[0]
    outs = []
    for flat in (False, True):
        ta, ts, tv = (torch.from_numpy(x).to(DEV) for x in (a, s_full, v0))
        s_next = torch.empty(nrows, dtype=TD[dt], device=DEV)
        state = dev.new_state(DEV)
        if flat:
            part = dev.flat_scratch(nrows, ncols, TD[dt], DEV)
            dev.flat_round(ta, ts, s_next, part, tv, state, row0=row0, eps=1e-3, k=2,
                           semantics=sem)
        else:
            dev.fused_round(ta, ts, s_next, tv, state, row0=row0, eps=1e-3, k=2, semantics=sem)
        outs.append((to_np(ta), to_np(s_next), to_np(tv), dev.read_state(state)))
    (a0, s0, v0_, st0), (a1, s1, v1, st1) = outs
    ref = orc.compute_next(a, s_full, row0=row0, order=0 if sem == _lib.ST_SEM_SYCL else 1)
    assert np.array_equal(a1, ref) and np.array_equal(a1, a0)
    assert np.array_equal(v1, v0_) and st1 == st0
    tol = 1e-13 if dt == np.float64 else 2e-6
    ref_s = orc.rowsum(ref)
    assert np.max(np.abs(s1 - ref_s) / np.abs(ref_s)) <= tol


def test_flat_round_stats_and_gating(orc):
    """k_stats: max ignores negatives and NaN (find_max starts at 0), a NaN
    pair fails the stop test, the stopping round sets end = k+1 and later
    flat rounds are no-ops; the scratch words are left zeroed."""
    n = 700
    a = torch.from_numpy(orc.random_matrix(n, 1)).to(DEV)
    s = torch.full((n,), 4.0, dtype=torch.float64, device=DEV)     # constant: stops
    s_next = torch.empty_like(s)
    v = torch.ones_like(s)
    part = dev.flat_scratch(n, n, torch.float64, DEV)
    state = dev.new_state(DEV)
    dev.flat_round(a, s, s_next, part, v, state, k=0)
    st = dev.read_state(state)
    assert st["stop"] == 1 and st["done"] == 1 and st["end"] == 1 and st["max"] == 4.0
    keep = a.clone()
    dev.flat_round(a, s * 2.0, s_next, part, v, state, k=1)       # gated
    assert torch.equal(a, keep)
    raw = _lib.st_state.from_buffer_copy(state.cpu().numpy().tobytes())
    assert raw.arrivals == 0 and raw.max_bits == 0 and raw.fail == 0
    s2 = torch.full((n,), 2.0, dtype=torch.float64, device=DEV)
    s2[5], s2[6] = -7.0, float("nan")
    state2 = dev.new_state(DEV)
    dev.flat_round(a, s2, s_next, part, v, state2, k=0, max_itr=10)
    st2 = dev.read_state(state2)
    assert st2["max"] == 2.0 and st2["stop"] == 0 and st2["done"] == 0


def test_round_stop_and_gating(orc):
    n = 600
    a = torch.from_numpy(orc.random_matrix(n, 1)).to(DEV)
    keep = a.clone()
    s = torch.full((n,), 4.0, dtype=torch.float64, device=DEV)   # constant: stops at once
    s_next = torch.empty_like(s)
    v = torch.ones_like(s)
    state = dev.new_state(DEV)
    dev.fused_round(a, s, s_next, v, state, k=0)
    st = dev.read_state(state)
    assert st["stop"] == 1 and st["done"] == 1 and st["end"] == 1 and st["iters"] == 0
    after = a.clone()
    assert torch.equal(after, keep)           # D^-1 A D with constant s is the identity map
    dev.fused_round(a, s * 2.0, s_next, v, state, k=1)    # a later round: no-op
    assert torch.equal(a, after) and dev.read_state(state)["end"] == 1
    # max_itr exhaustion on round k = max_itr - 1
    state2 = dev.new_state(DEV)
    s2 = torch.from_numpy(orc.random_matrix(n, 2, nrows=1)[0] + 1.0).to(DEV)
    dev.fused_round(a, s2, s_next, v, state2, k=4, max_itr=5)
    st2 = dev.read_state(state2)
    assert st2["done"] == 1 and st2["stop"] == 0 and st2["iters"] == 5 and st2["end"] == 5


@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("nrows,ncols,row0", [(512, 1536, 512), (1500, 1500, 0), (7, 257, 100),
                                              (2049, 6000, 3000)])
def test_split_round_matches_round(orc, dt, nrows, ncols, row0):
    """st_round_split_* local + remote == st_round_*: A_{k+1}, v and the
    state bit for bit; s_{k+1} to rounding (two column sets summed apart),
    and bit for bit when the local set is every column."""
    a = orc.random_matrix(ncols, 3, dt, nrows=nrows)
    s_full = np.ascontiguousarray((orc.random_matrix(ncols, 9, dt, nrows=1)[0]
                                   + dt(0.5)).astype(dt))
    v0 = orc.random_matrix(ncols, 5, dt, nrows=1)[0]
    outs = []
    for col0, col1 in ((None, None), (row0, row0 + nrows), (0, ncols)):
        ta, ts, tv = (torch.from_numpy(x).to(DEV) for x in (a, s_full, v0))
        s_next = torch.empty(nrows, dtype=TD[dt], device=DEV)
        state = dev.new_state(DEV)
        if col0 is None:
            dev.fused_round(ta, ts, s_next, tv, state, row0=row0, eps=1e-3, k=3)
        else:
            part = torch.empty(nrows, dtype=TD[dt], device=DEV)
            dev.split_round(ta, ts, None, part, None, state, span=dev.SPAN_LOCAL, row0=row0,
                            col0=col0, col1=col1, eps=1e-3, k=3)
            dev.split_round(ta, ts, s_next, part, tv, state, span=dev.SPAN_REMOTE, row0=row0,
                            col0=col0, col1=col1, eps=1e-3, k=3)
        outs.append((to_np(ta), to_np(s_next), to_np(tv), dev.read_state(state)))
    base = outs[0]
    for got in outs[1:]:
        assert np.array_equal(got[0], base[0]) and np.array_equal(got[2], base[2])
        assert got[3] == base[3]
        tol = 1e-14 if dt == np.float64 else 1e-6
        assert np.max(np.abs(got[1] - base[1]) / base[1]) <= tol
    assert np.array_equal(outs[2][1], base[1])           # local = all columns


@pytest.mark.parametrize("dt", [np.float64, np.float32])
@pytest.mark.parametrize("nrows,ncols,row0,col0,col1", [
    (512, 1536, 512, 512, 1024), (1500, 1500, 0, 0, 1500), (1500, 1500, 0, 700, 700),
    (7, 257, 100, 100, 107), (2049, 6000, 3000, 3000, 5049), (300, 3001, 5, 5, 305),
    (64, 4096, 1024, 1000, 1030)])
def test_split_flat_round_matches_flat(orc, dt, nrows, ncols, row0, col0, col1):
    """st_round_split_flat_* local + remote == st_round_flat_*: A_{k+1}, v
    and the state bit for bit; s_{k+1} to rounding (a piece straddling the
    local range is summed in two parts), and bit for bit when the local
    range is every column or empty."""
    a = orc.random_matrix(ncols, 3, dt, nrows=nrows)
    s_full = np.ascontiguousarray((orc.random_matrix(ncols, 9, dt, nrows=1)[0]
                                   + dt(0.5)).astype(dt))
    v0 = orc.random_matrix(ncols, 5, dt, nrows=1)[0]
    outs = []
    for split in (False, True):
        ta, ts, tv = (torch.from_numpy(x).to(DEV) for x in (a, s_full, v0))
        s_next = torch.empty(nrows, dtype=TD[dt], device=DEV)
        state = dev.new_state(DEV)
        if split:
            part = dev.split_flat_scratch(nrows, ncols, col0, col1, TD[dt], DEV)
            part.fill_(float("nan"))              # every slot read must be written
            dev.split_flat_round(ta, ts, None, part, None, state, span=dev.SPAN_LOCAL,
                                 row0=row0, col0=col0, col1=col1, eps=1e-3, k=3)
            dev.split_flat_round(ta, ts, s_next, part, tv, state, span=dev.SPAN_REMOTE,
                                 row0=row0, col0=col0, col1=col1, eps=1e-3, k=3)
        else:
            part = dev.flat_scratch(nrows, ncols, TD[dt], DEV)
            dev.flat_round(ta, ts, s_next, part, tv, state, row0=row0, eps=1e-3, k=3)
        outs.append((to_np(ta), to_np(s_next), to_np(tv), dev.read_state(state)))
    (a0, s0, v0_, st0), (a1, s1, v1, st1) = outs
    ref = orc.compute_next(a, s_full, row0=row0)
    assert np.array_equal(a1, ref) and np.array_equal(a1, a0)
    assert np.array_equal(v1, v0_) and st1 == st0
    tol = 1e-14 if dt == np.float64 else 1e-6
    assert np.max(np.abs(s1 - s0) / s0) <= tol
    if col0 == col1 or (col0, col1) == (0, ncols):
        assert np.array_equal(s1, s0)


def test_split_flat_round_gating(orc):
    """Both halves are no-ops once a previous round stopped."""
    n = 700
    a = torch.from_numpy(orc.random_matrix(n, 1)).to(DEV)
    s = torch.full((n,), 4.0, dtype=torch.float64, device=DEV)     # constant: stops
    s_next = torch.empty_like(s)
    v = torch.ones_like(s)
    part = dev.split_flat_scratch(n, n, 100, 300, torch.float64, DEV)
    state = dev.new_state(DEV)
    for span in (dev.SPAN_LOCAL, dev.SPAN_REMOTE):
        dev.split_flat_round(a, s, s_next, part, v, state, span=span, col0=100, col1=300, k=0)
    assert dev.read_state(state)["end"] == 1
    keep, vkeep = a.clone(), v.clone()
    for span in (dev.SPAN_LOCAL, dev.SPAN_REMOTE):
        dev.split_flat_round(a, s * 3.0, s_next, part, v, state, span=span, col0=100,
                             col1=300, k=1)
    assert torch.equal(a, keep) and torch.equal(v, vkeep)


@pytest.mark.parametrize("n", [3000, 9216])
def test_sharded_overlap_single_gpu_bitwise(solver, n):
    """overlap=True at P = 1 (streams, events and the split launches; the
    gather is empty) gives bitwise the unsplit result: one-launch round at
    3000, the flat round at 9216 (648 MiB)."""
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    res = []
    for overlap in (False, True):
        sh = ShardedSimilarityTransform(n, torch.float64, overlap=overlap)
        sh.load("hilbert")
        res.append(sh.solve(eps=1e-3))
    (l0, v0, i0, r0), (l1, v1, i1, r1) = res
    assert l0 == l1 and i0 == i1 and r0 == r1 and torch.equal(v0, v1)


@pytest.mark.parametrize("n", [3000, 16384])
def test_sharded_single_gpu_matches_device_solver(solver, n):
    """P = 1 sharded driver == the library's solve loop, bit for bit, for the
    one-launch round (3000²) and the flat round (16384², 2 GiB)."""
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    sh = ShardedSimilarityTransform(n, torch.float64)
    sh.load("hilbert")
    lam, v, iters, rounds = sh.solve(eps=1e-3)
    a = dev.generate("hilbert", n, torch.float64, device=DEV)
    lam2, v2, it2, st2 = solver.solve(a)
    assert lam == lam2 and iters == it2 and rounds == st2["rounds"]
    assert torch.equal(v, v2)


@pytest.mark.parametrize("n,mf", [(3000, False), (8192, False), (8192, True), (2048, True)])
def test_sharded_rounds_fast_path_bitwise(n, mf):
    """sh.rounds(K) (pre-resolved launches, the bench's timed loop) enqueues
    exactly what K calls of sh.round() do: matrix, row sums, v and state
    bitwise, on the one-launch round, the flat round and the matrix-free
    form, including the gated rounds past a stop."""
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    out = []
    for fast in (False, True):
        sh = ShardedSimilarityTransform(n, torch.float64, matrix_free=mf)
        sh.load("hilbert")
        sh.start()
        for eps, k in ((0.0, 5), (1e-3, 30)):          # fixed rounds, then a stop
            if fast:
                sh.rounds(k, eps, 100)
            else:
                for _ in range(k):
                    sh.round(eps, 100)
        torch.cuda.synchronize()
        out.append((sh.mat.clone(), [x.clone() for x in sh.s], [x.clone() for x in sh.vb],
                    dev.read_state(sh.state), sh.k, sh.cur))
        sh.close()
    a, b = out
    assert torch.equal(a[0], b[0]) and a[3] == b[3] and a[4:] == b[4:]
    assert all(torch.equal(x, y) for x, y in zip(a[1] + a[2], b[1] + b[2]))
    assert a[3]["done"] == 1


@pytest.mark.parametrize("kw", [dict(eps=1e-3), dict(eps=0.0, max_itr=7), dict(eps=0.0, max_itr=9)])
def test_sharded_deferred_writes_bitwise(kw):
    """The sharded driver's solve with deferred writes (the default on flat
    blocks) == storing every round: λ, v, iterations and the final block."""
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    out = []
    for dw in (True, False):
        sh = ShardedSimilarityTransform(4352, torch.float64, deferred_writes=dw)
        assert sh.deferred_writes == dw
        mat = sh.load("random", seed=8)
        out.append((*sh.solve(**kw), mat.clone()))
        sh.close()
    (l0, v0, i0, r0, m0), (l1, v1, i1, r1, m1) = out
    assert l0 == l1 and i0 == i1 and r0 == r1 and torch.equal(v0, v1) and torch.equal(m0, m1)


def _gpu_gloo_worker(rank, world, port, n, outdir, overlap=False):
    import torch.distributed as dist
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = ShardedSimilarityTransform(n, torch.float64, overlap=overlap)
        sh.load("random", seed=6)
        lam, v, iters, rounds = sh.solve(eps=1e-3)
        np.save(os.path.join(outdir, f"v{rank}.npy"), v.cpu().numpy())
        np.save(os.path.join(outdir, f"m{rank}.npy"), np.array([lam, iters, rounds]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n", [2501, 9216])
def test_sharded_two_ranks_on_one_gpu(tmp_path, solver, n):
    """The row-block path with P = 2 (both ranks on cuda:0, gloo exchange)
    gives bitwise the single-GPU result: per-row sums do not depend on the
    partition and every rank derives identical m_k / stop_k.  2501: ragged
    blocks on k_round; 9216: 324 MiB blocks on the flat round (and 648 MiB
    single-GPU, also flat)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_gpu_gloo_worker, args=(2, port, n, str(tmp_path)), nprocs=2, join=True)
    a = dev.generate("random", n, torch.float64, seed=6, device=DEV)
    lam, v, it, st = solver.solve(a)
    for r in range(2):
        lam_r, it_r, rounds_r = np.load(tmp_path / f"m{r}.npy")
        assert lam_r == lam and int(it_r) == it and int(rounds_r) == st["rounds"]
        assert np.array_equal(np.load(tmp_path / f"v{r}.npy"), to_np(v))


@pytest.mark.parametrize("n", [2502, 9216])
def test_sharded_overlap_two_ranks_on_one_gpu(tmp_path, solver, n):
    """P = 2 with the overlapped exchange (communication stream, events,
    split launches; gloo on one GPU): same iterations and rounds as the
    single-GPU solve, λ and v to fp64 rounding, identical on both ranks.
    2502: 1251 rows each on the grid-stride split; 9216: 324 MiB blocks on
    the flat split."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_gpu_gloo_worker, args=(2, port, n, str(tmp_path), True), nprocs=2, join=True)
    a = dev.generate("random", n, torch.float64, seed=6, device=DEV)
    lam, v, it, st = solver.solve(a)
    v0 = np.load(tmp_path / "v0.npy")
    for r in range(2):
        lam_r, it_r, rounds_r = np.load(tmp_path / f"m{r}.npy")
        assert int(it_r) == it and int(rounds_r) == st["rounds"]
        assert abs(lam_r - lam) <= 1e-13 * lam
        vr = np.load(tmp_path / f"v{r}.npy")
        assert np.array_equal(vr, v0) and np.max(np.abs(vr - to_np(v))) <= 1e-13


def test_fused_step_is_gated_by_done(orc):
    a = orc.random_matrix(300, 1)
    ta = torch.from_numpy(a).to(DEV)
    s = torch.full((300,), 2.0, dtype=torch.float64, device=DEV)
    state = dev.new_state(DEV)
    # mark done: epilogue on a constant vector stops immediately
    dev.epilogue(s, None, state, eps=1e-3)
    assert dev.read_state(state)["done"] == 1
    dev.scale_rowsum(ta, s * 3.0, torch.empty_like(s), state=state)
    assert np.array_equal(to_np(ta), a)


def test_row_sums_independent_of_partition(orc):
    # per-row reduction order does not depend on ROWS / launch split, so a
    # row block gives bitwise the same sums as the full matrix
    a = orc.random_matrix(3000, 5)
    full = to_np(dev.rowsum(torch.from_numpy(a).to(DEV)))
    part = to_np(dev.rowsum(torch.from_numpy(a[1234:1240]).to(DEV)))
    assert np.array_equal(full[1234:1240], part)


# ---------------------------------------------------------------------------
# whole solves through the drop-in API
# ---------------------------------------------------------------------------
def test_dropin_kat3(eigen, golden):
    kat = golden[2]["kat3"]
    lam, v, ts, itr = eigen.similarity_transform(np.array(kat["matrix"], dtype=np.float32))
    assert isinstance(lam, np.float32) and v.dtype == np.float32 and ts >= 0
    assert abs(lam - kat["eigen_val"]) < kat["tol"]                # test.cpp:99
    assert np.all(np.abs(v - np.array(kat["eigen_vec"])) < kat["tol"])
    assert itr == 4


def test_dropin_hilbert_round_counts_fp32(eigen, orc, golden):
    p = golden[2]["hilbert_round_counts_fp32"]
    for n, rounds in zip(p["sizes"], p["rounds"]):
        mat = orc.hilbert(n, np.float32)
        lam, v, ts, itr = eigen.similarity_transform(mat)
        assert itr == rounds, (n, itr, rounds)                     # README.md:70-76
        ref = orc.similarity_transform(mat, orc.SEM_SYCL)
        assert abs(lam - ref.eigen_val) <= 1e-5 * ref.eigen_val
        assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-4


@pytest.mark.parametrize("kind,n", [("hilbert", 128), ("hilbert", 1000), ("hilbert", 4096),
                                    ("random", 333), ("random", 1024), ("random", 4099)])
def test_dropin_fp64_vs_oracle(eigen, orc, kind, n):
    mat = orc.hilbert(n) if kind == "hilbert" else orc.random_matrix(n, 11)
    lam, v, ts, itr = eigen.similarity_transform(mat)
    ref = orc.similarity_transform(mat, orc.SEM_SYCL)
    assert isinstance(lam, np.float64)
    assert itr == ref.iter_count
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-10


def test_mainpy_semantics_vs_reference_golden(eigen, orc, golden):
    cases, vecs, _ = golden
    for name, case in cases.items():
        mat = golden_input(case, orc)
        lam, v, ts, itr, stats = eigen.similarity_transform_ex(mat, semantics=_lib.ST_SEM_MAINPY)
        assert itr == case["itr"], name
        assert abs(lam - case["eigen_val"]) <= 1e-12 * abs(case["eigen_val"]), name
        assert np.max(np.abs(v - vecs[name])) <= 1e-12, name


def test_residual_random_fp32(eigen):
    # wrapper/python/test.py:3-18: DIM = 1024, 4 runs, A v ≈ λ v (atol 1e-3)
    rng = np.random.default_rng(2021)
    mat = rng.random((1024, 1024)).astype("f")
    for _ in range(4):
        lam, v, ts, itr = eigen.similarity_transform(mat)
        assert np.all(np.isclose(mat @ v, lam * v, atol=1e-3)), "Av = λv assertion failed !"


@pytest.mark.parametrize("n", [32, 64, 128, 256, 512, 1024])
def test_random_vs_numpy_eigvals(eigen, orc, n):
    """main.py:62-70's randomized check (λ − max eig < EPS, one-sided) on the
    HIP path, two-sided, and the north star's 1e-6 relative bound once λ
    (≈ N/2) is large against the absolute EPS = 1e-3 stop (N >= 512; at
    N = 32 the reference's own stop leaves 1.5e-5), and 128² Hilbert against
    eigvalsh at the reference's EPS (≈1e-4 relative)."""
    mat = orc.random_matrix(n, 7)
    lam, v, ts, itr = eigen.similarity_transform(mat)
    true = float(np.max(np.linalg.eigvals(mat).real))
    assert abs(lam - true) < 1e-3
    if n >= 512:
        assert abs(lam - true) / true < 1e-6
    if n == 128:
        h = orc.hilbert(128)
        lam_h = eigen.similarity_transform(h)[0]
        true_h = float(np.max(np.linalg.eigvalsh(h)))
        assert abs(lam_h - true_h) / true_h < 3e-4


def test_deterministic(eigen, orc):
    mat = orc.random_matrix(2000, 4)
    a = eigen.similarity_transform(mat)
    b = eigen.similarity_transform(mat)
    assert a[0] == b[0] and np.array_equal(a[1], b[1]) and a[3] == b[3]


def test_input_not_modified(eigen, orc):
    mat = orc.hilbert(300, np.float32)
    keep = mat.copy()
    eigen.similarity_transform(mat)
    assert np.array_equal(mat, keep)       # similarity_transform.cpp:14,19


def test_dropin_input_checks(eigen, orc, solver):
    """What the reference's wrapper rejects, this one rejects the same way
    (wrapper/python/similarity_transform.py:55-57: square, float32 - float64
    added), and what it cannot express is an error, not a crash: an empty
    matrix is a negative return with a message (the reference would divide
    its work-group count by zero); a non-contiguous view is solved as its
    C-contiguous copy; the device surface refuses a host tensor."""
    with pytest.raises(AssertionError, match="square"):
        eigen.similarity_transform(np.ones((3, 4), np.float32))
    for bad in (np.int32, np.float16):
        with pytest.raises(AssertionError, match="dtype"):
            eigen.similarity_transform(np.ones((3, 3), bad))
    with pytest.raises(ev.EigenValueError, match="dim must be > 0"):
        eigen.similarity_transform(np.zeros((0, 0), np.float32))
    mat = orc.random_matrix(130, 4, np.float32)
    want = eigen.similarity_transform(mat)
    got = eigen.similarity_transform(np.asfortranarray(mat))          # column-major
    assert got[0] == want[0] and got[3] == want[3] and np.array_equal(got[1], want[1])
    with pytest.raises(ValueError, match="HIP device"):
        solver.solve(torch.from_numpy(mat))


@pytest.mark.parametrize("dt", [np.float32, np.float64])
@pytest.mark.parametrize("n", [1, 2, 3, 5, 17, 63, 65, 257])
def test_edge_sizes(eigen, orc, dt, n):
    mat = orc.random_matrix(n, n, dt)
    lam, v, ts, itr = eigen.similarity_transform(mat)
    ref = orc.similarity_transform(mat, orc.SEM_SYCL)
    assert itr == ref.iter_count
    tol = 1e-10 if dt == np.float64 else 1e-5
    assert abs(lam - ref.eigen_val) <= tol * ref.eigen_val
    assert np.max(np.abs(v - ref.eigen_vec)) <= 10 * tol


@pytest.mark.parametrize("dt", [np.float32, np.float64])
def test_max_itr_exhaustion(eigen, orc, dt):
    mat = orc.random_matrix(100, 3, dt)
    lam, v, ts, itr, st = eigen.similarity_transform_ex(mat, eps=0.0, max_itr=5, batch=2)
    ref = orc.similarity_transform(mat, orc.SEM_SYCL, eps=0.0, max_itr=5)
    assert itr == ref.iter_count == 5 and st["converged"] == 0 and st["rounds"] == 5
    tol = 1e-12 if dt == np.float64 else 1e-5
    assert abs(lam - ref.eigen_val) <= tol * ref.eigen_val
    assert np.max(np.abs(v - ref.eigen_vec)) <= tol


@pytest.mark.parametrize("batch", [1, 3, 8, 64])
def test_batch_size_does_not_change_results(eigen, orc, batch):
    mat = orc.hilbert(512)
    base = eigen.similarity_transform(mat)
    lam, v, ts, itr, st = eigen.similarity_transform_ex(mat, batch=batch, time_kernels=True)
    assert lam == base[0] and np.array_equal(v, base[1]) and itr == base[3] == 12
    assert st["fused_launches"] == itr + 1 and st["fused_ms_total"] > 0  # rounds 0..itr
    rt = eigen.last_round_times()                      # per-round times of that solve
    assert rt.size == itr + 1 and np.all(rt > 0)
    assert abs(rt.sum() - st["fused_ms_total"]) <= 1e-3 * st["fused_ms_total"] + 1e-6
    eigen.similarity_transform(mat)                     # untimed solve clears them
    assert eigen.last_round_times().size == 0


def test_device_solver(solver, orc):
    a = dev.generate("hilbert", 2048, torch.float64, device=DEV)
    keep = a.clone()
    lam, v, itr, st = solver.solve(a)
    assert torch.equal(a, keep)                               # not in place by default
    ref = orc.similarity_transform(orc.hilbert(2048), orc.SEM_SYCL)
    assert itr == ref.iter_count == 14
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(to_np(v) - ref.eigen_vec)) <= 1e-10
    lam2, v2, itr2, _ = solver.solve(a, inplace=True)
    assert lam2 == lam and torch.equal(v2, v)
    # any DLPack producer on the device, zero copy
    class Producer:
        def __init__(self, t):
            self.t = t

        def __dlpack__(self, **kw):
            return self.t.__dlpack__(**kw)

        def __dlpack_device__(self):
            return self.t.__dlpack_device__()
    lam3, v3, itr3, _ = solver.solve(Producer(keep.clone()))
    assert lam3 == lam and torch.equal(v3, v) and itr3 == itr
    with pytest.raises(ValueError):
        solver.solve(keep.t(), inplace=True)                  # non-contiguous in place


def test_large_random_vs_oracle(solver, orc):
    n = 16384
    a = dev.generate("random", n, torch.float64, seed=0, device=DEV)
    lam, v, itr, _ = solver.solve(a, inplace=True)
    ref = orc.similarity_transform(orc.random_matrix(n, 0), orc.SEM_SYCL, nthreads=16)
    assert itr == ref.iter_count
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(to_np(v) - ref.eigen_vec)) <= 1e-10


def test_full_size_properties(solver):
    # BASELINE config 3 size (32768^2 fp64 = 8 GiB): size-independent checks
    n = 32768
    a = dev.generate("random", n, torch.float64, seed=0, device=DEV)
    lam, v, itr, _ = solver.solve(a, inplace=True)
    dev.generate("random", n, torch.float64, seed=0, device=DEV, out=a)
    av = torch.mv(a, v)                                # torch fp64 as the checker only
    r = av - lam * v
    assert (r.abs().max() / (lam * v.abs().max())).item() < 1e-9
    # Collatz–Wielandt: for a positive matrix and v > 0 the true Perron root
    # lies in [min (Av)_i/v_i, max (Av)_i/v_i]; the bracket proves the
    # north star's "within 1e-6 rel. of the true eigenvalue" at full size
    q = av / v
    lo, hi = q.min().item(), q.max().item()
    assert v.min().item() > 0 and lo <= hi
    assert max(abs(lam - lo), abs(lam - hi)) / lam < 1e-6   # |λ - λ_true| / λ bound
    # and against the committed CPU Perron root of the same matrix
    pin = large_pin(n, "f64")
    assert abs(lam - pin["lambda"]) / pin["lambda"] < 1e-6
    assert pin["cw_lo"] <= hi and lo <= pin["cw_hi"]            # brackets overlap
    # homogeneity over a fixed number of rounds: every quantity of the
    # iteration on 2A is exactly twice (s, λ) or equal to (v, D^-1 A D
    # ratios) that on A, bit for bit
    dev.generate("random", n, torch.float64, seed=0, device=DEV, out=a)
    lam4, v4, it4, _ = solver.solve(a, eps=0.0, max_itr=4, inplace=True)
    dev.generate("random", n, torch.float64, seed=0, device=DEV, out=a)
    a.mul_(2.0)
    lam8, v8, it8, _ = solver.solve(a, eps=0.0, max_itr=4, inplace=True)
    assert it4 == it8 == 4
    assert lam8 == 2.0 * lam4 and torch.equal(v8, v4)
    del a
    torch.cuda.empty_cache()


# ---------------------------------------------------------------------------
# matrix-free form
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("kind,n", [("hilbert", 128), ("hilbert", 1000), ("hilbert", 4096),
                                    ("random", 333), ("random", 1024), ("random", 4099),
                                    ("random", 3)])
def test_matrix_free_fp64_vs_oracle(eigen, orc, kind, n):
    mat = orc.hilbert(n) if kind == "hilbert" else orc.random_matrix(n, 11)
    lam, v, ts, itr, st = eigen.similarity_transform_ex(mat, matrix_free=True)
    ref = orc.similarity_transform(mat, orc.SEM_SYCL)
    assert itr == ref.iter_count and st["rounds"] == ref.rounds_evaluated
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-10


def test_matrix_free_mainpy_vs_golden(eigen, orc, golden):
    cases, vecs, _ = golden
    for name, case in cases.items():
        mat = golden_input(case, orc)
        lam, v, ts, itr, _ = eigen.similarity_transform_ex(mat, semantics=_lib.ST_SEM_MAINPY,
                                                           matrix_free=True)
        assert itr == case["itr"], name
        assert abs(lam - case["eigen_val"]) <= 1e-11 * abs(case["eigen_val"]), name
        assert np.max(np.abs(v - vecs[name])) <= 1e-11, name


def test_matrix_free_fp32_round_counts(eigen, orc, golden):
    p = golden[2]["hilbert_round_counts_fp32"]
    for n, rounds in zip(p["sizes"], p["rounds"]):
        mat = orc.hilbert(n, np.float32)
        lam, v, ts, itr, _ = eigen.similarity_transform_ex(mat, matrix_free=True)
        assert itr == rounds, (n, itr, rounds)
        ref = orc.similarity_transform(mat, orc.SEM_SYCL)
        assert abs(lam - ref.eigen_val) <= 1e-5 * ref.eigen_val


def test_matrix_free_leaves_input_and_matches_transform(solver):
    n = 6000
    a = dev.generate("random", n, torch.float64, seed=2, device=DEV)
    keep = a.clone()
    lam, v, it, st = solver.solve(a, matrix_free=True, batch=3)
    assert torch.equal(a, keep)                       # A_0 is never written
    lam_t, v_t, it_t, st_t = solver.solve(a)
    assert it == it_t and st["rounds"] == st_t["rounds"]
    assert abs(lam - lam_t) <= 1e-12 * lam_t
    assert (v - v_t).abs().max().item() <= 1e-12
    lam_x, v_x, it_x, st_x = solver.solve(a, matrix_free=True, eps=0.0, max_itr=7)
    assert it_x == 7 and st_x["rounds"] == 7 and st_x["converged"] == 0


@pytest.mark.parametrize("dt,nr,n,row0", [(np.float64, 4352, 4352, 0),    # cached, 8 KB pieces
                                          (np.float64, 2049, 6001, 3000),  # rank block, W = 1
                                          (np.float32, 6144, 6144, 0),
                                          (np.float64, 16385, 16385, 0)])  # 2 GiB: non-temporal
def test_mfree_flat_form_matches_mfree(orc, dt, nr, n, row0):
    """st_mfree_round_flat (k_flat<MF> + k_mparts, the flat form of the
    matrix-free launch) against st_mfree_round over 9 launches from the same
    block: the stats, λ, v and the row sums agree to the dtype's rounding
    (the two sum a row in another association), the gated launch after a
    stop is a no-op in both, and the flat form's sums do not depend on the
    launch: two runs are bit-identical."""
    tdt = TD[dt]
    a = dev.generate("random", n, tdt, nrows=nr, row0=row0, seed=12, device=DEV)
    part = dev.flat_scratch(nr, n, tdt, DEV)
    s_full = torch.from_numpy(orc.random_matrix(n, 13, np.float64, nrows=1)[0] + 0.5).to(DEV)

    def run(flat, eps=0.0, launches=9):
        s = [s_full.to(tdt).clone(), s_full.to(tdt).clone()]
        v = [torch.ones(n, dtype=tdt, device=DEV) for _ in range(2)]
        st = dev.new_state(DEV)
        dev.rowsum(a, out=s[0][row0:row0 + nr])
        for k in range(1, launches + 1):
            args = (a, s[(k - 1) & 1], s[k & 1][row0:row0 + nr], v[(k - 1) & 1], v[k & 1])
            if flat:
                dev.mfree_round_flat(*args, part, st, row0=row0, eps=eps, k=k, max_itr=1000)
            else:
                dev.mfree_round(*args, st, row0=row0, eps=eps, k=k, max_itr=1000)
        torch.cuda.synchronize()
        return s[launches & 1].clone(), v[launches & 1].clone(), dev.read_state(st)

    tol = 1e-12 if dt == np.float64 else 2e-5
    sf, vf, stf = run(True)
    sk, vk, stk = run(False)
    assert (stf["round"], stf["stop"], stf["done"]) == (stk["round"], stk["stop"], stk["done"])
    assert abs(stf["eigen_val"] - stk["eigen_val"]) <= tol * abs(stk["eigen_val"])
    assert abs(stf["max"] - stk["max"]) <= tol * abs(stk["max"])
    assert ((vf - vk).abs() / vk.abs()).max().item() <= tol
    rows = slice(row0, row0 + nr)
    assert ((sf[rows] - sk[rows]).abs() / sk[rows].abs()).max().item() <= tol
    sf2, vf2, _ = run(True)
    assert torch.equal(sf, sf2) and torch.equal(vf, vf2)              # deterministic
    # a huge eps stops at round 0: launch 1 records it, launches 2.. are gated
    # (v_0 and s_1, in the odd buffers, stay as launch 1 left them)
    sf3, vf3, st3 = run(True, eps=1e30, launches=5)
    sk3, vk3, sk3st = run(False, eps=1e30, launches=5)
    assert st3["done"] == sk3st["done"] == 1 and st3["end"] == sk3st["end"] == 1
    assert ((vf3 - vk3).abs() / vk3.abs()).max().item() <= tol


def _gpu_gloo_mfree_worker(rank, world, port, n, outdir):
    import torch.distributed as dist
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = ShardedSimilarityTransform(n, torch.float64, matrix_free=True)
        sh.load("hilbert")
        lam, v, iters, rounds = sh.solve(eps=1e-3, batch=5)
        np.save(os.path.join(outdir, f"v{rank}.npy"), v.cpu().numpy())
        np.save(os.path.join(outdir, f"m{rank}.npy"), np.array([lam, iters, rounds]))
    finally:
        dist.destroy_process_group()


def test_matrix_free_sharded_two_ranks(tmp_path, solver):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    n = 3001
    mp.spawn(_gpu_gloo_mfree_worker, args=(2, port, n, str(tmp_path)), nprocs=2, join=True)
    a = dev.generate("hilbert", n, torch.float64, device=DEV)
    lam, v, it, st = solver.solve(a, matrix_free=True)
    for r in range(2):
        lam_r, it_r, rounds_r = np.load(tmp_path / f"m{r}.npy")
        assert lam_r == lam and int(it_r) == it and int(rounds_r) == st["rounds"]
        assert np.array_equal(np.load(tmp_path / f"v{r}.npy"), to_np(v))


def test_fp32_large_never_converges_at_reference_eps(solver):
    """fp32 row sums ≈ N/2 at N = 16384 have an ulp (2^-10 ≈
    9.8e-4 at 8192, 2^-9 at 16384) at the EPS scale, so the reference's fp32
    stop test never passes and the loop runs MAX_ITR = 1000 rounds; λ still
    agrees with the fp64 solve to fp32 precision."""
    n = 16384
    a32 = dev.generate("random", n, torch.float32, seed=0, device=DEV)
    lam32, v32, it32, st32 = solver.solve(a32, inplace=True, batch=64)
    assert it32 == 1000 and st32["converged"] == 0 and st32["rounds"] == 1000
    a64 = dev.generate("random", n, torch.float64, seed=0, device=DEV)
    lam64, v64, it64, _ = solver.solve(a64, inplace=True)
    assert it64 == 3
    assert abs(lam32 - lam64) <= 2e-6 * lam64
    # v is a product over 1000 rounds of fp32 ratios s/m whose noise is the
    # fp32 ulp of s (≈1e-7 relative): it drifts to ~1e-4 (measured 1.7e-4)
    assert (v32.double() - v64).abs().max().item() <= 1e-3


def test_config4_size_on_one_gpu(solver):
    """BASELINE configs[3] size, 65536² fp64 = 32 GiB (N² = 2^32 elements:
    exercises every 64-bit index path), on one GPU through DeviceSolver:
    converges, residual small, matrix-free agrees.  The row-block driver at
    P = 1 on the same size, against the oracle's solve, is
    test_gpu_fullsize.py::test_config3_sharded_p1_vs_oracle."""
    n = 65536
    a = dev.generate("random", n, torch.float64, seed=0, device=DEV)
    lam_mf, v_mf, it_mf, _ = solver.solve(a, matrix_free=True)
    r = torch.mv(a, v_mf) - lam_mf * v_mf
    assert (r.abs().max() / (lam_mf * v_mf.abs().max())).item() < 1e-9
    pin = large_pin(n, "f64")                                  # CPU Perron root
    assert abs(lam_mf - pin["lambda"]) / pin["lambda"] < 1e-6
    lam, v, it, _ = solver.solve(a, inplace=True)
    assert it == it_mf and abs(lam - lam_mf) <= 1e-12 * lam
    assert (v - v_mf).abs().max().item() <= 1e-12
    del a, r
    torch.cuda.empty_cache()


def test_error_paths_and_degenerate_inputs(eigen):
    L = _lib.load()
    one = np.ones((1, 1), np.float32)
    ev_, vec_, it_ = np.zeros(1, np.float32), np.zeros(1, np.float32), np.zeros(1, np.uint32)
    # dim = 0: negative return and a message, never a crash or a hang
    assert L.max_eigen_value(eigen.sycl_q, one.ctypes.data, ev_.ctypes.data,
                             vec_.ctypes.data, 0, it_.ctypes.data) < 0
    assert "dim" in _lib.last_error()
    with pytest.raises(_lib.EigenValueError):
        eigen.similarity_transform_ex(np.ones((3, 3), np.float32), semantics=7)
    # all-zero matrix: s = 0 everywhere -> the cyclic stop test passes at
    # round 0 (|0 - 0| < EPS), λ = 0, as the reference's loop would
    lam, v, ts, itr = eigen.similarity_transform(np.zeros((64, 64), np.float32))
    assert lam == 0 and itr == 0
    # NaN input: the stop test never passes (NaN compares false), the loop
    # runs to max_itr and reports it — no hang
    bad = np.ones((32, 32), np.float64)
    bad[3, 4] = np.nan
    lam, v, ts, itr, st = eigen.similarity_transform_ex(bad, max_itr=6)
    assert itr == 6 and st["converged"] == 0 and np.isnan(lam)


def _rccl_worker(rank, port, outdir):
    import torch.distributed as dist
    from eigen_value_amd.sharded import ShardedSimilarityTransform, _allgather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        # the in-slot all-gather the sharded loop issues every round, on RCCL
        out = torch.arange(12, dtype=torch.float64, device="cuda")
        _allgather(out, out[0:12])
        assert torch.equal(out, torch.arange(12, dtype=torch.float64, device="cuda"))
        # the library-owned communicator (presence and id over the group's
        # store, then st_comm_init's own rendezvous)
        from eigen_value_amd.sharded import RcclComm
        rc = RcclComm()
        info = rc.info()
        assert {k: info[k] for k in ("nranks", "rank", "device")} == \
            {"nranks": 1, "rank": 0, "device": 0}
        # in a torch process the library's RCCL calls bind torch's bundled RCCL
        assert "torch" in info["rccl_path"] and info["rccl_version_code"] >= 22000, info
        for dt in (torch.float64, torch.float32):
            out = torch.arange(12, dtype=dt, device="cuda")
            rc.allgather(out, out[0:12])
            torch.cuda.synchronize()
            assert torch.equal(out, torch.arange(12, dtype=dt, device="cuda"))
        rc.close()
        sh = ShardedSimilarityTransform(2048, torch.float64)
        sh.load("hilbert")
        lam, v, iters, rounds = sh.solve()
        np.save(os.path.join(outdir, "rccl.npy"), np.array([lam, iters, rounds]))
        sh.close()
        # a flat block: the deferred-write solve's ring of gathered row sums
        # on the library communicator == storing every round
        res = []
        for dw in (True, False):
            sh = ShardedSimilarityTransform(4352, torch.float64, deferred_writes=dw)
            assert sh.deferred_writes == dw and sh.rccl is None   # P = 1: no comm needed
            sh.load("random", seed=2)
            res.append(sh.solve(eps=0.0, max_itr=10))
            sh.close()
        (l0, v0, i0, r0), (l1, v1, i1, r1) = res
        np.save(os.path.join(outdir, "rccl_defer.npy"),
                np.array([l0 == l1 and i0 == i1 and r0 == r1 and bool(torch.equal(v0, v1))]))
    finally:
        dist.destroy_process_group()


def test_rccl_process_group_single_rank(tmp_path, orc):
    """P = 1 over the nccl (= RCCL) backend: the sharded driver under an
    initialised RCCL process group, and the in-place all-gather call."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_rccl_worker, args=(port, str(tmp_path)), nprocs=1, join=True)
    lam, iters, rounds = np.load(tmp_path / "rccl.npy")
    ref = orc.similarity_transform(orc.hilbert(2048), orc.SEM_SYCL)
    assert int(iters) == ref.iter_count == 14
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert bool(np.load(tmp_path / "rccl_defer.npy")[0])


@pytest.mark.parametrize("matrix_free", [False, True])
def test_native_multi_gpu_solve(orc, matrix_free):
    """st_solve_multi_* (one process, RCCL communicator over the visible
    devices; P = 1 here, the all-gather still issued) vs the oracle."""
    from eigen_value_amd.multi import solve_multi
    ngpu = torch.cuda.device_count()
    n = 3001
    lam, v, it, st = solve_multi(n, "random", ngpus=ngpu, seed=3, matrix_free=matrix_free)
    ref = orc.similarity_transform(orc.random_matrix(n, 3), orc.SEM_SYCL)
    assert it == ref.iter_count and st["rounds"] == ref.rounds_evaluated
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(v - ref.eigen_vec)) <= 1e-10
    # host-matrix input, fp32 Hilbert: the reference's published 9 rounds
    mat = orc.hilbert(128, np.float32)
    lam32, v32, it32, _ = solve_multi(128, mat, ngpus=ngpu, matrix_free=matrix_free)
    assert it32 == 9 and abs(lam32 - 2.2171896) < 1e-5
    with pytest.raises(_lib.EigenValueError, match="without rows"):
        solve_multi(1, "hilbert", devices=[0, 0])


def test_native_multi_gpu_flat_round(solver):
    """st_solve_multi_* on a block that takes the flat round (9216², 648 MiB)
    equals the library's single-GPU solve loop bit for bit."""
    from eigen_value_amd.multi import solve_multi
    n = 9216
    lam, v, it, st = solve_multi(n, "random", ngpus=1, seed=3)
    a = dev.generate("random", n, torch.float64, seed=3, device=DEV)
    lam1, v1, it1, st1 = solver.solve(a, inplace=True)
    assert lam == lam1 and it == it1 and st["rounds"] == st1["rounds"]
    assert np.array_equal(v, to_np(v1))
    # deferred writes (the default) against storing every round, converging
    # and fixed-round solves
    for kw in (dict(), dict(eps=0.0, max_itr=8)):
        r1 = solve_multi(n, "random", ngpus=1, seed=3, **kw)
        r2 = solve_multi(n, "random", ngpus=1, seed=3, write_every_round=True, **kw)
        assert r1[0] == r2[0] and r1[2] == r2[2] and np.array_equal(r1[1], r2[1]), kw
    del a
    torch.cuda.empty_cache()


def test_fuzz_vs_oracle(eigen, orc):
    """Seeded random sweep over size, dtype, semantics, form, batch and
    eps: iteration counts equal to the oracle's, λ / v within the dtype's
    tolerance.  Sizes straddle the launch-shape switches (rows per group,
    remainder groups, 16-byte vs element access).  Every case runs traced on
    both sides (tests/stop_parity.py): a count may differ only where the
    two solves' own row sums put a round's max |Δs| on opposite sides of
    eps, and that must be explained by their measured row-sum deviation
    (at most DEV_ULPS ulps of max s)."""
    import stop_parity as sp
    rng = np.random.default_rng(1234)
    straddles = []
    for case in range(40):
        n = int(rng.choice([1, 2, 3, 7, 64, 127, 255, 1023, 1024, 1025, 2047, 2048, 2049,
                            2051, 3000]))
        dt = np.float64 if rng.random() < 0.6 else np.float32
        sem = int(rng.integers(0, 2))
        mf = bool(rng.random() < 0.4)
        batch = int(rng.choice([1, 2, 5, 8, 16]))
        eps = float(rng.choice([1e-3, 1e-6, 1e-2]))
        kind = "hilbert" if rng.random() < 0.5 else "random"
        mat = orc.hilbert(n, dt) if kind == "hilbert" else orc.random_matrix(n, case, dt)
        lam, v, ts, itr, st = eigen.similarity_transform_ex(
            mat, eps=eps, semantics=sem, matrix_free=mf, batch=batch, max_itr=200,
            trace_sums=True)
        ref = orc.similarity_transform(mat, sem, eps=dt(eps), max_itr=200, trace=True)
        tag = (case, n, dt.__name__, sem, mf, batch, eps, kind)
        cmp = sp.compare(eigen.last_round_sums(), ref.row_sums, dt(eps),
                         sem == _lib.ST_SEM_SYCL, 200, matrix_free=mf)
        if not sp.assert_stop_parity(cmp, tag):
            straddles.append((tag, cmp["straddle"]))
            continue
        assert itr == ref.iter_count, tag
        tol = 1e-10 if dt == np.float64 else 2e-5
        assert abs(lam - ref.eigen_val) <= tol * abs(ref.eigen_val) + 1e-30, tag
        assert np.max(np.abs(v - ref.eigen_vec)) <= (1e-10 if dt == np.float64 else 5e-4), tag
    assert len(straddles) <= 2, straddles


@pytest.mark.parametrize("n", [512, 1024, 2048, 4096])
def test_dropin_fp32_random_at_reference_eps(eigen, orc, n):
    """The reference's wrapper test shape (wrapper/python/test.py:3-18: fp32
    random matrices through max_eigen_value, EPS = 1e-3f from
    include/similarity_transform.hpp:4, the cyclic stop of
    similarity_transform.cpp:413-421) against the oracle: iteration count
    equal, λ within 1e-5 relative, v within 1e-4, and the per-round stop
    decisions traced on both sides (no round straddles EPS)."""
    import stop_parity as sp
    rng = np.random.default_rng(2021 + n)
    mat = rng.random((n, n)).astype("f")          # wrapper/python/test.py:9
    lam, v, ts, itr = eigen.similarity_transform(mat)            # the drop-in call
    ref = orc.similarity_transform(mat, orc.SEM_SYCL, trace=True)
    lam2, v2, _, itr2, st = eigen.similarity_transform_ex(mat, trace_sums=True)
    assert lam2 == lam and itr2 == itr and np.array_equal(v2, v)  # tracing moves nothing
    cmp = sp.compare(eigen.last_round_sums(), ref.row_sums, orc.EPS_F32, True, orc.MAX_ITR)
    assert sp.assert_stop_parity(cmp, n), cmp
    assert itr == ref.iter_count
    assert abs(float(lam) - float(ref.eigen_val)) <= 1e-5 * float(ref.eigen_val)
    assert np.max(np.abs(v.astype(np.float64) - ref.eigen_vec)) <= 1e-4
    assert np.all(np.isclose(mat @ v, lam * v, atol=1e-3))       # the reference's own check


def test_trace_sums_round_trip(eigen, solver, orc):
    """ST_FLAG_TRACE_SUMS records s_0 .. s_{end-1} on every form (one-launch
    round, flat deferred, matrix-free; drop-in and device paths) without
    changing a result, and an untraced solve clears the trace."""
    import stop_parity as sp
    for n, dt, kw in ((300, np.float64, {}), (300, np.float32, dict(matrix_free=True)),
                      (4352, np.float64, {}), (2048, np.float32, dict(matrix_free=True))):
        mat = orc.hilbert(n, dt)
        base = eigen.similarity_transform_ex(mat, **kw)
        lam, v, _, itr, st = eigen.similarity_transform_ex(mat, trace_sums=True, **kw)
        sums = eigen.last_round_sums()
        assert lam == base[0] and itr == base[3] and np.array_equal(v, base[1])
        assert sums.shape == (st["rounds"], n) and sums.dtype == dt
        ref = orc.similarity_transform(mat, orc.SEM_SYCL, trace=True)
        cmp = sp.compare(sums, ref.row_sums, dt(1e-3), True, orc.MAX_ITR,
                         matrix_free=kw.get("matrix_free", False))
        assert sp.assert_stop_parity(cmp, n) and itr == ref.iter_count
        t = torch.from_numpy(mat).to(DEV)
        lam_d, v_d, it_d, st_d = solver.solve(t, trace_sums=True, **kw)
        assert lam_d == lam and it_d == itr and np.array_equal(solver.last_round_sums(), sums)
        eigen.similarity_transform_ex(mat, **kw)
        assert eigen.last_round_sums().shape[0] == 0
    with pytest.raises(ev.EigenValueError, match="TRACE_SUMS"):
        eigen.similarity_transform_ex(orc.hilbert(4096), trace_sums=True, max_itr=100000)


def test_config1_hilbert8192_fp64_vs_oracle(solver, orc):
    """BASELINE configs[1]: 8192² Hilbert fp64 on one GPU, both forms, vs
    the oracle's same-semantics solve (17 rounds, README.md:76)."""
    a = dev.generate("hilbert", 8192, torch.float64, device=DEV)
    ref = orc.similarity_transform(orc.hilbert(8192), orc.SEM_SYCL, nthreads=16)
    assert ref.iter_count == 17
    for mf in (False, True):
        lam, v, it, st = solver.solve(a, matrix_free=mf)
        assert it == 17 and st["rounds"] == 18
        assert abs(lam - ref.eigen_val) <= 1e-12 * ref.eigen_val
        assert np.max(np.abs(to_np(v) - ref.eigen_vec)) <= 1e-12


def test_config5_fp32_32768_tracks_fp64(solver):
    """BASELINE configs[4]: 32768² fp32 (float4 accesses) over a fixed
    number of rounds agrees with the fp64 iteration on the same input to
    fp32 precision (the tolerance study, profiles/r01_fp32_study.json)."""
    n = 32768
    a32 = dev.generate("random", n, torch.float32, seed=0, device=DEV)
    lam32, v32, it32, _ = solver.solve(a32, inplace=True, eps=0.0, max_itr=8)
    del a32
    torch.cuda.empty_cache()
    a64 = dev.generate("random", n, torch.float64, seed=0, device=DEV)
    lam64, v64, it64, _ = solver.solve(a64, inplace=True, eps=0.0, max_itr=8)
    del a64
    torch.cuda.empty_cache()
    assert it32 == it64 == 8
    assert abs(lam32 - lam64) <= 1e-6 * lam64
    assert (v32.double() - v64).abs().max().item() <= 1e-5
    # each against the CPU Perron root of its own generated matrix
    for lam_, dt in ((lam32, "f32"), (lam64, "f64")):
        pin = large_pin(n, dt)
        assert abs(lam_ - pin["lambda"]) / pin["lambda"] < 1e-6, dt


def test_cpp_kernel_tests():
    # tests/cpp/test_kernels.cpp mirrors the reference's tests/test.cpp
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run(["make", "-s", "-C", os.path.join(here, "cpp")], check=True)
    out = subprocess.run([os.path.join(here, "cpp", "test_kernels")], capture_output=True,
                         text=True, timeout=300)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "similarity transform worked" in out.stdout


def test_wave_reductions_bitwise():
    """tests/cpp/test_reduce.hip: every wave-reduction form of st_device.h
    (broadcast tree, lane-63 tree, the two-row tree of k_flat, stepwise
    rows) gives the same bits on 4096 waves of mixed-magnitude data."""
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run(["make", "-s", "-C", os.path.join(here, "cpp"), "test_reduce"], check=True)
    out = subprocess.run([os.path.join(here, "cpp", "test_reduce")], capture_output=True,
                         text=True, timeout=120)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "wave reductions bit-identical" in out.stdout


def test_parts_segments_bitwise():
    """tests/cpp/test_parts.hip: k_parts_seg (4 / 2 rows per wave for rows of
    at most 16 / 32 partials, the flat round's partial-sum launch on cached
    and short blocks) against k_parts (a wave per row): s_{k+1}, 1/s_{k+1}
    and the eigenvector update bit for bit, every partial count 1 ... 32,
    row counts that leave waves partly empty, fp64 and fp32."""
    import subprocess
    here = os.path.dirname(os.path.abspath(__file__))
    subprocess.run(["make", "-s", "-C", os.path.join(here, "cpp"), "test_parts"], check=True)
    out = subprocess.run([os.path.join(here, "cpp", "test_parts")], capture_output=True,
                         text=True, timeout=120)
    print(out.stdout)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "k_parts_seg bit-identical to k_parts" in out.stdout


# ---------------------------------------------------------------------------
# the whole solve in one workgroup (k_solve_small, n <= 128 fp64 / 256 fp32)
# against the per-round launch loop: bit-identical λ, v, iteration count and
# final matrix
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dt,n", [(np.float64, 2), (np.float64, 8), (np.float64, 62),
                                  (np.float64, 100), (np.float64, 128),
                                  (np.float32, 4), (np.float32, 128), (np.float32, 252),
                                  (np.float32, 256)])
@pytest.mark.parametrize("sem", [_lib.ST_SEM_SYCL, _lib.ST_SEM_MAINPY])
@pytest.mark.parametrize("kind", ["hilbert", "random"])
def test_single_launch_solve_matches_round_loop(solver, orc, dt, n, sem, kind):
    mat = orc.hilbert(n, dt) if kind == "hilbert" else orc.random_matrix(n, 5, dt)
    a1 = torch.from_numpy(mat).to(DEV)
    a2 = a1.clone()
    r1 = solver.solve(a1, inplace=True, semantics=sem)
    r2 = solver.solve(a2, inplace=True, semantics=sem, round_loop=True)
    assert r1[2] == r2[2] and r1[3]["rounds"] == r2[3]["rounds"]
    assert r1[0] == r2[0]                                   # λ bitwise
    assert torch.equal(r1[1], r2[1])                        # v bitwise
    assert torch.equal(a1, a2)                              # final matrix bitwise
    ref = orc.similarity_transform(mat, orc.SEM_SYCL if sem == _lib.ST_SEM_SYCL
                                   else orc.SEM_MAINPY)
    assert r1[2] == ref.iter_count
    tol = 1e-10 if dt == np.float64 else 1e-5
    assert abs(r1[0] - ref.eigen_val) <= tol * ref.eigen_val


@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_single_launch_exhaustion_and_eps(solver, orc, dt):
    mat = orc.random_matrix(64, 9, dt)
    for kw in (dict(eps=0.0, max_itr=5), dict(eps=1e-6), dict(max_itr=1)):
        a1 = torch.from_numpy(mat).to(DEV)
        a2 = a1.clone()
        r1 = solver.solve(a1, inplace=True, **kw)
        r2 = solver.solve(a2, inplace=True, round_loop=True, **kw)
        assert (r1[0], r1[2], r1[3]["rounds"], r1[3]["converged"]) == \
               (r2[0], r2[2], r2[3]["rounds"], r2[3]["converged"]), kw
        assert torch.equal(r1[1], r2[1]) and torch.equal(a1, a2), kw
    r = solver.solve(torch.from_numpy(mat).to(DEV), eps=0.0, max_itr=5)
    assert r[2] == 5 and r[3]["rounds"] == 5 and r[3]["converged"] == 0


def test_single_launch_dropin_is_one_launch(eigen, orc):
    # the drop-in call at configs[0]'s size: Hilbert 128 fp32 (README.md:70,
    # 9 rounds) — the single launch and the loop agree, and the single launch
    # finishes the loop in less time than the per-round form
    h = orc.hilbert(128, np.float32)
    lam, v, ts, itr, st = eigen.similarity_transform_ex(h)
    lam2, v2, ts2, itr2, st2 = eigen.similarity_transform_ex(h, round_loop=True)
    assert itr == itr2 == 9 and lam == lam2 and np.array_equal(v, v2)
    best = min(eigen.similarity_transform_ex(h)[4]["loop_ms"] for _ in range(5))
    best_loop = min(eigen.similarity_transform_ex(h, round_loop=True)[4]["loop_ms"]
                    for _ in range(5))
    print(f"hilbert128 f32 loop_ms: single launch {best:.4f}, per round {best_loop:.4f}")
    assert best < best_loop


# ---------------------------------------------------------------------------
# deferred writes (blocks >= 144 MiB: the flat round stores A every 6th round
# and re-applies the pending scalings) against storing every round:
# bit-identical λ, v, iteration count, row-sum bookkeeping and final matrix
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dt,n", [(np.float64, 4352), (np.float32, 6144),
                                  (np.float64, 8192),    # configs[1]: 1-row tiles of 8
                                  (np.float64, 4353),    # odd: element-wide access
                                  # just past 2 GiB: non-temporal, 6 rounds per
                                  # store, element-wide (n % 16 B != 0)
                                  (np.float64, 16385), (np.float32, 23171)])
@pytest.mark.parametrize("sem", [_lib.ST_SEM_SYCL, _lib.ST_SEM_MAINPY])
def test_deferred_writes_bitwise(solver, dt, n, sem):
    assert dev.flat_round_pays(n, n, TD[dt])
    base = dev.generate("random", n, TD[dt], seed=4, device=DEV)
    # fixed round counts ending at every residue mod 6 (the final flush), a
    # converging solve, and max_itr = 1
    for kw in (dict(eps=0.0, max_itr=7), dict(eps=0.0, max_itr=8), dict(eps=0.0, max_itr=9),
               dict(eps=0.0, max_itr=10), dict(eps=0.0, max_itr=11), dict(eps=0.0, max_itr=12),
               dict(), dict(eps=1e-9), dict(max_itr=1)):
        a1, a2 = base.clone(), base.clone()
        r1 = solver.solve(a1, inplace=True, semantics=sem, **kw)
        r2 = solver.solve(a2, inplace=True, semantics=sem, write_every_round=True, **kw)
        assert (r1[0], r1[2], r1[3]["rounds"], r1[3]["converged"]) == \
               (r2[0], r2[2], r2[3]["rounds"], r2[3]["converged"]), kw
        assert torch.equal(r1[1], r2[1]), kw                # v bitwise
        assert torch.equal(a1, a2), kw                      # final matrix bitwise


def test_max_single_gpu_size(solver):
    """131072² fp64 = 128 GiB on one GPU: the flat launches' 2^24 workgroups
    exceed one dispatch dimension (2-D grid).  The deferred and every-round
    transforms agree bit for bit, the matrix-free form to rounding, and λ
    lies between the smallest and largest row sum (Perron-Frobenius)."""
    n = 131072
    torch.cuda.empty_cache()
    a = dev.generate("random", n, torch.float64, seed=0, device=DEV)
    rs = a.sum(dim=1)
    lo, hi = rs.min().item(), rs.max().item()
    del rs
    lam_mf, v_mf, it_mf, _ = solver.solve(a, matrix_free=True)
    lam, v, it, st = solver.solve(a, inplace=True)                       # deferred
    assert lo <= lam <= hi and it == it_mf and it >= 2
    assert abs(lam - lam_mf) <= 1e-12 * lam and (v - v_mf).abs().max().item() <= 1e-12
    dev.generate("random", n, torch.float64, seed=0, device=DEV, out=a)
    lam2, v2, it2, _ = solver.solve(a, inplace=True, write_every_round=True)
    assert (lam2, it2) == (lam, it) and torch.equal(v2, v)
    print(f"131072^2 f64: lambda {lam!r} in [{lo}, {hi}], {it} rounds, "
          f"loop {st['loop_ms']:.1f} ms")
    del a
    torch.cuda.empty_cache()


def test_deferred_writes_dropin_and_batches(eigen, orc):
    # the host-matrix path (private copy, no final flush) and batch sizes
    # that stop mid-group: identical to storing every round
    mat = orc.hilbert(6144, np.float32)
    ref = eigen.similarity_transform_ex(mat, write_every_round=True)
    for batch in (1, 2, 5):
        got = eigen.similarity_transform_ex(mat, batch=batch)
        assert got[0] == ref[0] and np.array_equal(got[1], ref[1]) and got[3] == ref[3]
