"""CPU: pin the oracle before trusting it (no GPU needed).

* SEM_MAINPY fp64 solves are BIT-identical to the reference's main.py
  (golden vectors made by tests/golden/make_golden.py from
  /root/reference/main.py:30-47).
* SEM_SYCL fp32 reproduces the reference's published Hilbert round counts
  (README.md:70-76) and the 3x3 known answer (tests/test.cpp:99-102).
* Per-kernel pins follow tests/test.cpp:22-73.
"""
import numpy as np
import pytest

from conftest import golden_input


def test_pairwise_sum_matches_numpy(orc):
    rng = np.random.default_rng(0)
    for n in list(range(0, 140)) + [255, 256, 257, 1000, 4097, 32768]:
        for dt in (np.float64, np.float32):
            a = rng.random(n).astype(dt)
            assert orc.pairwise_sum(a) == np.sum(a), (n, dt)


@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_generators_numpy_equals_c(orc, dt):
    L = orc.lib()
    sfx = "f64" if dt == np.float64 else "f32"
    for n, nrows, row0, seed in ((7, 7, 0, 0), (64, 10, 13, 5), (129, 3, 126, 123456789)):
        h = np.empty((nrows, n), dtype=dt)
        getattr(L, f"orc_hilbert_{sfx}")(h.ctypes.data, nrows, n, row0)
        assert np.array_equal(h, orc.hilbert(n, dt, nrows=nrows, row0=row0))
        r = np.empty((nrows, n), dtype=dt)
        getattr(L, f"orc_random_{sfx}")(r.ctypes.data, nrows, n, row0, seed)
        ref = orc.random_matrix(n, seed, dt, nrows=nrows, row0=row0)
        assert np.array_equal(r, ref)
        assert r.min() > 0 and r.max() <= 1


def test_hilbert_matches_reference_formula(orc):
    # utils.cpp:150: 1.f / (float)(r + c + 1)
    n = 50
    h = orc.hilbert(n, np.float32)
    for r in (0, 7, 49):
        for c in (0, 3, 49):
            assert h[r, c] == np.float32(1.0) / np.float32(r + c + 1)


def test_mainpy_golden_bit_exact(orc, golden):
    cases, vecs, _ = golden
    assert len(cases) >= 20
    for name, case in cases.items():
        mat = golden_input(case, orc)
        r = orc.similarity_transform(mat, orc.SEM_MAINPY)
        assert r.eigen_val == case["eigen_val"], name
        assert float(r.eigen_val).hex() == case["eigen_val_hex"], name
        assert np.array_equal(r.eigen_vec, vecs[name]), name
        assert r.iter_count == case["itr"], name


def test_kat3_reference_pins(orc, golden):
    _, _, pins = golden
    kat = pins["kat3"]
    mat = np.array(kat["matrix"], dtype=np.float32)
    r = orc.similarity_transform(mat, orc.SEM_SYCL)
    assert abs(r.eigen_val - kat["eigen_val"]) < kat["tol"]
    assert np.all(np.abs(r.eigen_vec - np.array(kat["eigen_vec"])) < kat["tol"])


def test_hilbert_round_counts_readme(orc, golden):
    _, _, pins = golden
    p = pins["hilbert_round_counts_fp32"]
    for n, rounds in zip(p["sizes"], p["rounds"]):
        if n > 4096:
            continue   # 8192 is covered by test_hilbert_8192_round_count
        r = orc.similarity_transform(orc.hilbert(n, np.float32), orc.SEM_SYCL)
        assert r.iter_count == rounds, (n, r.iter_count, rounds)
        r64 = orc.similarity_transform(orc.hilbert(n, np.float64), orc.SEM_SYCL)
        assert r64.iter_count == rounds, n


def test_hilbert_8192_round_count(orc):
    r = orc.similarity_transform(orc.hilbert(8192, np.float32), orc.SEM_SYCL)
    assert r.iter_count == 17                       # README.md:76
    assert abs(r.eigen_val - 2.599992) < 1e-5


def test_kernel_unit_pins(orc):
    n = 1024                                          # tests/test.cpp:7
    # rowsum of the identity is 1 (tests/test.cpp:22-30)
    assert np.all(orc.rowsum(np.eye(n, dtype=np.float32)) == 1.0)
    # max of r+1 is N (tests/test.cpp:32-41)
    vec = np.arange(1, n + 1, dtype=np.float32)
    mx = orc.find_max(vec)
    assert mx == n
    # eigenvector update from v = 1 is s/m (tests/test.cpp:43-54)
    v = orc.compute_eigen_vector(vec, np.float32(mx), np.ones(n, np.float32))
    assert np.max(np.abs(vec / mx - v)) == 0.0
    # stop: constant 1+1e-4 -> 1; (r+1)*1e-4 -> 0 only via the cyclic wrap
    ok = np.full(n, np.float32(1) + np.float32(1e-4), dtype=np.float32)
    assert orc.stop(ok, cyclic=True) is True
    fail = (np.arange(n, dtype=np.float32) + 1) * np.float32(1e-4)
    assert orc.stop(fail, cyclic=True) is False
    assert orc.stop(fail, cyclic=False) is True      # main.py:25-27 semantics


def test_find_max_starts_at_zero(orc):
    # similarity_transform.cpp:185 initialises the running max to 0.f
    assert orc.find_max(np.array([-3.0, -1.0])) == 0.0


def test_compute_next_orders(orc):
    rng = np.random.default_rng(3)
    a = rng.random((5, 7))
    s = rng.random(7) + 0.5
    sycl = orc.compute_next(a[:, :7][:5], s, row0=2, order=0)
    py = orc.compute_next(a[:, :7][:5], s, row0=2, order=1)
    for r in range(5):
        inv = 1.0 / s[2 + r]
        assert np.array_equal(sycl[r], a[r] * (inv * s))
        assert np.array_equal(py[r], (inv * a[r]) * s)


def test_max_itr_exhaustion(orc):
    # eps = 0 never stops: iter_count = MAX_ITR, λ = s[0] of the last evaluation
    mat = orc.random_matrix(16, 1)
    r = orc.similarity_transform(mat, orc.SEM_SYCL, eps=0.0, max_itr=7)
    assert r.iter_count == 7 and r.rounds_evaluated == 7
    r2 = orc.similarity_transform(mat, orc.SEM_SYCL, eps=0.0, max_itr=8)
    assert r2.rounds_evaluated == 8 and r2.eigen_val != 0


def test_single_element(orc):
    r = orc.similarity_transform(np.array([[3.5]]), orc.SEM_SYCL)
    assert r.eigen_val == 3.5 and r.iter_count == 0 and r.eigen_vec[0] == 1.0
    r = orc.similarity_transform(np.array([[3.5]]), orc.SEM_MAINPY)
    assert r.iter_count == 1


def test_thread_count_invariance(orc):
    mat = orc.random_matrix(300, 2)
    a = orc.similarity_transform(mat, orc.SEM_SYCL, nthreads=1)
    b = orc.similarity_transform(mat, orc.SEM_SYCL, nthreads=4)
    assert a.eigen_val == b.eigen_val and np.array_equal(a.eigen_vec, b.eigen_vec)


def test_random_fp64_meets_north_star_accuracy(orc):
    # north_star: eigenvalue within 1e-6 rel. of numpy (random positive fp64)
    mat = orc.random_matrix(512, 0)
    r = orc.similarity_transform(mat, orc.SEM_SYCL)
    true = np.max(np.linalg.eigvals(mat).real)
    assert abs(r.eigen_val - true) / true < 1e-6


def test_large_pins(orc):
    """tests/golden/large_pins.json: CPU Perron roots of the full-size
    BASELINE random matrices (SURVEY.md §8c large-N reference).  The
    Collatz–Wielandt brackets are tight, λ sits near N/2 (U(0,1] entries),
    and the C generator the pins were computed from reproduces the numpy
    generator bit for bit on sampled rows of those very matrices."""
    import ctypes

    from conftest import large_pin
    for n, dt in ((32768, "f64"), (32768, "f32"), (65536, "f64")):
        p = large_pin(n, dt)
        assert p["cw_lo"] <= p["lambda"] <= p["cw_hi"]
        assert p["cw_rel_width"] < 1e-13
        assert abs(p["lambda"] / (n / 2) - 1) < 1e-3
        npdt = np.float64 if dt == "f64" else np.float32
        for row0 in (0, n // 2 + 1, n - 1):
            c = np.empty((1, n), npdt)
            getattr(orc.lib(), f"orc_random_{dt}")(c.ctypes.data_as(ctypes.c_void_p), 1, n, row0, 0)
            ref = orc.random_matrix(n, 0, npdt, nrows=1, row0=row0)
            assert np.array_equal(c, ref)


@pytest.mark.parametrize("kind,n,dtype,semantics,eps,max_itr", [
    ("random", 1000, np.float64, 0, None, 64),
    ("hilbert", 777, np.float64, 1, None, 64),
    ("hilbert", 1024, np.float32, 0, None, 64),
    ("random", 2000, np.float64, 1, 0.0, 5),
    ("random", 513, np.float32, 0, 0.0, 8),
])
def test_generated_solve_bit_identical(orc, kind, n, dtype, semantics, eps, max_itr):
    """The streaming oracle for generated inputs too large to hold twice
    (orc_similarity_transform_gen_*: A_0 regenerated in row blocks each round,
    recorded transforms re-applied) equals the plain oracle loop bit for bit;
    it produces the configs[3] pins (tests/golden/make_large_pins.py)."""
    a = orc.generate_c(kind, n, 3, dtype)
    ref = orc.hilbert(n, dtype) if kind == "hilbert" else orc.random_matrix(n, 3, dtype)
    assert np.array_equal(a, ref)
    r1 = orc.similarity_transform(a, semantics, eps=eps, max_itr=max_itr)
    r2 = orc.similarity_transform_gen(kind, n, 3, dtype, semantics, eps=eps,
                                      max_itr=max_itr, chunk_rows=97)
    assert (r1.iter_count, r1.rounds_evaluated) == (r2.iter_count, r2.rounds_evaluated)
    assert r1.eigen_val == r2.eigen_val
    assert np.array_equal(r1.eigen_vec, r2.eigen_vec)


def test_oracle_under_sanitizers(tmp_path):
    """The checker itself under AddressSanitizer + UndefinedBehaviorSanitizer
    (SURVEY.md §5): tests/cpp/oracle_sanitize.c drives every oracle entry
    point across its internal boundaries (pairwise leaves of 128, the
    8192-element numpy buffer, ragged rows, n = 1, the streaming solve's
    uneven chunks) and the reference's 3x3 known answer; any report aborts."""
    import os
    import shutil
    import subprocess
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "oracle_sanitize")
    subprocess.run(["gcc", "-O1", "-g", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-fopenmp",
                    "-ffp-contract=off", "-std=c11", "-Wall", "-Wextra", "-Wno-unknown-pragmas",
                    os.path.join(repo, "tests", "cpp", "oracle_sanitize.c"),
                    os.path.join(repo, "oracle", "st_oracle.c"), "-lm", "-o", exe],
                   check=True, capture_output=True, text=True)
    env = dict(os.environ, OMP_NUM_THREADS="2")
    # the environment may preload a library ahead of the ASan runtime
    env["ASAN_OPTIONS"] = "verify_asan_link_order=0"
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "clean" in out.stdout


def test_stop_parity_rule():
    """tests/stop_parity.py on synthetic traces (fp32, cyclic, eps = 1.0):
    identical traces agree; a round whose max |ds| straddles eps by less
    than the row sums' deviation excuses different counts; a deviation past
    DEV_ULPS (plus the round index for the matrix-free form) fails; a trace
    that does not stop where its solve stopped fails."""
    import stop_parity as sp
    f = np.float32
    orc = np.array([[1, 4, 1, 4], [2, 2.5, 2, 2.5]], f)          # stops in round 1
    assert sp.first_stop(orc, f(1.0), True) == 1
    c = sp.compare(orc, orc.copy(), f(1.0), True, 100)
    assert sp.assert_stop_parity(c) and c["straddle"] is None and c["max_dev_ulps"] == 0
    # the device's round-1 sums 3 ulps apart put max |ds| just past eps
    u = np.spacing(f(2.5))
    gpu = np.array([[1, 4, 1, 4],
                    [2, 2.5, 2, 2.5],
                    [2, 2.25, 2, 2.25]], f)
    gpu[1, 1] = gpu[1, 3] = f(3.0) + u        # max |ds| 1 + u: no stop
    orc2 = orc.copy()
    orc2[1, 1] = orc2[1, 3] = f(3.0) - u      # max |ds| 1 - u: stops
    gpu[1, 1] = gpu[1, 3] = f(3.0) + 2 * u
    c = sp.compare(gpu, orc2, f(1.0), True, 100)
    assert c["straddle"] is not None and c["straddle"]["round"] == 1
    assert sp.assert_stop_parity(c) is False                   # listed, not failed
    # a deviation of 1000 ulps is not rounding
    bad = orc2.copy()
    bad[0, 1] += 1000 * np.spacing(f(4.0))
    with pytest.raises(AssertionError, match="row sums deviate"):
        sp.assert_stop_parity(sp.compare(bad, orc2, f(1.0), True, 100))
    # ... but over many rounds the solves may drift apart by one ulp per round
    drift = np.repeat(orc2[:1], 40, axis=0)
    drift[:, 0] = f(1.0)
    late = drift.copy()
    late[39, 1] += 40 * np.spacing(f(4.0))
    assert sp.compare(late, drift, f(1.0), True, 40)["dev_excess"] == []
    late[39, 1] += 40 * np.spacing(f(4.0))
    assert sp.compare(late, drift, f(1.0), True, 40)["dev_excess"] == [39]
    # a trace that passes the stop test before its last round is inconsistent
    with pytest.raises(AssertionError, match="does not stop"):
        sp.assert_stop_parity(sp.compare(np.vstack([orc, orc[1:]]), orc, f(1.0), True, 100))
