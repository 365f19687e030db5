"""The launch-table knobs (include/st_tuning.h) move no result.

These run against the TUNING build, libsimilarity_transform_tuning.so: the
same kernels as libsimilarity_transform.so plus the process-wide setters of
its launch tables, which the product library does not export (VERDICT r05
#5).  Collected by the main GPU run, this file is one test there
(test_tuning_build_knobs) that re-runs the file in a child process whose
default library is the tuning build (EIGEN_VALUE_LIB), where the knob tests
themselves are collected: every solve of a knob test then goes through the
library whose tables it sets.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no HIP device", allow_module_level=True)

from eigen_value_amd import _lib  # noqa: E402
from eigen_value_amd import device as dev  # noqa: E402

DEV = "cuda:0"
TD = {np.float64: torch.float64, np.float32: torch.float32}
IN_TUNING = os.path.realpath(_lib.lib_path()) == os.path.realpath(_lib.TUNING_LIB)


if not IN_TUNING:
    def test_tuning_build_knobs():
        """Run this file's knob tests in a child whose library is the
        tuning build; the tuning build's kernels equal the product's (same
        sources), checked here on one solve."""
        assert os.path.exists(_lib.TUNING_LIB), "run make: the tuning build is missing"
        env = dict(os.environ, EIGEN_VALUE_LIB=_lib.TUNING_LIB)
        out = subprocess.run([sys.executable, "-u", "-m", "pytest", "-x", "-q", "-p",
                              "no:cacheprovider", "--timeout", "600", "--timeout-method",
                              "thread", "-m", "gpu", os.path.abspath(__file__)],
                             env=env, capture_output=True, text=True, timeout=900,
                             cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        print(out.stdout[-3000:])
        assert out.returncode == 0, out.stdout[-6000:] + out.stderr[-3000:]
        assert " passed" in out.stdout and "failed" not in out.stdout

    def test_tuning_build_kernels_are_the_products():
        """The same solve through both libraries, bit for bit (the tuning
        build differs in its exports only)."""
        env = dict(os.environ, EIGEN_VALUE_LIB=_lib.TUNING_LIB)
        code = ("import sys, torch; sys.path.insert(0, sys.argv[1]);"
                "from eigen_value_amd import device as dev;"
                "a = dev.generate('random', 4352, torch.float64, seed=2, device='cuda:0');"
                "lam, v, it, st = dev.DeviceSolver('cuda:0').solve(a, eps=0.0, max_itr=8);"
                "torch.save(v.cpu(), sys.argv[2]); print('LAM', repr(lam), it)")
        repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"tuning_v_{os.getpid()}.pt")
        out = subprocess.run([sys.executable, "-c", code, repo, path], env=env,
                             capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-3000:]
        a = dev.generate("random", 4352, torch.float64, seed=2, device=DEV)
        lam, v, it, st = dev.DeviceSolver(DEV).solve(a, eps=0.0, max_itr=8)
        line = [ln for ln in out.stdout.splitlines() if ln.startswith("LAM")][-1].split()
        assert float(line[1]) == lam and int(line[2]) == it
        assert torch.equal(torch.load(path, weights_only=True), v.cpu())
        os.remove(path)

else:
    @pytest.fixture(scope="module")
    def solver():
        s = dev.DeviceSolver(DEV)
        yield s
        s.close()

    @pytest.mark.parametrize("dt,n", [(np.float64, 4352), (np.float64, 16385),
                                      (np.float32, 6144), (np.float32, 23171)])
    def test_deferred_caps_do_not_change_results(solver, dt, n):
        """The workgroups-per-CU caps of the deferred launches (st_set_defer_caps,
        dynamic LDS reserved per workgroup) change residency only: a solve under
        the shipped table, with every cap removed and with every slot at 2 / 8
        per CU is bit-identical (λ, v, iterations, final matrix)."""
        L = _lib.load()
        d = 1 if dt == np.float64 else 0
        nt = 1 if n * n * np.dtype(dt).itemsize >= (2 << 30) else 0
        base = dev.generate("random", n, TD[dt], seed=8, device=DEV)
        slots = (0, 1, 2, 3, 4, 6)
        saved = {sl: L.st_set_defer_caps(d, nt, sl, 0) for sl in slots}     # read + clear
        try:
            for sl in slots:
                L.st_set_defer_caps(d, nt, sl, saved[sl])                   # shipped table
            out = []
            for cap in (None, 0, 2, 8):
                if cap is not None:
                    for sl in slots:
                        assert L.st_set_defer_caps(d, nt, sl, cap) >= 0
                a = base.clone()
                r = solver.solve(a, inplace=True, eps=0.0, max_itr=9)
                out.append((r[0], r[2], r[1].cpu(), a))
            for o in out[1:]:
                assert o[0] == out[0][0] and o[1] == out[0][1]
                assert torch.equal(o[2], out[0][2]) and torch.equal(o[3], out[0][3])
        finally:
            for sl in slots:
                L.st_set_defer_caps(d, nt, sl, saved[sl])


    @pytest.mark.parametrize("n", [4352, 8192, 10240])
    def test_deferred_ntload_does_not_change_results(solver, n):
        """Non-temporal matrix loads in the cached fp64 deferred rounds
        (st_set_defer_ntload, per block size class) change the cache policy
        only: a solve under the shipped mask, with cached loads throughout, with
        every round's loads non-temporal and with the storing round's stores
        non-temporal too (bit 7) is bit-identical (λ, v, iterations, final
        matrix)."""
        L = _lib.load()
        cls = L.st_defer_ntload_class(n, n, 1)
        assert cls == {4352: 0, 8192: 1, 10240: 2}[n]
        base = dev.generate("random", n, torch.float64, seed=9, device=DEV)
        saved = L.st_set_defer_ntload(cls, 0)
        try:
            out = []
            for mask in (saved, 0, 0x5f, 0xdf):
                assert L.st_set_defer_ntload(cls, mask) >= 0
                a = base.clone()
                r = solver.solve(a, inplace=True, eps=0.0, max_itr=9)
                out.append((r[0], r[2], r[1].cpu(), a))
            for o in out[1:]:
                assert o[0] == out[0][0] and o[1] == out[0][1]
                assert torch.equal(o[2], out[0][2]) and torch.equal(o[3], out[0][3])
        finally:
            L.st_set_defer_ntload(cls, saved)


    @pytest.mark.parametrize("n,dtype", [(8192, "f32"), (16384, "f64"), (23200, "f32")])
    def test_deferred_cache_flip_does_not_change_results(solver, n, dtype):
        """The deferred rounds' cache policy on the other forms
        (st_set_defer_cache: cached fp32 blocks, and the non-temporal form from
        2 GiB, whose loads / stores a mask turns cached) moves no result: λ, v,
        iterations and the final matrix are bit-identical under every mask."""
        L = _lib.load()
        d = 1 if dtype == "f64" else 0
        dt = torch.float64 if d else torch.float32
        cls = L.st_every_cache_class(n, n, d)
        assert cls == {8192: 0, 16384: 3, 23200: 3}[n]
        base = dev.generate("random", n, dt, seed=12, device=DEV)
        saved = L.st_set_defer_cache(d, cls, 0)
        try:
            out = []
            for mask in (saved, 0x1f, 0x41, 0xdf):
                assert L.st_set_defer_cache(d, cls, mask) >= 0
                a = base.clone()
                r = solver.solve(a, inplace=True, eps=0.0, max_itr=9)
                out.append((r[0], r[2], r[1].cpu(), a))
            for o in out[1:]:
                assert o[0] == out[0][0] and o[1] == out[0][1]
                assert torch.equal(o[2], out[0][2]) and torch.equal(o[3], out[0][3])
        finally:
            L.st_set_defer_cache(d, cls, saved)


    @pytest.mark.parametrize("n,dtype", [(6144, "f64"), (4608, "f64"), (8192, "f32")])
    def test_mfree_shapes_do_not_change_results(solver, n, dtype):
        """Every launch shape of the matrix-free round (st_set_mfree_shape:
        cached 2 / 4 rows per group, non-temporal 4 rows, the table) gives the
        same solve bit for bit (λ, v, iterations): the rows a workgroup takes
        change no row's summation order."""
        L = _lib.load()
        dt = torch.float64 if dtype == "f64" else torch.float32
        a = dev.generate("random", n, dt, seed=14, device=DEV)
        saved = L.st_set_mfree_shape(0)
        try:
            out = []
            for shape in (0, 1, 2, 3):
                assert L.st_set_mfree_shape(shape) >= 0
                r = solver.solve(a, matrix_free=True, eps=0.0, max_itr=7)
                out.append((r[0], r[2], r[1].cpu()))
            for o in out[1:]:
                assert o[0] == out[0][0] and o[1] == out[0][1] and torch.equal(o[2], out[0][2])
        finally:
            L.st_set_mfree_shape(saved)


    @pytest.mark.parametrize("n", [4352, 8192, 10240])
    def test_every_cache_does_not_change_results(solver, n):
        """The every-round flat launch's cache policy (st_set_every_cache: the
        loads', the stores' or both policies turned over, per block size class)
        changes where lines are kept only: a solve that stores every round is
        bit-identical under every policy (λ, v, iterations, final matrix)."""
        L = _lib.load()
        cls = L.st_every_cache_class(n, n, 1)
        assert cls == {4352: 0, 8192: 1, 10240: 2}[n]
        base = dev.generate("random", n, torch.float64, seed=11, device=DEV)
        saved = L.st_set_every_cache(cls, 0)
        try:
            out = []
            # (policy, piece tile, workgroups per CU): st_set_every_tile and
            # st_set_every_caps are for tools, and move no result either
            for pol, tile, cap in ((saved, 0, 0), (0, 0, 0), (1, 0, 0), (2, 0, 0), (3, 0, 0),
                                   (saved, 1, 0), (saved, 16, 3)):
                assert L.st_set_every_cache(cls, pol) >= 0
                assert L.st_set_every_tile(cls, tile) >= 0 and L.st_set_every_caps(cls, cap) >= 0
                a = base.clone()
                r = solver.solve(a, inplace=True, eps=0.0, max_itr=7, write_every_round=True)
                out.append((r[0], r[2], r[1].cpu(), a))
            for o in out[1:]:
                assert o[0] == out[0][0] and o[1] == out[0][1]
                assert torch.equal(o[2], out[0][2]) and torch.equal(o[3], out[0][3])
        finally:
            L.st_set_every_cache(cls, saved)
            L.st_set_every_tile(cls, 0)
            L.st_set_every_caps(cls, 0)


    @pytest.mark.parametrize("limit", [8, 1000, 4096])
    def test_flat_2d_grid_bitwise(solver, orc, limit):
        """A flat launch of more workgroups than one dispatch dimension holds
        (2^32 - 1 work-items: fp64 from 131072², test_max_single_gpu_size) goes
        2-D.  Forced 2-D at small sizes (st_set_flat_grid_limit; widths that
        divide the grid and ones that leave padding workgroups) every launch
        form - the every-round and deferred solves, the two split halves - is
        bit-identical to the 1-D grid."""
        n = 4352                                                  # 144.5 MiB: flat
        base = dev.generate("random", n, torch.float64, seed=6, device=DEV)
        a = orc.random_matrix(6000, 3, np.float64, nrows=2049)    # split block
        s_full = torch.from_numpy(orc.random_matrix(6000, 9, np.float64, nrows=1)[0] + 0.5).to(DEV)

        def run():
            out = []
            for every in (False, True):
                m = base.clone()
                r = solver.solve(m, inplace=True, eps=0.0, max_itr=5, write_every_round=every)
                out += [r[0], r[2], r[1].cpu(), m]
            ta, tv = torch.from_numpy(a).to(DEV), torch.ones(6000, dtype=torch.float64, device=DEV)
            s_next = torch.empty(2049, dtype=torch.float64, device=DEV)
            part = dev.split_flat_scratch(2049, 6000, 3000, 5049, torch.float64, DEV)
            state = dev.new_state(DEV)
            for span in (dev.SPAN_LOCAL, dev.SPAN_REMOTE):
                dev.split_flat_round(ta, s_full, s_next if span == dev.SPAN_REMOTE else None,
                                     part, tv if span == dev.SPAN_REMOTE else None, state,
                                     span=span, row0=3000, col0=3000, col1=5049, eps=1e-3, k=1)
            return out + [ta, s_next, tv, dev.read_state(state)]

        ref = run()
        try:
            assert dev.set_flat_grid_limit(limit) == limit
            got = run()
        finally:
            assert dev.set_flat_grid_limit(0) == 16777208
        for x, y in zip(ref, got):
            assert (torch.equal(x, y) if isinstance(x, torch.Tensor) else x == y)
