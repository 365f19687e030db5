"""GPU parity at the BASELINE full sizes against the CPU oracle (not only
through size-independent properties), and the communicator's deadline and
failure paths on one device (the multi-device tests are in
tests/test_zz_multi_device.py, which collects last).

Tolerances (as tests/test_gpu_parity.py):
  * fp64 vs the oracle's same-semantics solve: iteration count equal, λ
    relative <= 1e-10, eigenvector max-abs <= 1e-10 (the GPU sums rows in a
    fixed tree, the oracle in numpy's pairwise order);
  * fp32: iteration count equal, λ relative <= 1e-5, eigenvector max-abs
    <= 1e-5 (fp32 row sums of ~16384 carry ulps of 2^-9).

The oracle runs on the box's host cores inside the test where the input fits
the host twice (32768², 8 GiB fp64 / 4 GiB fp32) and must reproduce the
committed pins (tests/golden/large_oracle.json, make_large_oracle.py) bit
for bit; 65536² (32 GiB) is checked against the committed pin only.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no HIP device", allow_module_level=True)

from eigen_value_amd import _lib  # noqa: E402
from eigen_value_amd import device as dev  # noqa: E402
from conftest import host_threads, large_oracle, large_pin  # noqa: E402

DEV = "cuda:0"
NDEV = torch.cuda.device_count()
HOST_THREADS = host_threads()


@pytest.fixture(scope="module")
def solver():
    s = dev.DeviceSolver(DEV)
    yield s
    s.close()


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _host_oracle(orc, name, n, npdt, max_itr):
    """The oracle's SYCL-semantics solve of the seeded input on this host,
    checked bit for bit against the committed pin."""
    mat = orc.generate_c("random", n, 0, npdt)
    ref = orc.similarity_transform(mat, orc.SEM_SYCL, max_itr=max_itr, nthreads=HOST_THREADS)
    del mat
    pin, v_pin = large_oracle(name)
    assert (ref.iter_count, ref.rounds_evaluated) == (pin["iter_count"], pin["rounds_evaluated"])
    assert float(ref.eigen_val) == pin["eigen_val"]
    assert np.array_equal(ref.eigen_vec, v_pin)
    return ref


def test_config2_random32768_f64_vs_oracle(solver, orc):
    """configs[2]: 32768² random fp64 (seed 0), the library's solve loop
    (deferred writes), against the oracle's solve of the same matrix run on
    the host (similarity_transform.cpp:39-53, stop :413-421, count :54)."""
    n = 32768
    ref = _host_oracle(orc, "random32768_f64", n, np.float64, 1000)
    a = dev.generate("random", n, torch.float64, seed=0, device=DEV)
    lam, v, it, st = solver.solve(a, inplace=True)
    assert it == ref.iter_count == 3 and st["rounds"] == ref.rounds_evaluated
    assert abs(lam - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(v.cpu().numpy() - ref.eigen_vec)) <= 1e-10
    # the matrix-free form on a fresh copy of the input
    dev.generate("random", n, torch.float64, seed=0, device=DEV, out=a)
    lam_mf, v_mf, it_mf, _ = solver.solve(a, matrix_free=True)
    assert it_mf == ref.iter_count
    assert abs(lam_mf - ref.eigen_val) <= 1e-10 * ref.eigen_val
    assert np.max(np.abs(v_mf.cpu().numpy() - ref.eigen_vec)) <= 1e-10
    del a, v, v_mf
    _free()


def test_config4_random32768_f32_vs_oracle(solver, orc):
    """configs[4]: 32768² random fp32 over 8 rounds at the reference's
    EPS = 1e-3f (the fp32 iteration does not stop at this size, so both
    exhaust max_itr = 8) against the oracle's fp32 solve run on the host."""
    n = 32768
    ref = _host_oracle(orc, "random32768_f32_8rounds", n, np.float32, 8)
    a = dev.generate("random", n, torch.float32, seed=0, device=DEV)
    lam, v, it, st = solver.solve(a, inplace=True, max_itr=8)
    assert it == ref.iter_count == 8 and st["rounds"] == 8 and st["converged"] == 0
    assert abs(float(lam) - float(ref.eigen_val)) <= 1e-5 * float(ref.eigen_val)
    assert np.max(np.abs(v.cpu().numpy().astype(np.float64) - ref.eigen_vec)) <= 1e-5
    del a, v
    _free()


def test_config3_sharded_p1_vs_oracle():
    """configs[3] size, 65536² random fp64 (32 GiB), through the row-block
    driver (ShardedSimilarityTransform, P = 1: no process group, the block is
    the whole matrix) with its default deferred-write solve, against the
    oracle's solve of the same matrix (committed pin: the streaming oracle,
    bit-identical to the plain loop) and the true Perron root."""
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    pin, v_pin = large_oracle("random65536_f64")
    n = 65536
    sh = ShardedSimilarityTransform(n, torch.float64)
    assert sh.part.nrows == n and sh.deferred_writes
    sh.load("random", seed=0)
    lam, v, it, rounds = sh.solve()
    assert it == pin["iter_count"] == 3 and rounds == pin["rounds_evaluated"]
    assert abs(lam - pin["eigen_val"]) <= 1e-10 * pin["eigen_val"]
    assert np.max(np.abs(v.cpu().numpy() - v_pin)) <= 1e-10
    perron = large_pin(n, "f64")["lambda"]
    assert abs(lam - perron) / perron < 1e-6
    sh.close()
    del sh, v
    _free()


# ---------------------------------------------------------------------------
# the RCCL deadline (st_set_comm_timeout): a communicator whose peer never
# arrives is aborted and named instead of hanging the caller
# ---------------------------------------------------------------------------
_DEADLINE_PROBE = r"""
import ctypes, sys, time
sys.path.insert(0, sys.argv[1])
import torch                      # as in a torch process: torch's RCCL is the one bound
from eigen_value_amd import _lib
L = _lib.load()
L.st_set_comm_timeout(3.0)
uid = ctypes.create_string_buffer(128)
assert L.st_comm_unique_id(uid) == 0
comm = ctypes.c_void_p()
t0 = time.time()
rc = L.st_comm_init(ctypes.byref(comm), 2, 0, uid.raw, 0)   # rank 1 never joins
print("RC", rc, "EL", round(time.time() - t0, 2), "NULL", comm.value is None)
print("ERR", _lib.last_error())
print("RCCL", _lib.rccl_info()["rccl_version"], flush=True)
"""


def test_comm_init_deadline_names_the_stalled_rank(tmp_path):
    """st_comm_init as rank 0 of 2 with no rank 1: the presence check before
    RCCL (st_rendezvous.hip) waits the 3 s deadline, returns -1, leaves the
    handle NULL and names rank 1; no rank entered RCCL, so the process ends
    with a NORMAL interpreter exit and returncode 0 (round 4
    entered RCCL's init, whose abort left a thread that crashed the exit).
    In a child process, bounded, so a hang cannot take the test runner."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _DEADLINE_PROBE, repo], capture_output=True,
                         text=True, timeout=150)
    assert out.returncode == 0, (out.returncode, out.stdout[-2000:], out.stderr[-3000:])
    lines = dict(ln.split(" ", 1) for ln in out.stdout.splitlines()
                 if ln[:3] in ("RC ", "ERR") or ln.startswith("RCCL "))
    rc, _, el, _, null = lines["RC"].split()
    assert int(rc) < 0 and null == "True"
    assert 2.9 <= float(el) < 10.0
    assert "RCCL rank 1 of 2 did not reach st_comm_init" in lines["ERR"], lines["ERR"]
    assert "no rank entered RCCL" in lines["ERR"]
    print("probe:", lines)


_SAME_DEVICE_PROBE = r"""
import ctypes, os, sys, time
sys.path.insert(0, sys.argv[1])
import torch
from eigen_value_amd import _lib
mode, idfile = sys.argv[2], sys.argv[3]
L = _lib.load()
L.st_set_comm_timeout(30.0)
if mode == "host":
    uid = ctypes.create_string_buffer(128)
    assert L.st_comm_unique_id(uid) == 0
    open(idfile + ".tmp", "w").write(uid.raw.hex())
    os.replace(idfile + ".tmp", idfile)
    raw, rank = uid.raw, 0
else:
    while not os.path.exists(idfile):
        time.sleep(0.05)
    raw, rank = bytes.fromhex(open(idfile).read()), 1
comm = ctypes.c_void_p()
t0 = time.time()
rc = L.st_comm_init(ctypes.byref(comm), 2, rank, raw, 0)
print("RC", rc, "EL", round(time.time() - t0, 2), flush=True)
print("ERR", _lib.last_error(), flush=True)
if rc == 0:
    print("DESTROY", L.st_comm_destroy(comm), flush=True)
"""


def test_comm_init_two_ranks_one_device_exit_normally(tmp_path):
    """Two processes join one rendezvous as ranks 0 and 1, both on device 0:
    the presence check passes and both enter ncclCommInitRankConfig, which
    RCCL refuses for a device used twice (profiles/r04_rccl_same_gpu_probe.log)
    - or accepts; either way the init thread reports, owns and aborts the
    failed communicator itself, the call returns promptly, and BOTH
    processes end with a normal exit, returncode 0 (the single-owner init,
    ADVICE r04 st_multi.hip:194)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    idfile = str(tmp_path / "id")
    procs = [subprocess.Popen([sys.executable, "-c", _SAME_DEVICE_PROBE, repo, m, idfile],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for m in ("host", "peer")]
    outs = [p.communicate(timeout=150) for p in procs]
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 0, (p.returncode, so[-2000:], se[-3000:])
        lines = dict(ln.split(" ", 1) for ln in so.splitlines() if ln[:3] in ("RC ", "ERR"))
        rc, _, el = lines["RC"].split()
        assert float(el) < 60.0
        assert "did not reach" not in lines["ERR"] and "no word" not in lines["ERR"]
        if int(rc) < 0:
            assert "ncclCommInitRankConfig" in lines["ERR"], lines["ERR"]
        print("probe:", lines)


_DUPLICATE_PROBE = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
from eigen_value_amd import _lib
from eigen_value_amd.multi import solve_multi
_lib.load().st_set_comm_timeout(20.0)
t0 = time.time()
try:
    solve_multi(3001, "random", devices=[0, 0], seed=3)
    print("RESULT ok")
except _lib.EigenValueError as e:
    print("RESULT error", round(time.time() - t0, 2), str(e).replace("\n", " "))
"""


def test_native_multi_gpu_grouped_init_failure_is_prompt(tmp_path):
    """st_solve_multi_* over two ranks on one device (RCCL refuses a device
    twice): the grouped non-blocking init on the helper thread reports the
    failure as an error naming the call, promptly, instead of hanging - the
    multi-device init path's failure handling, exercised on a one-GPU box.
    (If a future RCCL accepts it, the solve simply has to succeed.)"""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _DUPLICATE_PROBE, repo], capture_output=True,
                         text=True, timeout=150)
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("RESULT")][-1]
    if line.startswith("RESULT error"):
        el = float(line.split()[2])
        assert el < 60 and "st_solve_multi" in line, line
