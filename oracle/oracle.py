"""CPU oracle for the similarity-transform max-eigenvalue iteration.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the
checker (or as the timed CPU baseline).  The product path
(``eigen_value_amd`` / ``libsimilarity_transform.so``) never imports it.

Two layers:

* ``st_oracle.c`` (ctypes, built by ``oracle/Makefile``) — the O(N^2) C
  restatement, OpenMP over rows, numpy pairwise row-sum order.  See the C
  file header for the reference file:line each function follows.
* numpy forms of the input generators (``hilbert``, ``random_matrix``) that
  are bit-identical to the C and HIP generators.

Parity pins (tests/golden/): bit-identical to the reference's ``main.py``
(fp64, SEM_MAINPY) on the 3x3 KAT, Hilbert 32..1024 and seeded random
matrices; SEM_SYCL reproduces the reference's published Hilbert round counts
(README.md:70-76) and the tests/test.cpp:99-102 3x3 known answer.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import NamedTuple, Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libst_oracle.so")

SEM_SYCL = 0    # cyclic stop, A *= (1/s_r)*s_c, count = break index
SEM_MAINPY = 1  # non-cyclic stop, ((1/s_r)*A)*s_c, count = itr + 1

EPS_F32 = np.float32(1e-3)   # include/similarity_transform.hpp:4 (float)
EPS_F64 = np.float64(1e-3)   # main.py:6
MAX_ITR = 1000               # include/similarity_transform.hpp:5

_lib: Optional[ctypes.CDLL] = None


def build(force: bool = False) -> str:
    """Compile st_oracle.c with the committed Makefile (gcc only)."""
    if force or not os.path.exists(LIB_PATH) or (
            os.path.getmtime(LIB_PATH) < os.path.getmtime(os.path.join(HERE, "st_oracle.c"))):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB_PATH)
        _declare(_lib)
    return _lib


def _declare(L: ctypes.CDLL) -> None:
    P = ctypes.c_void_p
    u32, u64, i32, i64 = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int, ctypes.c_int64
    for sfx, T in (("f64", ctypes.c_double), ("f32", ctypes.c_float)):
        getattr(L, f"orc_pairwise_sum_{sfx}").argtypes = [P, i64]
        getattr(L, f"orc_pairwise_sum_{sfx}").restype = T
        getattr(L, f"orc_hilbert_{sfx}").argtypes = [P, u32, u32, u32]
        getattr(L, f"orc_random_{sfx}").argtypes = [P, u32, u32, u32, u64]
        getattr(L, f"orc_rowsum_{sfx}").argtypes = [P, P, u32, u32]
        getattr(L, f"orc_find_max_{sfx}").argtypes = [P, u32]
        getattr(L, f"orc_find_max_{sfx}").restype = T
        getattr(L, f"orc_compute_eigen_vector_{sfx}").argtypes = [P, T, P, u32]
        getattr(L, f"orc_stop_{sfx}").argtypes = [P, u32, T, i32]
        getattr(L, f"orc_stop_{sfx}").restype = i32
        getattr(L, f"orc_compute_next_{sfx}").argtypes = [P, P, u32, u32, u32, i32]
        getattr(L, f"orc_similarity_transform_{sfx}").argtypes = [
            P, u32, T, u32, i32, i32, P, P, P, P, P, P]
        getattr(L, f"orc_similarity_transform_{sfx}").restype = i32
        getattr(L, f"orc_similarity_transform_trace_{sfx}").argtypes = [
            P, u32, T, u32, i32, i32, P, P, P, P, P, P, P]
        getattr(L, f"orc_similarity_transform_trace_{sfx}").restype = i32
        getattr(L, f"orc_similarity_transform_gen_{sfx}").argtypes = [
            i32, u64, u32, T, u32, i32, i32, u32, P, P, P, P, P]
        getattr(L, f"orc_similarity_transform_gen_{sfx}").restype = i32
    L.orc_max_threads.restype = i32


def _sfx(dtype) -> str:
    dtype = np.dtype(dtype)
    if dtype == np.float64:
        return "f64"
    if dtype == np.float32:
        return "f32"
    raise TypeError(f"oracle supports float32/float64, got {dtype}")


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


# --------------------------------------------------------------------------
# generators (numpy forms; bit-identical to orc_* and the HIP generators)
# --------------------------------------------------------------------------
def hilbert(n: int, dtype=np.float64, nrows: Optional[int] = None, row0: int = 0) -> np.ndarray:
    """utils.cpp:137-154 — A[r][c] = 1/(r+c+1) computed in ``dtype``."""
    nrows = n if nrows is None else nrows
    r = np.arange(row0, row0 + nrows, dtype=np.int64)[:, None]
    c = np.arange(n, dtype=np.int64)[None, :]
    d = (r + c + 1).astype(dtype)
    return (np.asarray(1, dtype=dtype) / d).astype(dtype)


_SM1 = np.uint64(0x9E3779B97F4A7C15)
_SM2 = np.uint64(0xBF58476D1CE4E5B9)
_SM3 = np.uint64(0x94D049BB133111EB)


def splitmix(seed: int, idx: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * _SM1
        z = (z ^ (z >> np.uint64(30))) * _SM2
        z = (z ^ (z >> np.uint64(27))) * _SM3
        return z ^ (z >> np.uint64(31))


def random_matrix(n: int, seed: int = 0, dtype=np.float64,
                  nrows: Optional[int] = None, row0: int = 0) -> np.ndarray:
    """Seeded U(0,1] counter-hash matrix (replaces utils.cpp:125-134)."""
    nrows = n if nrows is None else nrows
    idx = (np.arange(row0, row0 + nrows, dtype=np.uint64)[:, None] * np.uint64(n)
           + np.arange(n, dtype=np.uint64)[None, :])
    z = splitmix(seed, idx)
    if np.dtype(dtype) == np.float64:
        return ((z >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * 2.0 ** -53
    return (((z >> np.uint64(40)) + np.uint64(1)).astype(np.float32)
            * np.float32(2.0 ** -24)).astype(np.float32)


# --------------------------------------------------------------------------
# per-kernel restatements (C)
# --------------------------------------------------------------------------
def pairwise_sum(a: np.ndarray):
    a = np.ascontiguousarray(a)
    return getattr(lib(), f"orc_pairwise_sum_{_sfx(a.dtype)}")(_ptr(a), a.size)


def rowsum(mat: np.ndarray) -> np.ndarray:
    mat = np.ascontiguousarray(mat)
    s = np.empty(mat.shape[0], dtype=mat.dtype)
    getattr(lib(), f"orc_rowsum_{_sfx(mat.dtype)}")(_ptr(mat), _ptr(s), mat.shape[0], mat.shape[1])
    return s


def find_max(s: np.ndarray):
    s = np.ascontiguousarray(s)
    return getattr(lib(), f"orc_find_max_{_sfx(s.dtype)}")(_ptr(s), s.size)


def compute_eigen_vector(s: np.ndarray, m, v: np.ndarray) -> np.ndarray:
    v = np.array(v, dtype=s.dtype, copy=True)
    getattr(lib(), f"orc_compute_eigen_vector_{_sfx(s.dtype)}")(_ptr(np.ascontiguousarray(s)), m, _ptr(v), s.size)
    return v


def stop(s: np.ndarray, eps=None, cyclic: bool = True) -> bool:
    s = np.ascontiguousarray(s)
    if eps is None:
        eps = EPS_F32 if s.dtype == np.float32 else EPS_F64
    return bool(getattr(lib(), f"orc_stop_{_sfx(s.dtype)}")(_ptr(s), s.size, eps, int(cyclic)))


def compute_next(mat: np.ndarray, s_full: np.ndarray, row0: int = 0, order: int = 0) -> np.ndarray:
    out = np.array(mat, copy=True, order="C")
    s_full = np.ascontiguousarray(s_full, dtype=mat.dtype)
    getattr(lib(), f"orc_compute_next_{_sfx(mat.dtype)}")(
        _ptr(out), _ptr(s_full), out.shape[0], out.shape[1], row0, order)
    return out


class Solve(NamedTuple):
    eigen_val: float
    eigen_vec: np.ndarray
    iter_count: int
    rounds_evaluated: int
    loop_ms: float
    max_dsum: np.ndarray   # per evaluated round, max |s_i - s_next| inspected
    row_sums: Optional[np.ndarray] = None  # (rounds_evaluated, n) with trace=True


def similarity_transform(mat: np.ndarray, semantics: int = SEM_SYCL, eps=None,
                         max_itr: int = MAX_ITR, nthreads: int = 0,
                         trace: bool = False) -> Solve:
    """Whole solve (similarity_transform.cpp:5-75 or main.py:30-47).
    ``trace`` also returns every evaluated round's row sums s_k
    (``row_sums``, the vectors the stop test compared)."""
    mat = np.ascontiguousarray(mat)
    if mat.dtype not in (np.float32, np.float64):
        mat = mat.astype(np.float64)
    n = mat.shape[0]
    assert mat.shape == (n, n), "must be square"
    sfx = _sfx(mat.dtype)
    if eps is None:
        eps = EPS_F32 if sfx == "f32" else EPS_F64
    ev = np.zeros(1, dtype=mat.dtype)
    vec = np.zeros(n, dtype=mat.dtype)
    it = np.zeros(1, dtype=np.uint32)
    ev_n = np.zeros(1, dtype=np.uint32)
    ms = np.zeros(1, dtype=np.float64)
    dsum = np.zeros(max(max_itr, 1), dtype=np.float64)
    args = (_ptr(mat), n, eps, max_itr, semantics, nthreads,
            _ptr(ev), _ptr(vec), _ptr(it), _ptr(dsum), _ptr(ms), _ptr(ev_n))
    sums = None
    if trace:
        sums = np.zeros((max(max_itr, 1), n), dtype=mat.dtype)
        rc = getattr(lib(), f"orc_similarity_transform_trace_{sfx}")(*args, _ptr(sums))
    else:
        rc = getattr(lib(), f"orc_similarity_transform_{sfx}")(*args)
    if rc != 0:
        raise ValueError("oracle solve failed (bad arguments or out of memory)")
    r = int(ev_n[0])
    return Solve(ev[0], vec, int(it[0]), r, float(ms[0]), dsum[:r],
                 None if sums is None else sums[:r])


def max_threads() -> int:
    return int(lib().orc_max_threads())


def generate_c(kind: str, n: int, seed: int = 0, dtype=np.float64,
               nrows: Optional[int] = None, row0: int = 0) -> np.ndarray:
    """The C generators (orc_hilbert_* / orc_random_*, OpenMP): the same bits
    as hilbert() / random_matrix(), without numpy's temporaries — for the
    full-size configs (8 GiB at 32768^2 fp64)."""
    nrows = n if nrows is None else nrows
    out = np.empty((nrows, n), dtype=dtype)
    L = lib()
    if kind == "hilbert":
        getattr(L, f"orc_hilbert_{_sfx(dtype)}")(_ptr(out), nrows, n, row0)
    elif kind == "random":
        getattr(L, f"orc_random_{_sfx(dtype)}")(_ptr(out), nrows, n, row0, seed)
    else:
        raise ValueError(f"unknown kind {kind!r}")
    return out


def similarity_transform_gen(kind: str, n: int, seed: int = 0, dtype=np.float64,
                             semantics: int = SEM_SYCL, eps=None, max_itr: int = 64,
                             nthreads: int = 0, chunk_rows: int = 2048) -> Solve:
    """Whole solve of a GENERATED input without holding it (orc_similarity_
    transform_gen_*): each round regenerates A_0 in row blocks and re-applies
    the recorded transforms.  Bit-identical to similarity_transform() on the
    same matrix; for the sizes that do not fit the host twice (configs[3]).
    ``max_itr`` also bounds the row-sum history kept (max_itr * n)."""
    sfx = _sfx(dtype)
    T = np.dtype(dtype).type
    if eps is None:
        eps = EPS_F32 if T is np.float32 else EPS_F64
    ev = np.zeros(1, dtype=dtype)
    vec = np.zeros(n, dtype=dtype)
    it = np.zeros(1, dtype=np.uint32)
    ms = np.zeros(1, dtype=np.float64)
    ev_n = np.zeros(1, dtype=np.uint32)
    k = {"hilbert": 1, "random": 2}[kind]
    rc = getattr(lib(), f"orc_similarity_transform_gen_{sfx}")(
        k, seed, n, T(eps), max_itr, semantics, nthreads, chunk_rows,
        _ptr(ev), _ptr(vec), _ptr(it), _ptr(ms), _ptr(ev_n))
    if rc != 0:
        raise ValueError("oracle generated solve failed (bad arguments or out of memory)")
    return Solve(ev[0], vec, int(it[0]), int(ev_n[0]), float(ms[0]),
                 np.zeros(0, dtype=np.float64))
