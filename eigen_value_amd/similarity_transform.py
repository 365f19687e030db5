"""Drop-in Python wrapper: same class, method and return tuple as the
reference's ``wrapper/python/similarity_transform.py`` (class ``EigenValue``,
lines 18-78), backed by the MI355X library instead of the SYCL one.

    import eigen_value_amd.similarity_transform as st
    ev = st.EigenValue()
    λ, v, ts, itr = ev.similarity_transform(mat)     # mat: float32 (n, n)

Differences, all additive:

* ``so_path`` resolves to the in-tree ``eigen_value_amd/lib/`` build
  (``EIGEN_VALUE_LIB`` overrides); the reference used a CWD-relative
  ``'../libsimilarity_transform.so'`` (line 19).
* float64 matrices are accepted and dispatched to ``max_eigen_value_f64``
  (the reference asserts float32, line 57); float32 behaviour is unchanged.
* ``iter_cnt`` is a ``uint32`` buffer, matching the C ``uint*`` (the
  reference passes ``np.uint`` = uint64, lines 63-64,73).
* a negative return from the library raises ``EigenValueError`` with the
  library's message (the reference had no error path).
* ``close()`` / context manager release the device context (the reference
  leaks its queue).
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib


class EigenValue:
    so_path: str = _lib.lib_path()
    sycl_q: ctypes.c_void_p = None   # name kept for drop-in compatibility
    so_lib: ctypes.CDLL = None

    def __init__(self) -> None:
        """Load the shared library and create a device context (queue)."""
        import os
        if not os.path.exists(self.so_path):
            raise Exception(
                f'failed to find shared library `{os.path.abspath(self.so_path)}`')
        self.so_lib = _lib.load(None if self.so_path == _lib.lib_path() else self.so_path)
        self.sycl_q = ctypes.c_void_p()
        self.so_lib.make_queue(ctypes.byref(self.sycl_q))
        if self.sycl_q.value is None:
            raise Exception(f'failed to get default HIP queue: {_lib.last_error(self.so_lib)}')

    # ------------------------------------------------------------------
    def similarity_transform(self, mat: np.ndarray) -> Tuple[np.floating, np.ndarray, int, int]:
        """Largest eigenvalue λ and eigenvector v of a positive square matrix.

        Returns ``(λ, v, ts_ms, iterations)`` exactly as the reference
        (wrapper/python/similarity_transform.py:42-78): λ is ``np.float32``
        for float32 input (``np.float64`` for float64), ``ts`` the elapsed
        milliseconds reported by the library (host->device copy included,
        as in similarity_transform.cpp:36-58), ``iterations`` the number of
        similarity transforms applied before convergence.  ``A v ≈ λ v``.
        """
        m, n = mat.shape
        assert m == n, "must be square matrix of floating points !"
        assert mat.dtype.num in (11, 12), "dtype of input matrix must be float32 (or float64) !"
        mat = np.ascontiguousarray(mat)
        eigen_val = np.empty(1, dtype=mat.dtype)
        eigen_vec = np.empty(n, dtype=mat.dtype)
        iter_cnt = np.zeros(1, dtype=np.uint32)
        fn = self.so_lib.max_eigen_value if mat.dtype == np.float32 else self.so_lib.max_eigen_value_f64
        ts = fn(self.sycl_q, mat.ctypes.data, eigen_val.ctypes.data,
                eigen_vec.ctypes.data, n, iter_cnt.ctypes.data)
        _lib.check(ts, "max_eigen_value", self.so_lib)
        return eigen_val[0], eigen_vec, int(ts), int(iter_cnt[0])

    # ------------------------------------------------------------------
    def similarity_transform_ex(self, mat: np.ndarray, *, eps: Optional[float] = None,
                                max_itr: int = 0, semantics: int = _lib.ST_SEM_SYCL,
                                batch: int = 0, time_kernels: bool = False,
                                matrix_free: bool = False, round_loop: bool = False,
                                write_every_round: bool = False, trace_sums: bool = False):
        """Extended call: options + statistics (``max_eigen_value_ex``).
        ``round_loop`` keeps one launch per round where the whole solve would
        fit one workgroup (``ST_FLAG_ROUND_LOOP``; identical results);
        ``write_every_round`` stores the matrix every round where the flat
        round would store it every 6th (``ST_FLAG_WRITE_EVERY_ROUND``;
        identical results); ``trace_sums`` records every evaluated round's
        row sums (``ST_FLAG_TRACE_SUMS``; identical results), read back with
        ``last_round_sums()``.

        Returns ``(λ, v, ts_ms, iterations, stats_dict)``."""
        m, n = mat.shape
        assert m == n, "must be square matrix of floating points !"
        mat = np.ascontiguousarray(mat)
        if mat.dtype not in (np.float32, np.float64):
            raise TypeError("float32 or float64 matrix required")
        flags = ((_lib.ST_FLAG_TIME_KERNELS if time_kernels else 0)
                 | (_lib.ST_FLAG_MATRIX_FREE if matrix_free else 0)
                 | (_lib.ST_FLAG_ROUND_LOOP if round_loop else 0)
                 | (_lib.ST_FLAG_WRITE_EVERY_ROUND if write_every_round else 0)
                 | (_lib.ST_FLAG_TRACE_SUMS if trace_sums else 0))
        self._trace = (n, mat.dtype)
        opt = _lib.st_options(-1.0 if eps is None else float(eps), max_itr, semantics,
                              batch, flags)
        stats = _lib.st_stats()
        eigen_val = np.empty(1, dtype=mat.dtype)
        eigen_vec = np.empty(n, dtype=mat.dtype)
        iter_cnt = np.zeros(1, dtype=np.uint32)
        dtype = _lib.DTYPE_F32 if mat.dtype == np.float32 else _lib.DTYPE_F64
        ts = self.so_lib.max_eigen_value_ex(
            self.sycl_q, dtype, mat.ctypes.data, eigen_val.ctypes.data,
            eigen_vec.ctypes.data, n, iter_cnt.ctypes.data,
            ctypes.byref(opt), ctypes.byref(stats))
        _lib.check(ts, "max_eigen_value_ex", self.so_lib)
        return eigen_val[0], eigen_vec, int(ts), int(iter_cnt[0]), stats.as_dict()

    def last_round_times(self) -> np.ndarray:
        """Per-round kernel times (ms) of the last ``similarity_transform_ex``
        call made with ``time_kernels=True`` (empty otherwise)."""
        L = self.so_lib
        n = _lib.check(L.st_last_round_times(self.sycl_q, None, 0), "st_last_round_times", L)
        out = np.zeros(n, dtype=np.float32)
        if n:
            _lib.check(L.st_last_round_times(self.sycl_q, out.ctypes.data, n),
                       "st_last_round_times", L)
        return out

    def last_round_sums(self) -> np.ndarray:
        """Row sums s_0 .. s_{rounds-1} of the last ``similarity_transform_ex``
        call made with ``trace_sums=True``, shape (rounds, n) (empty
        otherwise)."""
        n, dt = getattr(self, "_trace", (0, np.float32))
        return _lib.round_sums(self.so_lib, self.sycl_q, n, dt)

    # ------------------------------------------------------------------
    def close(self) -> None:
        if self.so_lib is not None and self.sycl_q is not None and self.sycl_q.value:
            self.so_lib.destroy_queue(self.sycl_q)
            self.sycl_q = ctypes.c_void_p()

    def __enter__(self) -> "EigenValue":
        return self

    def __exit__(self, *exc) -> None:
        self.close()
