"""Native single-process multi-GPU solve (``st_solve_multi_*``): P devices
driven from one host thread, row-block sharded, one RCCL all-gather of the
row-sum vector per round.  The one-process-per-GPU form over
torch.distributed is ``eigen_value_amd.sharded``; both run the same kernels.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Union

import numpy as np

from . import _lib

_GEN = {"host": 0, "hilbert": 1, "random": 2}


def solve_multi(n: int, matrix: Union[str, np.ndarray] = "hilbert", *, ngpus: int = 1,
                devices: Optional[Sequence[int]] = None, seed: int = 0, dtype=np.float64,
                eps: Optional[float] = None, max_itr: int = 0,
                semantics: int = _lib.ST_SEM_SYCL, matrix_free: bool = False, batch: int = 0,
                write_every_round: bool = False):
    """Returns (λ, v: ndarray, iterations, stats).

    ``matrix`` is a host (n, n) array, or "hilbert" / "random" to generate
    each device's rows in its own HBM (no host copy of the matrix)."""
    L = _lib.load()
    if isinstance(matrix, np.ndarray):
        mat = np.ascontiguousarray(matrix)
        assert mat.shape == (n, n), "must be square"
        dtype = mat.dtype
        kind, ptr = 0, mat.ctypes.data
    else:
        kind, ptr, mat = _GEN[matrix], None, None
    dtype = np.dtype(dtype)
    if dtype not in (np.float32, np.float64):
        raise TypeError("float32 or float64 required")
    sfx = "f32" if dtype == np.float32 else "f64"
    if devices is not None:
        ngpus = len(devices)
        dev_arr = (ctypes.c_int * ngpus)(*devices)
    else:
        dev_arr = None
    ev = np.zeros(1, dtype=dtype)
    v = np.zeros(n, dtype=dtype)
    it = ctypes.c_uint32()
    flags = ((_lib.ST_FLAG_MATRIX_FREE if matrix_free else 0)
             | (_lib.ST_FLAG_WRITE_EVERY_ROUND if write_every_round else 0))
    opt = _lib.st_options(-1.0 if eps is None else float(eps), max_itr, semantics, batch, flags)
    stats = _lib.st_stats()
    rc = getattr(L, f"st_solve_multi_{sfx}")(ptr, n, ngpus, dev_arr, kind, seed,
                                             ev.ctypes.data, v.ctypes.data, ctypes.byref(it),
                                             ctypes.byref(opt), ctypes.byref(stats))
    _lib.check(rc, "st_solve_multi")
    return ev[0], v, int(it.value), stats.as_dict()
