"""The drop-in boundary driven through the reference wrapper's OWN ctypes
binding (wrapper/python/similarity_transform.py:33-37,59-76), written out
here from its published declarations (not copied):

* ``make_queue`` with ``argtypes = [POINTER(c_void_p)]`` (:35-37);
* ``max_eigen_value`` with ``restype = c_int64`` and ``argtypes = [c_void_p,
  ndpointer(float32, 2-D, CONTIGUOUS), ndpointer(float32, 1-D),
  ndpointer(float32, 1-D), c_uint, ndpointer(np.uint, 1-D)]`` (:59-69);
* a zeroed ``np.uint`` (= uint64 on LP64) iteration-count buffer (:73) behind
  the C ``unsigned int*`` (wrapper/similarity_transform.cpp:14-37): the
  library writes its low 32 bits, the zeroed high half keeps the value.

The library is opened with a fresh ``ctypes.CDLL`` (its own function
objects, so these argtypes do not touch eigen_value_amd._lib's), and the
results must equal ``EigenValue.similarity_transform`` bit for bit.
"""
import ctypes

import numpy as np
import pytest

from eigen_value_amd import _lib

pytestmark = pytest.mark.gpu


class ReferenceBinding:
    """What a maintainer of the reference gets by pointing its wrapper's
    ``so_path`` at libsimilarity_transform.so."""

    def __init__(self):
        self.so_lib = ctypes.CDLL(_lib.lib_path())
        self.so_lib.make_queue.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.q = ctypes.c_void_p()
        self.so_lib.make_queue(ctypes.byref(self.q))
        assert self.q.value is not None, "make_queue wrote NULL"

    def similarity_transform(self, mat):
        m, n = mat.shape
        assert m == n and mat.dtype.num == 11
        mat_t = np.ctypeslib.ndpointer(dtype=np.float32, ndim=2, flags="CONTIGUOUS")
        vec_t = np.ctypeslib.ndpointer(dtype=np.float32, ndim=1, flags="CONTIGUOUS")
        itr_t = np.ctypeslib.ndpointer(dtype=np.uint, ndim=1, flags="CONTIGUOUS")
        f = self.so_lib.max_eigen_value
        f.restype = ctypes.c_int64
        f.argtypes = [ctypes.c_void_p, mat_t, vec_t, vec_t, ctypes.c_uint, itr_t]
        eigen_val = np.empty(1, dtype=np.float32)
        eigen_vec = np.empty(n, dtype=np.float32)
        iter_cnt = np.zeros(1, dtype=np.uint)
        ts = f(self.q, mat, eigen_val, eigen_vec, n, iter_cnt)
        return eigen_val[0], eigen_vec, ts, iter_cnt[0], iter_cnt

    def close(self):
        # the reference leaks its queue; the library's addition frees it
        self.so_lib.destroy_queue.argtypes = [ctypes.c_void_p]
        self.so_lib.destroy_queue(self.q)


def _hilbert(n):
    i = np.arange(n, dtype=np.int64)
    return np.float32(1.0) / (i[:, None] + i[None, :] + 1).astype(np.float32)


@pytest.mark.parametrize("case", ["kat3", "random1024", "hilbert128", "hilbert1000"])
def test_reference_wrapper_binding(orc, golden, case):
    kat = golden[2]["kat3"]
    if case == "kat3":
        # tests/test.cpp:84-102 (the reference's 3x3 known answer)
        mat = np.array(kat["matrix"], dtype=np.float32)
    elif case == "random1024":
        mat = orc.random_matrix(1024, 11, np.float32)
    elif case == "hilbert128":
        mat = _hilbert(128)            # configs[0]'s size: the single-launch solve
    else:
        mat = _hilbert(1000)           # a dim the reference would reject (1000 % 32)
    mine = ReferenceBinding()
    try:
        lam, vec, ts, itr, itr_buf = mine.similarity_transform(mat)
    finally:
        mine.close()
    assert itr_buf.dtype == np.uint64 and itr_buf.shape == (1,)
    assert ts >= 0, _lib.last_error()
    from eigen_value_amd.similarity_transform import EigenValue
    with EigenValue() as ev:
        lam2, vec2, _, itr2 = ev.similarity_transform(mat)
    assert isinstance(lam, np.float32) and lam == lam2
    assert np.array_equal(vec, vec2)
    assert int(itr) == itr2
    ref = orc.similarity_transform(mat.astype(np.float32), orc.SEM_SYCL)
    assert int(itr) == ref.iter_count
    assert abs(float(lam) - float(ref.eigen_val)) <= 1e-5 * abs(float(ref.eigen_val))
    if case == "kat3":                                   # test.cpp:99-102
        assert abs(float(lam) - kat["eigen_val"]) < kat["tol"]
        assert np.all(np.abs(vec - np.array(kat["eigen_vec"])) < kat["tol"])
