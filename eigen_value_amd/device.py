"""Device-resident API over torch-ROCm tensors.

Torch is plumbing here (HBM allocation, streams); every kernel is the HIP
code in ``libsimilarity_transform.so`` launched through the C-ABI on the
caller's current torch stream.  Nothing in this module computes on the CPU:
a missing library raises, a non-CUDA tensor raises.
"""
from __future__ import annotations

import ctypes
from typing import Optional

from . import _lib

_SFX = {}


def _torch():
    import torch
    return torch


def _sfx(t) -> str:
    torch = _torch()
    if t.dtype == torch.float64:
        return "f64"
    if t.dtype == torch.float32:
        return "f32"
    raise TypeError(f"float32/float64 tensor required, got {t.dtype}")


def _check_cuda(*ts) -> None:
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("device API needs tensors on a HIP device (cuda:N)")


def _stream(device=None) -> int:
    torch = _torch()
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()


# --------------------------------------------------------------------------
# state
# --------------------------------------------------------------------------
def new_state(device="cuda"):
    """A zeroed 64-byte ``st_state`` on the device (uint8 tensor)."""
    torch = _torch()
    return torch.zeros(64, dtype=torch.uint8, device=device)


def reset_state(state) -> None:
    _check_cuda(state)
    _lib.check(_lib.load().st_state_reset(_ptr(state), _stream(state.device)), "st_state_reset")


def read_state(state) -> dict:
    raw = bytes(state.cpu().numpy().tobytes())
    s = _lib.st_state.from_buffer_copy(raw)
    return dict(done=s.done, round=s.round, iters=s.iters, stop=s.stop,
                eigen_val=s.lambda_, max=s.max, end=s.end)


# --------------------------------------------------------------------------
# generators
# --------------------------------------------------------------------------
def generate(kind: str, n: int, dtype=None, nrows: Optional[int] = None, row0: int = 0,
             seed: int = 0, device="cuda", out=None):
    """Rows [row0, row0+nrows) of an n-wide input matrix generated on device.

    kind: 'hilbert' (utils.cpp:137-154), 'random' (seeded splitmix64 U(0,1]),
    'identity' (utils.cpp:5-27)."""
    torch = _torch()
    dtype = dtype or torch.float64
    nrows = n if nrows is None else nrows
    if out is None:
        out = torch.empty((nrows, n), dtype=dtype, device=device)
    _check_cuda(out)
    L, sfx, st = _lib.load(), _sfx(out), _stream(out.device)
    if kind == "hilbert":
        rc = getattr(L, f"st_generate_hilbert_{sfx}")(_ptr(out), nrows, n, row0, st)
    elif kind == "random":
        rc = getattr(L, f"st_generate_random_{sfx}")(_ptr(out), nrows, n, row0, seed, st)
    elif kind == "identity":
        rc = getattr(L, f"st_generate_identity_{sfx}")(_ptr(out), nrows, n, row0, st)
    else:
        raise ValueError(f"unknown generator {kind!r}")
    _lib.check(rc, f"generate_{kind}")
    return out


def fill(x, value: float) -> None:
    _check_cuda(x)
    _lib.check(getattr(_lib.load(), f"st_fill_{_sfx(x)}")(_ptr(x), x.numel(), value,
                                                          _stream(x.device)), "fill")


# --------------------------------------------------------------------------
# step-level kernels
# --------------------------------------------------------------------------
def rowsum(mat, out=None):
    """s[r] = Σ_c A[r][c] for the rows of ``mat`` (sum_across_rows)."""
    _check_cuda(mat)
    assert mat.is_contiguous() and mat.dim() == 2
    if out is None:
        out = mat.new_empty(mat.shape[0])
    _lib.check(getattr(_lib.load(), f"st_rowsum_{_sfx(mat)}")(
        _ptr(mat), _ptr(out), mat.shape[0], mat.shape[1], _stream(mat.device)), "rowsum")
    return out


def rowsum_flat(mat, out, part) -> None:
    """out[r] = sum_c mat[r][c] in the flat form (st_rowsum_flat): the
    solve loops' initial pass for blocks where ``flat_round_pays``; ``part``
    is ``flat_scratch(nrows, ncols)``."""
    _check_cuda(mat, out, part)
    _lib.check(getattr(_lib.load(), f"st_rowsum_flat_{_sfx(mat)}")(
        _ptr(mat), _ptr(out), _ptr(part), mat.shape[0], mat.shape[1],
        _stream(mat.device)), "rowsum_flat")


def scale_rowsum(mat, s_cur, s_next=None, row0: int = 0,
                 semantics: int = _lib.ST_SEM_SYCL, state=None) -> None:
    """Fused round body, in place on ``mat`` (local rows row0..): see
    ``st_scale_rowsum_*`` in include/similarity_transform.h."""
    _check_cuda(mat, s_cur, s_next, state)
    assert mat.is_contiguous() and mat.dim() == 2
    nrows, ncols = mat.shape
    assert s_cur.numel() >= ncols and s_cur.numel() >= row0 + nrows
    if s_next is not None:
        assert s_next.numel() >= nrows
    _lib.check(getattr(_lib.load(), f"st_scale_rowsum_{_sfx(mat)}")(
        _ptr(mat), _ptr(s_cur), _ptr(s_next), nrows, ncols, row0, semantics,
        _ptr(state), _stream(mat.device)), "scale_rowsum")


def fused_round(mat, s_cur, s_next, v, state, row0: int = 0, eps: float = 1e-3, k: int = 0,
          max_itr: int = _lib.ST_MAX_ITR, semantics: int = _lib.ST_SEM_SYCL) -> None:
    """One whole round k in one launch (``st_round_*``): stats of the full
    s_cur, v update of the local rows, in-place transform, s_next."""
    _check_cuda(mat, s_cur, s_next, v, state)
    assert mat.is_contiguous() and mat.dim() == 2
    nrows, ncols = mat.shape
    assert s_cur.numel() >= ncols and v.numel() >= row0 + nrows and s_next.numel() >= nrows
    _lib.check(getattr(_lib.load(), f"st_round_{_sfx(mat)}")(
        _ptr(mat), _ptr(s_cur), _ptr(s_next), _ptr(v), nrows, ncols, row0, eps, k,
        max_itr, semantics, _ptr(state), _stream(mat.device)), "round")


def mfree_round(mat0, s_prev, s_next, v_prev, v_cur, state, row0: int = 0,
                eps: float = 1e-3, k: int = 1, max_itr: int = _lib.ST_MAX_ITR,
                semantics: int = _lib.ST_SEM_SYCL) -> None:
    """Matrix-free launch k >= 1 (``st_mfree_round_*``): round k-1's stats
    and v_{k-1} (full vector) from s_prev, and s_k for the local rows of A_0."""
    _check_cuda(mat0, s_prev, s_next, v_prev, v_cur, state)
    assert mat0.is_contiguous() and mat0.dim() == 2
    nrows, ncols = mat0.shape
    assert s_prev.numel() >= ncols and v_prev.numel() >= ncols and v_cur.numel() >= ncols
    assert s_next.numel() >= nrows and row0 + nrows <= ncols
    _lib.check(getattr(_lib.load(), f"st_mfree_round_{_sfx(mat0)}")(
        _ptr(mat0), _ptr(s_prev), _ptr(s_next), _ptr(v_prev), _ptr(v_cur), nrows, ncols,
        row0, eps, k, max_itr, semantics, _ptr(state), _stream(mat0.device)), "mfree_round")


def mfree_round_flat(mat0, s_prev, s_next, v_prev, v_cur, part, state, row0: int = 0,
                     eps: float = 1e-3, k: int = 1, max_itr: int = _lib.ST_MAX_ITR,
                     semantics: int = _lib.ST_SEM_SYCL) -> None:
    """mfree_round in the flat form (``st_mfree_round_flat_*``): partial dot
    products per 4 / 8 KB piece into ``part`` (flat_scratch), then s_k and
    v_{k-1}; the solve loops' form for blocks where flat_round_pays."""
    _check_cuda(mat0, s_prev, s_next, v_prev, v_cur, part, state)
    assert mat0.is_contiguous() and mat0.dim() == 2
    nrows, ncols = mat0.shape
    assert s_prev.numel() >= ncols and v_prev.numel() >= ncols and v_cur.numel() >= ncols
    assert s_next.numel() >= nrows and row0 + nrows <= ncols
    assert part.numel() >= int(_lib.load().st_round_flat_scratch(nrows, ncols))
    _lib.check(getattr(_lib.load(), f"st_mfree_round_flat_{_sfx(mat0)}")(
        _ptr(mat0), _ptr(s_prev), _ptr(s_next), _ptr(v_prev), _ptr(v_cur), _ptr(part), nrows,
        ncols, row0, eps, k, max_itr, semantics, _ptr(state), _stream(mat0.device)),
        "mfree_round_flat")


def flat_round_pays(nrows: int, ncols: int, dtype) -> bool:
    """Whether the flat round (st_round_flat) is the faster form for a block."""
    torch = _torch()
    return bool(_lib.load().st_round_flat_pays(nrows, ncols,
                                               1 if dtype == torch.float64 else 0))


def flat_scratch(nrows: int, ncols: int, dtype, device=None):
    """Partial-sum scratch for flat_round on this block."""
    torch = _torch()
    n = int(_lib.load().st_round_flat_scratch(nrows, ncols))
    return torch.empty(n, dtype=dtype, device=device or "cuda")


def flat_round(mat, s_cur, s_next, part, v, state, *, row0: int = 0, eps: float = 1e-3,
               k: int = 0, max_itr: int = _lib.ST_MAX_ITR,
               semantics: int = _lib.ST_SEM_SYCL) -> None:
    """Round k as two launches for large blocks (st_round_flat): the
    transform in short per-piece workgroups (the first row group also takes
    the stats of the full s_cur), then the pieces' partial sums into s_next
    and the v update.  Same contract as fused_round."""
    _check_cuda(mat, s_cur, s_next, part, v, state)
    assert mat.is_contiguous() and mat.dim() == 2
    nrows, ncols = mat.shape
    assert s_cur.numel() >= ncols and s_next.numel() >= nrows and v.numel() >= ncols
    assert row0 + nrows <= ncols
    assert part.numel() >= int(_lib.load().st_round_flat_scratch(nrows, ncols))
    _lib.check(getattr(_lib.load(), f"st_round_flat_{_sfx(mat)}")(
        _ptr(mat), _ptr(s_cur), _ptr(s_next), _ptr(part), _ptr(v), nrows, ncols, row0,
        eps, k, max_itr, semantics, _ptr(state), _stream(mat.device)), "round_flat")


def set_flat_grid_limit(max_x: int = 0) -> int:
    """Testing hook (st_set_flat_grid_limit, include/st_tuning.h): the width
    past which the flat launches go 2-D (0 = the default, the dispatch
    limit).  Returns the limit in force.  The tuning build only: the
    package's library must be libsimilarity_transform_tuning.so
    (EIGEN_VALUE_LIB), whose launches the limit then moves."""
    L = _lib.load()
    if not hasattr(L, "st_set_flat_grid_limit"):
        raise _lib.EigenValueError("st_set_flat_grid_limit: the tuning build only "
                                   "(EIGEN_VALUE_LIB=" + _lib.TUNING_LIB + ")")
    return int(L.st_set_flat_grid_limit(max_x))


def defer_rounds(nrows: int, ncols: int, dtype) -> int:
    """Rounds per store of the deferred flat round on a block
    (st_defer_rounds)."""
    torch = _torch()
    return int(_lib.load().st_defer_rounds(nrows, ncols,
                                           1 if dtype == torch.float64 else 0))


def recip(s, inv) -> None:
    """inv = 1 / s elementwise (st_recip), the reciprocals the deferred round
    re-applies."""
    _check_cuda(s, inv)
    assert inv.numel() >= s.numel() and inv.dtype == s.dtype
    _lib.check(getattr(_lib.load(), f"st_recip_{_sfx(s)}")(
        _ptr(s), _ptr(inv), s.numel(), _stream(s.device)), "recip")


def flat_round_deferred(mat, s_cur, inv_cur, s_next, inv_next, part, v, state,
                        pend_s=(), pend_inv=(), *, store: bool, flush: bool = False,
                        row0: int = 0, eps: float = 1e-3, k: int = 0,
                        max_itr: int = _lib.ST_MAX_ITR,
                        semantics: int = _lib.ST_SEM_SYCL) -> None:
    """Round k of the flat round with deferred writes
    (st_round_flat_deferred): ``mat`` holds the last STORED matrix A_j,
    ``pend_s`` / ``pend_inv`` the pending rounds' full row-sum vectors
    s_j .. s_{k-1} and their reciprocals; A_{k+1} is stored when ``store``.
    s_next / inv_next are the block's slots (as in flat_round).  ``flush``
    (with ``store``) only stores A_{k+1}.  Bit-identical to flat_round on a
    matrix stored every round."""
    import ctypes
    _check_cuda(mat, s_cur, inv_cur, part, v, state, *pend_s, *pend_inv)
    m = defer_rounds(*mat.shape, mat.dtype)
    assert len(pend_s) == len(pend_inv) < m
    # the round with m - 1 pending is the group's storing round
    assert store or len(pend_s) + 1 < m, "a round with m - 1 pending rounds must store"
    assert mat.is_contiguous() and mat.dim() == 2
    nrows, ncols = mat.shape
    assert s_cur.numel() >= ncols and inv_cur.numel() >= ncols and v.numel() >= ncols
    assert all(x.numel() >= ncols for x in (*pend_s, *pend_inv))
    assert row0 + nrows <= ncols
    assert part.numel() >= int(_lib.load().st_round_flat_scratch(nrows, ncols))
    if not flush:
        _check_cuda(s_next, inv_next)
        assert s_next.numel() >= nrows and inv_next.numel() >= nrows
    np_ = len(pend_s)
    arr_s = (ctypes.c_void_p * max(1, np_))(*[_ptr(x) for x in pend_s])
    arr_i = (ctypes.c_void_p * max(1, np_))(*[_ptr(x) for x in pend_inv])
    _lib.check(getattr(_lib.load(), f"st_round_flat_deferred_{_sfx(mat)}")(
        _ptr(mat), _ptr(s_cur), _ptr(inv_cur), None if flush else _ptr(s_next),
        None if flush else _ptr(inv_next), _ptr(part), _ptr(v), nrows, ncols, row0, eps, k,
        max_itr, semantics, arr_s, arr_i, np_, int(store), int(flush), _ptr(state),
        _stream(mat.device)), "round_flat_deferred")


SPAN_LOCAL = 1
SPAN_REMOTE = 2


def split_round(mat, s_cur, s_next, part, v, state, *, span: int, row0: int = 0,
                col0: int = 0, col1: Optional[int] = None, eps: float = 1e-3, k: int = 0,
                max_itr: int = _lib.ST_MAX_ITR, semantics: int = _lib.ST_SEM_SYCL) -> None:
    """Half of a round (st_round_split): ``span=SPAN_LOCAL`` transforms the
    columns [col0, col1) and writes their row sums to ``part``;
    ``span=SPAN_REMOTE`` does the rest of the round (m/stop/v/state from
    the full ``s_cur``, the other columns, ``s_next = part + their sum``)."""
    _check_cuda(mat, s_cur, s_next, part, v, state)
    assert mat.is_contiguous() and mat.dim() == 2
    nrows, ncols = mat.shape
    col1 = ncols if col1 is None else col1
    assert s_cur.numel() >= ncols and part.numel() >= nrows and row0 + nrows <= ncols
    assert span == SPAN_LOCAL or (s_next is not None and s_next.numel() >= nrows
                                  and v is not None and v.numel() >= ncols)
    _lib.check(getattr(_lib.load(), f"st_round_split_{_sfx(mat)}")(
        _ptr(mat), _ptr(s_cur), _ptr(s_next), _ptr(part), _ptr(v), nrows, ncols, row0,
        col0, col1, eps, k, max_itr, semantics, span, _ptr(state),
        _stream(mat.device)), "round_split")


def split_flat_scratch(nrows: int, ncols: int, col0: int, col1: int, dtype, device=None):
    """Partial-sum scratch for split_flat_round on this block and local range."""
    torch = _torch()
    n = int(_lib.load().st_round_split_flat_scratch(nrows, ncols, col0, col1))
    return torch.empty(n, dtype=dtype, device=device or "cuda")


def split_flat_round(mat, s_cur, s_next, part, v, state, *, span: int, row0: int = 0,
                     col0: int = 0, col1: Optional[int] = None, eps: float = 1e-3,
                     k: int = 0, max_itr: int = _lib.ST_MAX_ITR,
                     semantics: int = _lib.ST_SEM_SYCL) -> None:
    """split_round in the flat form (st_round_split_flat): ``part`` is the
    split_flat_scratch of this block and range, shared by both halves."""
    _check_cuda(mat, s_cur, s_next, part, v, state)
    assert mat.is_contiguous() and mat.dim() == 2
    nrows, ncols = mat.shape
    col1 = ncols if col1 is None else col1
    need = int(_lib.load().st_round_split_flat_scratch(nrows, ncols, col0, col1))
    assert s_cur.numel() >= ncols and part.numel() >= need and row0 + nrows <= ncols
    assert span == SPAN_LOCAL or (s_next is not None and s_next.numel() >= nrows
                                  and v is not None and v.numel() >= ncols)
    _lib.check(getattr(_lib.load(), f"st_round_split_flat_{_sfx(mat)}")(
        _ptr(mat), _ptr(s_cur), _ptr(s_next), _ptr(part), _ptr(v), nrows, ncols, row0,
        col0, col1, eps, k, max_itr, semantics, span, _ptr(state),
        _stream(mat.device)), "round_split_flat")


def epilogue(s, v, state, eps: float, max_itr: int = _lib.ST_MAX_ITR,
             semantics: int = _lib.ST_SEM_SYCL) -> None:
    """Round epilogue: max, v *= s/m, stop test, λ = s[0], bookkeeping."""
    _check_cuda(s, v, state)
    _lib.check(getattr(_lib.load(), f"st_epilogue_{_sfx(s)}")(
        _ptr(s), _ptr(v), s.numel(), eps, max_itr, semantics, _ptr(state),
        _stream(s.device)), "epilogue")


# --------------------------------------------------------------------------
# whole solve on a device-resident matrix
# --------------------------------------------------------------------------
class DeviceSolver:
    """Owns one library context bound to the current torch stream."""

    def __init__(self, device=None):
        torch = _torch()
        self.device = torch.device(device or "cuda")
        self.L = _lib.load()
        with torch.cuda.device(self.device):
            self.q = ctypes.c_void_p()
            self.L.make_queue(ctypes.byref(self.q))
        if not self.q.value:
            raise _lib.EigenValueError(f"make_queue failed: {_lib.last_error()}")

    def solve(self, mat, *, inplace: bool = False, eps: Optional[float] = None,
              max_itr: int = 0, semantics: int = _lib.ST_SEM_SYCL, batch: int = 0,
              time_kernels: bool = False, matrix_free: bool = False,
              round_loop: bool = False, write_every_round: bool = False,
              trace_sums: bool = False):
        """Returns (λ: float, v: tensor, iterations: int, stats: dict).

        Matrices of n <= 128 (fp64) / 256 (fp32) run the whole solve in one
        workgroup launch (bit-identical); ``round_loop`` forces one launch per
        round instead (``ST_FLAG_ROUND_LOOP``).  Matrices of >= 144 MiB
        store the transformed matrix every 6th round
        (``defer_rounds``) and re-apply the pending scalings in registers
        (identical results and final matrix, a third to 3/8 fewer bytes);
        ``write_every_round`` stores it every round
        (``ST_FLAG_WRITE_EVERY_ROUND``).

        ``mat`` is transformed in place when ``inplace`` (it is the private
        working copy the reference makes, similarity_transform.cpp:14,19)
        and then ends at A_end, end = ``stats["rounds"]``: the stopping
        round's launch still applies its transform, one more than the
        reference loop, which breaks before compute_next_matrix (cpp:45-52).
        ``matrix_free`` runs the read-only form: the
        input is never written, so no copy is made.  ``mat`` may be a torch
        tensor or any DLPack producer (``__dlpack__``) on this device.
        ``trace_sums`` records every evaluated round's row sums
        (``ST_FLAG_TRACE_SUMS``; identical results): ``last_round_sums()``."""
        torch = _torch()
        if not isinstance(mat, torch.Tensor) and hasattr(mat, "__dlpack__"):
            mat = torch.from_dlpack(mat)   # any DLPack producer, zero copy
        _check_cuda(mat)
        if mat.device.index != (self.device.index if self.device.index is not None
                                else torch.cuda.current_device()):
            raise ValueError(f"matrix on {mat.device}, solver context on {self.device}")
        n = mat.shape[0]
        assert mat.dim() == 2 and mat.shape == (n, n), "must be square"
        if inplace and not mat.is_contiguous():
            raise ValueError("inplace needs a contiguous (row-major) matrix")
        work = mat if (inplace or matrix_free) else mat.clone()
        work = work.contiguous()
        v = torch.empty(n, dtype=mat.dtype, device=mat.device)
        ev = (ctypes.c_double if mat.dtype == torch.float64 else ctypes.c_float)()
        it = ctypes.c_uint32()
        flags = ((_lib.ST_FLAG_TIME_KERNELS if time_kernels else 0)
                 | (_lib.ST_FLAG_MATRIX_FREE if matrix_free else 0)
                 | (_lib.ST_FLAG_ROUND_LOOP if round_loop else 0)
                 | (_lib.ST_FLAG_WRITE_EVERY_ROUND if write_every_round else 0)
                 | (_lib.ST_FLAG_TRACE_SUMS if trace_sums else 0))
        opt = _lib.st_options(-1.0 if eps is None else float(eps), max_itr, semantics,
                              batch, flags)
        stats = _lib.st_stats()
        self._trace = (n, mat.dtype)
        _lib.check(self.L.st_set_stream(self.q, _stream(mat.device)), "st_set_stream")
        rc = getattr(self.L, f"st_solve_device_{_sfx(mat)}")(
            self.q, _ptr(work), n, _ptr(v), None, ctypes.byref(ev), ctypes.byref(it),
            ctypes.byref(opt), ctypes.byref(stats))
        _lib.check(rc, "st_solve_device")
        return float(ev.value), v, int(it.value), stats.as_dict()

    def last_round_sums(self):
        """Row sums s_0 .. s_{rounds-1} of the last ``solve(trace_sums=True)``
        as a (rounds, n) numpy array (empty if that solve was not traced)."""
        import numpy as np
        n, dt = getattr(self, "_trace", (0, None))
        npdt = np.float64 if dt is not None and dt == _torch().float64 else np.float32
        return _lib.round_sums(self.L, self.q, n, npdt)

    def close(self) -> None:
        if self.q is not None and self.q.value:
            self.L.destroy_queue(self.q)
            self.q = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
