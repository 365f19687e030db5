"""ctypes binding of ``libsimilarity_transform.so`` (include/similarity_transform.h).

The library is built in-tree by ``make`` / ``__graft_entry__.build()`` into
``eigen_value_amd/lib/``.  There is no fallback: if the shared object is
missing, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
DEFAULT_LIB = os.path.join(PKG_DIR, "lib", "libsimilarity_transform.so")
# the tuning build: the same kernels plus the launch-table setters of
# include/st_tuning.h (tools and the knob tests only)
TUNING_LIB = os.path.join(PKG_DIR, "lib", "libsimilarity_transform_tuning.so")
HEADER = os.path.join(REPO_DIR, "include", "similarity_transform.h")
TUNING_HEADER = os.path.join(REPO_DIR, "include", "st_tuning.h")

ST_SEM_SYCL = 0
ST_SEM_MAINPY = 1
ST_FLAG_TIME_KERNELS = 1
ST_FLAG_MATRIX_FREE = 2
ST_FLAG_ROUND_LOOP = 4
ST_FLAG_WRITE_EVERY_ROUND = 8
ST_FLAG_TRACE_SUMS = 16
ST_MAX_ITR = 1000

DTYPE_F32 = 0
DTYPE_F64 = 1


class EigenValueError(RuntimeError):
    """A call into libsimilarity_transform.so reported an error."""


class st_options(ctypes.Structure):
    _fields_ = [("eps", ctypes.c_double),
                ("max_itr", ctypes.c_uint32),
                ("semantics", ctypes.c_uint32),
                ("batch", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


class st_stats(ctypes.Structure):
    _fields_ = [("h2d_ms", ctypes.c_double),
                ("loop_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double),
                ("fused_ms_total", ctypes.c_double),
                ("rowsum_ms", ctypes.c_double),
                ("fused_launches", ctypes.c_uint32),
                ("rounds", ctypes.c_uint32),
                ("converged", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class st_launch_policy(ctypes.Structure):
    """include/similarity_transform.h st_launch_policy."""
    _fields_ = [("kernel", ctypes.c_int), ("rows", ctypes.c_int), ("tile", ctypes.c_uint),
                ("cap", ctypes.c_uint), ("grid", ctypes.c_uint), ("piece_bytes", ctypes.c_uint),
                ("load_nt", ctypes.c_int), ("store_nt", ctypes.c_int), ("alt", ctypes.c_int)]


ST_FORM_ROUND, ST_FORM_DEFER_READ, ST_FORM_DEFER_STORE, ST_FORM_MFREE = 0, 1, 2, 3
ST_FORM_ROWSUM = 4
KERNEL_NAMES = {0: "k_round", 1: "k_flat", 2: "k_flat<NP>", 3: "k_mfree", 4: "k_fused",
                5: "k_flat_sum"}


def launch_policy(dtype: str, nrows: int, ncols: int, form: int, npend: int = 0) -> dict:
    """What the solve loops launch for an nrows x ncols block
    (st_launch_policy_query): kernel, rows per workgroup / group, piece
    tile, workgroups-per-CU cap, grid cap, piece bytes, cache policy."""
    L = load()
    out = st_launch_policy()
    check(L.st_launch_policy_query(1 if dtype == "f64" else 0, nrows, ncols, form, npend,
                                   ctypes.byref(out)), "st_launch_policy_query")
    d = {f: getattr(out, f) for f, _ in st_launch_policy._fields_}
    d["kernel"] = KERNEL_NAMES[d["kernel"]]
    return d


class st_state(ctypes.Structure):
    _fields_ = [("done", ctypes.c_uint32),
                ("round", ctypes.c_uint32),
                ("iters", ctypes.c_uint32),
                ("stop", ctypes.c_uint32),
                ("lambda_", ctypes.c_double),
                ("max", ctypes.c_double),
                ("end", ctypes.c_uint32),
                ("arrivals", ctypes.c_uint32),
                ("max_bits", ctypes.c_uint64),
                ("fail", ctypes.c_uint32),
                ("pad0", ctypes.c_uint32),
                ("pad", ctypes.c_uint64 * 1)]


assert ctypes.sizeof(st_state) == 64
assert ctypes.sizeof(st_options) == 24
assert ctypes.sizeof(st_stats) == 56

_lib: Optional[ctypes.CDLL] = None
_by_path: dict = {}   # every library loaded, by real path (one CDLL each)


def lib_path() -> str:
    return os.environ.get("EIGEN_VALUE_LIB") or DEFAULT_LIB


def load(path: Optional[str] = None) -> ctypes.CDLL:
    """Load (once) and declare the C-ABI.  Raises if the .so is missing."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or lib_path()
    if not os.path.exists(p):
        raise FileNotFoundError(
            f"libsimilarity_transform.so not found at {p!r}: run `make` or "
            "`python -c 'import __graft_entry__ as g; g.build()'` first "
            "(there is no CPU fallback)")
    key = os.path.realpath(p)
    L = _by_path.get(key)
    if L is None:
        L = ctypes.CDLL(p)
        _declare(L)
        if hasattr(L, "st_set_defer_caps"):     # the tuning build
            declare_tuning(L)
        _by_path[key] = L
    if path is None:
        _lib = L
    return L


def load_tuning() -> ctypes.CDLL:
    """The tuning build (libsimilarity_transform_tuning.so), declared with
    the main ABI and the setters of include/st_tuning.h.  A separate library
    with its own launch tables: a knob set here moves only the launches made
    through it (run a knob study with EIGEN_VALUE_LIB pointing at it, so
    that the package's default library is this one)."""
    L = load(TUNING_LIB)
    declare_tuning(L)
    return L


def declare_tuning(L: ctypes.CDLL) -> None:
    """argtypes of the st_tuning.h setters (raises AttributeError on the
    product library, which exports none)."""
    u32, i32 = ctypes.c_uint32, ctypes.c_int
    L.st_set_flat_grid_limit.argtypes = [u32]
    L.st_set_flat_grid_limit.restype = u32
    L.st_set_defer_caps.argtypes = [i32, i32, u32, u32]
    L.st_set_defer_caps.restype = i32
    L.st_set_defer_ntload.argtypes = [u32, u32]
    L.st_set_defer_ntload.restype = i32
    L.st_defer_ntload_class.argtypes = [u32, u32, i32]
    L.st_defer_ntload_class.restype = i32
    L.st_set_every_cache.argtypes = [u32, u32]
    L.st_set_every_cache.restype = i32
    L.st_every_cache_class.argtypes = [u32, u32, i32]
    L.st_every_cache_class.restype = i32
    L.st_set_every_tile.argtypes = [u32, u32]
    L.st_set_every_tile.restype = i32
    L.st_set_every_caps.argtypes = [u32, u32]
    L.st_set_every_caps.restype = i32
    L.st_set_defer_cache.argtypes = [i32, u32, u32]
    L.st_set_defer_cache.restype = i32
    L.st_set_mfree_shape.argtypes = [u32]
    L.st_set_mfree_shape.restype = i32
    L.st_set_k0_reverse.argtypes = [i32]
    L.st_set_k0_reverse.restype = i32


def _declare(L: ctypes.CDLL) -> None:
    P, u32, u64, i32, i64 = (ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64,
                             ctypes.c_int, ctypes.c_int64)
    f32, f64 = ctypes.c_float, ctypes.c_double
    L.make_queue.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
    L.make_queue.restype = None
    L.destroy_queue.argtypes = [P]
    L.destroy_queue.restype = None
    L.eigen_last_error.argtypes = []
    L.eigen_last_error.restype = ctypes.c_char_p
    L.st_version.restype = ctypes.c_char_p
    L.st_probe_switches.restype = ctypes.c_char_p
    L.st_device_count.restype = i32
    L.max_eigen_value.argtypes = [P, P, P, P, u32, P]
    L.max_eigen_value.restype = i64
    L.max_eigen_value_f64.argtypes = [P, P, P, P, u32, P]
    L.max_eigen_value_f64.restype = i64
    L.max_eigen_value_ex.argtypes = [P, i32, P, P, P, u32, P, P, P]
    L.max_eigen_value_ex.restype = i64
    L.st_last_round_times.argtypes = [P, P, u32]
    L.st_last_round_times.restype = i32
    L.st_last_round_sums.argtypes = [P, P, u32]
    L.st_last_round_sums.restype = i32
    L.st_set_stream.argtypes = [P, P]
    L.st_set_stream.restype = i32
    L.st_use_own_stream.argtypes = [P]
    L.st_use_own_stream.restype = i32
    for sfx, T in (("f32", f32), ("f64", f64)):
        fm = getattr(L, f"st_solve_multi_{sfx}")
        fm.argtypes = [P, u32, i32, P, i32, u64, P, P, P, P, P]
        fm.restype = i64
        fn = getattr(L, f"st_solve_device_{sfx}")
        fn.argtypes = [P, P, u32, P, P, P, P, P, P]
        fn.restype = i64
        getattr(L, f"st_generate_hilbert_{sfx}").argtypes = [P, u32, u32, u32, P]
        getattr(L, f"st_generate_random_{sfx}").argtypes = [P, u32, u32, u32, u64, P]
        getattr(L, f"st_generate_identity_{sfx}").argtypes = [P, u32, u32, u32, P]
        getattr(L, f"st_fill_{sfx}").argtypes = [P, u64, T, P]
        getattr(L, f"st_rowsum_{sfx}").argtypes = [P, P, u32, u32, P]
        getattr(L, f"st_rowsum_flat_{sfx}").argtypes = [P, P, P, u32, u32, P]
        getattr(L, f"st_scale_rowsum_{sfx}").argtypes = [P, P, P, u32, u32, u32, u32, P, P]
        getattr(L, f"st_epilogue_{sfx}").argtypes = [P, P, u32, T, u32, u32, P, P]
        getattr(L, f"st_round_{sfx}").argtypes = [P, P, P, P, u32, u32, u32, T, u32, u32,
                                                  u32, P, P]
        getattr(L, f"st_mfree_round_flat_{sfx}").argtypes = [P, P, P, P, P, P, u32, u32, u32,
                                                              T, u32, u32, u32, P, P]
        getattr(L, f"st_mfree_round_flat_{sfx}").restype = i32
        getattr(L, f"st_mfree_round_{sfx}").argtypes = [P, P, P, P, P, u32, u32, u32, T, u32,
                                                        u32, u32, P, P]
        getattr(L, f"st_round_split_{sfx}").argtypes = [P, P, P, P, P, u32, u32, u32, u32,
                                                        u32, T, u32, u32, u32, i32, P, P]
        getattr(L, f"st_round_split_flat_{sfx}").argtypes = [P, P, P, P, P, u32, u32, u32,
                                                             u32, u32, T, u32, u32, u32,
                                                             i32, P, P]
        getattr(L, f"st_round_flat_{sfx}").argtypes = [P, P, P, P, P, u32, u32, u32, T, u32,
                                                       u32, u32, P, P]
        getattr(L, f"st_round_flat_deferred_{sfx}").argtypes = [
            P, P, P, P, P, P, P, u32, u32, u32, T, u32, u32, u32, P, P, u32, i32, i32, P, P]
        getattr(L, f"st_recip_{sfx}").argtypes = [P, P, u32, P]
        for name in ("generate_hilbert", "generate_random", "generate_identity",
                     "fill", "rowsum", "rowsum_flat", "scale_rowsum", "epilogue", "round", "mfree_round",
                     "round_split", "round_split_flat", "round_flat", "round_flat_deferred",
                     "recip"):
            getattr(L, f"st_{name}_{sfx}").restype = i32
    L.st_round_flat_scratch.argtypes = [u32, u32]
    L.st_round_flat_scratch.restype = u64
    L.st_round_split_flat_scratch.argtypes = [u32, u32, u32, u32]
    L.st_round_split_flat_scratch.restype = u64
    L.st_round_flat_pays.argtypes = [u32, u32, i32]
    L.st_round_flat_pays.restype = i32
    L.st_defer_rounds.argtypes = [u32, u32, i32]
    L.st_defer_rounds.restype = u32
    L.st_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.st_comm_unique_id.restype = i32
    L.st_comm_unique_id_addr.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    L.st_comm_unique_id_addr.restype = i32
    L.st_comm_init.argtypes = [ctypes.POINTER(ctypes.c_void_p), i32, i32, ctypes.c_char_p, i32]
    L.st_comm_init.restype = i32
    L.st_comm_id_release.argtypes = [ctypes.c_char_p]
    L.st_comm_id_release.restype = i32
    L.st_comm_destroy.argtypes = [P]
    L.st_comm_destroy.restype = i32
    L.st_set_comm_timeout.argtypes = [ctypes.c_double]
    L.st_set_comm_timeout.restype = ctypes.c_double
    L.st_comm_info.argtypes = [P, P, P, P]
    L.st_comm_info.restype = i32
    L.st_get_comm_timeout.argtypes = []
    L.st_get_comm_timeout.restype = ctypes.c_double
    L.st_rccl_version.argtypes = [P, ctypes.c_char_p, i32]
    L.st_rccl_version.restype = i32
    for sfx in ("f32", "f64"):
        getattr(L, f"st_allgather_{sfx}").argtypes = [P, P, P, u64, P]
        getattr(L, f"st_allgather_{sfx}").restype = i32
    L.st_launch_policy_query.argtypes = [i32, u32, u32, i32, u32, P]
    L.st_launch_policy_query.restype = i32
    L.st_state_reset.argtypes = [P, P]
    L.st_state_reset.restype = i32


def round_sums(L: ctypes.CDLL, q, n: int, dtype):
    """st_last_round_sums of queue ``q`` as a (rounds, n) array of ``dtype``."""
    import numpy as np
    r = check(L.st_last_round_sums(q, None, 0), "st_last_round_sums", L)
    out = np.zeros((r, n), dtype=dtype)
    if r and n:
        check(L.st_last_round_sums(q, out.ctypes.data, r), "st_last_round_sums", L)
    return out


def rccl_info(L: Optional[ctypes.CDLL] = None) -> dict:
    """The RCCL the library's calls are bound to in THIS process
    (st_rccl_version): {"rccl_version": "X.Y.Z", "rccl_version_code": int,
    "rccl_path": file holding the bound ncclAllGather}.  Inside a torch
    process that is torch's bundled librccl; for a C caller the /opt/rocm one."""
    L = L or load()
    code = ctypes.c_int(0)
    path = ctypes.create_string_buffer(4096)
    L.st_rccl_version(ctypes.byref(code), path, len(path))
    v = code.value
    return {"rccl_version": f"{v // 10000}.{v // 100 % 100}.{v % 100}",
            "rccl_version_code": v, "rccl_path": path.value.decode(errors="replace")}


def last_error(L: Optional[ctypes.CDLL] = None) -> str:
    """The thread-local message of the library that made the failing call
    (``L``; the default library when None)."""
    msg = (L or load()).eigen_last_error()
    return msg.decode() if msg else ""


def check(rc: int, what: str, L: Optional[ctypes.CDLL] = None) -> int:
    """Raise EigenValueError for a negative return of a call into ``L``."""
    if rc < 0:
        raise EigenValueError(f"{what} failed: {last_error(L) or 'unknown error'}")
    return rc


def declared_symbols(header: str = HEADER) -> list[str]:
    """Function names declared inside the extern "C" block of the header."""
    import re
    text = open(header).read()
    body = text.split('extern "C" {', 1)[1].split('} /* extern "C" */', 1)[0]
    body = body.split("#ifdef __cplusplus", 1)[0]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", body)
    skip = {"sizeof"}
    return sorted({n for n in names if n not in skip and not n.isupper()})
