"""CPU: the C-ABI library loads and exports every symbol the header declares;
host-side wrapper logic.  No compute calls (no GPU here)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from eigen_value_amd import _lib


def test_library_exists_and_loads():
    assert os.path.exists(_lib.lib_path()), "run `make` first"
    L = _lib.load()
    assert L.st_version().decode().startswith("eigen_value_amd")


def test_exports_every_declared_symbol():
    declared = _lib.declared_symbols()
    # the two drop-in names bound by wrapper/python/similarity_transform.py
    assert "make_queue" in declared and "max_eigen_value" in declared
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.lib_path()],
                         capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    L = _lib.load()
    for s in declared:
        assert getattr(L, s) is not None


def _exported(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path],
                         capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if " T " in line}


def test_product_library_exports_no_tuning_setter():
    """The library drop-in callers load exports the product ABI only
    (VERDICT r05 #5): no launch-table setter of include/st_tuning.h, no
    st_set_* but the context's stream and the RCCL deadline."""
    exported = _exported(_lib.lib_path())
    tuning = _lib.declared_symbols(_lib.TUNING_HEADER)
    assert len(tuning) == 11 and not (set(tuning) & exported), set(tuning) & exported
    assert sorted(e for e in exported if e.startswith("st_set_")) == \
        ["st_set_comm_timeout", "st_set_stream"]
    assert not (exported - set(_lib.declared_symbols())), exported - set(_lib.declared_symbols())


def test_tuning_build_exports_the_tuning_abi():
    """libsimilarity_transform_tuning.so: the product ABI plus st_tuning.h."""
    assert os.path.exists(_lib.TUNING_LIB), "run `make` first"
    exported = _exported(_lib.TUNING_LIB)
    want = set(_lib.declared_symbols()) | set(_lib.declared_symbols(_lib.TUNING_HEADER))
    assert not (want - exported), want - exported
    L = _lib.load_tuning()
    assert L.st_set_flat_grid_limit(0) == 16777208
    # K0's walk order: previous mode back, any negative = the policy (-1)
    dflt = L.st_set_k0_reverse(1)
    assert dflt in (-1, 0, 1) and L.st_set_k0_reverse(7) == 1
    assert L.st_set_k0_reverse(-5) == 1 and L.st_set_k0_reverse(0) == -1
    assert L.st_set_k0_reverse(dflt) == 0


def test_drop_in_signatures_are_c_abi():
    # extern "C" names are unmangled; the drop-in pair keeps the reference's
    # argument list (wrapper/similarity_transform.cpp:3-37)
    hdr = open(_lib.HEADER).read()
    assert "void make_queue(void** wq);" in hdr
    assert ("int64_t max_eigen_value(void* wq, float* mat, float* eigen_val,\n"
            "                        float* eigen_vec, unsigned int dim,\n"
            "                        unsigned int* iter_cnt);") in hdr


def test_struct_layouts():
    assert ctypes.sizeof(_lib.st_state) == 64
    assert ctypes.sizeof(_lib.st_options) == 24
    assert ctypes.sizeof(_lib.st_stats) == 56


def test_no_device_errors_are_clean():
    L = _lib.load()
    if L.st_device_count() > 0:
        pytest.skip("a GPU is present")
    q = ctypes.c_void_p(123)
    L.make_queue(ctypes.byref(q))
    assert q.value is None
    assert "no HIP device" in _lib.last_error()
    # NULL queue -> negative return + message, never a crash
    m = np.ones((4, 4), np.float32)
    ev, vec, it = np.zeros(1, np.float32), np.zeros(4, np.float32), np.zeros(1, np.uint32)
    rc = L.max_eigen_value(None, m.ctypes.data, ev.ctypes.data, vec.ctypes.data, 4, it.ctypes.data)
    assert rc < 0 and "null queue" in _lib.last_error()
    with pytest.raises(Exception, match="queue"):
        import eigen_value_amd
        eigen_value_amd.EigenValue()


def test_step_api_argument_errors():
    L = _lib.load()
    assert L.st_rowsum_f64(None, None, 4, 4, None) < 0
    assert "null" in _lib.last_error()
    assert L.st_epilogue_f32(None, None, 0, 1e-3, 10, 0, None, None) < 0
    assert L.st_scale_rowsum_f64(None, None, None, 4, 4, 0, 7, None, None) < 0
    # zero-sized work is a no-op, not an error
    assert L.st_fill_f64(None, 0, 1.0, None) == 0


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setenv("EIGEN_VALUE_LIB", str(tmp_path / "nope.so"))
    with pytest.raises(FileNotFoundError, match="no CPU fallback"):
        _lib.load(_lib.lib_path())


def test_header_compiles_as_c_and_cxx(tmp_path):
    src_c = tmp_path / "t.c"
    src_c.write_text('#include "similarity_transform.h"\nint main(void){return (int)sizeof(st_state)-64;}\n')
    inc = os.path.dirname(_lib.HEADER)
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", f"-I{inc}", str(src_c), "-o", str(tmp_path / "tc")], check=True)
    src_cc = tmp_path / "t.cc"
    src_cc.write_text('#include "similarity_transform.h"\n'
                      'int main(){ int64_t (*f)(void*, const double*, double*, double*,\n'
                      '  unsigned, unsigned, unsigned*) = &similarity_transform;\n'
                      '  return f ? (int)sizeof(st_options)-24 : 1; }\n')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", f"-I{inc}", "-c", str(src_cc),
                    "-o", str(tmp_path / "tcc.o")], check=True)


def test_wrapper_argument_checks_match_reference():
    # wrapper/python/similarity_transform.py:55-57: square, float32 asserted
    # before any library call (float64 is additionally accepted here)
    from eigen_value_amd.similarity_transform import EigenValue
    ev = object.__new__(EigenValue)          # no device needed for the checks
    with pytest.raises(AssertionError, match="square"):
        ev.similarity_transform(np.ones((3, 4), np.float32))
    with pytest.raises(AssertionError, match="float32"):
        ev.similarity_transform(np.ones((3, 3), np.int64))
    with pytest.raises(TypeError):
        ev.similarity_transform_ex(np.ones((3, 3), np.float16))


def test_sharded_partition_rejects_empty_rank():
    torch = pytest.importorskip("torch")
    from eigen_value_amd.sharded import ShardedSimilarityTransform

    class Dummy:
        def empty(self, shape, dtype):
            return torch.zeros(shape, dtype=dtype)

        def new_state(self):
            return {}

    import torch.distributed as dist
    assert not dist.is_initialized()
    sh = ShardedSimilarityTransform(5, torch.float64, ops=Dummy())   # world 1
    assert (sh.part.row0, sh.part.nrows, sh.part.chunk) == (0, 5, 5)


def test_launch_policy_queries():
    """Host-side policy exported by the library (no device needed): the flat
    round from 144 MiB and the deferred-write depth
    (6 rounds per store on every block since round 2's launch shapes)."""
    L = _lib.load()
    assert L.st_round_flat_pays(6144, 6144, 0) == 1        # 144 MiB fp32
    assert L.st_round_flat_pays(4096, 4096, 1) == 0        # 128 MiB fp64
    assert L.st_round_flat_pays(8192, 8192, 1) == 1
    assert L.st_defer_rounds(8192, 8192, 1) == 6
    assert L.st_defer_rounds(8192, 8192, 0) == 6
    assert L.st_defer_rounds(32768, 32768, 1) == 6
    assert L.st_defer_rounds(16384, 16384, 1) == 6         # 2 GiB: non-temporal


def test_probe_switches_are_the_shipped_defaults():
    """A library build carries no A/B probe switch (st_kernels.hip fails to
    compile with one unless -DST_PROBES=1), and st_version says so."""
    L = _lib.load()
    assert L.st_probe_switches() == b"defaults"
    assert b"probe switches: defaults" in L.st_version()


def test_deferred_round_without_store_is_rejected_at_m_minus_1():
    """st_round_flat_deferred: the round with m - 1 pending rounds is the
    group's storing round; asked not to store it returns -1 with a message
    (before this check it silently launched the 4-pending kernel and dropped
    the 5th scaling).  Rejected on the host before any device call."""
    L = _lib.load()
    m = L.st_defer_rounds(8192, 8192, 1)
    dummy = ctypes.c_void_p(4096)                 # never dereferenced: rejected first
    arr = (ctypes.c_void_p * m)(*([4096] * m))
    for fn in (L.st_round_flat_deferred_f64, L.st_round_flat_deferred_f32):
        rc = fn(dummy, dummy, dummy, dummy, dummy, dummy, dummy, 8192, 8192, 0, 1e-3, 0, 1000, 0, arr, arr, m - 1, 0, 0, dummy, None)
        assert rc < 0 and "without a store" in _lib.last_error()
        rc = fn(dummy, dummy, dummy, dummy, dummy, dummy, dummy, 8192, 8192, 0, 1e-3, 0, 1000, 0, arr, arr, m, 1, 0, dummy, None)
        assert rc < 0 and "pending rounds" in _lib.last_error()


def test_defer_caps_setter():
    """(the tuning build, include/st_tuning.h) st_set_defer_caps (workgroups per CU of the deferred launches): bad
    arguments are refused, a value set is returned by the next call (the
    previous one), and the default is restored."""
    L = _lib.load_tuning()
    assert L.st_set_defer_caps(2, 0, 0, 4) < 0 and "st_set_defer_caps" in _lib.last_error(L)
    assert L.st_set_defer_caps(1, 1, 7, 4) < 0
    assert L.st_set_defer_caps(1, 1, 6, 1) < 0
    assert L.st_set_defer_caps(1, 1, 6, 33) < 0
    old = L.st_set_defer_caps(1, 1, 6, 5)
    assert old >= 0
    assert L.st_set_defer_caps(1, 1, 6, old) == 5


def test_defer_ntload_setter():
    """st_set_defer_ntload (non-temporal loads of the cached fp64 deferred
    rounds) and its size classes: bad arguments are refused, the shipped
    masks are the measured ones, a mask set is returned by the
    next call."""
    L = _lib.load_tuning()
    assert L.st_set_defer_ntload(3, 0) < 0 and "st_set_defer_ntload" in _lib.last_error(L)
    assert L.st_set_defer_ntload(0, 0x20) < 0 and L.st_set_defer_ntload(0, 0x100) < 0
    assert L.st_defer_ntload_class(8192, 8192, 2) < 0
    assert [L.st_defer_ntload_class(r, c, 1) for r, c in
            ((4096, 8192), (8192, 8192), (2880, 23040), (10240, 10240), (12288, 12288))] == [0, 1, 1, 2, 2]
    assert L.st_defer_ntload_class(8192, 8192, 0) == 0          # fp32: 256 MiB
    shipped = []
    for cls in range(3):
        old = L.st_set_defer_ntload(cls, 0x41)
        shipped.append(old)
        assert L.st_set_defer_ntload(cls, old) == 0x41
    assert shipped == [0, 0x41, 0x5f]
    # the general form: fp64 classes 0..2 are the same masks
    assert L.st_set_defer_cache(2, 0, 0) < 0 and L.st_set_defer_cache(1, 4, 0) < 0
    assert L.st_set_defer_cache(0, 0, 0x20) < 0
    assert L.st_set_defer_cache(1, 1, 0x41) == 0x41
    shipped = [[L.st_set_defer_cache(d, c, 0) for c in range(4)] for d in (0, 1)]
    for d in (0, 1):
        for c in range(4):
            assert L.st_set_defer_cache(d, c, shipped[d][c]) == 0
    assert shipped == [[0, 0x41, 0x41, 0], [0, 0x41, 0x5f, 0]]


def test_every_cache_setter():
    """st_set_every_cache (the every-round flat launch's cache policy on
    cached blocks) and its size classes: bad arguments are refused, the
    shipped policies are the measured ones, a policy set is
    returned by the next call."""
    L = _lib.load_tuning()
    assert L.st_set_every_cache(4, 0) < 0 and "st_set_every_cache" in _lib.last_error(L)
    assert L.st_set_every_cache(0, 4) < 0
    assert L.st_every_cache_class(8192, 8192, 2) < 0
    assert [L.st_every_cache_class(r, c, 1) for r, c in
            ((4096, 8192), (8192, 8192), (2880, 23040), (10240, 10240), (32768, 32768))] \
        == [0, 1, 1, 2, 3]
    assert L.st_set_every_cache(4, 0) < 0
    shipped = []
    for cls in range(4):
        old = L.st_set_every_cache(cls, 3)
        shipped.append(old)
        assert L.st_set_every_cache(cls, old) == 3
    assert shipped == [2, 2, 0, 0]
    assert L.st_set_every_tile(4, 0) < 0 and L.st_set_every_tile(0, 4097) < 0
    assert L.st_set_every_tile(1, 16) == 0 and L.st_set_every_tile(1, 0) == 16
    assert L.st_set_every_caps(4, 0) < 0 and L.st_set_every_caps(0, 1) < 0
    assert L.st_set_every_caps(0, 33) < 0
    caps = [L.st_set_every_caps(c, 3) for c in range(4)]
    assert [L.st_set_every_caps(c, caps[c]) for c in range(4)] == [3, 3, 3, 3]
    assert L.st_set_mfree_shape(4) < 0 and "st_set_mfree_shape" in _lib.last_error(L)
    assert L.st_set_mfree_shape(2) == 0 and L.st_set_mfree_shape(0) == 2


def test_comm_timeout_setter_and_env(monkeypatch):
    """st_set_comm_timeout: the RCCL deadline every waiting communicator step
    is polled under (default ST_COMM_TIMEOUT_S, else 120 s); a value <= 0
    restores the default.  No GPU needed: the setter is host state."""
    L = _lib.load()
    base = L.st_set_comm_timeout(0.0)                   # reset, read the default
    assert base == float(os.environ.get("ST_COMM_TIMEOUT_S", "120") or 120)
    assert L.st_set_comm_timeout(7.5) == base
    assert L.st_set_comm_timeout(-1.0) == 7.5
    assert L.st_set_comm_timeout(0.0) == base


def test_comm_calls_reject_bad_arguments_without_a_device():
    """st_comm_init validates before touching RCCL or HIP, and a NULL
    communicator is an error everywhere but st_comm_destroy (a no-op)."""
    L = _lib.load()
    comm = ctypes.c_void_p(123)
    assert L.st_comm_init(ctypes.byref(comm), 2, 2, b"\0" * 128, 0) < 0
    assert "bad rank" in _lib.last_error()
    assert L.st_comm_init(None, 1, 0, b"\0" * 128, 0) < 0
    assert L.st_comm_info(None, None, None, None) < 0
    assert L.st_comm_destroy(None) == 0
    buf = (ctypes.c_double * 4)()
    assert L.st_allgather_f64(None, buf, buf, 1, None) < 0


def test_comm_unique_id_addr():
    """st_comm_unique_id_addr advertises the caller's IPv4 address (the
    Python driver passes 127.0.0.1 for a single-host group instead of
    setting ST_COMM_ADDR in a running process); a malformed one is refused."""
    import socket
    import struct
    L = _lib.load()
    uid = ctypes.create_string_buffer(128)
    assert L.st_comm_unique_id_addr(uid, b"127.0.0.1") == 0
    assert uid.raw[:7] == b"st-rdv2"
    assert socket.inet_ntoa(uid.raw[16:20]) == "127.0.0.1"        # RdvId.addr
    assert struct.unpack(">H", uid.raw[20:22])[0] > 0               # RdvId.port
    assert L.st_comm_unique_id_addr(uid, b"not-an-address") < 0
    assert "not an IPv4 address" in _lib.last_error()


def test_comm_init_rejects_a_foreign_id():
    """An id that st_comm_unique_id did not make (e.g. raw RCCL id bytes) is
    refused before any socket, HIP or RCCL call."""
    L = _lib.load()
    comm = ctypes.c_void_p()
    assert L.st_comm_init(ctypes.byref(comm), 2, 0, b"\1" * 128, 0) < 0
    assert "not made by st_comm_unique_id" in _lib.last_error()
    assert comm.value is None


def test_comm_rendezvous_names_the_missing_ranks_without_a_device():
    """st_comm_init's presence check runs before RCCL and HIP (VERDICT r04
    #1): as rank 0 of 3 with ranks 1 and 2 absent it returns -1 after the
    deadline (2 s here), names both, and no RCCL state exists; with every
    rank present (three threads of this process) the rendezvous passes and
    the call gets as far as the RCCL id (which needs a device: on CPU the
    error is about that, never about a missing rank)."""
    import threading
    import time
    L = _lib.load()
    old = L.st_set_comm_timeout(2.0)
    try:
        uid = ctypes.create_string_buffer(128)
        assert L.st_comm_unique_id(uid) == 0
        comm = ctypes.c_void_p()
        t0 = time.time()
        assert L.st_comm_init(ctypes.byref(comm), 3, 0, uid.raw, 0) < 0
        el = time.time() - t0
        err = _lib.last_error()
        assert 1.9 <= el < 8.0, el
        assert "ranks 1, 2 of 3 did not reach st_comm_init" in err, err
        assert "no rank entered RCCL" in err and comm.value is None
        # all present: the id's host is whichever thread claims the listener
        assert L.st_comm_unique_id(uid) == 0
        res = {}

        def join(r):
            c = ctypes.c_void_p()
            res[r] = (L.st_comm_init(ctypes.byref(c), 3, r, uid.raw, 0), _lib.last_error(), c)
        th = [threading.Thread(target=join, args=(r,)) for r in (2, 0, 1)]
        t0 = time.time()
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        assert sorted(res) == [0, 1, 2]
        for rc, err, c in res.values():
            assert "did not reach" not in err and "no word" not in err, err
            if rc == 0:
                L.st_comm_destroy(c)
    finally:
        L.st_set_comm_timeout(old)


_PEER_ALONE = r"""
import ctypes, sys, time
sys.path.insert(0, sys.argv[1])
from eigen_value_amd import _lib
L = _lib.load()
L.st_set_comm_timeout(1.0)
c = ctypes.c_void_p()
t0 = time.time()
rc = L.st_comm_init(ctypes.byref(c), 2, 1, bytes.fromhex(sys.argv[2]), 0)
print("RC", rc, "EL", round(time.time() - t0, 2))
print("ERR", _lib.last_error(), flush=True)
"""


def test_comm_rendezvous_peer_names_an_absent_host():
    """A rank whose id's maker never joins: it connects to the maker's
    listener (this process), says hello, hears nothing and returns -1 after
    at most two deadlines, saying so - and exits normally (rc 0)."""
    import sys
    L = _lib.load()
    uid = ctypes.create_string_buffer(128)
    assert L.st_comm_unique_id(uid) == 0
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _PEER_ALONE, repo, uid.raw.hex()],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = dict(ln.split(" ", 1) for ln in out.stdout.splitlines() if ln[:3] in ("RC ", "ERR"))
    rc, _, el = lines["RC"].split()
    assert int(rc) < 0 and 1.0 <= float(el) < 10.0
    assert "no word from the id's host" in lines["ERR"], lines["ERR"]


_JOIN = r"""
import ctypes, sys, time
sys.path.insert(0, sys.argv[1])
from eigen_value_amd import _lib
L = _lib.load()
L.st_set_comm_timeout(20.0)
rank, nranks = int(sys.argv[3]), int(sys.argv[4])
c = ctypes.c_void_p()
t0 = time.time()
rc = L.st_comm_init(ctypes.byref(c), nranks, rank, bytes.fromhex(sys.argv[2]), 0)
print("RC", rc, "EL", round(time.time() - t0, 2))
print("ERR", _lib.last_error(), flush=True)
"""


def test_comm_rendezvous_eight_processes_without_a_device():
    """The driver's 8-GPU shape of st_comm_init's rendezvous, on CPU: this
    process makes the id and joins as rank 0 while seven other processes
    join as ranks 1..7 (in any order).  Every rank gets past the presence
    check together - on a box without a device the id's host then cannot
    make the RCCL id, and all eight report exactly that, promptly (never a
    missing rank, never a hang)."""
    import sys
    import time
    L = _lib.load()
    uid = ctypes.create_string_buffer(128)
    assert L.st_comm_unique_id(uid) == 0
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = [subprocess.Popen([sys.executable, "-c", _JOIN, repo, uid.raw.hex(), str(r), "8"],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in (7, 3, 1, 5, 2, 6, 4)]
    old = L.st_set_comm_timeout(20.0)
    try:
        comm = ctypes.c_void_p()
        t0 = time.time()
        rc0 = L.st_comm_init(ctypes.byref(comm), 8, 0, uid.raw, 0)
        err0, el0 = _lib.last_error(), time.time() - t0
    finally:
        L.st_set_comm_timeout(old)
    outs = [p.communicate(timeout=60) for p in procs]
    if rc0 == 0:                               # a box with a device: RCCL ran
        L.st_comm_destroy(comm)
    else:
        assert "could not make the RCCL id" in err0, err0
    assert el0 < 15.0
    for p, (so, se) in zip(procs, outs):
        assert p.returncode == 0, se[-2000:]
        lines = dict(ln.split(" ", 1) for ln in so.splitlines() if ln[:3] in ("RC ", "ERR"))
        assert "did not reach" not in lines["ERR"] and "no word" not in lines["ERR"], lines
        if rc0 != 0:
            assert "could not make the RCCL id" in lines["ERR"], lines


def _id_addr(raw: bytes):
    """(IPv4 address, port) a rendezvous id advertises (bytes 16..21)."""
    import socket
    return socket.inet_ntoa(raw[16:20]), int.from_bytes(raw[20:22], "big")


def test_comm_rendezvous_ignores_stray_connectors():
    """Connections that never say hello, or send something else, do not
    delay the ranks' admission (the host used to read hellos
    one connection at a time, 5 s each): three ranks as threads get past the
    presence check within a second or two beside two such connectors."""
    import socket
    import threading
    import time
    L = _lib.load()
    old = L.st_set_comm_timeout(20.0)
    try:
        uid = ctypes.create_string_buffer(128)
        assert L.st_comm_unique_id(uid) == 0
        addr = _id_addr(uid.raw)
        stray = socket.create_connection(addr)
        noisy = socket.create_connection(addr)
        noisy.sendall(b"GET / HTTP/1.0\r\n\r\n")
        res = {}

        def join(r):
            c = ctypes.c_void_p()
            res[r] = (L.st_comm_init(ctypes.byref(c), 3, r, uid.raw, 0), _lib.last_error(), c)
        th = [threading.Thread(target=join, args=(r,)) for r in (1, 2, 0)]
        t0 = time.time()
        for t in th:
            t.start()
        for t in th:
            t.join(60)
        el = time.time() - t0
        stray.close()
        noisy.close()
        assert sorted(res) == [0, 1, 2] and el < 4.0, (el, res)
        for rc, err, c in res.values():
            assert "did not reach" not in err and "no word" not in err, err
            if rc == 0:
                L.st_comm_destroy(c)
    finally:
        L.st_set_comm_timeout(old)


_PEER_GIVES_UP = r"""
import ctypes, sys, time
sys.path.insert(0, sys.argv[1])
from eigen_value_amd import _lib
L = _lib.load()
L.st_set_comm_timeout(1.0)
c = ctypes.c_void_p()
t0 = time.time()
rc = L.st_comm_init(ctypes.byref(c), 2, 1, bytes.fromhex(sys.argv[2]), 0)
print("RC", rc, "EL", round(time.time() - t0, 2))
print("ERR", _lib.last_error(), flush=True)
"""


def test_comm_rendezvous_host_after_the_peers_deadline():
    """a peer that gave up at its own deadline and
    closed its socket leaves its hello in the listen backlog; the id's host,
    arriving later, must not count it as present (that used to send the
    RCCL id to a dead rank and enter RCCL without it).  Here the host joins
    after the peer exited: it names rank 1 as missing (it hung up after its
    hello) and never gets as far as making the RCCL id."""
    import sys
    import time
    L = _lib.load()
    uid = ctypes.create_string_buffer(128)
    assert L.st_comm_unique_id(uid) == 0
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", _PEER_GIVES_UP, repo, uid.raw.hex()],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "RC -1" in out.stdout, out.stdout
    time.sleep(0.5)
    old = L.st_set_comm_timeout(2.0)
    try:
        comm = ctypes.c_void_p()
        t0 = time.time()
        rc = L.st_comm_init(ctypes.byref(comm), 2, 0, uid.raw, 0)
        err, el = _lib.last_error(), time.time() - t0
    finally:
        L.st_set_comm_timeout(old)
    assert rc < 0 and comm.value is None
    assert "rank 1 of 2 did not reach st_comm_init" in err, err
    assert "hung up after arriving: 1" in err and "could not make the RCCL id" not in err, err
    assert el < 8.0


def test_comm_id_release():
    """st_comm_id_release closes the listener of an id its maker will not
    join: 0 the first time, 1 after; a peer can no longer
    connect; a foreign id is refused."""
    import socket
    L = _lib.load()
    uid = ctypes.create_string_buffer(128)
    assert L.st_comm_unique_id_addr(uid, b"127.0.0.1") == 0
    addr = _id_addr(uid.raw)
    assert addr[0] == "127.0.0.1"
    socket.create_connection(addr, timeout=2).close()          # listening
    assert L.st_comm_id_release(uid.raw) == 0
    assert L.st_comm_id_release(uid.raw) == 1
    with pytest.raises(OSError):
        socket.create_connection(addr, timeout=2)
    assert L.st_comm_id_release(b"\1" * 128) < 0


def test_comm_listener_binds_the_advertised_address():
    """the listener of an id advertising 127.0.0.1 listens on
    the loopback address only, not on every interface."""
    import socket
    L = _lib.load()
    uid = ctypes.create_string_buffer(128)
    assert L.st_comm_unique_id_addr(uid, b"127.0.0.1") == 0
    port = _id_addr(uid.raw)[1]
    try:
        others = {a[4][0] for a in socket.getaddrinfo(socket.gethostname(), None, socket.AF_INET)}
    except OSError:
        others = set()
    others = [a for a in others if not a.startswith("127.")]
    for a in others:
        with pytest.raises(OSError):
            socket.create_connection((a, port), timeout=2)
    socket.create_connection(("127.0.0.1", port), timeout=2).close()
    assert L.st_comm_id_release(uid.raw) == 0


def test_rccl_version_is_reported():
    """st_rccl_version / _lib.rccl_info / st_version name the RCCL the
    library's calls bind to: X.Y.Z and the file holding the
    bound ncclAllGather.  No GPU needed."""
    import re
    L = _lib.load()
    info = _lib.rccl_info(L)
    assert re.fullmatch(r"2\.\d+\.\d+", info["rccl_version"]), info
    assert info["rccl_version_code"] >= 22000
    assert re.search(r"librccl\.so", info["rccl_path"]) and os.path.isabs(info["rccl_path"])
    v = L.st_version().decode()
    assert f"RCCL {info['rccl_version']} ({info['rccl_path']})" in v, v


def test_package_and_library_versions_agree():
    """eigen_value_amd.__version__ is the version st_version() reports."""
    import eigen_value_amd
    L = _lib.load()
    assert L.st_version().decode().split()[1] == eigen_value_amd.__version__


def test_launch_policy_map_is_pinned():
    """The whole launch policy - kernel, rows per workgroup, piece tile,
    workgroups-per-CU cap, grid cap, load / store cache policy of every
    launch form the solve loops use, over blocks covering every size class
    (tools/launch_policy_table.py) - equals the committed map
    tests/golden/launch_policy.json: a change to any shape or policy table
    in st_kernels.hip shows up here and in the JSON's diff."""
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools"))
    import launch_policy_table as lpt
    golden = json.load(open(lpt.GOLDEN))
    live = lpt.table()
    assert len(live) == len(golden)
    diff = [(g, l) for g, l in zip(golden, live) if g != l]
    assert not diff, diff[:3]


def test_launch_policy_rejects_bad_queries():
    L = _lib.load()
    out = _lib.st_launch_policy()
    assert L.st_launch_policy_query(2, 8192, 8192, 0, 0, ctypes.byref(out)) < 0
    assert L.st_launch_policy_query(1, 8192, 8191, 0, 0, ctypes.byref(out)) < 0
    assert L.st_launch_policy_query(1, 4096, 4096, 1, 0, ctypes.byref(out)) < 0   # no flat
    assert "144 MiB" in _lib.last_error()
    assert L.st_launch_policy_query(1, 8192, 8192, 1, 5, ctypes.byref(out)) < 0   # 5 w/o store
    assert L.st_launch_policy_query(1, 8192, 8192, 2, 5, ctypes.byref(out)) == 0
    assert out.rows == 8 and out.tile == 16 and out.store_nt == 0


def test_launch_policy_matches_the_hardware_traces():
    """The pinned map against what actually ran on the GPU: every k_flat and
    k_mfree instantiation in the committed rocprof kernel statistics of the
    headline workloads (profiles/r04_*_kernel_stats.csv, `bench.py --kind K
    --n N --dtype D`) has the rows per workgroup, piece bytes and load /
    store cache policy st_launch_policy_query gives for its form (the
    every-round round, a deferred read-only round, a storing round or a
    flush with NP pending, the matrix-free round)."""
    import csv
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cases = (("r04_hilbert8192_f64_kernel_stats.csv", "f64", 8192),
             ("r04_random32768_f64_kernel_stats.csv", "f64", 32768),
             ("r04_random32768_f32_kernel_stats.csv", "f32", 32768))
    checked = 0
    for fname, dt, n in cases:
        size = 8 if dt == "f64" else 4
        for row in csv.DictReader(open(os.path.join(root, "profiles", fname))):
            name = row["Name"]
            m = re.search(r"k_flat<([^>]*)>", name)
            if m:
                a = [x.strip() for x in m.group(1).split(",")]
                W, NT, R, BLK, NP, U, DS, FL = (int(a[1]), a[3] == "true", int(a[4]),
                                                int(a[8]), int(a[11]), int(a[12]),
                                                int(a[14]), int(a[16]))
                form = (_lib.ST_FORM_ROUND if NP < 0 else
                        _lib.ST_FORM_DEFER_STORE if DS == 1 else _lib.ST_FORM_DEFER_READ)
                p = _lib.launch_policy(dt, n, n, form, max(NP, 0))
                assert p["rows"] == R and p["piece_bytes"] == BLK * W * U * size, (fname, a)
                assert p["load_nt"] == int(NT != bool(FL & 1)), (fname, a)
                if form != _lib.ST_FORM_DEFER_READ:
                    assert p["store_nt"] == int(NT != bool(FL & 2)), (fname, a)
                checked += 1
            m = re.search(r"k_mfree<([^>]*)>", name)
            if m:
                a = [x.strip() for x in m.group(1).split(",")]
                p = _lib.launch_policy(dt, n, n, _lib.ST_FORM_MFREE)
                assert p["rows"] == int(a[1]) and p["load_nt"] == int(a[4] == "true"), (fname, a)
                checked += 1
    assert checked >= 20
