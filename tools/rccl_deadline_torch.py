#!/usr/bin/env python3
"""The RCCL deadline characterisation of round 4 (tools/comm_deadline_probe,
RCCL 2.27.7 from /opt/rocm), repeated on the RCCL a TORCH process binds -
torch's bundled librccl (2.26.6 in this image), the one the GPU suite, the
sharded driver and the driver's SCALE run use.

Rank 0 of 2 joins a fresh RCCL unique id and rank 1 never arrives:
ncclCommInitRankConfig(blocking = 0) on a helper thread, this thread waits
--wait s, reads the handle RCCL wrote, optionally ncclCommAbort()s it, and the
process exits normally; every step is timestamped.  Run each variant in a
process of its own under `timeout` (a crash at exit is the finding).

    timeout -k 5 40 python3 tools/rccl_deadline_torch.py --abort 0
    timeout -k 5 40 python3 tools/rccl_deadline_torch.py --abort 1

This is what the library's st_comm_init no longer does: it checks presence
first (st_rendezvous.hip) and enters RCCL only with every rank there.
"""
import argparse
import ctypes
import sys
import threading
import time

T0 = time.monotonic()


def log(msg):
    print(f"[{time.monotonic() - T0:7.3f}] {msg}", flush=True)


class NcclConfig(ctypes.Structure):   # ncclConfig_v22700 (rccl.h), append-only
    _fields_ = [("size", ctypes.c_size_t), ("magic", ctypes.c_uint), ("version", ctypes.c_uint),
                ("blocking", ctypes.c_int), ("cgaClusterSize", ctypes.c_int),
                ("minCTAs", ctypes.c_int), ("maxCTAs", ctypes.c_int),
                ("netName", ctypes.c_char_p), ("splitShare", ctypes.c_int),
                ("trafficClass", ctypes.c_int), ("commName", ctypes.c_char_p),
                ("collnetEnable", ctypes.c_int), ("CTAPolicy", ctypes.c_int),
                ("shrinkShare", ctypes.c_int), ("nvlsCTAs", ctypes.c_int)]


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--abort", type=int, default=1)
    ap.add_argument("--wait", type=float, default=3.0)
    a = ap.parse_args()
    import os

    import torch
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    R = ctypes.CDLL(path)                       # the copy torch already loaded
    v = ctypes.c_int()
    R.ncclGetVersion(ctypes.byref(v))
    log(f"RCCL {v.value // 10000}.{v.value // 100 % 100}.{v.value % 100} ({path})")
    uid = UniqueId()
    log(f"ncclGetUniqueId -> {R.ncclGetUniqueId(ctypes.byref(uid))}")
    undef = -2147483648
    cfg = NcclConfig(ctypes.sizeof(NcclConfig), 0xcafebeef, v.value, 0, undef, undef, undef,
                     None, undef, undef, None, undef, undef, undef, undef)
    comm = ctypes.c_void_p()
    done = threading.Event()
    R.ncclCommInitRankConfig.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                         UniqueId, ctypes.c_int, ctypes.POINTER(NcclConfig)]

    def init():
        torch.cuda.set_device(0)
        q = R.ncclCommInitRankConfig(ctypes.byref(comm), 2, uid, 0, ctypes.byref(cfg))
        log(f"helper: ncclCommInitRankConfig(nranks 2, rank 0, blocking 0) -> {q}")
        done.set()

    log("helper: ncclCommInitRankConfig ...")
    threading.Thread(target=init, daemon=True).start()
    done.wait(a.wait)
    log(f"after {a.wait} s: helper done {int(done.is_set())}, handle "
        f"{hex(comm.value) if comm.value else None}")
    if comm.value:
        st = ctypes.c_int(-1)
        log(f"ncclCommGetAsyncError -> {R.ncclCommGetAsyncError(comm, ctypes.byref(st))}, "
            f"state {st.value}")
        if a.abort:
            log("ncclCommAbort ...")
            log(f"ncclCommAbort -> {R.ncclCommAbort(comm)}")
            done.wait(10.0)
            log(f"helper done {int(done.is_set())} within 10 s of the abort")
    log("main returns (normal interpreter exit)")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
