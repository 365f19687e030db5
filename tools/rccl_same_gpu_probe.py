#!/usr/bin/env python3
"""Can two ranks of the library's RCCL communicator share one GPU?

The pool's boxes have one MI355X, so the P > 1 RCCL paths (st_comm_init with
nranks > 1, st_allgather across ranks) only run on the driver's 8-GPU node.
This probe starts two processes on device 0 that join one communicator
(unique id through a file), all-gather a short vector and check it, with
the library's deadline (st_set_comm_timeout) bounding every wait: either
RCCL accepts two ranks on one device (then the exchange itself is tested
here) or it refuses them - promptly, with the error named.

    timeout -k 10 120 python3 tools/rccl_same_gpu_probe.py [--ranks 2] [--timeout 30]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def rank_main(rank, world, d, limit):
    import torch
    from eigen_value_amd import _lib
    L = _lib.load()
    L.st_set_comm_timeout(limit)
    torch.cuda.set_device(0)
    idf = os.path.join(d, "id")
    uid = ctypes.create_string_buffer(128)
    if rank == 0:
        _lib.check(L.st_comm_unique_id(uid), "st_comm_unique_id")
        with open(idf + ".tmp", "wb") as f:
            f.write(uid.raw)
        os.replace(idf + ".tmp", idf)
    else:
        t0 = time.time()
        while not os.path.exists(idf):
            if time.time() - t0 > limit:
                raise SystemExit("no unique id from rank 0")
            time.sleep(0.05)
        uid = ctypes.create_string_buffer(open(idf, "rb").read(), 128)
    comm = ctypes.c_void_p()
    t0 = time.time()
    rc = L.st_comm_init(ctypes.byref(comm), world, rank, uid.raw, 0)
    out = {"rank": rank, "init_rc": rc, "init_s": round(time.time() - t0, 3)}
    if rc != 0:
        out["error"] = _lib.last_error()
        print(json.dumps(out), flush=True)
        return
    n, r, dv = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    L.st_comm_info(comm, ctypes.byref(n), ctypes.byref(r), ctypes.byref(dv))
    out["rccl"] = {"nranks": n.value, "rank": r.value, "device": dv.value}
    x = torch.full((world * 5,), -1.0, dtype=torch.float64, device="cuda")
    x[rank * 5:(rank + 1) * 5] = torch.arange(rank * 5, rank * 5 + 5, dtype=torch.float64)
    s = torch.cuda.current_stream().cuda_stream
    t0 = time.time()
    rc = L.st_allgather_f64(comm, ctypes.c_void_p(x[rank * 5:].data_ptr()),
                            ctypes.c_void_p(x.data_ptr()), 5, ctypes.c_void_p(s))
    torch.cuda.synchronize()
    out["allgather_rc"] = rc
    out["allgather_s"] = round(time.time() - t0, 3)
    out["allgather_ok"] = bool(torch.equal(x.cpu(), torch.arange(world * 5, dtype=torch.float64)))
    if rc != 0:
        out["error"] = _lib.last_error()
    out["destroy_rc"] = L.st_comm_destroy(comm)
    print(json.dumps(out), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ranks", type=int, default=2)
    p.add_argument("--timeout", type=float, default=30.0)
    p.add_argument("--rank", type=int, default=None)
    p.add_argument("--dir", default=None)
    a = p.parse_args()
    if a.rank is not None:
        return rank_main(a.rank, a.ranks, a.dir, a.timeout)
    d = tempfile.mkdtemp(prefix="rccl_probe_")
    procs = [subprocess.Popen([sys.executable, __file__, "--rank", str(r), "--ranks",
                               str(a.ranks), "--dir", d, "--timeout", str(a.timeout)],
                              stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for r in range(a.ranks)]
    for r, pr in enumerate(procs):
        try:
            o, e = pr.communicate(timeout=3 * a.timeout + 60)
        except subprocess.TimeoutExpired:
            pr.kill()
            o, e = pr.communicate()
        print(f"rank {r} exit {pr.returncode}")
        print(o.strip())
        tail = [ln for ln in e.splitlines() if "WARN" in ln or "rror" in ln][-8:]
        if tail:
            print("  stderr: " + "\n  stderr: ".join(tail))


if __name__ == "__main__":
    main()
