#!/usr/bin/env python3
"""Per-round cost of the exchange step on one GPU: the fused round alone,
round + torch.distributed all_gather_into_tensor (ProcessGroupNCCL: its own
stream, event hand-offs), and round + the library's RCCL communicator on
the launch stream, and the host time inside each exchange call (the
library's communicators are non-blocking since round 4: a call that
returns ncclInProgress is polled to completion of its enqueue).  World
size 1 (the collective still runs), n = 8192 (N=...)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import torch.distributed as dist
    from eigen_value_amd.sharded import RcclComm, ShardedSimilarityTransform, _allgather
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    n, K = int(os.environ.get("N", "8192")), 300
    sh = ShardedSimilarityTransform(n, torch.float64)
    sh.load("hilbert")
    rccl = RcclComm()
    res = {}
    for mode in ("none", "torch", "native", "none", "torch", "native"):
        sh.start()
        for _ in range(10):
            sh.round(0.0, 2**31)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = 0.0      # time inside the exchange call itself (host enqueue)
        for _ in range(K):
            sh.round(0.0, 2**31)
            s = sh.s[sh.cur]
            t1 = time.perf_counter()
            if mode == "torch":
                _allgather(s, s[:sh.part.chunk])
            elif mode == "native":
                rccl.allgather(s, s[:sh.part.chunk])
            host += time.perf_counter() - t1
        torch.cuda.synchronize()
        res.setdefault(mode, []).append((time.perf_counter() - t0) / K * 1e3)
        res.setdefault(mode + "_host_us", []).append(host / K * 1e6)
    for m, v in res.items():
        if m.endswith("_host_us"):
            print(f"{m:>15}: exchange call on the host {min(v):.1f} us per round")
        else:
            print(f"{m:>15}: ms/round {min(v):.5f}  (runs {', '.join(f'{x:.5f}' for x in v)})")
    rccl.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
