#!/usr/bin/env python3
"""Where the bench's host-clock overhead comes from: the
timed region is t0 -> K rounds -> torch.cuda.synchronize(), so ms_per_step
carries a fixed start + stop latency that K = 20 (the driver's) amortises
over 20 rounds and K = 200 (the builder's old default) over 200.  For the
configs[1] round (k_flat + k_parts, Hilbert 8192^2 fp64) this prints, per K:
host ms per round, HIP-event ms per round and the difference times K (the
fixed part), plus the cost of an idle synchronize and of an event round
trip, and K = 20 once more with an amdgpu sysfs clock read right before t0
(`20+clocks`).  Run as is and with HSA_ENABLE_INTERRUPT=0 (the runtime then polls
completion signals instead of sleeping on an interrupt).

    python3 tools/sync_probe.py [--json OUT]
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from eigen_value_amd.sharded import ShardedSimilarityTransform
    torch.cuda.set_device(0)
    out = {"HSA_ENABLE_INTERRUPT": os.environ.get("HSA_ENABLE_INTERRUPT")}
    # an idle synchronize, and an event recorded on an idle stream
    torch.cuda.synchronize()
    t = []
    for _ in range(200):
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    out["idle_sync_us"] = round(sorted(t)[len(t) // 2] * 1e6, 2)
    e = torch.cuda.Event()
    t = []
    for _ in range(200):
        t0 = time.perf_counter()
        e.record()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    out["event_roundtrip_us"] = round(sorted(t)[len(t) // 2] * 1e6, 2)
    sh = ShardedSimilarityTransform(8192, torch.float64)
    sh.load("hilbert")
    import bench
    res = {}
    for k in (1, 5, 20, 200, "20+clocks"):
        clocks = isinstance(k, str)
        kk = 20 if clocks else k
        rows = []
        for _ in range(a.reps):
            sh.load("hilbert")
            sh.start()
            sh.rounds(5, 0.0, 2 ** 31)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
            torch.cuda.synchronize()
            if clocks:   # an amdgpu sysfs clock read right before t0 (round 6's first bench)
                bench.gpu_clocks(torch, 0)
            t0 = time.perf_counter()
            ev[0].record()
            sh.rounds(kk, 0.0, 2 ** 31)
            ev[1].record()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            evm = ev[0].elapsed_time(ev[1])
            rows.append((el * 1e3 / kk, evm / kk, (el * 1e3 - evm) * 1e3))
        rows.sort(key=lambda r: r[0])
        med = rows[len(rows) // 2]
        res[str(k)] = {"host_ms_per_round": round(med[0], 5), "event_ms_per_round": round(med[1], 5),
                       "fixed_us": round(med[2], 1)}
        print(k, res[str(k)], flush=True)
    out["by_k"] = res
    sh.close()
    print(json.dumps(out), flush=True)
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
