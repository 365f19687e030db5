#!/usr/bin/env python3
"""ms per round of aligned vs ragged sizes (element-wide access when a row
is not a whole number of 16-byte vectors): fixed-round device solves
(eps = 0, --rounds rounds; loop_ms / rounds, K0 included), best of 3.

    python3 tools/ragged_probe.py [--mfree] [--small]
"""
import argparse
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from eigen_value_amd import device as dev  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--rounds", type=int, default=24)
p.add_argument("--small", action="store_true", help="one-launch k_round sizes (< 144 MiB)")
p.add_argument("--mfree", action="store_true", help="the matrix-free form")
a = p.parse_args()
if a.small:
    cases = ((torch.float64, (2048, 2047, 4096, 4095)), (torch.float32, (4096, 4094, 6000, 6001)))
else:
    cases = ((torch.float64, (8192, 8191, 16384, 16385, 32768, 32767)),
             (torch.float32, (8192, 8190, 23168, 23171)))
modes = ((dict(matrix_free=True), "mfree", 1),) if a.mfree else \
    ((dict(write_every_round=True), "every=True", 2), (dict(), "every=False", 2))
s = dev.DeviceSolver("cuda:0")
for dt, sizes in cases:
    for n in sizes:
        a0 = dev.generate("random", n, dt, seed=0, device="cuda:0")
        for kw, name, passes in modes:
            best = 1e9
            for rep in range(3):
                m = a0 if a.mfree else a0.clone()
                torch.cuda.synchronize()
                _, _, it, st = s.solve(m, inplace=True, eps=0.0, max_itr=a.rounds, **kw)
                best = min(best, st["loop_ms"] / a.rounds)
                del m
            print(f"{str(dt)[6:]} n={n} {name}: {best:.4f} ms/round "
                  f"({passes * n * n * a0.element_size() / best / 1e6:.0f} GB/s on {passes}N^2b)",
                  flush=True)
        del a0
        torch.cuda.empty_cache()
