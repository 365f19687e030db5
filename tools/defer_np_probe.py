#!/usr/bin/env python3
"""Cost of the pending rounds in a read-only deferred flat round
(st_round_flat_deferred, store = 0): npend = 0, 1, 2 with the pending row
sums in their own vectors (as the solve keeps them) or aliased to s_k
(same addresses as the current round's column scales: L1 hits), 32768^2
fp64 by default.  Tells the pending loads' cost from the extra arithmetic.

    python3 tools/defer_np_probe.py [--n 32768] [--f32]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from eigen_value_amd import device as dev  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--n", type=int, default=32768)
p.add_argument("--f32", action="store_true")
p.add_argument("--reps", type=int, default=10)
a = p.parse_args()
dt = torch.float32 if a.f32 else torch.float64
n, D = a.n, "cuda:0"
mat = dev.generate("random", n, dt, seed=0, device=D)
g = torch.Generator(device="cpu").manual_seed(1)
m = dev.defer_rounds(n, n, dt)
# s_k plus m - 1 pending vectors (the storing round re-applies m - 1)
vecs = [(torch.rand(n, generator=g, dtype=torch.float64) * n / 2 + n / 4).to(dt).to(D)
        for _ in range(m)]
invs = [1.0 / x for x in vecs]
s_next, inv_next = torch.empty(n, dtype=dt, device=D), torch.empty(n, dtype=dt, device=D)
v = torch.ones(n, dtype=dt, device=D)
part = dev.flat_scratch(n, n, dt, D)
state = dev.new_state(D)
print(f"n={n} {dt} rounds per store {m}", flush=True)


def run(npend, alias, store=False, k0=1):
    ps = [vecs[0] if alias else vecs[1 + i] for i in range(npend)]
    pi = [invs[0] if alias else invs[1 + i] for i in range(npend)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = []
    for r in range(a.reps + 2):
        dev.reset_state(state)
        ev[0].record()
        dev.flat_round_deferred(mat, vecs[0], invs[0], s_next, inv_next, part, v, state,
                                ps, pi, store=store, k=k0 + 2 * r, max_itr=1 << 30, eps=0.0)
        ev[1].record()
        torch.cuda.synchronize()
        if r >= 2:
            times.append(ev[0].elapsed_time(ev[1]))
    return min(times), sorted(times)[len(times) // 2]


# read-only rounds carry 0 .. m - 2 pending scalings (m - 1 pending is the
# storing round, which a non-storing call is refused)
for npend in range(m - 1):
    for alias in (False, True):
        if npend == 0 and alias:
            continue
        best, med = run(npend, alias)
        print(f"npend={npend} {'aliased to s_k' if alias else 'own vectors   '}: "
              f"best {best:.4f} ms, median {med:.4f} ms "
              f"({n * n * mat.element_size() / best / 1e6:.0f} GB/s read)", flush=True)
best, med = run(m - 1, False, store=True)
print(f"npend={m - 1} storing            : best {best:.4f} ms, median {med:.4f} ms", flush=True)
