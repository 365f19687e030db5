#!/usr/bin/env python3
"""The library's launch policy as one map (st_launch_policy_query): for a
set of blocks that covers every size class and launch form the solve loops
use - fp32 / fp64, cached and non-temporal flat blocks, k_round below 144
MiB, the weak-scaled and configs[3] rank blocks - the kernel, rows per
workgroup, piece tile, workgroups-per-CU cap and load / store cache policy
of the every-round, deferred (by pending count) and matrix-free launches.

    python3 tools/launch_policy_table.py            # print a markdown table
    python3 tools/launch_policy_table.py --write    # regenerate tests/golden/launch_policy.json

tests/test_capi.py pins the library against the committed JSON, so any
change of a launch shape or cache policy shows in the diff."""
import json
import os
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
GOLDEN = os.path.join(HERE, "tests", "golden", "launch_policy.json")

# (dtype, nrows, ncols, what)
BLOCKS = [
    ("f64", 2048, 2048, "L2-sized"), ("f64", 4096, 4096, "128 MiB"),
    ("f64", 6144, 6144, "288 MiB, flat cached"), ("f64", 8192, 8192, "configs[1]"),
    ("f64", 5824, 11648, "weak P=2 rank block"), ("f64", 4096, 16384, "weak P=4 rank block"),
    ("f64", 2880, 23040, "weak P=8 rank block"), ("f64", 10240, 10240, "800 MiB"),
    ("f64", 12288, 12288, "1.1 GiB"), ("f64", 32768, 32768, "north star"),
    ("f64", 8192, 65536, "configs[3] P=8 rank block"), ("f64", 65536, 65536, "configs[3] P=1"),
    ("f32", 4096, 4096, "64 MiB"), ("f32", 8192, 8192, "256 MiB, flat cached"),
    ("f32", 12288, 12288, "576 MiB"), ("f32", 16384, 16384, "1 GiB"),
    ("f32", 32768, 32768, "configs[4]"),
]
FORMS = [("round", 0, 0)] + [(f"read NP={k}", 1, k) for k in range(5)] + \
    [("store NP=5", 2, 5), ("mfree", 3, 0), ("K0 rowsum", 4, 0)]


def table():
    from eigen_value_amd import _lib
    out = []
    for dt, nr, nc, what in BLOCKS:
        flat = bool(_lib.load().st_round_flat_pays(nr, nc, 1 if dt == "f64" else 0))
        for name, form, np_ in FORMS:
            if form in (1, 2) and not flat:
                continue
            p = _lib.launch_policy(dt, nr, nc, form, np_)
            out.append({"block": f"{nr}x{nc}", "dtype": dt, "what": what, "form": name, **p})
    return out


def markdown(rows):
    hdr = ("| block | dtype | form | kernel | rows | tile | cap | grid | piece B | "
           "load nt | store nt | alt |\n|---|---|---|---|---|---|---|---|---|---|---|---|")
    lines = [hdr]
    for r in rows:
        lines.append(f"| {r['block']} ({r['what']}) | {r['dtype']} | {r['form']} | {r['kernel']} | "
                     f"{r['rows']} | {r['tile']} | {r['cap']} | {r['grid']} | {r['piece_bytes']} | "
                     f"{r['load_nt']} | {r['store_nt']} | {r['alt']} |")
    return "\n".join(lines)


if __name__ == "__main__":
    rows = table()
    if "--write" in sys.argv:
        with open(GOLDEN, "w") as f:
            json.dump(rows, f, indent=0)
            f.write("\n")
        print(f"wrote {GOLDEN} ({len(rows)} launches)")
    else:
        print(markdown(rows))
