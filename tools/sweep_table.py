#!/usr/bin/env python3
"""Tabulate tools/sweep_dir output: each variant's time relative to the
best variant at that size (1.000 = best).

    python3 tools/sweep_table.py profiles/r01_sweep_dir.log
"""
import re
import sys


def parse(path):
    cur, res = None, {}
    for line in open(path):
        m = re.match(r"n=(\d+)(?:x(\d+))? (f\d\d)", line)
        if m:
            rows = int(m[1])
            cols = int(m[2]) if m[2] else rows
            cur = (rows, cols, m[3])
            continue
        m = re.match(r"\s+(k_round|k_mfree) rows=(\d) nt=(\d) alt=(\d) grid=\s*(\d+)\s+([\d.]+) ms", line)
        if m:
            key = (int(m[2]), int(m[3]), int(m[4]), int(m[5]))
            res.setdefault((cur, m[1]), {})[key] = float(m[6])
    return res


def main(path):
    res = parse(path)
    for kern in ("k_round", "k_mfree"):
        sizes = sorted({c for (c, k) in res if k == kern})
        keys = sorted({v for (c, k), d in res.items() if k == kern for v in d})
        label = lambda c: (f"{c[0]}" if c[0] == c[1] else f"{c[0]}x{c[1]}") + f" {c[2][1:]}"
        w = max(10, max(len(label(c)) for c in sizes) + 2)
        print(kern, "(rows, nt, alt, grid)")
        print("variant".ljust(20) + "".join(label(c).rjust(w) for c in sizes))
        for v in keys:
            row = str(v).ljust(20)
            for c in sizes:
                d = res[(c, kern)]
                row += (f"{d[v] / min(d.values()):.3f}".rjust(w) if v in d else " " * w)
            print(row)
        print("best ms".ljust(20) + "".join(f"{min(res[(c, kern)].values()):.4f}".rjust(w) for c in sizes))
        print()


if __name__ == "__main__":
    main(sys.argv[1])
