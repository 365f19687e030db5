#!/usr/bin/env python3
"""Tabulate flat_map_sweep A/B logs: python3 tools/ab_table.py DIR [min_np]
(files NAME_REP.log, NAME = flat_map_sweep[_old][_f32]); one line per
block x NP x rows x tile with every variant's time."""
import collections
import glob
import re
import sys

d = sys.argv[1]
min_np = int(sys.argv[2]) if len(sys.argv) > 2 else -1
tab = collections.defaultdict(dict)
for f in sorted(glob.glob(f"{d}/*.log")):
    base = f.split("/")[-1][:-4]
    name, rep = base.rsplit("_", 1)
    var = "old" if "_old" in name else "new"
    cur = None
    for ln in open(f):
        if not ln.startswith(" "):
            cur = " ".join(ln.split()[:2])
            continue
        m = re.search(r"NP=\s*(-?\d+) R=(\d) PT=\s*(\d+).*?([\d.]+) ms", ln)
        if m:
            np_, r, pt, ms = m.groups()
            tab[(cur, int(np_), int(r), int(pt))][var + rep] = float(ms)
for k, v in sorted(tab.items()):
    if k[1] >= min_np:
        print(f"{k[0]:18s} NP={k[1]:2d} R={k[2]} PT={k[3]:2d}  " +
              " ".join(f"{a}:{b:.4f}" for a, b in sorted(v.items())))
