#!/usr/bin/env python3
"""List the files under profiles/ that no document, test or bench code
cites (README.md, INTEGRATION.md, bench.py, tests/,
eigen_value_amd/, include/).  Citations may use shell
patterns (`r02_flat_map_every_*.log`, `r02_defer_pmc_random32768_{f64,f32}.json`),
which are expanded against the directory.

    python3 tools/check_citations.py          # prints the uncited files
    python3 tools/check_citations.py --rm     # and removes them (git rm)
"""
import fnmatch
import glob
import itertools
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# what counts as a citation: the documents, the bench and the tests (the
# index profiles/README.md and the tools that WRITE the files do not: a file
# only they name is evidence nothing relies on)
SOURCES = ["DESIGN.md", "README.md", "INTEGRATION.md", "bench.py", "tests/*.py",
           "eigen_value_amd/*.py", "eigen_value_amd/csrc/*", "include/*.h"]
TOKEN = re.compile(r"r0\d_[A-Za-z0-9_*{},.\-\[\]]+")


def braces(p):
    """Expand {a,b} alternatives (no nesting)."""
    m = re.search(r"\{([^{}]*)\}", p)
    if not m:
        return [p]
    return list(itertools.chain.from_iterable(
        braces(p[:m.start()] + alt + p[m.end():]) for alt in m.group(1).split(",")))


ELLIPSIS = re.compile(r"…(_[A-Za-z0-9_*{},.\-\[\]]+)")


def expand_ellipsis(prev, tail):
    """`…_X` after a full name on the same line: the shared prefix of `prev`
    up to where X's first word starts in it (`r01_sweep_dir_blocks.log`,
    `…_blocks_table.txt` -> `r01_sweep_dir_blocks_table.txt`), else prev
    without its extension + tail (`r03_defer_cycle_x.json` + `…_launches.csv`)."""
    tail = tail.rstrip(".,")
    word = re.match(r"_[A-Za-z0-9]+", tail).group(0)
    i = prev.rfind(word)
    if i > 0:
        return prev[:i] + tail
    return os.path.splitext(prev)[0] + tail


def cited_patterns():
    pats = set()
    for pat in SOURCES:
        for f in glob.glob(os.path.join(HERE, pat)):
            if not os.path.isfile(f):
                continue
            for line in open(f, errors="replace").read().splitlines():
                prev = None
                for m in re.finditer(TOKEN.pattern + "|" + ELLIPSIS.pattern, line):
                    if m.group(0).startswith("…"):
                        if prev is None:
                            continue
                        tok = expand_ellipsis(prev, m.group(1))
                    else:
                        tok = prev = m.group(0).rstrip(".,")
                    for p in braces(tok):
                        pats.add(p)
    return pats


def uncited():
    files = sorted(os.listdir(os.path.join(HERE, "profiles")))
    pats = cited_patterns()
    out = []
    for f in files:
        if f == "README.md":
            continue
        stem = os.path.splitext(f)[0]
        hit = any(fnmatch.fnmatch(f, p) or fnmatch.fnmatch(stem, p) or f.startswith(p)
                  or (("*" in p or "?" in p) and fnmatch.fnmatch(f, p + "*"))
                  for p in pats)
        if not hit:
            out.append(f)
    return out


if __name__ == "__main__":
    left = uncited()
    for f in left:
        print(f"profiles/{f}")
    if "--rm" in sys.argv and left:
        subprocess.run(["git", "rm", "-q", *[f"profiles/{f}" for f in left]], cwd=HERE,
                       check=True)
