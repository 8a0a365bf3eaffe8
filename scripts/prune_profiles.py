#!/usr/bin/env python
"""List (or remove with --apply) the files under profiles/ that no document cites.

    python scripts/prune_profiles.py [--apply]

A file is kept when DESIGN.md, README.md, INTEGRATION.md or bench.py names it -- literally, or through
the shell-style patterns those documents use (`r05_pmc_d4ic{,_g}_{fetch,write}_*`, `r02_bench_v*.log`,
a name cited without its extension) -- or when it is profiles/pmc_traffic.json (bench.py reads it).
With --apply the others are removed with `git rm` (they stay in the history)."""
import fnmatch
import itertools
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOCS = ["DESIGN.md", "README.md", "INTEGRATION.md", "bench.py"]


def expand_braces(pat):
    m = re.search(r"\{([^{}]*)\}", pat)
    if not m:
        return [pat]
    out = []
    for alt in m.group(1).split(","):
        out += expand_braces(pat[:m.start()] + alt + pat[m.end():])
    return out


def cited_patterns():
    pats = set()
    for doc in DOCS:
        text = open(os.path.join(ROOT, doc)).read()
        for tok in re.findall(r"(?:profiles/)?(r0\d_[A-Za-z0-9_*{},.\-]+)", text):
            tok = tok.rstrip(".,")
            for p in expand_braces(tok):
                pats.add(p)
    return pats


def main(apply):
    files = sorted(os.listdir(os.path.join(ROOT, "profiles")))
    pats = cited_patterns()
    keep, drop = [], []
    for f in files:
        if f == "pmc_traffic.json":
            keep.append(f)
            continue
        base = f.rsplit(".", 1)[0]
        ok = any(fnmatch.fnmatch(f, p) or fnmatch.fnmatch(base, p) or f.startswith(p.rstrip("*") + ".") or
                 (p.endswith("*") and f.startswith(p[:-1])) for p in pats)
        (keep if ok else drop).append(f)
    print("%d files, %d cited, %d not cited" % (len(files), len(keep), len(drop)))
    for f in drop:
        print("  drop", f)
    if apply and drop:
        for chunk in (drop[i:i + 100] for i in range(0, len(drop), 100)):
            subprocess.check_call(["git", "rm", "-q", "--"] + [os.path.join("profiles", f) for f in chunk], cwd=ROOT)


if __name__ == "__main__":
    main("--apply" in sys.argv[1:])
