#!/usr/bin/env python
"""Per-kernel HBM counters of rocprofv3 --pmc passes, condensed for bench.py.

    python scripts/pmc_traffic.py profiles/rNN_pmc_<cfg>_{fetch,write}_counter_collection.csv ...

Reads the per-dispatch counter CSVs (one FETCH_SIZE pass, one WRITE_SIZE pass: separate runs, as
MI355X_MICROARCH.md's HBM section prescribes) and merges into profiles/pmc_traffic.json one record per
(round, config, kernel, grid size): the mean FETCH_SIZE / WRITE_SIZE per dispatch in KiB and the
dispatch counts.  bench.py's pmc_traffic() prices a kernel's HBM bytes from these records (FETCH x 2,
the gfx950 under-count, + WRITE), so the GPU runs need not carry the multi-megabyte raw passes (they
stay committed under profiles/ and are listed in .gpurunignore)."""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "profiles", "pmc_traffic.json")


def kernel_base(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.split(r"[<(]", name, 1)[0].split("::")[-1].strip()
    return name.split()[-1]  # "void k_bwd_merged" -> k_bwd_merged


def main(paths):
    recs = json.load(open(OUT)) if os.path.exists(OUT) else []
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in paths:
        m = re.match(r"r(\d+)_pmc_(.+?)_(fetch|write)_", os.path.basename(path))
        if not m:
            raise SystemExit("unexpected file name %s" % path)
        rnd, cfg = int(m.group(1)), re.sub(r"_[gs]$", "", m.group(2))  # d4ic_g: the grid run of d4ic
        for row in csv.DictReader(open(path)):
            key = (rnd, cfg, kernel_base(row["Kernel_Name"]), int(row.get("Grid_Size") or 0))
            acc[key][row["Counter_Name"]].append(float(row["Counter_Value"]))
    new = []
    for (rnd, cfg, k, grid), cs in sorted(acc.items()):
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        new.append({"round": rnd, "config": cfg, "kernel": k, "grid_size": grid,
                    "fetch_kib": sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]),
                    "write_kib": sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]),
                    "dispatches": [len(cs["FETCH_SIZE"]), len(cs["WRITE_SIZE"])]})
    keys = set((r["round"], r["config"], r["kernel"], r["grid_size"]) for r in new)
    recs = [r for r in recs if (r["round"], r["config"], r["kernel"], r["grid_size"]) not in keys] + new
    recs.sort(key=lambda r: (r["round"], r["config"], r["kernel"], r["grid_size"]))
    with open(OUT, "w") as f:
        json.dump(recs, f, indent=0)
    print("%d records (%d new) -> %s" % (len(recs), len(new), OUT))


if __name__ == "__main__":
    main(sys.argv[1:])
