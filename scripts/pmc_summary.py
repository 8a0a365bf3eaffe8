import csv, sys, collections, re
rows = []
for f in sys.argv[1:]:
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])[:40]
    agg[name][r["Counter_Name"]].append((r["Dispatch_Id"], float(r["Counter_Value"])))
for k, cs in sorted(agg.items()):
    out = []
    for cn, vals in sorted(cs.items()):
        per = collections.defaultdict(float)
        for d, v in vals: per[d] += v
        m = sum(per.values()) / len(per)
        out.append("%s=%.4g" % (cn, m))
    print(k, "|", " ".join(out))
