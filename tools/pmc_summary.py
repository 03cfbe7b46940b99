"""Summarize rocprofv3 --pmc csv passes: per kernel, mean counter value per dispatch."""
import collections
import csv
import glob
import sys

pat = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(pat, recursive=True)):
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"][:48]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    w = v.get("SQ_WAVES", [1])
    print(k, " waves/dispatch", w[0])
    for c, vals in sorted(v.items()):
        m = sum(vals) / len(vals)
        print(f"    {c:24s} {m:16.0f}   per wave {m / max(w[0], 1):12.1f}")
