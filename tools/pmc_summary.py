"""Summarize rocprofv3 --pmc csv passes: per kernel INSTANTIATION (full Kernel_Name),
the mean counter value per dispatch.

  python tools/pmc_summary.py "<glob of counter_collection.csv>" [--json OUT_JSON]

Text to stdout (per wave too); --json writes {kernel name: {counter: mean per dispatch}}
for bench.py --pmc-json.
"""
import collections
import csv
import glob
import json
import sys


def summarize(pat):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(pat, recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def main():
    res = summarize(sys.argv[1])
    for k, v in res.items():
        w = v.get("SQ_WAVES", 1.0)
        print(k[:96], " waves/dispatch", w)
        for c, m in sorted(v.items()):
            print(f"    {c:28s} {m:16.0f}   per wave {m / max(w, 1):12.1f}")
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
