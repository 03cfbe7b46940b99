"""HBM bytes per launch from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE),
corrected as MI355X_MICROARCH.md (HBM section) prescribes for gfx950:
FETCH_SIZE counts half the bytes of wide coalesced reads -> x2; WRITE_SIZE as is.
Both counters are in KiB.  Output: {stage: bytes per launch} for bench.py
--traffic-json (stages as in bench.STAGES).

  python tools/hbm_traffic.py FETCH_DIR WRITE_DIR OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import sys


def stage_of(kernel):
    if "select_kernel" in kernel:
        return "select"
    if "finish_kernel" in kernel or "dense_rows_kernel" in kernel:
        return "finish"
    if "attn_prep_kernel" in kernel or "rows_prep_kernel" in kernel or "cols_prep_kernel" in kernel:
        return "prep"
    if "qkv_proj_kernel" in kernel:
        return "proj"
    return None


def per_stage(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            st = stage_of(r["Kernel_Name"])
            if st:
                vals[st].append(float(r["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fetch = per_stage(sys.argv[1], "FETCH_SIZE")
    write = per_stage(sys.argv[2], "WRITE_SIZE")
    out = {}
    for st in set(fetch) | set(write):
        out[st] = 2.0 * fetch.get(st, 0.0) + write.get(st, 0.0)
    out["_raw"] = {"fetch_bytes_x1": fetch, "write_bytes": write,
                   "note": "traffic = 2 * FETCH_SIZE + WRITE_SIZE (KiB -> bytes), gfx950 correction"}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
