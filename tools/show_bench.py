import json, sys
for c in sys.argv[1:]:
    d = json.load(open(f"gpurun_out/b_{c}.json"))
    print(c, round(d["value"] / 1e6, 2), "Mtok/s", round(d["ms_per_step"], 3), "ms",
          {k: round(v, 3) for k, v in d["stages_ms"].items()}, d["parity"])
