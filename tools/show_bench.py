"""Print the headline fields of bench JSON files (paths), and of their secondary lines."""
import json
import sys

r = lambda x: round(x, 3) if isinstance(x, float) else x
for path in sys.argv[1:]:
    d = json.load(open(path))
    if "value" in d:
        print(path, round(d["value"] / 1e6, 2), "Mtok/s", r(d["ms_per_step"]), "ms",
              {k: r(v) for k, v in d.get("stages_ms", {}).items()}, d.get("parity"),
              d.get("roofline", {}).get("mfma", {}).get("engine"))
    for s in d.get("secondary", []):
        print("  ", s["config"], round(s["value"] / 1e6, 2), "Mtok/s", r(s["ms_per_step"]), "ms",
              {k: r(v) for k, v in s.get("stages_ms", {}).items()},
              {k: (r(v) if not isinstance(v, dict) else {a: r(b) for a, b in v.items() if not isinstance(b, dict)})
               for k, v in s.items() if k in ("mfma", "parity", "idx_equal_fused")})
