"""Print the headline and the secondary figures of a bench.py JSON line (tooling)."""
import json
import sys

d = json.load(open(sys.argv[1]))
print("headline", round(d["value"] / 1e6, 1), "M", d["unit"], "ms/step", round(d["ms_per_step"], 4),
      "frac", (d.get("roofline") or {}).get("frac"))
for k, v in d.items():
    if isinstance(v, dict) and "value" in v:
        print(" ", k, round(v["value"] / 1e6, 2), "M", v.get("launch_ms") or (v.get("fwd_ms"), v.get("bwd_ms")))
