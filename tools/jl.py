#!/usr/bin/env python3
"""Print chosen fields of the last JSON line of bench outputs (experiment tooling).
  python tools/jl.py file.json [file2.json ...]"""
import json
import sys

for f in sys.argv[1:]:
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(f, "unreadable:", type(e).__name__)
        continue
    r = d.get("roofline") or {}
    print(f, "ms/step", round(d.get("ms_per_step", 0), 4), "value %.4g" % d.get("value", 0), "frac",
          round(r.get("frac", 0) or 0, 4), "traffic", r.get("traffic"))
