#!/usr/bin/env python3
"""Prints the key fields of bench JSON lines found in the given log files."""
import json
import sys

for path in sys.argv[1:]:
    for line in open(path):
        line = line.strip()
        if not line.startswith("{"):
            continue
        r = json.loads(line)
        print(r["config"].get("workload"), r["value"], r["unit"], "ms/step", r["ms_per_step"],
              "e2e", r.get("e2e_ms"), "f+tb GCUPS", r.get("gcups_fill_plus_traceback"), "fill", r.get("fill_ms_per_launch", {}).get("median"),
              "roofline", {k: r.get("roofline", {}).get(k) for k in ("achieved", "frac")})
