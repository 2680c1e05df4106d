#!/usr/bin/env python3
"""Steady-state per-kernel durations from a rocprofv3 kernel trace: drops each kernel's first
`--skip` dispatches (warmup: clock ramp, cold caches) and reports mean/median of the rest, so
the figure is comparable with bench.py's live per-launch timing of its profiled step."""
import argparse
import csv
import json
import statistics
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--skip-frac", type=float, default=0.3, help="fraction of each kernel's dispatches dropped")
a = ap.parse_args()
by = defaultdict(list)
for r in csv.DictReader(open(a.trace)):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    by[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
out = {}
for k, v in by.items():
    s = v[int(len(v) * a.skip_frac):]
    out[k] = {"dispatches": len(v), "used": len(s), "mean_us": round(statistics.mean(s), 2),
              "median_us": round(statistics.median(s), 2), "total_us_used": round(sum(s), 1)}
print(json.dumps(dict(sorted(out.items(), key=lambda kv: -kv[1]["total_us_used"])), indent=1))
