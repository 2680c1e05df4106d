#!/usr/bin/env python3
"""Copy one tools/evidence.sh run (gpurun_out/<run>/) into profiles/ under round-R names (R = $ROUND, default 6), and give its
bench line the traffic / VALU figures of the same run (the PMC passes run after the line is printed,
so the line itself could only cite the previous round's files):
  bench.json                      -> profiles/rR_bench_<cfg>.json (roofline.traffic / compute from below)
  prof_dual/*kernel_stats.csv     -> profiles/rR_<cfg>_bench_kernel_stats.csv
  prof_single/*kernel_stats.csv   -> profiles/rR_<cfg>_bench_kernel_stats_single_lane.csv
  steady.json                     -> profiles/rR_<cfg>_trace_steady_single_lane.json
  traffic.json / valu.json        -> profiles/rR_<cfg>_traffic.json / rR_<cfg>_valu_counters.json
usage: ROUND=6 python3 tools/collect.py <run dir under gpurun_out> <cfg>"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
run, cfg = sys.argv[1], sys.argv[2]
R = "r" + os.environ.get("ROUND", "6")
src = os.path.join(ROOT, "gpurun_out", run)
prof = os.path.join(ROOT, "profiles")


def one(pattern):
    hits = sorted(glob.glob(os.path.join(src, pattern)))
    return hits[0] if hits else None


copies = {"prof_dual/*kernel_stats.csv": f"{R}_{cfg}_bench_kernel_stats.csv",
          "prof_single/*kernel_stats.csv": f"{R}_{cfg}_bench_kernel_stats_single_lane.csv",
          "steady.json": f"{R}_{cfg}_trace_steady_single_lane.json",
          "traffic.json": f"{R}_{cfg}_traffic.json", "valu.json": f"{R}_{cfg}_valu_counters.json"}
for pat, dst in copies.items():
    f = one(pat) or one(pat.replace("/*", "/*/*"))
    if f:
        shutil.copy(f, os.path.join(prof, dst))
        print("copied", os.path.relpath(f, ROOT), "->", dst)
line = json.load(open(os.path.join(src, "bench.json")))
roof = line.get("roofline") or {}
tr = json.load(open(os.path.join(src, "traffic.json"))).get("kernels", {})
vc = json.load(open(os.path.join(src, "valu.json"))).get("kernels", {})
top = roof.get("kernel", "").split(" + ")[0]   # the library's own name of what ran (exacto_prof_kernels)
key = top.split("<")[0]
hit = [v for k, v in tr.items() if k == top] or [v for k, v in tr.items() if key and key in k]
if hit:
    roof["traffic"] = round(hit[0]["traffic_bytes_avg"], 1)
    roof["traffic_over_algorithmic"] = round(hit[0]["traffic_bytes_avg"] / roof["bytes_per_launch"], 4)
    roof["traffic_source"] = f"profiles/{R}_{cfg}_traffic.json"
hit = [v for k, v in vc.items() if k == top] or [v for k, v in vc.items() if key and key in k]
if hit:
    v = hit[0]
    need = v["valu_insts"] * 4.4 / 1024.0
    roof["compute"] = {"bound": "valu", "valu_insts_per_launch": round(v["valu_insts"]), "cycles_per_valu": 4.4,
                       "gpu_cycles_per_launch": round(v["gpu_cycles"]), "frac": round(need / v["gpu_cycles"], 3),
                       "source": f"profiles/{R}_{cfg}_valu_counters.json"}
line["evidence_run"] = run
json.dump(line, open(os.path.join(prof, f"{R}_bench_{cfg}.json"), "w"))
print("wrote", f"{R}_bench_{cfg}.json", line["value"], roof.get("kernel"), roof.get("frac"),
      roof.get("traffic_over_algorithmic"))
