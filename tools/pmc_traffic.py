#!/usr/bin/env python3
"""Per-launch HBM bytes of every kernel of a bench.py run, from the FETCH_SIZE / WRITE_SIZE passes of
tools/evidence.sh (one counter per rocprofv3 run).

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and reports half of the bytes
of wide coalesced streaming reads (16 B/lane `global_load` and `... lds` alike), so read bytes =
2 * 1024 * FETCH_SIZE; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.  Several kernels store
8 B per lane, so both factors are also measured on a known byte count: tools/ntt_bench.py's forward
transforms read and write exactly 8 n bytes per polynomial (cal_*), and the measured factors are
reported next to the prescribed ones.  Output: per kernel, averages over its dispatches; bench.py
divides them by its own algorithmic bytes per launch over the same launch mix.

usage: python3 tools/pmc_traffic.py <dir with fetch/ write/ [cal_fetch/ cal_write/]> > traffic.json
"""
import collections
import csv
import glob
import gzip
import json
import os
import sys


GRID = {}   # (file, dispatch id) -> grid size in threads


def per_dispatch(path, counter):
    """{kernel name: {dispatch id: value}} (counter summed over the dimensions rocprofv3 reports)."""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv*"), recursive=True):
        for r in csv.DictReader(gzip.open(f, "rt") if f.endswith(".gz") else open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name][(f, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
            GRID[(f, int(r["Dispatch_Id"]))] = int(r.get("Grid_Size") or 0)
    return vals


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else None


out = sys.argv[1]
res = {"correction": "read = 2 x 1024 x FETCH_SIZE (guide), write = 1024 x WRITE_SIZE", "kernels": {}}
cf = per_dispatch(os.path.join(out, "cal_fetch"), "FETCH_SIZE")
cw = per_dispatch(os.path.join(out, "cal_write"), "WRITE_SIZE")
if cf:
    # calibration: ntt_bench runs 1 + 2 forward launches over 16384 polys of n = 4096
    known = 16384 * 8 * 4096
    fk = [v for k, d in cf.items() if "ntt_fwd" in k for v in d.values()]
    wk = [v for k, d in cw.items() if "ntt_fwd" in k for v in d.values()]
    res["calibration"] = {"known_bytes_per_launch_each_way": known,
                          "fetch_factor_measured": known / (1024 * med(fk)) if fk else None,
                          "write_factor_measured": known / (1024 * med(wk)) if wk else None}
fetch = per_dispatch(os.path.join(out, "fetch"), "FETCH_SIZE")
write = per_dispatch(os.path.join(out, "write"), "WRITE_SIZE")
# The passes run the bench command with --no-latency (tools/evidence.sh), so every dispatch belongs
# to a full batch.  A full batch launches several sizes (e.g. a 7168-product chunk and a 1024-product
# rest, or transforms of different polynomial counts) and bench.py's algorithmic bytes per launch
# average over that mix: the top-level figures average every dispatch, weighted by dispatch;
# "largest_grid" keeps the largest size alone.  (A run with the latency block also holds batch-1
# dispatches: pass --min-grid-frac F to drop grids below F x the largest.)
MIN_FRAC = float(sys.argv[sys.argv.index("--min-grid-frac") + 1]) if "--min-grid-frac" in sys.argv else 0.0
res["note"] = ("top-level figures per kernel: averages over all its dispatches of a bench.py --no-latency run "
               "(the launch mix bench.py averages its algorithmic bytes over); largest_grid: that size alone; "
               "by_grid: every size")
for name in sorted(set(fetch) | set(write)):
    fd, wd = fetch.get(name, {}), write.get(name, {})
    if not fd or not wd:
        continue
    by = {}
    for grid in sorted({GRID[k] for k in fd} | {GRID[k] for k in wd}):
        rd = [2 * 1024 * v for k, v in fd.items() if GRID[k] == grid]
        wr = [1024 * v for k, v in wd.items() if GRID[k] == grid]
        if rd and wr:
            by[grid] = {"dispatches": len(rd), "read_bytes_avg": sum(rd) / len(rd),
                        "write_bytes_avg": sum(wr) / len(wr),
                        "traffic_bytes_avg": sum(rd) / len(rd) + sum(wr) / len(wr)}
    if not by:
        continue
    big = max(by)
    mix = [g for g in by if g >= MIN_FRAC * big]
    nd = sum(by[g]["dispatches"] for g in mix)
    top = {"dispatches": nd}
    for key in ("read_bytes_avg", "write_bytes_avg", "traffic_bytes_avg"):
        top[key] = sum(by[g][key] * by[g]["dispatches"] for g in mix) / nd
    top["grid_threads_mix"] = sorted(mix)
    top["largest_grid"] = dict(by[big], grid_threads=big)
    if len(by) > 1:
        top["by_grid"] = {str(g): v for g, v in by.items()}
    res["kernels"][name] = top
print(json.dumps(res, indent=1))
