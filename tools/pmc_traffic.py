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
import json
import os
import sys


def per_dispatch(path, counter):
    """{kernel name: {dispatch id: value}} (counter summed over the dimensions rocprofv3 reports)."""
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals[name][(f, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
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
for name in sorted(set(fetch) | set(write)):
    rd = [2 * 1024 * v for v in fetch.get(name, {}).values()]
    wr = [1024 * v for v in write.get(name, {}).values()]
    if not rd or not wr:
        continue
    res["kernels"][name] = {"dispatches": len(rd), "read_bytes_avg": sum(rd) / len(rd),
                            "write_bytes_avg": sum(wr) / len(wr),
                            "traffic_bytes_avg": sum(rd) / len(rd) + sum(wr) / len(wr)}
print(json.dumps(res, indent=1))
