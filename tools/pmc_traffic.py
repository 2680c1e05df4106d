#!/usr/bin/env python3
"""Per-launch HBM bytes of the forward NTT from the FETCH_SIZE / WRITE_SIZE passes of
tools/pmc_traffic.sh.

Corrections (MI355X_MICROARCH.md, HBM section): FETCH_SIZE is in KiB and reports half of the bytes
of wide coalesced streaming reads (16 B/lane `global_load` and `... lds` alike), so read bytes =
2 * 1024 * FETCH_SIZE; WRITE_SIZE is exact for 16-B-per-lane stores, and other widths are
uncalibrated.  The forward kernel stores 8 B per lane, so both factors are also measured here on a
known byte count: tools/ntt_bench.py's forward transforms read and write exactly 8 n bytes per
polynomial (cal_*), and the measured factors are reported next to the prescribed ones.  Output:
averages over every forward-NTT dispatch of the bench run; bench.py divides by its own
algorithmic bytes per launch (8 n written per polynomial, 8 n read, or 2 n for the int16 digit
sources) over the same launch mix.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(path, counter):
    vals = {}
    name = None
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ntt_fwd" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0]
            key = int(r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return vals, name


out = sys.argv[1]
# calibration: ntt_bench runs 1 + 2 forward launches over 16384 polys of n = 4096
cal_f, _ = per_dispatch(os.path.join(out, "cal_fetch"), "FETCH_SIZE")
cal_w, _ = per_dispatch(os.path.join(out, "cal_write"), "WRITE_SIZE")
known = 16384 * 8 * 4096
f_factor = known / (1024 * sorted(cal_f.values())[len(cal_f) // 2]) if cal_f else None
w_factor = known / (1024 * sorted(cal_w.values())[len(cal_w) // 2]) if cal_w else None
fetch, name = per_dispatch(os.path.join(out, "fetch"), "FETCH_SIZE")
write, _ = per_dispatch(os.path.join(out, "write"), "WRITE_SIZE")
rd = [2 * 1024 * v for v in fetch.values()]       # prescribed factor 2
wr = [1024 * v for v in write.values()]            # prescribed factor 1
res = {
    "kernel": name,
    "dispatches": len(rd),
    "read_bytes_avg": sum(rd) / len(rd),
    "write_bytes_avg": sum(wr) / len(wr),
    "traffic_bytes_avg": sum(rd) / len(rd) + sum(wr) / len(wr),
    "correction": "read = 2 x FETCH_SIZE (guide), write = WRITE_SIZE",
    "calibration": {"known_bytes_per_launch_each_way": known,
                    "fetch_factor_measured": f_factor, "write_factor_measured": w_factor},
}
print(json.dumps(res, indent=1))
