#!/usr/bin/env python3
"""Per-launch HBM bytes of the forward NTT from the FETCH_SIZE / WRITE_SIZE passes.

gfx950 corrections (MI355X_MICROARCH.md, HBM section, and our own calibration on a known byte
count: tools/ntt_bench.py over 16384 polys reads exactly 16384 * 8n bytes): FETCH_SIZE is in KiB
and counts half of the bytes of these coalesced streaming reads, so read bytes = 2 * FETCH_SIZE;
WRITE_SIZE (KiB) is exact.  Output: averages over every ntt_fwd_kernel dispatch of the run, and
bench.py divides by its own algorithmic bytes per launch (8 n written per polynomial, 8 n read, or
2 n for the int16 digit sources) over the same launch mix.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(path, counter):
    vals = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "ntt_fwd" not in r["Kernel_Name"] or r["Counter_Name"] != counter:
                continue
            key = int(r["Dispatch_Id"])
            grid = int(r.get("Grid_Size", 0) or 0)
            wg = int(r.get("Workgroup_Size", 0) or 0)
            v = vals.setdefault(key, [0.0, grid, wg])
            v[0] += float(r["Counter_Value"])
    return vals


out = sys.argv[1]
fetch = per_dispatch(os.path.join(out, "fetch"), "FETCH_SIZE")
write = per_dispatch(os.path.join(out, "write"), "WRITE_SIZE")
rd = [2 * 1024 * v[0] for v in fetch.values()]
wr = [1024 * v[0] for v in write.values()]
res = {
    "kernel": "ntt_fwd_asm_kernel (hand-scheduled forward NTT)",
    "dispatches": len(rd),
    "read_bytes_avg": sum(rd) / len(rd),
    "write_bytes_avg": sum(wr) / len(wr),
    "traffic_bytes_avg": sum(rd) / len(rd) + sum(wr) / len(wr),
}
print(json.dumps(res, indent=1))
