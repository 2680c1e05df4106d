#!/usr/bin/env python3
"""Summarise tools/probe_clock.sh output: per kernel, mean duration (kernel trace), GRBM cycles
per dispatch (summed over the 8 XCDs by rocprofv3, divided back) and the effective clock."""
import collections
import csv
import glob
import os
import sys

base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for d in sorted(glob.glob(os.path.join(base, "clk_*"))):
    kt = glob.glob(os.path.join(d, "kt", "**", "*kernel_trace.csv"), recursive=True)
    pm = glob.glob(os.path.join(d, "pmc", "**", "*counter_collection.csv"), recursive=True)
    if not kt or not pm:
        print(d, "incomplete")
        continue
    dur = collections.defaultdict(list)
    for r in csv.DictReader(open(kt[0])):
        dur[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(pm[0])):
        ctr[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, ds in dur.items():
        if "ntt" not in k:
            continue
        ds = sorted(ds)[len(ds) // 4:]          # drop the warm-up quarter
        t = sum(ds) / len(ds)
        c = ctr.get(k, {})
        gui = c.get("GRBM_GUI_ACTIVE", [0])
        cyc = sum(gui) / len(gui) / 8
        valu = c.get("SQ_INSTS_VALU", [0])
        print(f"{os.path.basename(d):14s} {k.split('(')[0][-28:]:28s} {t/1e3:8.1f} us  {cyc:10.0f} cyc  "
              f"{cyc / t if t else 0:5.2f} GHz  valu/disp {sum(valu)/len(valu):.3e}")
