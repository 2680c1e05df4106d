"""Per-kernel VALU issue counters from a `rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE
SQ_BUSY_CYCLES` run of bench.py -> the JSON bench.py reads as profiles/r2_<cfg>_valu_counters.json.

usage: python3 tools/valu_report.py <pmc dir> <source description> > out.json
"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = (f, int(r["Dispatch_Id"]))
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = r["Kernel_Name"].split("(")[0]
agg = collections.defaultdict(list)
for k, v in vals.items():
    agg[names[k]].append(v)
out = {"source": sys.argv[2] if len(sys.argv) > 2 else d,
       "note": "per-dispatch averages; SQ_INSTS_VALU and SQ_WAVES are chip totals; "
               "GRBM_GUI_ACTIVE summed over 8 XCDs (divided back)",
       "kernels": {}}
for name, lst in sorted(agg.items(), key=lambda kv: sum(x["GRBM_GUI_ACTIVE"] for x in kv[1])):
    n = len(lst)
    vi = sum(x["SQ_INSTS_VALU"] for x in lst) / n
    w = sum(x["SQ_WAVES"] for x in lst) / n
    out["kernels"][name] = {"dispatches": n, "valu_insts": vi, "waves": w,
                            "gpu_cycles": sum(x["GRBM_GUI_ACTIVE"] for x in lst) / n / 8,
                            "valu_per_wave": vi / max(w, 1)}
json.dump(out, sys.stdout, indent=1)
print()
