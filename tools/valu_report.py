"""Per-kernel issue counters from `rocprofv3 --pmc ...` runs of bench.py (one or more pass
directories) -> the JSON bench.py reads as profiles/r3_<cfg>_valu_counters.json.

Every counter found is averaged per dispatch.  Derived, where the counters are present:
  valu_per_wave        SQ_INSTS_VALU / SQ_WAVES
  gpu_cycles           GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs)
  wave_cycles          SQ_WAVE_CYCLES * 4 / SQ_WAVES (SQ_* cycle counters count quad-cycles)
  frac_active / frac_wait_any / frac_wait_inst   SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY (parked:
                       s_waitcnt / barrier), SQ_WAIT_INST_ANY (issue stall) over SQ_WAVE_CYCLES
                       (the three are disjoint and sum to about 1)
  frac_valu            SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES

usage: python3 tools/valu_report.py "<source description>" <pmc dir> [<pmc dir> ...] > out.json
"""
import collections
import csv
import glob
import gzip
import json
import sys

src = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
grids = {}
for d in sys.argv[2:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv*", recursive=True):
        op = gzip.open(f, "rt") if f.endswith(".gz") else open(f)
        for r in csv.DictReader(op):
            k = (d, int(r["Dispatch_Id"]))
            vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
            names[k] = r["Kernel_Name"].split("(")[0].replace("void ", "")
            grids[k] = int(r.get("Grid_Size") or 0)
# the passes run bench.py --no-latency (tools/evidence.sh, tools/r4_pmc.sh): every dispatch is part
# of a full batch, and the averages are over all of them (the launch mix bench.py's own per-launch
# averages cover).  --min-grid-frac F drops grids below F x the kernel's largest (a run that still
# has the batch-1 latency block).
MIN_FRAC = float(sys.argv[sys.argv.index("--min-grid-frac") + 1]) if "--min-grid-frac" in sys.argv else 0.0
if "--min-grid-frac" in sys.argv:
    i = sys.argv.index("--min-grid-frac")
    del sys.argv[i:i + 2]
top = {}
for k, nm in names.items():
    top[nm] = max(top.get(nm, 0), grids[k])
vals = {k: v for k, v in vals.items() if grids[k] >= MIN_FRAC * top[names[k]]}
# the passes are separate runs of the same program: dispatch ids line up per kernel name in order
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for k, v in sorted(vals.items()):
    for c, x in v.items():
        agg[names[k]][c].append(x)
out = {"source": src,
       "note": "per-dispatch averages over each kernel's largest-grid dispatches; SQ_* counts are chip totals (cycle counters in quad-cycles); "
               "GRBM_GUI_ACTIVE summed over 8 XCDs (divided back in gpu_cycles)",
       "kernels": {}}


def avg(c, name):
    lst = agg[name].get(c)
    return sum(lst) / len(lst) if lst else None


for name in sorted(agg, key=lambda nm: -(avg("GRBM_GUI_ACTIVE", nm) or 0) * len(agg[nm].get("GRBM_GUI_ACTIVE", [1]))):
    e = {"dispatches": max(len(x) for x in agg[name].values())}
    for c in sorted(agg[name]):
        e[c] = avg(c, name)
    w = e.get("SQ_WAVES") or 0
    if e.get("SQ_INSTS_VALU") is not None:
        e["valu_insts"] = e["SQ_INSTS_VALU"]
        e["valu_per_wave"] = e["SQ_INSTS_VALU"] / max(w, 1)
    if e.get("GRBM_GUI_ACTIVE") is not None:
        e["gpu_cycles"] = e["GRBM_GUI_ACTIVE"] / 8
    if w:
        e["waves"] = w
    wc = e.get("SQ_WAVE_CYCLES")
    if wc:
        e["wave_cycles"] = wc * 4 / max(w, 1)
        for c, key in (("SQ_ACTIVE_INST_ANY", "frac_active"), ("SQ_WAIT_ANY", "frac_wait_any"),
                       ("SQ_WAIT_INST_ANY", "frac_wait_inst"), ("SQ_ACTIVE_INST_VALU", "frac_valu"),
                       ("SQ_WAIT_INST_LDS", "frac_wait_lds")):
            if e.get(c) is not None:
                e[key] = e[c] / wc
    out["kernels"][name] = e
json.dump(out, sys.stdout, indent=1)
print()
