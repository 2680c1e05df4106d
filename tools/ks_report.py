import csv, collections, glob, json, sys
O = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ks"
print(open(f"{O}/pytest.log").read().strip().splitlines()[-1])
d = json.load(open(f"{O}/steady.json"))
vals = collections.defaultdict(lambda: collections.defaultdict(float)); names = {}
for f in glob.glob(f"{O}/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"]); vals[k][r["Counter_Name"]] += float(r["Counter_Value"]); names[k] = r["Kernel_Name"].split("(")[0]
agg = collections.defaultdict(list)
for k, v in vals.items(): agg[names[k]].append(v)
for k, v in d.items():
    pm = agg.get(k) or agg.get("void " + k) or []
    vw = sum(x["SQ_INSTS_VALU"] for x in pm) / max(sum(x["SQ_WAVES"] for x in pm), 1)
    print(f"{k[:52]:52s} {v['dispatches']:4d} {v['mean_us']:8.1f} us  VALU/wave {vw:7.0f}")
for v in (1, 0):
    print("ks32" if v else "60-bit MAC", json.load(open(f"{O}/b3_{v}.json"))["value"], json.load(open(f"{O}/b5_{v}.json"))["value"])
