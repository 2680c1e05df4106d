"""Table of steady-state kernel time (single lane) and VALU per wave from tools/r2_prof.sh output."""
import json
import sys

O = sys.argv[1]
st = json.load(open(f"{O}/steady.json"))
vc = json.load(open(f"{O}/valu.json"))["kernels"]
tot = sum(v["total_us_used"] for v in st.values())
for k, v in sorted(st.items(), key=lambda kv: -kv[1]["total_us_used"]):
    m = vc.get(k) or vc.get("void " + k) or {}
    print(f"{k[:58]:58s} {v['dispatches']:4d} {v['mean_us']:8.1f} us {100 * v['total_us_used'] / tot:5.1f}%  "
          f"VALU/wave {m.get('valu_per_wave', 0):7.0f}  waves {m.get('waves', 0):8.0f}")
