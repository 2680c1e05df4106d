#!/bin/bash
# Same-box A/B of library builds on bench.py lines: the in-tree library against build/ab/<variant>.so
# (tools/build_variants.sh), alternating, per config.  usage: bash tools/ab_lib.sh <name> "<variants>" [configs]
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-ablib}; VARS=${2:-}; shift 2
mkdir -p $O
cd $R
for c in ${@:-cfg3}; do
  for rep in 1 2; do
    for v in cur $VARS; do
      L=""; [ $v != cur ] && L=$R/build/ab/$v.so
      EXACTO_HIP_LIB=$L timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --min-time 1.5 > $O/${v}_${c}_$rep.json 2>> $O/err.log || exit 1
      python3 - $O/${v}_${c}_$rep.json $v $c <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = " ".join(f"{k}={v['avg_launch_us']:.0f}x{v['launches']}" for k, v in (d.get("kernels") or {}).items())
print(sys.argv[2], sys.argv[3], d["value"], "|", ks)
PY
    done
  done
done
echo done
