#!/bin/bash
# Same-box A/B of runtime switches on bench.py lines: each variant is a comma-separated list of
# VAR=value settings ("-" = the defaults), run alternately, two repetitions per config.
# usage: bash tools/ab_env.sh <name> "<variant> <variant> ..." [configs]
#   e.g. bash tools/ab_env.sh pin "- EXACTO_TENSOR_PIN=0 EXACTO_TENSOR_PIN=1" cfg3 cfg5
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-abenv}; VARS=${2:--}; shift 2
mkdir -p $O
cd $R
for c in ${@:-cfg3}; do
  for rep in 1 2; do
    for v in $VARS; do
      tag=$(echo "$v" | tr ',=/' '___')
      envs=(); [ "$v" != "-" ] && IFS=',' read -ra envs <<< "$v"
      env "${envs[@]}" timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --min-time 1.5 \
        > $O/${tag}_${c}_$rep.json 2>> $O/err.log || exit 1
      python3 - $O/${tag}_${c}_$rep.json "$v" $c <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ks = " ".join(f"{k}={v['avg_launch_us']:.0f}x{v['launches']}" for k, v in (d.get("kernels") or {}).items())
print(sys.argv[2], sys.argv[3], d["value"], "|", ks)
PY
    done
  done
done
echo done
