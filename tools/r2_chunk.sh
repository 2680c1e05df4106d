#!/bin/bash
# cfg5 chunk size A/B: one chunk per dbfv_mul (default) vs two or four (both pipeline lanes busy).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/chunk; mkdir -p $O
cd $R
for rep in 1 2; do
  for ch in 0 144 72; do
    timeout -k 10 200 python3 bench.py --config cfg5 --no-cpu-baseline --chunk $ch > $O/cfg5_${ch}_$rep.json 2>>$O/err.log || exit 1
    python3 -c "import json; d=json.load(open('$O/cfg5_${ch}_$rep.json')); print('cfg5 chunk=$ch rep$rep', d['value'])"
  done
done
