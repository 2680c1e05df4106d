#!/bin/bash
# bench.py lines of one config over several batch sizes (throughput vs GPU fill).
# usage: bash tools/sweep_batch.sh <name> <config> <batch...>
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-sweep}; CFG=$2; shift 2
mkdir -p $O
cd $R
for b in "$@"; do
  timeout -k 10 200 python3 bench.py --config $CFG --batch $b --no-cpu-baseline --min-time 1.5 > $O/${CFG}_b$b.json 2>> $O/err.log || exit 1
  python3 -c "import json; d=json.load(open('$O/${CFG}_b$b.json')); print('$CFG batch $b', d['value'], d['unit'], d['roofline']['kernel'], d['roofline']['frac'])"
done
