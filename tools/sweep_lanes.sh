#!/bin/bash
# bench.py lines of one config over (pipeline lanes, chunk) pairs.
# usage: bash tools/sweep_lanes.sh <name> <config> <lanes:chunk ...>
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-lanes}; CFG=$2; shift 2
mkdir -p $O
cd $R
for lc in "$@"; do
  l=${lc%:*}; ch=${lc#*:}
  EXACTO_LANES=$l timeout -k 10 200 python3 bench.py --config $CFG --chunk $ch --no-cpu-baseline --min-time 1.5 > $O/${CFG}_l${l}_c$ch.json 2>> $O/err.log || exit 1
  python3 -c "import json; d=json.load(open('$O/${CFG}_l${l}_c$ch.json')); print('$CFG lanes $l chunk $ch', d['value'])"
done
