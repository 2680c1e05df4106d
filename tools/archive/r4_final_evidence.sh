#!/bin/bash
# Round-4 final pass, part 2: tools/evidence.sh (kernel trace stats with two lanes and with one, HBM
# traffic, VALU counters) for the configurations named -> gpurun_out/<name>_<cfg>/
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=${1:-r4ev}; shift
for c in ${@:-cfg3 cfg1 u64dbfv}; do
  timeout -k 10 600 bash $R/tools/evidence.sh ${NAME}_$c $c > $R/gpurun_out/${NAME}_$c.log 2>&1 || { echo "evidence $c failed"; tail -20 $R/gpurun_out/${NAME}_$c.log; exit 1; }
  echo "evidence $c done"
done
