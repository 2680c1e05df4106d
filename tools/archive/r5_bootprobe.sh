#!/bin/bash
# whether this box shows the intermittent bootstrap zeros, and if it does, one
# failing run with the EXACTO_DEBUG_BOOT logs (allocations and releases with their runtime ranges, the
# c0pt write watch, the stream snapshots).  The C++ host-API test binary, one pool per context with
# destroyed contexts kept alive (the configuration that failed most in round 4):
#   1. up to P plain runs; none failing: "box does not reproduce", stop;
#   2. up to D runs with the diagnostics $DBG (default EXACTO_DEBUG_BOOT=1: snapshots and the c0pt
#      write watch; EXACTO_DEBUG_ALLOC=1/2: the allocation log), the first failing log kept (debug.log);
#   3. K runs of the library default (one pool per device) on the same box.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-bootprobe}; P=${2:-4}; D=${3:-8}; K=${4:-10}
mkdir -p $O/fx
cd $R
python3 - "$O/fx" > $O/names.txt <<'PY' || exit 1
import sys
sys.path.insert(0, "tests")
from test_cpp_api import _write_fixtures
print(" ".join(_write_fixtures(sys.argv[1])))
PY
NAMES=$(cat $O/names.txt)
run() {   # run <log> <env...>
  local log=$1; shift
  env "$@" timeout -k 10 60 ./build/test_api $O/fx $NAMES > $log 2>&1
  local rc=$?
  [ $rc -gt 1 ] && { echo "rc=$rc: stopping"; tail -5 $log; exit 1; }
  return $rc
}
DBG=${DBG:-EXACTO_DEBUG_BOOT=1}
hit=0
for i in $(seq 1 $P); do
  if ! run $O/plain.$i.log EXACTO_SCRATCH_POOL=own EXACTO_LEAK_CTX=1; then hit=$i; break; fi
done
[ $hit -eq 0 ] && { echo "box does not reproduce: 0 of $P plain runs failed"; exit 0; }
echo "plain run $hit failed"
for i in $(seq 1 $D); do
  if ! run $O/debug.$i.log EXACTO_SCRATCH_POOL=own EXACTO_LEAK_CTX=1 $DBG; then
    cp $O/debug.$i.log $O/debug.log; echo "debug run $i failed"; break
  fi
  echo "debug run $i passed"
done
f=0
for i in $(seq 1 $K); do run $O/shared.$i.log || f=$((f+1)); done
echo "library default (one pool per device): $f of $K runs failed"
