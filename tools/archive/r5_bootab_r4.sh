#!/bin/bash
# the round-4 library (build/r4lib, commit a2ea7f6, with its own C++ test
# binary build/test_api_r4) against the current one (build/test_api) on the same box, alternating,
# in the configuration that failed 13 of 20 runs in round 4 (one pool per context, destroyed contexts
# kept alive).  Prints the failing-run count per library.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-bootab_r4}; K=${2:-10}
mkdir -p $O/fx
cd $R
python3 - "$O/fx" > $O/names.txt <<'PY' || exit 1
import sys
sys.path.insert(0, "tests")
from test_cpp_api import _write_fixtures
print(" ".join(_write_fixtures(sys.argv[1])))
PY
NAMES=$(cat $O/names.txt)
f4=0; f5=0
for i in $(seq 1 $K); do
  for b in r4 cur; do
    bin=./build/test_api; [ $b = r4 ] && bin=./build/test_api_r4
    EXACTO_SCRATCH_POOL=own EXACTO_LEAK_CTX=1 timeout -k 10 60 $bin $O/fx $NAMES > $O/$b.$i.log 2>&1
    rc=$?
    [ $rc -gt 1 ] && { echo "$b run $i rc=$rc: stopping"; tail -5 $O/$b.$i.log; exit 1; }
    if [ $rc -ne 0 ]; then [ $b = r4 ] && f4=$((f4+1)) || f5=$((f5+1)); grep -h "FAIL" $O/$b.$i.log | head -3; fi
  done
done
echo "round-4 library: $f4 of $K runs failed; current library: $f5 of $K runs failed"
