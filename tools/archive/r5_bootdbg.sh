#!/bin/bash
# the failing configuration of the intermittent bootstrap zeros (one pool per
# context, destroyed contexts kept alive: 13 of 20 runs failed in round 4) with EXACTO_DEBUG_BOOT=1,
# which now also logs every allocation / release of the library (pointer, size, pool, stream and the
# runtime's allocation range) and watches the bootstrap's c0pt block for writes by the library's
# generic writers.  The C++ host-API test binary (every golden case, then the bootstrap case) runs up
# to N times and stops at the first failing run, whose log is kept.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-bootdbg5}; N=${2:-5}
mkdir -p $O/fx
cd $R
python3 - "$O/fx" > $O/names.txt <<'PY' || exit 1
import sys
sys.path.insert(0, "tests")
from test_cpp_api import _write_fixtures
print(" ".join(_write_fixtures(sys.argv[1])))
PY
NAMES=$(cat $O/names.txt)
for i in $(seq 1 $N); do
  EXACTO_SCRATCH_POOL=own EXACTO_LEAK_CTX=1 EXACTO_DEBUG_BOOT=1 timeout -k 10 60 ./build/test_api $O/fx $NAMES > $O/run$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"
  [ $rc -gt 1 ] && { tail -5 $O/run$i.log; exit 1; }
  if grep -q "FAIL" $O/run$i.log; then grep -n "FAIL\|boot-dbg watch\|boot-dbg ptrs" $O/run$i.log | tail -20; exit 0; fi
done
echo "no failure in $N runs"
