#!/bin/bash
# Diagnostic of DESIGN.md §3's intermittent bootstrap result: the C++ host-API test (all its cases,
# as the GPU suite runs it) with EXACTO_DEBUG_BOOT=1, up to N times, stopping at the first failing
# run; the snapshots of every bootstrap intermediate are in the failing run's log.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-bootdbg}; N=${2:-6}
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  EXACTO_DEBUG_BOOT=1 timeout -k 10 120 python3 -u -m pytest tests/test_cpp_api.py -m gpu -q -x --timeout 100 > $O/run$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"
  [ $rc -ne 0 ] && { grep -n "boot-dbg\|boot v=\|FAIL" $O/run$i.log | tail -80; exit 0; }
done
echo "no failure in $N runs"
