#!/bin/bash
# Verification pass: extraction repro (pool scratch, with and without the 0xFF fill), C++ API
# suite 3x with the fill, then the whole GPU suite.  Stops at the first crash/timeout.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/verify; mkdir -p $O
cd $R
stop() { [ $1 -ge 124 ] && { echo "step rc=$1: stopping"; exit $1; }; return 0; }
timeout -k 10 150 python3 tools/r2_repro_extract.py > $O/repro.log 2>&1; rc=$?; echo "repro rc=$rc"; stop $rc
EXACTO_DEBUG_SCRATCH=1 timeout -k 10 150 python3 tools/r2_repro_extract.py > $O/repro_fill.log 2>&1; rc=$?; echo "repro fill rc=$rc"; stop $rc
for i in 1 2 3; do
  EXACTO_DEBUG_SCRATCH=1 timeout -k 10 120 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_cpp_api.py > $O/cpp_$i.log 2>&1
  rc=$?; echo "cpp $i rc=$rc"; stop $rc
done
timeout -k 10 500 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest.log; stop $rc
exit 0
