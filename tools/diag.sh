#!/bin/bash
# The C++ host-API suite (bootstrap case included) three times: own scratch pool, own pool with
# EXACTO_DEBUG_SCRATCH=1 (0xFF-filled blocks), the device's default pool.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-diag}; mkdir -p $O
cd $R
for v in own debug default; do
  case $v in debug) export EXACTO_DEBUG_SCRATCH=1 ;; default) unset EXACTO_DEBUG_SCRATCH; export EXACTO_SCRATCH_POOL=default ;; esac
  timeout -k 10 300 python3 -u -m pytest tests/test_cpp_api.py -q -x --timeout 200 --timeout-method thread > $O/cpp_$v.log 2>&1
  echo "cpp $v rc=$?"; grep -E "FAIL|ERROR" $O/cpp_$v.log | head -3
done
