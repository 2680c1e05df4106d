#!/bin/bash
# Round-2 refresh on the current tree: whole GPU suite, then every bench configuration.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/refresh; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -5 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
for c in ${BENCH_CONFIGS:-cfg3 cfg4 cfg5 cfg2 galois}; do
  timeout -k 10 300 python3 bench.py --config $c > $O/bench_$c.json 2>> $O/bench_err.log || exit 1
  cat $O/bench_$c.json
done
echo done
