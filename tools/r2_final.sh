#!/bin/bash
# End-of-round evidence: whole GPU suite, every bench configuration, single-lane kernel traces.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/final; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in cfg3 cfg4 cfg5 cfg2 galois; do
  timeout -k 10 300 python3 bench.py --config $c > $O/bench_$c.json 2>> $O/bench_err.log || exit 1
  cat $O/bench_$c.json
done
SPLIT_CONFIGS="cfg5 cfg4" bash tools/r2_split.sh || exit 1
mkdir -p $O/prof_cfg5_dual
bash tools/prof_bench.sh final/prof_cfg5_dual --config cfg5 --steps 6 || exit 1
echo done
