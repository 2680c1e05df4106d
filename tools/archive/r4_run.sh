#!/bin/bash
# Round 4 GPU pass: the -m gpu suite (or the tests PYTEST_K selects), then one bench line per config.
# usage: bash tools/r4_run.sh <outdir-name> [configs...]   (PYTEST_K=skip: no tests)
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-r4run}; shift
mkdir -p $O
cd $R
if [ "$PYTEST_K" != "skip" ]; then
  K=(); [ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for c in "$@"; do
  timeout -k 10 400 python3 bench.py --config $c $BENCH_ARGS > $O/bench_$c.json 2>> $O/bench_err.log || { echo "bench $c failed"; tail -20 $O/bench_err.log; exit 1; }
  cat $O/bench_$c.json
done
echo done
