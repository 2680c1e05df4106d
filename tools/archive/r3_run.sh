#!/bin/bash
# Round 3 GPU pass: whole -m gpu suite, then the bench line of each BASELINE config.
# usage: bash tools/r3_run.sh <outdir-name> [configs...]
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-r3run}; shift
mkdir -p $O
cd $R
K=(); [ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in ${@:-cfg3}; do
  timeout -k 10 400 python3 bench.py --config $c > $O/bench_$c.json 2>> $O/bench_err.log || exit 1
  cat $O/bench_$c.json
done
echo done
