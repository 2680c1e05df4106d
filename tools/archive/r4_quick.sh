#!/bin/bash
# Round-4 quick check: the GPU tests PYTEST_K selects (all with PYTEST_K unset), then one bench line
# (no CPU leg) per config named -> gpurun_out/<name>/.  usage: bash tools/r4_quick.sh <name> cfg...
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=$1; shift
O=$R/gpurun_out/$NAME; mkdir -p $O
cd $R
K=(); [ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench_err.log || { echo "bench $c failed"; tail $O/bench_err.log; exit 1; }
  python3 -c "import json;b=json.load(open('$O/bench_$c.json'));print('$c',b['value'],'|',' '.join(f\"{k}:{v['avg_launch_us']}us/{v['frac']}\" for k,v in b['kernels'].items()))"
done
echo quick done
