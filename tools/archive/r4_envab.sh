#!/bin/bash
# Same-box A/B of one library switch: the GPU tests PYTEST_K selects (if set), then alternating bench
# lines (no CPU leg) for each value of the switch.  usage: bash tools/r4_envab.sh <name> <VAR> "<v1 v2>" cfg...
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=$1; VAR=$2; VALS=$3; shift 3
O=$R/gpurun_out/$NAME; mkdir -p $O
cd $R
if [ -n "$PYTEST_K" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "$PYTEST_K" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
for c in "$@"; do
  for i in 1 2 3; do
    for v in $VALS; do
      env $VAR=$v timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline --no-latency > $O/${c}_${v}_$i.json 2>> $O/err.log || { echo "bench failed"; tail $O/err.log; exit 1; }
      python3 -c "import json;b=json.load(open('$O/${c}_${v}_$i.json'));k=b['kernels'];print('$c $VAR=$v',b['value'],' '.join(f\"{n}:{k[n]['avg_launch_us']}\" for n in ('fwd_ntt','inv_ntt','tensor_inv') if n in k))"
    done
  done
done
