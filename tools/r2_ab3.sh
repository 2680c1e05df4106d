#!/bin/bash
# A/B of one env switch on bench configurations (same box), after the GPU tests that cover it.
# usage: AB_VAR=NAME [AB_TESTS="tests/x.py ..."] [AB_CONFIGS="cfg3 cfg5"] bash tools/r2_ab3.sh
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ab; mkdir -p $O
cd $R
if [ -n "$AB_TESTS" ]; then
  timeout -k 10 300 python3 -u -m pytest $AB_TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for c in ${AB_CONFIGS:-cfg3 cfg5 cfg4}; do
  for rep in 1 2; do
    for v in 0 1; do
      env $AB_VAR=$v timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/${c}_${v}_$rep.json 2>>$O/err.log || exit 1
      python3 -c "import json,sys; d=json.load(open('$O/${c}_${v}_$rep.json')); print('$c $AB_VAR=$v rep$rep', d['value'], d['roofline']['avg_launch_us'])"
    done
  done
done
echo done
