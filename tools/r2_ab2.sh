#!/bin/bash
# Full GPU suite, then same-box A/B of env switches on bench configurations.
#   $@: env assignments to compare against the default (e.g. EXACTO_DOT30=0)
#   CONFIGS: bench configurations (default "cfg3 cfg5"); SUITE=0 skips the test suite.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ab2; mkdir -p $O
cd $R
stop() { [ $1 -ge 124 ] && { echo "step rc=$1: stopping"; exit $1; }; return 0; }
if [ "${SUITE:-1}" != 0 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > $O/pytest.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 $O/pytest.log; stop $rc; [ $rc -ne 0 ] && exit $rc
fi
for c in ${CONFIGS:-cfg3 cfg5}; do
  for rep in 1 2; do
    for v in default "$@"; do
      e=""; [ "$v" != default ] && e="$v"
      env $e timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/b_${c}_${v}_$rep.json 2>>$O/err.log; stop $?
      echo "$c $v rep$rep $(python3 -c "import json; d=json.load(open('$O/b_${c}_${v}_$rep.json')); print(d['value'], d['ms_per_step'])")"
    done
  done
done
exit 0
