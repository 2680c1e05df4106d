#!/bin/bash
# Round-4 final pass, part 1: the whole -m gpu suite, then every configuration's bench line as the
# driver runs it (CPU leg included) -> gpurun_out/<name>/
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-r4final}; shift
mkdir -p $O
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for c in ${@:-cfg3 cfg1 u64dbfv cfg2 cfg4 cfg5 galois}; do
  timeout -k 10 400 python3 bench.py --config $c > $O/bench_$c.json 2>> $O/bench_err.log || { echo "bench $c failed"; tail -20 $O/bench_err.log; exit 1; }
  python3 -c "import json;b=json.load(open('$O/bench_$c.json'));r=b['roofline'];cb=b.get('cpu_baseline') or {};print('$c',b['value'],b['unit'],r['kernel'],r['frac'],cb.get('value'),cb.get('unit'))"
done
echo done
