#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/r3base; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --config cfg3 --steps 20 --warmup 5 > $O/bench_cfg3.json 2> $O/bench_err.log || exit 1
cat $O/bench_cfg3.json
