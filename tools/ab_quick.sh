#!/bin/bash
# A/B gate: the given pytest files (must pass), then tools/ab_lib.sh over the configs.
# usage: bash tools/ab_quick.sh <name> "<tests>" "<variants>" [configs]
R=${GRAFT_REPO_ROOT:-/root/repo}
N=$1; TESTS=$2; VARS=$3; shift 3
mkdir -p $R/gpurun_out/$N
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS > $R/gpurun_out/$N/pytest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $R/gpurun_out/$N/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/ab_lib.sh $N "$VARS" "$@"
