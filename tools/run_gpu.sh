#!/bin/bash
# GPU pass: the -m gpu suite (or the tests PYTEST_K selects), then tools/evidence.sh for each
# configuration named (bench line, kernel-trace summaries with two lanes and one, HBM traffic and VALU
# counters) -> gpurun_out/<name>/ and gpurun_out/<name>_<cfg>/.
# usage: bash tools/run_gpu.sh <name> [configs...]   (PYTEST_K=skip: no tests)
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=${1:-run}; shift
O=$R/gpurun_out/$NAME
mkdir -p $O
cd $R
if [ "$PYTEST_K" != "skip" ]; then
  K=(); [ -n "$PYTEST_K" ] && K=(-k "$PYTEST_K")
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread "${K[@]}" > $O/pytest.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
for c in "$@"; do
  timeout -k 10 900 bash $R/tools/evidence.sh ${NAME}_$c $c > $O/evidence_$c.log 2>&1 || { echo "evidence $c failed"; tail -20 $O/evidence_$c.log; exit 1; }
  echo "evidence $c done"; head -c 300 $R/gpurun_out/${NAME}_$c/bench.json; echo
done
echo done
