#!/bin/bash
# A/B of DESIGN.md §3's intermittent bootstrap result: the C++ host-API test binary (every golden
# case, then the bootstrap case, as the GPU suite runs it) K times per environment variant; prints
# the number of failing runs per variant.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-bootab}; K=${2:-20}
mkdir -p $O/fx
cd $R
python3 - "$O/fx" > $O/names.txt <<'PY' || exit 1
import sys
sys.path.insert(0, "tests")
from test_cpp_api import _write_fixtures
print(" ".join(_write_fixtures(sys.argv[1])))
PY
NAMES=$(cat $O/names.txt)
for V in ${VARIANTS:-"shared:" "own:EXACTO_SCRATCH_POOL=own" "defpool:EXACTO_SCRATCH_POOL=default" "sharedleak:EXACTO_LEAK_CTX=1"}; do
  tag=${V%%:*}; envs=${V#*:}
  fails=0
  for i in $(seq 1 $K); do
    env $envs timeout -k 10 60 ./build/test_api $O/fx $NAMES > $O/$tag.$i.log 2>&1
    rc=$?
    [ $rc -ne 0 ] && fails=$((fails+1))
    [ $rc -gt 1 ] && { echo "$tag run $i rc=$rc: stopping"; tail -5 $O/$tag.$i.log; exit 1; }
    grep -h "FAIL" $O/$tag.$i.log | head -3
  done
  echo "variant $tag: $fails of $K runs failed"
done
