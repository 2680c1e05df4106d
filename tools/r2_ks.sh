#!/bin/bash
# ks32 iteration: parity, single-lane kernel profile, VALU counters, cfg3/cfg5 A/B.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ks; mkdir -p $O
cd $R
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ks32.py > $O/pytest.log 2>&1
EXACTO_DUAL_STREAM=0 bash tools/prof_bench.sh ks/prof --steps 6
python3 tools/trace_steady.py $O/prof/run_kernel_trace.csv > $O/steady.json
(cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS -d $O/pmc -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc.log 2>&1)
for v in 1 0; do
  EXACTO_KS32=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/b3_$v.json
  EXACTO_KS32=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --config cfg5 > $O/b5_$v.json
done
echo ok
