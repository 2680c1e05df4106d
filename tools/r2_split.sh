#!/bin/bash
# Single-lane kernel traces of bench configurations -> steady-state per-kernel split.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
E=$R/gpurun_out/split; mkdir -p $E
for c in ${SPLIT_CONFIGS:-cfg5 cfg4 cfg3}; do
  EXACTO_DUAL_STREAM=0 bash $R/tools/prof_bench.sh split/prof_$c --config $c --steps 6
  python3 $R/tools/trace_steady.py $E/prof_$c/run_kernel_trace.csv > $E/steady_$c.json
  cp $E/prof_$c/run_kernel_stats.csv $E/stats_$c.csv
done
echo done
