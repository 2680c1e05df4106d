#!/bin/bash
# Round-4 evidence pass: tools/evidence.sh for each config named (bench line, dual / single-lane
# kernel summaries, HBM traffic and VALU counters) -> gpurun_out/r4_<config>/.  Stops at the first
# failing step.  usage: bash tools/r4_evidence.sh cfg1 u64dbfv ...   (LIST=1: also the counter list)
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
if [ "$LIST" = "1" ]; then
  mkdir -p gpurun_out
  (cd /tmp && TMPDIR=/tmp timeout -k 10 60 rocprofv3 -L > $R/gpurun_out/rocprofv3_counters.txt 2>&1) || echo "counter list rc=$?"
fi
for c in "$@"; do
  timeout -k 10 900 bash tools/evidence.sh r4_$c $c > gpurun_out/r4_$c.evidence.log 2>&1 || { echo "evidence $c failed"; tail -20 gpurun_out/r4_$c.evidence.log; exit 1; }
  head -c 600 gpurun_out/r4_$c/bench.json; echo
done
echo evidence done
