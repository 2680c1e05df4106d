#!/bin/bash
# Clock + duration of the standalone forward NTT: default build, per-polynomial kernel, and the
# persistent kernel's compute-only (p1) / memory-only (p2) probe builds.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/probe_clock.sh pipe
EXACTO_NTT_PIPE=0 bash tools/probe_clock.sh nopipe
bash tools/probe_clock.sh p1 $R/build/variants/pipe_p1.so
bash tools/probe_clock.sh p2 $R/build/variants/pipe_p2.so
python3 tools/clock_report.py gpurun_out > gpurun_out/clock_report.txt
cat gpurun_out/clock_report.txt
