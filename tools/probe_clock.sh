#!/bin/bash
# Kernel-trace durations and the PMC clock/issue counters of the standalone NTT bench for one
# library build.  $1 = output name, $2 = library .so (optional; default in-tree build)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/clk_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$2" ] && export EXACTO_HIP_LIB=$2
B="python3 $R/tools/ntt_bench.py --polys 32768 --reps 4"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/kt -o run --output-format csv -- $B > $OUT/kt.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU \
  -d $OUT/pmc -o run --output-format csv -- $B > $OUT/pmc.log 2>&1
