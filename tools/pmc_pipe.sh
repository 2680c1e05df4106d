#!/bin/bash
# PMC pass over the standalone forward NTT (tools/ntt_bench.py) for one library build:
# clock (GRBM_GUI_ACTIVE) and SQ issue / wait counters.  $1 = output name, $2 = library .so (optional)
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$2" ] && export EXACTO_HIP_LIB=$2
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU \
  -d $OUT -o run --output-format csv -- python3 $R/tools/ntt_bench.py --polys 32768 --reps 2 > $OUT/log 2>&1
