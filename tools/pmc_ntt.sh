#!/bin/bash
# PMC passes over tools/ntt_bench.py (separate rocprofv3 runs; no trace domains with --pmc).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${1:-pmc}
cd /tmp && export TMPDIR=/tmp
mkdir -p $OUT
B="python3 $R/tools/ntt_bench.py --reps 3"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/sq -o run --output-format csv -- $B > $OUT/sq.log 2>&1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/lds -o run --output-format csv -- $B > $OUT/lds.log 2>&1
echo done
