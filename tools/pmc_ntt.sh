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
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS -d $OUT/lds -o run --output-format csv -- $B > $OUT/lds.log 2>&1
timeout -k 10 200 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCC_HIT_sum TCC_MISS_sum -d $OUT/ta -o run --output-format csv -- $B > $OUT/ta.log 2>&1 || echo "ta pass failed"
timeout -k 10 200 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA -d $OUT/sq2 -o run --output-format csv -- $B > $OUT/sq2.log 2>&1 || echo "sq2 pass failed"
echo done
