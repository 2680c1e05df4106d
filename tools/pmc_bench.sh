#!/bin/bash
# PMC passes (one counter group per rocprofv3 run; no trace domains) over a short bench.py run.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${1:-pmcb}; shift || true
cd /tmp && export TMPDIR=/tmp
mkdir -p $OUT
B="python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 $*"
run() {  # name counters...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/$name -o run --output-format csv -- $B > $OUT/$name.log 2>&1
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE
run fetch FETCH_SIZE
run write WRITE_SIZE
run mem SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum
echo done
