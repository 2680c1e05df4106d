#!/bin/bash
# Per-kernel picture of one bench configuration: single-lane steady-state kernel trace, VALU
# counters per kernel, and a chunk-size sweep.  CONFIG (default cfg3), CHUNKS (default "256 512 1024").
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
C=${CONFIG:-cfg3}
O=$R/gpurun_out/prof_$C; mkdir -p $O
cd $R
EXACTO_DUAL_STREAM=0 bash tools/prof_bench.sh prof_$C/trace --config $C --steps 6
python3 tools/trace_steady.py $O/trace/run_kernel_trace.csv > $O/steady.json
(cd /tmp && TMPDIR=/tmp timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/pmc -o run --output-format csv -- python3 $R/bench.py --config $C --no-cpu-baseline --steps 2 --warmup 1 > $O/pmc.log 2>&1)
python3 tools/valu_report.py $O/pmc "$C" > $O/valu.json
for ch in ${CHUNKS:-256 512 1024}; do
  timeout -k 10 200 python3 bench.py --config $C --no-cpu-baseline --chunk $ch > $O/chunk_$ch.json
  echo "chunk $ch $(python3 -c "import json; print(json.load(open('$O/chunk_$ch.json'))['value'])")"
done
python3 tools/prof_report.py $O
