#!/bin/bash
# PMC passes only (tools/evidence.sh's counter part) for the configurations named: FETCH_SIZE and
# WRITE_SIZE (HBM bytes per dispatch, calibrated once on tools/ntt_bench.py) and the VALU issue
# counters, each its own rocprofv3 run over bench.py --no-latency -> gpurun_out/<name>_<cfg>/
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=${1:-r4pmc}; shift
cd /tmp && export TMPDIR=/tmp
C="python3 $R/tools/ntt_bench.py --polys 16384 --reps 2"
V1="SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for CFG in ${@:-cfg3 cfg1 u64dbfv cfg5}; do
  E=$R/gpurun_out/${NAME}_$CFG; mkdir -p $E
  P="python3 $R/bench.py --config $CFG --no-cpu-baseline --no-latency --steps 2 --warmup 1 --reps 1"
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $E/cal_fetch -o run --output-format csv -- $C > $E/cal_fetch.log 2>&1 || { echo "cal fetch failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $E/cal_write -o run --output-format csv -- $C > $E/cal_write.log 2>&1 || { echo "cal write failed"; exit 1; }
  EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $E/fetch -o run --output-format csv -- $P > $E/fetch.log 2>&1 || { echo "$CFG fetch failed"; tail $E/fetch.log; exit 1; }
  EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $E/write -o run --output-format csv -- $P > $E/write.log 2>&1 || { echo "$CFG write failed"; tail $E/write.log; exit 1; }
  EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc $V1 -d $E/valu -o run --output-format csv -- $P > $E/valu.log 2>&1 || { echo "$CFG valu failed"; tail $E/valu.log; exit 1; }
  python3 $R/tools/pmc_traffic.py $E > $E/traffic.json
  python3 $R/tools/valu_report.py "rocprofv3 --pmc $V1 -- bench.py --config $CFG --no-latency --steps 2 --warmup 1 --reps 1 (one lane)" $E/valu > $E/valu.json
  find $E -name "*counter_collection.csv" -size +2M -exec gzip -f {} \;
  echo "pmc $CFG done"
done
