#!/bin/bash
# Round-2 evidence for the cfg3 bench: HBM traffic of the forward NTT (calibrated), its VALU
# issue counters, and kernel-trace summaries (dual lane as timed, single lane per kernel).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
E=$R/gpurun_out/ev2; mkdir -p $E
bash $R/tools/pmc_traffic.sh ev2/traffic_cfg3
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $E/valu -o run \
  --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $E/valu.log 2>&1
bash $R/tools/prof_bench.sh ev2/prof_cfg3 --steps 10
EXACTO_DUAL_STREAM=0 bash $R/tools/prof_bench.sh ev2/prof_cfg3_single --steps 6
python3 $R/tools/trace_steady.py $E/prof_cfg3_single/run_kernel_trace.csv > $E/steady_single.json
python3 $R/tools/valu_report.py $E/valu "rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -- bench.py --steps 2 --warmup 1 (cfg3)" > $E/valu_counters.json
cd $R
for c in ${BENCH_CONFIGS:-cfg2 cfg3 cfg4 cfg5 galois}; do
  timeout -k 10 400 python3 bench.py --config $c > $E/bench_$c.json 2>> $E/bench_err.log
  cat $E/bench_$c.json
done
echo done
