#!/bin/bash
# Measurement evidence of one bench.py configuration -> gpurun_out/<name>/ (copy what is judged into
# profiles/).  usage: bash tools/evidence.sh <name> <config> [extra bench.py args]
#   bench.json          the bench line (as the driver runs it: dual lane, >= 2 s timed region)
#   prof_dual/          rocprofv3 --kernel-trace --stats of the bench command (two pipeline lanes)
#   prof_single/        ... with EXACTO_DUAL_STREAM=0 (one lane: each kernel alone, as the bench's own
#                       per-kernel events see it in its profiled batches) + steady.json (warm-up dropped)
#   traffic.json        HBM bytes per dispatch of every kernel (FETCH_SIZE / WRITE_SIZE passes,
#                       calibrated on tools/ntt_bench.py), valu.json  VALU issue counters per kernel
# Every PMC pass is its own rocprofv3 run with one counter group and no trace domain.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=${1:-evidence}; CFG=${2:-cfg3}; shift 2 || true
E=$R/gpurun_out/$NAME; mkdir -p $E
cd $R
timeout -k 10 400 python3 bench.py --config $CFG "$@" > $E/bench.json 2> $E/bench.err
cat $E/bench.json
cd /tmp && export TMPDIR=/tmp
# the bench command itself (default steps and timed region, no CPU leg): as the driver runs it
# (two lanes) and with one lane, whose per-kernel averages are what the bench line's profiled
# batches measure (its `roofline.avg_launch_us`); each run prints its own bench line
B="python3 $R/bench.py --config $CFG --no-cpu-baseline $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/prof_dual -o run --output-format csv -- $B > $E/prof_dual.log 2>&1
EXACTO_DUAL_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $E/prof_single -o run --output-format csv -- $B > $E/prof_single.log 2>&1
python3 $R/tools/trace_steady.py $(ls $E/prof_single/*kernel_trace.csv $E/prof_single/*/*kernel_trace.csv 2>/dev/null | head -1) > $E/steady.json
P="python3 $R/bench.py --config $CFG --no-cpu-baseline --no-latency --steps 2 --warmup 1 --reps 1 $*"
C="python3 $R/tools/ntt_bench.py --polys 16384 --reps 2"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $E/cal_fetch -o run --output-format csv -- $C > $E/cal_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $E/cal_write -o run --output-format csv -- $C > $E/cal_write.log 2>&1
EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $E/fetch -o run --output-format csv -- $P > $E/fetch.log 2>&1
EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $E/write -o run --output-format csv -- $P > $E/write.log 2>&1
V1="SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc $V1 -d $E/valu -o run --output-format csv -- $P > $E/valu.log 2>&1
python3 $R/tools/pmc_traffic.py $E > $E/traffic.json
python3 $R/tools/valu_report.py "rocprofv3 --pmc $V1 -- bench.py --config $CFG --steps 2 --warmup 1 --reps 1 (one lane)" $E/valu > $E/valu.json
# keep what comes back under gpurun's 64 MiB: the per-dispatch CSVs are summarised above
find $E -name "*kernel_trace.csv" -size +2M -delete
find $E -name "*counter_collection.csv" -size +2M -exec gzip -f {} \;
echo done
