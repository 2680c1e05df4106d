#!/bin/bash
# HBM traffic of the forward NTT (the roofline kernel) inside the real bench, corrected the way
# MI355X_MICROARCH.md's HBM section prescribes and calibrated on a known byte count:
#   cal/   FETCH_SIZE and WRITE_SIZE over tools/ntt_bench.py (16384 polynomials, each forward
#          transform reads and writes exactly 8n bytes per polynomial)
#   fetch/ write/  the same counters over bench.py (one pass each: they do not fit one pass)
# then tools/pmc_traffic.py.  $1 = output directory under gpurun_out, the rest goes to bench.py.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${1:-traffic}; shift || true
cd /tmp && export TMPDIR=/tmp
mkdir -p $OUT
C="python3 $R/tools/ntt_bench.py --polys 16384 --reps 2"
B="python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 $*"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/cal_fetch -o run --output-format csv -- $C > $OUT/cal_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/cal_write -o run --output-format csv -- $C > $OUT/cal_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
python3 $R/tools/pmc_traffic.py $OUT > $OUT/traffic.json
cat $OUT/traffic.json
