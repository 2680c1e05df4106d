#!/bin/bash
# HBM traffic of the roofline kernel inside the real bench: FETCH_SIZE and WRITE_SIZE in separate
# rocprofv3 passes (they do not fit one pass on gfx950), then tools/pmc_traffic.py.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${1:-traffic}; shift || true
cd /tmp && export TMPDIR=/tmp
mkdir -p $OUT
B="python3 $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 $*"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
python3 $R/tools/pmc_traffic.py $OUT > $OUT/traffic.json
