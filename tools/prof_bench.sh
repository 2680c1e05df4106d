#!/bin/bash
# rocprofv3 kernel-trace summary of one bench.py configuration -> gpurun_out/<name>/
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=${1:-prof}; shift
mkdir -p $(dirname $R/gpurun_out/$NAME)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$NAME -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline "$@" > $R/gpurun_out/$NAME.log 2>&1
