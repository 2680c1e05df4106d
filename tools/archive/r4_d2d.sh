#!/bin/bash
# The same-stream device-to-device copy question of DESIGN.md §3 in one run (tools/d2d_repro.cpp):
# the reproducer as is, with SDMA engines off (every copy a blit kernel), and under a rocprofv3
# kernel + memory-copy trace that shows which engine each hipMemcpyAsync took; then the scalar-cache
# reproducer (tools/kcache_repro.cpp).
# usage: bash tools/r4_d2d.sh <outdir-name> [iterations]
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-d2d}; IT=${2:-20000}
mkdir -p $O
cd $R
timeout -k 10 120 build/d2d_repro $IT > $O/d2d_default.txt 2>&1 || { echo "d2d default rc=$?"; cat $O/d2d_default.txt; exit 1; }
cat $O/d2d_default.txt
HSA_ENABLE_SDMA=0 timeout -k 10 120 build/d2d_repro $IT > $O/d2d_nosdma.txt 2>&1 || { echo "d2d nosdma rc=$?"; exit 1; }
cat $O/d2d_nosdma.txt
timeout -k 10 120 build/kcache_repro $IT > $O/kcache.txt 2>&1 || { echo "kcache rc=$?"; cat $O/kcache.txt; exit 1; }
cat $O/kcache.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/trace -o run --output-format csv -- $R/build/d2d_repro 300 > $O/trace.log 2>&1 || { echo "trace rc=$?"; tail $O/trace.log; exit 1; }
echo d2d done
