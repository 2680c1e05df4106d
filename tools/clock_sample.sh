#!/bin/bash
# GPU clock and power sampled (amd-smi, read-only queries) while one bench.py line runs.
# usage: bash tools/clock_sample.sh <name> <config> [bench args]
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-clk}; CFG=${2:-cfg3}; shift 2
mkdir -p $O
cd $R
( for i in $(seq 1 60); do echo "== $(date +%s.%N)"; timeout 5 amd-smi metric -g 0 --clock --power 2>&1 | grep -iE "gfx_0|clk|socket_power|power:|current_socket|GFX" | head -12; sleep 0.5; done ) > $O/smi.log 2>&1 &
S=$!
timeout -k 10 200 python3 bench.py --config $CFG --no-cpu-baseline --min-time 8 "$@" > $O/bench_$CFG.json 2> $O/bench.err
rc=$?
kill $S 2>/dev/null; wait $S 2>/dev/null
cat $O/bench_$CFG.json | cut -c1-200
exit $rc
