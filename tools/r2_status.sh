#!/bin/bash
# Status pass: GPU test suite, cfg3 bench with the persistent forward NTT on and off, standalone NTT.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/status; mkdir -p $O
cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 120 python3 tools/ntt_bench.py --polys 32768 --reps 10 > $O/ntt_pipe.json 2>$O/ntt.err
EXACTO_NTT_PIPE=0 timeout -k 10 120 python3 tools/ntt_bench.py --polys 32768 --reps 10 > $O/ntt_nopipe.json 2>>$O/ntt.err
timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_pipe.json 2>$O/bench.err
EXACTO_NTT_PIPE=0 timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_nopipe.json 2>>$O/bench.err
echo done
