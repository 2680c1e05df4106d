#!/bin/bash
# Round evidence: bench lines for every config, rocprofv3 kernel summary and HBM traffic PMC
# of the default (cfg3) bench.  Everything lands in gpurun_out/evidence/.
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
E=$R/gpurun_out/evidence; mkdir -p $E
cd $R
timeout -k 10 300 python3 bench.py > $E/bench_cfg3.json 2> $E/bench_cfg3.err
for c in cfg2 cfg4 cfg5; do
  timeout -k 10 300 python3 bench.py --config $c > $E/bench_$c.json 2> $E/bench_$c.err
done
tools/prof_bench.sh evidence/prof_cfg3 --steps 10
bash tools/pmc_traffic.sh evidence/traffic_cfg3
echo done
