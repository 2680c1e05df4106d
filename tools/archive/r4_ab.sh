#!/bin/bash
# Round-4 quick pass: GPU suite, NTT probes, bench lines of the configs named, and the cfg5 tensor's
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) -> gpurun_out/<name>/.  usage: bash tools/r4_ab.sh <name> cfg...
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=$1; shift
O=$R/gpurun_out/$NAME; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "suite failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 build/ntt_probe 20 > $O/ntt_probe.json 2>&1 || { echo "probe failed"; cat $O/ntt_probe.json; exit 1; }
cat $O/ntt_probe.json
for c in "$@"; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench_err.log || { echo "bench $c failed"; tail $O/bench_err.log; exit 1; }
  python3 -c "import json;b=json.load(open('$O/bench_$c.json'));r=b['roofline'];print('$c',b['value'],r['kernel'],r['avg_launch_us'],r['frac'])"
done
cd /tmp && export TMPDIR=/tmp
P="python3 $R/bench.py --config cfg5 --no-cpu-baseline --steps 2 --warmup 1 --reps 1"
EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- $P > $O/fetch.log 2>&1 || { echo fetch failed; exit 1; }
EXACTO_DUAL_STREAM=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- $P > $O/write.log 2>&1 || { echo write failed; exit 1; }
python3 $R/tools/pmc_traffic.py $O > $O/traffic.json
echo ab done
