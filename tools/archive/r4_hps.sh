#!/bin/bash
# HPS-path check: the GPU tests of the HPS configurations (and every variant), then two bench lines
# each of compact_bfv and u64_dbfv -> gpurun_out/<name>/
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-hps}; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -k "hps or compact or u64 or variant or golden or published" > $O/pytest.log 2>&1 || { echo "tests failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for c in cfg1 u64dbfv; do
    timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/${c}_$i.json 2>> $O/err.log || { echo "bench failed"; tail $O/err.log; exit 1; }
    python3 -c "import json;b=json.load(open('$O/${c}_$i.json'));k=b['kernels'];print('$c',b['value'],' '.join(f\"{n}:{k[n]['avg_launch_us']}\" for n in k))"
  done
done
