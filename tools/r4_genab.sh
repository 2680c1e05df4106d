#!/bin/bash
# Same-box A/B of the generated generic-prime inverse rounds (EXACTO_NTT_GEN) on u64_dbfv, the
# configuration whose HPS auxiliary primes take them: alternating bench lines, then the variant test.
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-genab}; mkdir -p $O
cd $R
for i in 1 2 3; do
  for g in 1 0; do
    EXACTO_NTT_GEN=$g timeout -k 10 300 python3 bench.py --config u64dbfv --no-cpu-baseline > $O/gen${g}_$i.json 2>> $O/err.log || { echo "bench failed"; tail $O/err.log; exit 1; }
    python3 -c "import json;b=json.load(open('$O/gen${g}_$i.json'));k=b['kernels'];print('gen=$g',b['value'],k['inv_ntt']['avg_launch_us'],k['tensor_inv']['avg_launch_us'])"
  done
done
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_variants.py -q -x --timeout 300 --timeout-method thread -k "gen or switch" > $O/variants.log 2>&1 || { echo "variants failed"; tail -30 $O/variants.log; exit 1; }
tail -1 $O/variants.log
