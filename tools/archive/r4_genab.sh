#!/bin/bash
# Same-box A/B of the generated generic-prime NTT rounds (EXACTO_NTT_GEN) on the configurations whose
# HPS primes take them: the GPU suite first, alternating bench lines, then the variant test.
# usage: bash tools/r4_genab.sh <name> cfg...
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=${1:-genab}; shift
O=$R/gpurun_out/$NAME; mkdir -p $O
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "suite failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in "$@"; do
  for i in 1 2 3; do
    for g in 1 0; do
      EXACTO_NTT_GEN=$g timeout -k 10 300 python3 bench.py --config $c --no-cpu-baseline > $O/${c}_gen${g}_$i.json 2>> $O/err.log || { echo "bench failed"; tail $O/err.log; exit 1; }
      python3 -c "import json;b=json.load(open('$O/${c}_gen${g}_$i.json'));k=b['kernels'];print('$c gen=$g',b['value'],' '.join(f\"{n}:{k[n]['avg_launch_us']}\" for n in ('fwd_ntt','inv_ntt','tensor_inv') if n in k))"
    done
  done
done
