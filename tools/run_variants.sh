#!/bin/bash
# A/B the NTT variants built by tools/build_variants.sh (one process per variant).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
mkdir -p $R/gpurun_out
for v in "$@"; do
  echo -n "$v " >> $R/gpurun_out/variants.log
  EXACTO_HIP_LIB=$R/build/variants/$v.so timeout -k 10 120 python3 $R/tools/ntt_bench.py --polys 32768 >> $R/gpurun_out/variants.log
done
