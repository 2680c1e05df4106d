#!/bin/bash
# tools/ntt_bench.py (fwd / inv / pointwise, n = 4096 and 8192) with the in-tree library and with
# build/ab/<variant>.so, alternating.  usage: bash tools/ab_ntt.sh <name> "<variants>"
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-abntt}; VARS=${2:-}
mkdir -p $O
cd $R
for rep in 1 2; do
  for n in 4096 8192; do
    for v in cur $VARS; do
      L=""; [ $v != cur ] && L=$R/build/ab/$v.so
      EXACTO_HIP_LIB=$L timeout -k 10 120 python3 tools/ntt_bench.py --n $n --polys $((268435456 / n / 8)) --reps 10 > $O/ntt_${v}_${n}_$rep.txt 2>&1 || exit 1
      echo "$v n=$n: $(grep polys $O/ntt_${v}_${n}_$rep.txt)"
    done
  done
done
