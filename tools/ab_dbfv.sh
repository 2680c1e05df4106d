#!/bin/bash
# Same-box A/B: (1) the NTT parity tests and tools/ntt_bench.py with the current library and with
# build/ab/noaddx.so (forward butterflies without the addend form); (2) the dBFV bench lines
# of the current tree (default timed region, and one batch per step as round 2 timed it) against
# the round-2 tree (build/r2tree: its bench.py + library) and the device's default scratch pool.
# usage: bash tools/ab_dbfv.sh <name> [configs]
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-ab}; shift
mkdir -p $O
cd $R
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ntt.py \
  tests/test_gpu_ntt_pipe.py tests/test_gpu_ntt_asm_inv.py tests/test_gpu_bfv.py > $O/pytest.log 2>&1
rc=$?; echo "ntt tests rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
for n in 4096 8192; do
  for v in cur noaddx; do
    L=""; [ $v = noaddx ] && L=$R/build/ab/noaddx.so
    EXACTO_HIP_LIB=$L timeout -k 10 120 python3 tools/ntt_bench.py --n $n --polys $((134217728 / n / 8 * 2)) --reps 10 > $O/ntt_${v}_$n.txt 2>&1 || exit 1
    echo "$v n=$n: $(tr '\n' ' ' < $O/ntt_${v}_$n.txt | cut -c1-300)"
  done
done
for c in ${@:-cfg4 cfg5}; do
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/cur_$c.json 2>> $O/err.log || exit 1
  timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --reps 1 --steps 20 > $O/cur_short_$c.json 2>> $O/err.log || exit 1
  (cd build/r2tree && timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline --steps 20 > $O/r2_$c.json 2>> $O/err.log) || exit 1
  EXACTO_SCRATCH_POOL=default timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/curpool_$c.json 2>> $O/err.log || exit 1
  EXACTO_HIP_LIB=$R/build/ab/noaddx.so timeout -k 10 200 python3 bench.py --config $c --no-cpu-baseline > $O/noaddx_$c.json 2>> $O/err.log || exit 1
  for f in cur cur_short r2 curpool noaddx; do
    python3 -c "import json,sys; d=json.load(open('$O/${f}_$c.json')); print('$f $c', d['value'], d['ms_per_step'], d.get('timed_s'))"
  done
done
echo done
