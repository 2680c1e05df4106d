#!/bin/bash
# Parity first (new inverse + NTT + BFV suites), then A/B of env switches on the standalone NTT
# and the cfg3 bench.  $@: env assignments to A/B against the default (e.g. EXACTO_NTT_ASM_INV=0).
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/ab; mkdir -p $O
cd $R
stop() { [ $1 -ge 124 ] && { echo "step rc=$1: stopping"; exit $1; }; return 0; }
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ntt_asm_inv.py \
  tests/test_gpu_ntt.py tests/test_gpu_ntt_pipe.py tests/test_gpu_bfv.py > $O/pytest.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 $O/pytest.log; stop $rc; [ $rc -ne 0 ] && exit $rc
for v in default "$@"; do
  e=""; [ "$v" != default ] && e="$v"
  env $e timeout -k 10 120 python3 tools/ntt_bench.py --polys 32768 --reps 10 > $O/ntt_$v.json 2>>$O/err.log; stop $?
  env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline > $O/bench_$v.json 2>>$O/err.log; stop $?
  echo "== $v"; cat $O/ntt_$v.json; python3 -c "import json,sys; d=json.load(open('$O/bench_$v.json')); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
exit 0
