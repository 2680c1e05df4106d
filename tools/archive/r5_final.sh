#!/bin/bash
# Round-5 final pass: the -m gpu suite, the NTT probes (build/ntt_probe: full / compute-only /
# memory-only forms of the library's transform and tensor kernels, with their VALU counters), then
# tools/evidence.sh for each configuration named.  usage: bash tools/r5_final.sh <name> [configs...]
# (PYTEST_K=skip: no tests; PROBE=0: no probes)
R=${GRAFT_REPO_ROOT:-/root/repo}
NAME=${1:-r5final}; shift
O=$R/gpurun_out/$NAME
mkdir -p $O
cd $R
if [ "$PYTEST_K" != "skip" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; echo "gpu suite rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
fi
if [ "$PROBE" != "0" ]; then
  timeout -k 10 120 build/ntt_probe 20 > $O/ntt_probe.json 2> $O/ntt_probe.err || { echo "probe failed"; tail -5 $O/ntt_probe.err; exit 1; }
  cat $O/ntt_probe.json
  (cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $O/probe_pmc -o run --output-format csv -- $R/build/ntt_probe 3 > $O/probe_pmc.log 2>&1) || { echo "probe pmc failed"; exit 1; }
  python3 tools/valu_report.py "build/ntt_probe 3 ($NAME)" $O/probe_pmc > $O/probe_valu.json || exit 1
fi
for c in "$@"; do
  timeout -k 10 900 bash $R/tools/evidence.sh ${NAME}_$c $c > $O/evidence_$c.log 2>&1 || { echo "evidence $c failed"; tail -20 $O/evidence_$c.log; exit 1; }
  echo "evidence $c done"; head -c 300 $R/gpurun_out/${NAME}_$c/bench.json; echo
done
echo done
