#!/bin/bash
# Round-4 GPU pass: the bootstrap regression tests, the NTT compute-only probes (build/ntt_probe,
# tools/ntt_probe.hip), then tools/evidence.sh for the configs named.  usage: bash tools/r4_probe.sh cfg5 ...
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/r4p
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bootstrap.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/r4p/pytest_boot.log 2>&1 || { echo "boot tests failed"; tail -30 gpurun_out/r4p/pytest_boot.log; exit 1; }
tail -2 gpurun_out/r4p/pytest_boot.log
timeout -k 10 120 build/ntt_probe 20 > gpurun_out/r4p/ntt_probe.json 2>&1 || { echo "probe failed"; cat gpurun_out/r4p/ntt_probe.json; exit 1; }
cat gpurun_out/r4p/ntt_probe.json
(cd /tmp && TMPDIR=/tmp timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r4p/probe_prof -o run --output-format csv -- $R/build/ntt_probe 20 > $R/gpurun_out/r4p/probe_prof.log 2>&1) || { echo "probe prof failed"; exit 1; }
(cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $R/gpurun_out/r4p/probe_pmc -o run --output-format csv -- $R/build/ntt_probe 3 > $R/gpurun_out/r4p/probe_pmc.log 2>&1) || { echo "probe pmc failed"; exit 1; }
[ $# -gt 0 ] && LIST=1 bash tools/r4_evidence.sh "$@"
echo r4_probe done
