#!/bin/bash
# VALU busy from the hardware counters, calibrated: the same counter pass over tools/op_rate.hip
# (kernels that only issue one VALU instruction in 8 independent chains: the issue-saturated
# reference) and over tools/ntt_probe.hip (the library's NTT kernels, full and compute-only forms),
# then the n = 8192 stagger sweep of ntt_probe without the profiler.  -> gpurun_out/<name>/
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-valubusy}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
C="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/op -o run --output-format csv -- $R/build/op_rate 2.4 > $O/op.log 2>&1 || { echo "op pass failed"; tail $O/op.log; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc $C -d $O/ntt -o run --output-format csv -- $R/build/ntt_probe 3 > $O/ntt.log 2>&1 || { echo "ntt pass failed"; tail $O/ntt.log; exit 1; }
python3 $R/tools/valu_report.py "op_rate" $O/op > $O/op.json && python3 $R/tools/valu_report.py "ntt_probe" $O/ntt > $O/ntt.json || exit 1
timeout -k 10 120 $R/build/ntt_probe 10 > $O/probe.json 2>&1 || { echo "probe failed"; cat $O/probe.json; exit 1; }
cat $O/probe.json
find $O -name "*counter_collection.csv" -size +2M -delete
echo valubusy done
