#!/bin/bash
# SQ counters of the standalone forward NTT, hand-scheduled (EXACTO_NTT_ASM=1) vs compiler (0).
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/${1:-pmc_ab}
cd /tmp && export TMPDIR=/tmp
mkdir -p $OUT
for a in 1 0; do
  export EXACTO_NTT_ASM=$a
  B="python3 $R/tools/ntt_bench.py --reps 3 --polys 8192"
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d $OUT/sq_$a -o run --output-format csv -- $B > $OUT/sq_$a.log 2>&1
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d $OUT/sq2_$a -o run --output-format csv -- $B > $OUT/sq2_$a.log 2>&1
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for a in ("1", "0"):
    agg = collections.defaultdict(float); n = collections.Counter()
    for d in ("sq_" + a, "sq2_" + a):
        for f in glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "ntt_fwd" not in r["Kernel_Name"]: continue
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                n[r["Counter_Name"]] += 1
    print("asm=" + a, {k: round(v / max(n[k], 1)) for k, v in sorted(agg.items())})
PY
