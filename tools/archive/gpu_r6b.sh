set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="variants or psum or golden or bench_shape and not cfg4_bench and not cfg5_bench or prof or bfv or ks32 or worstcase" bash tools/run_gpu.sh r6b
bash tools/ab_env.sh r6fpc "- EXACTO_FP_CRT=0" cfg3 cfg5 cfg4
bash tools/ab_lib.sh r6sh3 "sh3" cfg4
mkdir -p gpurun_out/r6c5
cd /tmp && export TMPDIR=/tmp
EXACTO_DUAL_STREAM=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r6c5 -o trace -- python3 $R/bench.py --config cfg5 --steps 2 --warmup 1 --reps 1 --no-cpu-baseline --no-latency > $R/gpurun_out/r6c5/bench.log 2>&1
echo trace done
