set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="variants and (fpq or fp_crt or covered) or golden or bench_shape or psum or chain or worstcase or bfv" bash tools/run_gpu.sh r6q
bash tools/ab_env.sh r6fpq "- EXACTO_FPQ=0" cfg3 cfg5 cfg4
