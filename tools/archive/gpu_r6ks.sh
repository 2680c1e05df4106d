set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="variants and (ks_fpc or covered) or golden or bench_shape or ks32 or worstcase or galois or psum or chain" bash tools/run_gpu.sh r6ks
bash tools/ab_env.sh r6ksfpc "- EXACTO_KS_FPC=0" cfg3 cfg5 cfg4
