set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="psum or chain or golden or variants or split or bench_shape and not cfg4_bench and not cfg5_bench" bash tools/run_gpu.sh r6c
bash tools/ab_env.sh r6fork "- EXACTO_PSUM_FORK=0" cfg5 cfg4
