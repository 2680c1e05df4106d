set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="variants and (fpq or fp_crt or psum or covered) or golden or bench_shape or psum or chain or worstcase" bash tools/run_gpu.sh r6p
bash tools/ab_lib.sh r6pdef "prev" cfg5 cfg4
