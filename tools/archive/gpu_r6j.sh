set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="bench_shape or ks32 or variants or worstcase or psum or golden" bash tools/run_gpu.sh r6j
bash tools/ab_lib.sh r6kn "kn0" cfg4 cfg5
