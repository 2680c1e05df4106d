set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="bench_shape or ks32 or worstcase or galois" bash tools/run_gpu.sh r6rp
bash tools/ab_lib.sh r6rpre "rpre0" cfg3 cfg4
