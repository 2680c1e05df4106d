set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="variants and (psum or fpq or covered) or golden or bench_shape or psum or chain or worstcase or dbfv" bash tools/run_gpu.sh r6ps
bash tools/ab_lib.sh r6psab "pd0" cfg5 cfg4
