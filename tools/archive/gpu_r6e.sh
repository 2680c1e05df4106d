set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="variants or bench_shape or psum or chain or dbfv" bash tools/run_gpu.sh r6e
bash tools/ab_env.sh r6split2 "- EXACTO_CHAIN_SPLIT=0" cfg4 u64dbfv
