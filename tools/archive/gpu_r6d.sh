set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="chain or golden or variants or psum or split or bench_shape" bash tools/run_gpu.sh r6d
bash tools/ab_env.sh r6split "- EXACTO_CHAIN_SPLIT=0" cfg5
