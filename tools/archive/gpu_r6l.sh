set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/ab_env.sh r6lanes "- EXACTO_LANES=1 EXACTO_LANES=3" cfg5 cfg4
