set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
bash tools/ab_lib.sh r6stag "stag" cfg3 cfg5 galois
