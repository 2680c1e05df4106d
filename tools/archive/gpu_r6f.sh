set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
PYTEST_K="variants or chain or bench_shape or psum" bash tools/run_gpu.sh r6f
EXACTO_LANE_STAGGER=4 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bench_shapes.py -m gpu -v -x --timeout 300 -k "cfg3_bench or cfg4_bench" > gpurun_out/r6f/stagger_pytest.log 2>&1
tail -2 gpurun_out/r6f/stagger_pytest.log
bash tools/ab_env.sh r6stag "- EXACTO_LANE_STAGGER=4 EXACTO_LANE_STAGGER=3" cfg3
bash tools/ab_env.sh r6split3 "- EXACTO_CHAIN_SPLIT=3 EXACTO_CHAIN_SPLIT=4" cfg5 cfg4 u64dbfv
