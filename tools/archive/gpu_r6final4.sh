set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
cd $R
mkdir -p gpurun_out/r6final4
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r6final4/pytest.log 2>&1
tail -2 gpurun_out/r6final4/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6final4/smoke.log 2>&1
tail -1 gpurun_out/r6final4/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/r6final4/bench.json 2> gpurun_out/r6final4/bench.err
head -c 400 gpurun_out/r6final4/bench.json
PYTEST_K=skip bash tools/run_gpu.sh r6f4 cfg5 cfg4
