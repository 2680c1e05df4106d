#!/bin/bash
R=${GRAFT_REPO_ROOT:-/root/repo}; O=$R/gpurun_out/sweep5; mkdir -p $O; cd $R
for a in "--batch 1024" "--batch 2048" "--batch 4096" "--batch 1024 --chunk 256" "--batch 1024" "--batch 2048"; do
  tag=$(echo $a | tr ' -' '__')
  timeout -k 10 200 python3 bench.py --config cfg3 --no-cpu-baseline --no-latency --min-time 1.5 $a > $O/$tag.json 2>> $O/err.log || exit 1
  python3 -c "import json,sys; d=json.load(open('$O/$tag.json')); print('$a', d['value'])"
done
