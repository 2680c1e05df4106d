set -e
mkdir -p gpurun_out
rm -f gpurun_out/sweep.log
for c in 512 1024; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --chunk $c --steps 10 >> gpurun_out/sweep.log 2>&1
done
for c in 1024 2048; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --batch 4096 --chunk $c --steps 5 >> gpurun_out/sweep.log 2>&1
done
