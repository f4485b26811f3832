#!/bin/bash
# Round-4 run 4: the full GPU suite with the column-stationary headline kernel
# as the default and the pipelined Lanczos walk; kbench A/B against the gather
# kernel (lib_gather); bench lines.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
K=arm-neon-opencv_amd
step tests
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/d_gpu_tests.log 2>&1 || { tail -30 gpurun_out/d_gpu_tests.log; exit 1; }
tail -2 gpurun_out/d_gpu_tests.log
step kbench
timeout -k 10 300 python3 tools/kbench.py --op lanczos --iters 20 | tee gpurun_out/d_kbench.jsonl || exit 1
for rep in 1 2; do
  for l in lib lib_gather; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize_normalize --iters 30 | sed "s/^/$l /" || exit 1
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize --only 640x360 --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/d_variants.txt
step bench
for w in 5 5 50; do
  timeout -k 10 300 python3 bench.py --warmup $w --steps 20 --no-cpu-baseline | tee -a gpurun_out/d_bench.jsonl || exit 1
done
timeout -k 10 300 python3 bench.py --workload cubic_stats --warmup 5 --steps 20 --no-cpu-baseline | tee -a gpurun_out/d_bench.jsonl || exit 1
step done
