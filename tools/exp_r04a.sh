#!/bin/bash
# Round-4 experiment run 1 (through gpurun from the repo root): GPU suite,
# the driver's bench command vs a longer warm-up, and kernel variants
# (tools/variants.sh builds): headline diagnosis / cache policies, warp ring
# diagnosis / policies, strip store policy; the new Lanczos kernel and cfg5.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
step tests
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/a_gpu_tests.log 2>&1 || { tail -30 gpurun_out/a_gpu_tests.log; exit 1; }
tail -2 gpurun_out/a_gpu_tests.log
step bench
for w in 5 50 5; do
  timeout -k 10 300 python3 bench.py --warmup $w --steps 20 --no-cpu-baseline > gpurun_out/a_bench_w$w.json || exit 1
  cat gpurun_out/a_bench_w$w.json
done
timeout -k 10 300 python3 bench.py --workload cubic_stats --warmup 5 --steps 20 --no-cpu-baseline | tee gpurun_out/a_bench_cubic.json || exit 1
step kbench_new
timeout -k 10 300 python3 tools/kbench.py --op lanczos --iters 20 | tee gpurun_out/a_kbench_new.jsonl || exit 1
timeout -k 10 300 python3 tools/kbench.py --op cvt_cv --iters 20 | tee -a gpurun_out/a_kbench_new.jsonl || exit 1
step variants
K=arm-neon-opencv_amd
for rep in 1 2; do
  for l in lib lib_nf lib_d1 lib_d3 lib_d4 lib_s0 lib_s1 lib_s16 lib_s18 lib_l16; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize_normalize --iters 30 | sed "s/^/$l /" || exit 1
  done
  for l in lib lib_wd1 lib_wd2 lib_wd4 lib_ws0 lib_wl0 lib_wl2; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op warp --only rot15 --iters 30 | sed "s/^/$l /" || exit 1
  done
  for l in lib lib_ts0 lib_ts1; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize --only 1280 --iters 30 | sed "s/^/$l /" || exit 1
  done
done | tee gpurun_out/a_variants.txt
step done
