#!/bin/bash
# Round-4 experiment run 3: Lanczos with rows in flight; the column-stationary
# headline kernel (lib_cols): parity through the resize tests, then A/B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "=== $1 $(date +%T)"; }
K=arm-neon-opencv_amd
step tests_default
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lanczos or resize" \
    > gpurun_out/c_tests.log 2>&1 || { tail -30 gpurun_out/c_tests.log; exit 1; }
tail -2 gpurun_out/c_tests.log
step tests_cols
VACV_LIB_DIR=$K/lib_cols timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "resize_linear or resize_normalize or resize_full or u8_kernels_agree or channel_sums" \
    > gpurun_out/c_tests_cols.log 2>&1 || { tail -30 gpurun_out/c_tests_cols.log; exit 1; }
tail -2 gpurun_out/c_tests_cols.log
step kbench
timeout -k 10 300 python3 tools/kbench.py --op lanczos --iters 20 | tee gpurun_out/c_kbench.jsonl || exit 1
for rep in 1 2 3; do
  for l in lib lib_cols lib_d3; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize_normalize --iters 30 | sed "s/^/$l /" || exit 1
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize --only 640x360 --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/c_variants.txt
step bench_cols
VACV_LIB_DIR=$K/lib_cols timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline | tee gpurun_out/c_bench_cols.json || exit 1
timeout -k 10 300 python3 bench.py --warmup 5 --steps 20 --no-cpu-baseline | tee gpurun_out/c_bench.json || exit 1
step done
