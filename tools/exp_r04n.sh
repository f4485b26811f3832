#!/bin/bash
# Round-4 run 14: uniform (per task) range check in the column gather kernels
# (resize_cols, cubic_cols) vs the per-load check (lib_hd), same box.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "resize or cubic or channel_sums" \
    > gpurun_out/n_tests.log 2>&1 || { tail -30 gpurun_out/n_tests.log; exit 1; }
tail -1 gpurun_out/n_tests.log
for rep in 1 2 3; do
  for l in lib lib_hd; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op resize_normalize --iters 30 | sed "s/^/$l /" || exit 1
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op cubic --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
