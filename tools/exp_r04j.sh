#!/bin/bash
# Round-4 run 10: Lanczos vertical pass by ring slot (default) vs in tap order
# (lib_ls0), same box, alternating.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lanczos" \
    > gpurun_out/j_tests.log 2>&1 || { tail -30 gpurun_out/j_tests.log; exit 1; }
tail -1 gpurun_out/j_tests.log
for rep in 1 2 3; do
  for l in lib lib_ls0; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op lanczos --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/j_variants.txt
