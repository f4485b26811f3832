#!/bin/bash
# Round-4 run 18: Lanczos waves per workgroup (4 / 2 / 1: LDS per workgroup
# 24 / 12 / 6 KiB, so more workgroups per CU), same box.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
for l in lib_lw2 lib_lw1; do
  VACV_LIB_DIR=$K/$l timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k lanczos > gpurun_out/w_tests_$l.log 2>&1 || { tail -20 gpurun_out/w_tests_$l.log; exit 1; }
  tail -1 gpurun_out/w_tests_$l.log
done
for rep in 1 2; do
  for l in lib lib_lw2 lib_lw1; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op lanczos --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
