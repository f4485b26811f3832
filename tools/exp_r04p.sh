#!/bin/bash
# Round-4 run 15: Lanczos u8 windows in flight per wave (3 / 4 / 6 / 8), same box.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
for l in lib_ld1 lib_ld2 lib_ld3; do
  VACV_LIB_DIR=$K/$l timeout -k 10 200 python3 -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k lanczos > gpurun_out/p_tests_$l.log 2>&1 || { tail -20 gpurun_out/p_tests_$l.log; exit 1; }
  tail -1 gpurun_out/p_tests_$l.log
done
for rep in 1 2; do
  for l in lib_ld1 lib_ld2 lib_ld3; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op lanczos --only u8 --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
