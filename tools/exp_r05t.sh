#!/bin/bash
# Round-5 run t: lanczos_u8_kernel with the emit outside the loop (no hoisted
# sign extensions) and 32K tasks; 64K-task build; tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -m gpu -k "lanczos or random_geometry_interpolations" > gpurun_out/t_tests.log 2>&1 || { tail -60 gpurun_out/t_tests.log; exit 1; }
tail -2 gpurun_out/t_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/lib /" || exit 1
  VACV_LIB_DIR=arm-neon-opencv_amd/lib_lzt64 timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/t64 /" || exit 1
done 2>&1 | grep -v amdgpu.ids
