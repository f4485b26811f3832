#!/bin/bash
# Round-5 run b: warp_exp_kernel v2 (compact spans, two raw slots, compact
# 4-byte image): the warp tests, then kbench warp: exp (default tiles), exp
# with the other tile height, ring (VACV_WARP_KERNEL=6).
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp" > gpurun_out/b_tests.log 2>&1 || { tail -60 gpurun_out/b_tests.log; exit 1; }
tail -3 gpurun_out/b_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/exp /" || exit 1
  VACV_WARP_TILE_H=16 timeout -k 10 120 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/exp_th16 /" || exit 1
  VACV_WARP_TILE_H=32 timeout -k 10 120 python3 tools/kbench.py --op warp --only normalize --iters 30 | sed "s/^/exp_th32 /" || exit 1
  VACV_WARP_KERNEL=6 timeout -k 10 120 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/ring /" || exit 1
done 2>&1 | grep -v amdgpu.ids | grep -v nearest
