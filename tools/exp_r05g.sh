#!/bin/bash
# Round-5 run g: relay with its reads batched: warp tests, kbench exp
# (default, 8 / 32 frames per workgroup, 16-row tiles), phase clocks.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp" > gpurun_out/g_tests.log 2>&1 || { tail -60 gpurun_out/g_tests.log; exit 1; }
tail -2 gpurun_out/g_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op warp --only _u8 --iters 30 | sed "s/^/exp /" || exit 1
  VACV_WARP_FRAMES=8 timeout -k 10 120 python3 tools/kbench.py --op warp --only rot15_u8 --iters 30 | sed "s/^/exp_kf8 /" || exit 1
  VACV_WARP_FRAMES=32 timeout -k 10 120 python3 tools/kbench.py --op warp --only rot15_u8 --iters 30 | sed "s/^/exp_kf32 /" || exit 1
  VACV_WARP_TILE_H=16 timeout -k 10 120 python3 tools/kbench.py --op warp --only rot15_u8 --iters 30 | sed "s/^/exp_th16 /" || exit 1
done 2>&1 | grep -v amdgpu.ids | grep -v nearest
timeout -k 10 120 python3 tools/warp_prof.py $K/lib_dbg16 > gpurun_out/prof16g.txt 2>&1 || exit 1
grep expprof gpurun_out/prof16g.txt | tail -8
