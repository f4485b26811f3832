#!/bin/bash
# Round-5 run z: area_lane_kernel (u8 INTER_AREA 3x3 over BGR / BGRA) --
# INTER_AREA tests, kbench against the LDS column-sum kernel (AREA_KERNEL=3).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "area or nearest" > gpurun_out/z_tests.log 2>&1 || { tail -60 gpurun_out/z_tests.log; exit 1; }
tail -2 gpurun_out/z_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op resize_other --iters 30 --sweep 'AREA_KERNEL=0,3' || exit 1
done 2>&1 | grep -v amdgpu.ids | grep area
