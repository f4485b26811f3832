#!/bin/bash
# Round-5 run ab: area_lane_kernel with lane-contiguous loads + LDS exchange
# (lib_ax1, VACV_AREA_XCH=1) against the per-lane windows (lib): tests on
# the variant, kbench both.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VACV_LIB_DIR=arm-neon-opencv_amd/lib_ax1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "area or nearest" > gpurun_out/ab_tests.log 2>&1 || { tail -60 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
for rep in 1 2; do
  for v in lib lib_ax1; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op resize_other --iters 30 --only area_1080p_640 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
