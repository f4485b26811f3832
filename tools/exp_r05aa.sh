#!/bin/bash
# Round-5 run aa: area_lane_kernel output rows per wave (RG 1 / 2 / 4 / 8,
# the next row's loads in flight); INTER_AREA tests on the default (RG 4).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "area or nearest" > gpurun_out/aa_tests.log 2>&1 || { tail -60 gpurun_out/aa_tests.log; exit 1; }
tail -2 gpurun_out/aa_tests.log
for rep in 1 2; do
  for v in lib lib_rg1 lib_rg2 lib_rg8; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op resize_other --iters 30 --only area_1080p_640 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
