#!/bin/bash
# Round-5 run am: area_lane_kernel exchange-path loads non-temporal (lib_al2) vs default.
set -o pipefail
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in lib lib_al2; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op resize_other --iters 40 --only area_1080p_640 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
