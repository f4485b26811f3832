#!/bin/bash
# Round-5 run v: warp_exp_kernel without its two per-frame barriers
# (VACV_RING_DBG=32: wrong results, timing only) against the product build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_dbg32; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
