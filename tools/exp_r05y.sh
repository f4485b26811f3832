#!/bin/bash
# Round-5 run y: warp_exp_kernel tap-read prefetch (pf2: 2-pixel groups, two
# register sets; pf1: 1-pixel groups, two sets) against the product build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_pf2 lib_pf1; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
