#!/bin/bash
# Round-5 run c: warp_exp_kernel diagnosis builds (tools/kbench_lib.py):
# dbg1 DMA only, dbg2 no DMA, dbg8 no output stores, dbg4 conflict-free taps.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
for rep in 1 2; do
  for l in lib lib_dbg1 lib_dbg2 lib_dbg8 lib_dbg4; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op warp --only rot15_u8 --iters 30 | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
