#!/bin/bash
# Round-5 run u: lanczos_u8_kernel occupancy (waves_per_eu 6) and band size
# (8-row bands, 128K tasks) variants.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_lzw6 lib_lzm8 lib_lzm8w6; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
