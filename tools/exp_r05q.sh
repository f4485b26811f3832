#!/bin/bash
# Round-5 run q: Lanczos diagnosis builds (VACV_LZ_DBG 1 no horizontal
# arithmetic, 2 no window loads, 4 one-lane dropped stores, 8 no output stores)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in 1 2; do
  for v in lib lib_lzb1 lib_lzb2 lib_lzb4 lib_lzb8; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
