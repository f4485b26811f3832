#!/bin/bash
# Round-5 run af: staged-run Lanczos, windows in flight D = 2 / 4 / 8.
set -o pipefail
export TMPDIR=/tmp
for rep in 1 2; do
  for v in lib lib_lzd8 lib_lzd2; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
