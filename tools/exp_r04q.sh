#!/bin/bash
# Round-4 run 16: warp ring kernel occupancy / tap-group variants and the
# tile-height x slots sweep, same box.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
for rep in 1 2; do
  for l in lib lib_wpe6 lib_g1 lib_g1w6 lib_g4; do
    timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op warp --only rot15_u8 --iters 30 | grep -v nearest | sed "s/^/$l /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python3 tools/kbench.py --op warp --only rot15_u8 --iters 30 --sweep 'WARP_TILE_H=16,32;WARP_SLOTS=2,3' 2>&1 | grep -v "amdgpu.ids\|nearest"
