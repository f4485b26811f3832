#!/bin/bash
# Round-5 run j: fp32-output warps with direct 12-byte stores (lib_f0) vs the
# LDS exchange: warp tests on lib_f0, kbench normalize both, 16 / 32-row tiles.
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
mkdir -p gpurun_out
VACV_LIB_DIR=$K/lib_f0 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp" > gpurun_out/j_tests.log 2>&1 || { tail -60 gpurun_out/j_tests.log; exit 1; }
tail -2 gpurun_out/j_tests.log
for rep in 1 2; do
  for l in lib lib_f0; do
    for th in 16 32; do
      VACV_WARP_TILE_H=$th timeout -k 10 120 python3 tools/kbench_lib.py $K/$l --op warp --only normalize --iters 30 | sed "s/^/$l th$th /" || exit 1
    done
  done
done 2>&1 | grep -v amdgpu.ids
