#!/bin/bash
# Round-5 run aq: area_u8_unit_kernel with packed outputs through the wave's
# LDS slice (lib) vs the lanes' own stores (lib_ap0): area tests, kbench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "area or nearest or random_geometry_interpolations" > gpurun_out/aq_tests.log 2>&1 || { tail -60 gpurun_out/aq_tests.log; exit 1; }
tail -2 gpurun_out/aq_tests.log
for rep in 1 2 3; do
  for v in lib lib_ap0; do
    VACV_LIB_DIR=arm-neon-opencv_amd/$v timeout -k 10 150 python3 tools/kbench.py --op resize_other --iters 40 --only area | sed "s/^/$v /" || exit 1
  done
done 2>&1 | grep -v amdgpu.ids
