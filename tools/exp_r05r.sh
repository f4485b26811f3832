#!/bin/bash
# Round-5 run r: lanczos_u8_kernel (register ring) -- Lanczos tests, kbench
# against the LDS-ring kernel (LANCZOS_KERNEL=1) and the D=2 build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -m gpu -k "lanczos or random_geometry_interpolations" > gpurun_out/r_tests.log 2>&1 || { tail -60 gpurun_out/r_tests.log; exit 1; }
tail -2 gpurun_out/r_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 --sweep 'LANCZOS_KERNEL=0,1' | sed "s/^/d4 /" || exit 1
  VACV_LIB_DIR=arm-neon-opencv_amd/lib_lzr2 timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 | sed "s/^/d2 /" || exit 1
done 2>&1 | grep -v amdgpu.ids
