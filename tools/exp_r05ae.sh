#!/bin/bash
# Round-5 run ae: lanczos_u8_kernel with staged source runs (lane-contiguous
# 16-byte loads + the wave's LDS slice) against per-lane windows
# (LANCZOS_KERNEL=2); Lanczos tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "lanczos or random_geometry_interpolations" > gpurun_out/ae_tests.log 2>&1 || { tail -60 gpurun_out/ae_tests.log; exit 1; }
tail -2 gpurun_out/ae_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op lanczos --iters 30 --sweep 'LANCZOS_KERNEL=0,2' || exit 1
done 2>&1 | grep -v amdgpu.ids
