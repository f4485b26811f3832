#!/bin/bash
# Round-5 run ad: gray_x_kernel (a wave per 64 units of a row, LDS exchange,
# 1-KiB stores) -- colour-code tests, kbench against gray_kernel.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "cvt_color" > gpurun_out/ad_tests.log 2>&1 || { tail -60 gpurun_out/ad_tests.log; exit 1; }
tail -2 gpurun_out/ad_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op cvt_cv --iters 30 --sweep 'RESIZE_DIRECT=0,2' || exit 1
done 2>&1 | grep -v amdgpu.ids
