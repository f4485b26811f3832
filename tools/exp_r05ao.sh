#!/bin/bash
# Round-5 run ao: match_corr_mfma_kernel with double-buffered operand sets
# (loads in flight during the MFMAs) -- match tests, kbench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "match" > gpurun_out/ao_tests.log 2>&1 || { tail -60 gpurun_out/ao_tests.log; exit 1; }
tail -2 gpurun_out/ao_tests.log
for rep in 1 2; do
  timeout -k 10 150 python3 tools/kbench.py --op match --iters 20 || exit 1
done 2>&1 | grep -v amdgpu.ids
