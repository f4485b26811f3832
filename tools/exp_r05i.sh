#!/bin/bash
# Round-5 run i: exact per-row spans (LDS min / max) and INTER_NEAREST on
# warp_exp_kernel: warp tests, kbench warp (all cases) default vs ring / gather.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp" > gpurun_out/i_tests.log 2>&1 || { tail -60 gpurun_out/i_tests.log; exit 1; }
tail -2 gpurun_out/i_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench.py --op warp --iters 30 | sed "s/^/exp /" || exit 1
  VACV_WARP_KERNEL=6 timeout -k 10 120 python3 tools/kbench.py --op warp --only _u8 --iters 30 | sed "s/^/ring /" || exit 1
done 2>&1 | grep -v amdgpu.ids
