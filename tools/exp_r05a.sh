#!/bin/bash
# Round-5 run a: the round's new GPU tests (warp_exp_kernel on every warp
# test, Lanczos w < 8, the cubic gather kernel's fence, bench main() with two
# ranks on one GPU), then the warp kbench: warp_exp_kernel (default) vs the
# ring kernel (VACV_WARP_KERNEL=6) vs write-back ring stores (lib_sa0).
set -o pipefail
export TMPDIR=/tmp
K=arm-neon-opencv_amd
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_bench.py -x -v --timeout 300 --timeout-method thread \
    -m gpu -k "warp or lanczos4 or cubic_direct_and_staged or two_ranks_on_one_gpu" > gpurun_out/a_tests.log 2>&1 \
    || { tail -60 gpurun_out/a_tests.log; exit 1; }
tail -3 gpurun_out/a_tests.log
for rep in 1 2; do
  timeout -k 10 120 python3 tools/kbench_lib.py $K/lib --op warp --iters 30 | sed "s/^/exp /" || exit 1
  VACV_WARP_KERNEL=6 timeout -k 10 120 python3 tools/kbench_lib.py $K/lib --op warp --iters 30 | sed "s/^/ring /" || exit 1
  VACV_WARP_KERNEL=6 timeout -k 10 120 python3 tools/kbench_lib.py $K/lib_sa0 --op warp --iters 30 | sed "s/^/ring_sa0 /" || exit 1
done 2>&1 | grep -v amdgpu.ids
